// Young-lottery histogram (build-defined row E2) for gfx950.
//
// The reference only has the Monte Carlo panel; BASELINE's stationary Table II sweep
// needs the distribution iteration of the stationary household:
//   hist_lottery_kernel   (s, j) -> a' = m - c_s(m), m = R a_j + w l_s, lottery
//                         (lo, weight on lo) onto a_grid; policy search is the
//                         wave-cooperative monotone search of the EGM kernel.
//   hist_push_kernel      T[s][d] += w * mass[s][j] for d in {lo, lo + 1}:
//                         wave-aggregated fp64 atomics -- lanes are sorted by lo
//                         (monotone savings policy), so a segmented shuffle-scan
//                         merges equal destinations and only segment tails add.
//   hist_mix_kernel       mass'[s'][j] = sum_s P[s,s'] T[s][j] (one lane per j,
//                         S x S register contraction), sup-norm change, T zeroed.
//   hist_K_kernel         K = sum mass * a (fixed order) after convergence.
#include "common.h"
#include "internal.h"

#include <algorithm>
#include <cstring>

namespace aiy {

constexpr int kSlots = 4;  // per-calibration convergence words (3 distance slots + flag)

__device__ __forceinline__ int upper_bound(const double* __restrict__ x, int lo, int hi, double q) {
  while (lo < hi) {
    int mid = lo + ((hi - lo) >> 1);
    if (x[mid] <= q) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void hist_lottery_kernel(int S, int n_a, const double* __restrict__ m_tab,
                                                           const double* __restrict__ c_tab,
                                                           const double* __restrict__ a_grid,
                                                           const double* __restrict__ R, const double* __restrict__ w,
                                                           const double* __restrict__ lab, int* __restrict__ lo,
                                                           double* __restrict__ wlo) {
  const int cal = blockIdx.z, s = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = j < n_a;
  const double* ag = a_grid + (size_t)cal * n_a;
  const double aj = ag[active ? j : n_a - 1];
  const double q = R[cal] * aj + w[cal] * lab[(size_t)cal * S + s];
  const size_t row = ((size_t)cal * S + s) * (n_a + 1);
  const double c = interp_row_wave(m_tab + row, c_tab + row, n_a, q, active);
  const double ap = q - c;
  int d = upper_bound(ag, 0, n_a, ap) - 1;        // searchsorted(a_grid, a', 'right') - 1
  d = d < 0 ? 0 : (d > n_a - 2 ? n_a - 2 : d);
  double wl = (ag[d + 1] - ap) / (ag[d + 1] - ag[d]);
  wl = wl < 0.0 ? 0.0 : (wl > 1.0 ? 1.0 : wl);
  if (active) {
    const size_t o = ((size_t)cal * S + s) * n_a + j;
    lo[o] = d;
    wlo[o] = wl;
  }
}

// Segmented (runs of equal key in adjacent active lanes) inclusive sum, Hillis-Steele
// style; returns true on the lane that closes its run (its sum is the run total).
// Every lane of the wave must call it.
__device__ __forceinline__ bool seg_sum(int key, bool active, double& v) {
  const int lane = threadIdx.x & (kWave - 1);
  const int act = active ? 1 : 0;
  const int pk = __shfl_up(key, 1, kWave);
  const int pa = __shfl_up(act, 1, kWave);
  const bool head = lane == 0 || !active || !pa || pk != key;
  int start = head ? lane : 0;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int s2 = __shfl_up(start, o, kWave);
    if (lane >= o) start = max(start, s2);
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double v2 = __shfl_up(v, o, kWave);
    if (lane - o >= start) v += v2;
  }
  const int nk = __shfl_down(key, 1, kWave);
  const int na = __shfl_down(act, 1, kWave);
  return active && (lane == kWave - 1 || !na || nk != key);
}

__global__ __launch_bounds__(256) void hist_push_kernel(int S, int n_a, const int* __restrict__ lo,
                                                        const double* __restrict__ wlo,
                                                        const double* __restrict__ mass, double* __restrict__ T,
                                                        const unsigned long long* dslots, int iter, double tol) {
  const int cal = blockIdx.z, s = blockIdx.y;
  if (dslots && iter >= 2) {   // same sticky protocol as the EGM solve (egm.hip)
    if (load_u64_agent(&dslots[cal * kSlots + 3]) != 0ull) return;
    const double dprev = __longlong_as_double((long long)load_u64_agent(&dslots[cal * kSlots + (iter - 1) % 3]));
    if (!(dprev >= tol)) return;
  }
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = j < n_a;
  const size_t o = ((size_t)cal * S + s) * n_a + (active ? j : 0);
  const int d = active ? lo[o] : -1;
  const double mj = active ? mass[o] : 0.0;
  const double wl = active ? wlo[o] : 0.0;
  double* Trow = T + ((size_t)cal * S + s) * n_a;
  double vlo = wl * mj;
  double vhi = (1.0 - wl) * mj;
  if (seg_sum(d, active, vlo)) unsafeAtomicAdd(&Trow[d], vlo);
  if (seg_sum(d, active, vhi)) unsafeAtomicAdd(&Trow[d + 1], vhi);
}

template <int SMAX>
__global__ __launch_bounds__(256) void hist_mix_kernel(int S, int n_a, const double* __restrict__ P,
                                                       double* __restrict__ T, const double* __restrict__ mass,
                                                       double* __restrict__ mass_out, unsigned long long* dslots,
                                                       int* last_iter, int iter, double tol) {
  const int cal = blockIdx.y;
  if (dslots && iter >= 2) {   // same sticky protocol as the EGM solve (egm.hip)
    if (load_u64_agent(&dslots[cal * kSlots + 3]) != 0ull) return;
    const double dprev = __longlong_as_double((long long)load_u64_agent(&dslots[cal * kSlots + (iter - 1) % 3]));
    if (!(dprev >= tol)) {
      if (blockIdx.x == 0 && threadIdx.x == 0) store_u64_agent(&dslots[cal * kSlots + 3], 1ull);
      return;
    }
  }
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = j < n_a;
  const size_t base = (size_t)cal * S * n_a;
  double t[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    t[s] = 0.0;
    if (s < S && active) {
      t[s] = T[base + (size_t)s * n_a + j];
      T[base + (size_t)s * n_a + j] = 0.0;
    }
  }
  const double* Pc = P + (size_t)cal * S * S;
  double dmax = 0.0;
  for (int sp = 0; sp < S; ++sp) {
    double acc = 0.0;
#pragma unroll
    for (int s = 0; s < SMAX; ++s)
      if (s < S) acc += Pc[(size_t)s * S + sp] * t[s];
    if (active) {
      const size_t o = base + (size_t)sp * n_a + j;
      dmax = nan_max(dmax, fabs(acc - mass[o]));
      mass_out[o] = acc;
    }
  }
  if (dslots) {
    __shared__ double red[256 / kWave];
    dmax = wave_nan_max(dmax);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = dmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      double d = red[0];
      for (int w2 = 1; w2 < (int)(blockDim.x / kWave); ++w2) d = nan_max(d, red[w2]);
      atomicMax(&dslots[cal * kSlots + iter % 3], (unsigned long long)__double_as_longlong(d));
      if (blockIdx.x == 0) {
        store_u64_agent(&dslots[cal * kSlots + (iter + 1) % 3], 0ull);
        last_iter[cal] = iter;
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Fused lottery step (push + mix in one launch, no global atomics, no T buffer).
// With a monotone savings policy lo[s][j] is non-decreasing in j, so the sources that
// land in a destination tile [d0, d1) are one contiguous range per s:
//   jb[s][d] = first j with lo[s][j] >= d   (hist_range_kernel, once per lottery)
//   sources of the tile: j in [jb[s][d0 - 1], jb[s][d1])
// One workgroup per (tile of kHistTile destinations, calibration): the tile's sources
// of every s are flattened into one index space (adjacent lanes -> adjacent j, keys
// (s, d) sorted), pushed with the same vlo = w m, vhi = (1 - w) m products as
// hist_push_kernel through the segmented wave sum into LDS atomics, then mixed over s
// exactly as hist_mix_kernel (same order of the S x S contraction, same distance and
// sticky protocol).  HBM per point and iteration: lo 4 + w 8 + mass 8 + mass' 8 = 28 B
// (the mass re-read of the distance hits L2).
// ---------------------------------------------------------------------------------
constexpr int kHistTile = 256;
constexpr int kHistUnroll = 4;

__global__ __launch_bounds__(256) void hist_range_kernel(int S, int n_a, const int* __restrict__ lo,
                                                         int* __restrict__ jb, int* flag) {
  const int cal = blockIdx.z, s = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > n_a) return;   // j == n_a closes the row: d in (lo[n_a - 1], n_a] -> n_a
  const size_t r = (size_t)cal * S + s;
  const int* L = lo + r * n_a;
  int* J = jb + r * (n_a + 1);
  const int prev = j == 0 ? -1 : L[j - 1];
  const int cur = j == n_a ? n_a : L[j];
  if (cur < prev || cur > n_a) {   // not monotone: the push/mix pair runs instead
    atomicOr(flag, 1);
    return;
  }
  for (int d = prev + 1; d <= cur; ++d) J[d] = j;
}

template <int SMAX>
__global__ __launch_bounds__(256) void hist_step_kernel(int S, int n_a, const int* __restrict__ lo,
                                                        const double* __restrict__ wlo, const int* __restrict__ jb,
                                                        const double* __restrict__ P,
                                                        const double* __restrict__ mass,
                                                        double* __restrict__ mass_out, unsigned long long* dslots,
                                                        int* last_iter, int iter, double tol) {
  const int cal = blockIdx.y;
  if (dslots && iter >= 2) {   // same sticky protocol as hist_mix_kernel
    if (load_u64_agent(&dslots[cal * kSlots + 3]) != 0ull) return;
    const double dprev = __longlong_as_double((long long)load_u64_agent(&dslots[cal * kSlots + (iter - 1) % 3]));
    if (!(dprev >= tol)) {
      if (blockIdx.x == 0 && threadIdx.x == 0) store_u64_agent(&dslots[cal * kSlots + 3], 1ull);
      return;
    }
  }
  extern __shared__ double Tl[];   // [S][kHistTile], dynamic (S x 2 KB)
  __shared__ int s_off[SMAX + 1];
  __shared__ int s_jlo[SMAX];
  const int tid = threadIdx.x;
  const int d0 = blockIdx.x * kHistTile;
  const int d1 = min(d0 + kHistTile, n_a);
  const size_t rows = (size_t)cal * S;
  for (int q = tid; q < S * kHistTile; q += blockDim.x) Tl[q] = 0.0;
  if (tid < S) {
    const int* J = jb + (rows + tid) * (n_a + 1);
    const int a = J[d0 > 0 ? d0 - 1 : 0];
    s_jlo[tid] = a;
    s_off[tid + 1] = J[d1] - a;
  }
  __syncthreads();
  if (tid == 0) {
    s_off[0] = 0;
    for (int q = 0; q < S; ++q) s_off[q + 1] += s_off[q];
  }
  __syncthreads();
  const int total = s_off[S];
  for (int k0 = 0; k0 < total; k0 += kHistUnroll * (int)blockDim.x) {
    int key[kHistUnroll], ss[kHistUnroll], dd[kHistUnroll];
    double mj[kHistUnroll], wl[kHistUnroll];
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u) {
      const int k = k0 + u * (int)blockDim.x + tid;
      const bool act = k < total;
      int sl = 0, sh = S - 1;   // s with s_off[s] <= k < s_off[s + 1]
      while (sl < sh) {
        const int mid = (sl + sh + 1) >> 1;
        if (s_off[mid] <= k) sl = mid; else sh = mid - 1;
      }
      const size_t o = (rows + sl) * n_a + (act ? s_jlo[sl] + (k - s_off[sl]) : 0);
      ss[u] = sl;
      dd[u] = act ? lo[o] : -1;
      key[u] = act ? sl * (n_a + 1) + dd[u] : -1;
      mj[u] = act ? mass[o] : 0.0;
      wl[u] = act ? wlo[o] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kHistUnroll; ++u) {
      const bool act = key[u] >= 0;
      double vlo = wl[u] * mj[u];
      double vhi = (1.0 - wl[u]) * mj[u];
      double* Ts = Tl + ss[u] * kHistTile;
      const int d = dd[u];
      if (seg_sum(key[u], act, vlo) && d >= d0) atomicAdd(&Ts[d - d0], vlo);
      if (seg_sum(key[u], act, vhi) && d + 1 < d1) atomicAdd(&Ts[d + 1 - d0], vhi);
    }
  }
  __syncthreads();
  const int j = d0 + tid;
  const bool active = j < d1;
  const size_t base = rows * n_a;
  double t[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s) t[s] = (s < S) ? Tl[s * kHistTile + tid] : 0.0;
  const double* Pc = P + (size_t)cal * S * S;
  double dmax = 0.0;
  for (int sp = 0; sp < S; ++sp) {
    double acc = 0.0;
#pragma unroll
    for (int s = 0; s < SMAX; ++s)
      if (s < S) acc += Pc[(size_t)s * S + sp] * t[s];
    if (active) {
      const size_t o = base + (size_t)sp * n_a + j;
      dmax = nan_max(dmax, fabs(acc - mass[o]));
      mass_out[o] = acc;
    }
  }
  if (dslots) {
    __shared__ double red[256 / kWave];
    dmax = wave_nan_max(dmax);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = dmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      double d = red[0];
      for (int w2 = 1; w2 < (int)(blockDim.x / kWave); ++w2) d = nan_max(d, red[w2]);
      atomicMax(&dslots[cal * kSlots + iter % 3], (unsigned long long)__double_as_longlong(d));
      if (blockIdx.x == 0) {
        store_u64_agent(&dslots[cal * kSlots + (iter + 1) % 3], 0ull);
        last_iter[cal] = iter;
      }
    }
  }
}

// K = sum_{s, j} mass[s][j] a_j per calibration (one 1024-thread block each): per node
// the S masses summed in state order, times a_j, then a fixed-order block reduction.
// K = sum_{s, j} mass[s][j] a[j]: kKBlocks blocks per calibration over contiguous column
// ranges (one block per calibration read 10 MB through one CU: ~360 us at configs[4]), then the
// blocks' partials summed in block order -- a fixed order, independent of the timing.
constexpr int kKThreads = 256;
constexpr int kKBlocks = 64;
__global__ __launch_bounds__(kKThreads) void hist_K_kernel(int S, int n_a, const double* __restrict__ mass,
                                                           const double* __restrict__ a_grid,
                                                           double* __restrict__ part) {
  const int cal = blockIdx.y, b = blockIdx.x;
  const int per = (n_a + kKBlocks - 1) / kKBlocks;
  const int j0 = b * per, j1 = min(j0 + per, n_a);
  double acc = 0.0;
  const double* ag = a_grid + (size_t)cal * n_a;
  const double* mc = mass + (size_t)cal * S * n_a;
  for (int j = j0 + (int)threadIdx.x; j < j1; j += kKThreads) {
    double ms = 0.0;
    for (int s = 0; s < S; ++s) ms += mc[(size_t)s * n_a + j];
    acc += ms * ag[j];
  }
  __shared__ double red[kKThreads / kWave];
  acc = wave_sum_fixed(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double k = 0.0;
    for (int w = 0; w < kKThreads / kWave; ++w) k += red[w];
    part[(size_t)cal * kKBlocks + b] = k;
  }
}
__global__ void hist_K_sum_kernel(int n_cal, const double* __restrict__ part, double* __restrict__ K) {
  const int cal = blockIdx.x * blockDim.x + threadIdx.x;
  if (cal >= n_cal) return;
  double k = 0.0;
  for (int b = 0; b < kKBlocks; ++b) k += part[(size_t)cal * kKBlocks + b];
  K[cal] = k;
}
// K of every calibration into h->d_K[0, n_cal) (partials behind it)
static void launch_hist_K(aiy_handle* h, int n_cal, int S, int n_a, const double* mass, const double* a_grid,
                          hipStream_t st) {
  double* part = h->d_K + n_cal;
  hipLaunchKernelGGL(hist_K_kernel, dim3(kKBlocks, n_cal), dim3(kKThreads), 0, st, S, n_a, mass, a_grid, part);
  hipLaunchKernelGGL(hist_K_sum_kernel, dim3((n_cal + 63) / 64), dim3(64), 0, st, n_cal, (const double*)part, h->d_K);
}

static int32_t ensure_hist_scratch(aiy_handle* h, int n_cal) {
  if ((size_t)n_cal <= h->hist_cap) return AIY_OK;
  if (h->d_hdist) { (void)hipFree(h->d_hdist); (void)hipFree(h->d_K); (void)hipFree(h->d_hlast); }
  if (h->h_hdist) { (void)hipHostFree(h->h_hdist); (void)hipHostFree(h->h_K); (void)hipHostFree(h->h_hlast); }
  h->d_hdist = nullptr; h->d_K = nullptr; h->d_hlast = nullptr;
  h->h_hdist = nullptr; h->h_K = nullptr; h->h_hlast = nullptr; h->hist_cap = 0;
  AIY_HIP(h, hipMalloc((void**)&h->d_hdist, sizeof(unsigned long long) * kSlots * n_cal));
  AIY_HIP(h, hipMalloc((void**)&h->d_K, sizeof(double) * n_cal * (1 + kKBlocks)));   // K, then partials
  AIY_HIP(h, hipMalloc((void**)&h->d_hlast, sizeof(int) * (n_cal + 1)));   // + monotone flag
  AIY_HIP(h, hipHostMalloc((void**)&h->h_hdist, sizeof(unsigned long long) * kSlots * n_cal, hipHostMallocDefault));
  AIY_HIP(h, hipHostMalloc((void**)&h->h_K, sizeof(double) * n_cal, hipHostMallocDefault));
  AIY_HIP(h, hipHostMalloc((void**)&h->h_hlast, sizeof(int) * (n_cal + 1), hipHostMallocDefault));
  h->hist_cap = n_cal;
  return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_hist_lottery(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_a, const double* m_tab,
                                    const double* c_tab, const double* a_grid, const double* R, const double* w,
                                    const double* lab, int32_t* lo, double* wlo, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_cal < 1 || S < 1 || n_a < 2 || n_cal > 65535 || S > 65535) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (!m_tab || !c_tab || !a_grid || !R || !w || !lab || !lo || !wlo) return fail(h, AIY_ERR_ARG, "null pointer");
  AIY_HIP(h, hipSetDevice(h->device));
  dim3 grid((n_a + 255) / 256, S, n_cal);
  hipLaunchKernelGGL(hist_lottery_kernel, grid, dim3(256), 0, as_stream(stream), S, n_a, m_tab, c_tab, a_grid, R, w,
                     lab, lo, wlo);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_hist_solve(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_a, const int32_t* lo,
                                  const double* wlo, const double* P, const double* a_grid, double tol,
                                  int32_t max_iter, int32_t chunk, double* mass, double* work, double* K_out,
                                  int32_t* iters_out, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_cal < 1 || S < 1 || n_a < 2 || n_cal > 65535 || S > AIY_MAX_STATES) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (!lo || !wlo || !P || !a_grid || !mass || !work || !K_out || !iters_out) return fail(h, AIY_ERR_ARG, "null pointer");
  if (max_iter < 1) return fail(h, AIY_ERR_ARG, "max_iter must be >= 1");
  if (chunk <= 0) chunk = 64;
  AIY_HIP(h, hipSetDevice(h->device));
  int32_t rc = ensure_hist_scratch(h, n_cal);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  const size_t per = (size_t)n_cal * S * n_a;
  double* T = work;          // [n_cal][S][n_a] push accumulator (kept zero between iterations)
  double* alt = work + per;  // [n_cal][S][n_a] ping-pong partner of `mass`
  AIY_HIP(h, hipMemsetAsync(h->d_hdist, 0, sizeof(unsigned long long) * kSlots * n_cal, st));
  AIY_HIP(h, hipMemsetAsync(h->d_hlast, 0, sizeof(int) * (n_cal + 1), st));
  if (h->hist_resident && !h->hist_fused) {
    // the whole iteration in one device-resident launch (hist_resident.hip)
    for (hipEvent_t& e : h->hc_ev)
      if (!e) AIY_HIP(h, hipEventCreate(&e));
    rc = hist_solve_resident(h, n_cal, S, n_a, lo, wlo, P, tol, max_iter, mass, h->d_hlast, st);
    if (rc == AIY_OK) {
      launch_hist_K(h, n_cal, S, n_a, mass, a_grid, st);
      AIY_CHECK_LAUNCH(h);
      AIY_HIP(h, hipMemcpyAsync(h->h_hlast, h->d_hlast, sizeof(int) * n_cal, hipMemcpyDeviceToHost, st));
      AIY_HIP(h, hipMemcpyAsync(h->h_K, h->d_K, sizeof(double) * n_cal, hipMemcpyDeviceToHost, st));
      AIY_HIP(h, hipStreamSynchronize(st));
      for (int c = 0; c < n_cal; ++c) {
        iters_out[c] = h->h_hlast[c];
        K_out[c] = h->h_K[c];
      }
      return AIY_OK;
    }
    if (rc != AIY_ERR_UNSUPPORTED) return rc;
    AIY_HIP(h, hipMemsetAsync(h->d_hlast, 0, sizeof(int) * (n_cal + 1), st));   // push/mix below
  }
  // Fused path: the tile source ranges jb [n_cal][S][n_a + 1] (int) live in T's space.
  int* jb = reinterpret_cast<int*>(T);
  const size_t step_lds = (size_t)S * kHistTile * sizeof(double);
  bool fused = h->hist_fused && step_lds <= 128 * 1024;
  if (fused) {
    hipLaunchKernelGGL(hist_range_kernel, dim3((n_a + 1 + 255) / 256, S, n_cal), dim3(256), 0, st, S, n_a, lo, jb,
                       h->d_hlast + n_cal);
    AIY_CHECK_LAUNCH(h);
    AIY_HIP(h, hipMemcpyAsync(h->h_hlast + n_cal, h->d_hlast + n_cal, sizeof(int), hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipStreamSynchronize(st));
    fused = h->h_hlast[n_cal] == 0;   // every row monotone
  }
  if (!fused) AIY_HIP(h, hipMemsetAsync(T, 0, per * sizeof(double), st));
  auto step_fn = S <= 8 ? (const void*)hist_step_kernel<8>
                        : S <= 16 ? (const void*)hist_step_kernel<16>
                                  : S <= 32 ? (const void*)hist_step_kernel<32> : (const void*)hist_step_kernel<64>;
  if (fused && step_lds > 48 * 1024)
    AIY_HIP(h, hipFuncSetAttribute(step_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)step_lds));
  dim3 gstep((n_a + kHistTile - 1) / kHistTile, n_cal);
  dim3 gpush((n_a + 255) / 256, S, n_cal);
  dim3 gmix((n_a + 255) / 256, n_cal);
  int it = 1;
  while (true) {
    const int end = std::min(it + chunk, max_iter + 1);
    for (int k = it; k < end; ++k) {
      const double* src = (k & 1) ? mass : alt;   // iteration k reads buffer (k-1)%2, writes k%2
      double* dst = (k & 1) ? alt : mass;
      if (fused) {
        void* args[] = {(void*)&S, (void*)&n_a, (void*)&lo, (void*)&wlo, (void*)&jb, (void*)&P, (void*)&src,
                        (void*)&dst, (void*)&h->d_hdist, (void*)&h->d_hlast, (void*)&k, (void*)&tol};
        AIY_HIP(h, hipLaunchKernel(step_fn, gstep, dim3(256), args, step_lds, st));
        continue;
      }
      hipLaunchKernelGGL(hist_push_kernel, gpush, dim3(256), 0, st, S, n_a, lo, wlo, src, T, h->d_hdist, k, tol);
      if (S <= 8)
        hipLaunchKernelGGL(hist_mix_kernel<8>, gmix, dim3(256), 0, st, S, n_a, P, T, src, dst, h->d_hdist, h->d_hlast, k, tol);
      else if (S <= 16)
        hipLaunchKernelGGL(hist_mix_kernel<16>, gmix, dim3(256), 0, st, S, n_a, P, T, src, dst, h->d_hdist, h->d_hlast, k, tol);
      else if (S <= 32)
        hipLaunchKernelGGL(hist_mix_kernel<32>, gmix, dim3(256), 0, st, S, n_a, P, T, src, dst, h->d_hdist, h->d_hlast, k, tol);
      else
        hipLaunchKernelGGL(hist_mix_kernel<64>, gmix, dim3(256), 0, st, S, n_a, P, T, src, dst, h->d_hdist, h->d_hlast, k, tol);
    }
    AIY_CHECK_LAUNCH(h);
    AIY_HIP(h, hipMemcpyAsync(h->h_hlast, h->d_hlast, sizeof(int) * n_cal, hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipMemcpyAsync(h->h_hdist, h->d_hdist, sizeof(unsigned long long) * kSlots * n_cal, hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipStreamSynchronize(st));
    bool all = true;
    for (int c = 0; c < n_cal; ++c) {
      const int last = h->h_hlast[c];
      double d;
      unsigned long long b = h->h_hdist[c * kSlots + last % 3];
      std::memcpy(&d, &b, sizeof(d));
      all = all && ((last >= 1 && !(d >= tol)) || last >= max_iter);
    }
    it = end;
    if (all || it > max_iter) break;
  }
  // bring every calibration's final distribution into `mass`
  for (int c = 0; c < n_cal; ++c) {
    const int last = h->h_hlast[c];
    iters_out[c] = last;
    if (last & 1) {
      const size_t off = (size_t)c * S * n_a;
      AIY_HIP(h, hipMemcpyAsync(mass + off, alt + off, (size_t)S * n_a * sizeof(double), hipMemcpyDeviceToDevice, st));
    }
  }
  launch_hist_K(h, n_cal, S, n_a, mass, a_grid, st);
  AIY_CHECK_LAUNCH(h);
  AIY_HIP(h, hipMemcpyAsync(h->h_K, h->d_K, sizeof(double) * n_cal, hipMemcpyDeviceToHost, st));
  AIY_HIP(h, hipStreamSynchronize(st));
  for (int c = 0; c < n_cal; ++c) K_out[c] = h->h_K[c];
  return AIY_OK;
}

extern "C" int32_t aiy_hist_launch_stats(aiy_handle* h, double* ms_sum, int64_t* launches, int32_t reset) {
  if (!h) return AIY_ERR_ARG;
  if (ms_sum) *ms_sum = h->hc_ms_sum;
  if (launches) *launches = h->hc_launches;
  if (reset) {
    h->hc_ms_sum = 0.0;
    h->hc_launches = 0;
  }
  return AIY_OK;
}
