// EGM backward step for gfx950.
//
// One launch == one call of solve_Aiyagari (Aiyagari_Support.py:1423-1520) for every
// calibration of a batch.  Work decomposition (MI355X-first, not a translation of the
// reference's 4-D NumPy tiling):
//   * the reference tiles mNext/Mnext/R/P to [a, M, s, s'] (precompute_arrays,
//     Aiyagari_Support.py:906-1037) and evaluates every next-period marginal value 28x
//     (once per current state s).  Here a 256-thread block owns one (calibration, M node
//     k, tile of kTile = 64 asset nodes) and evaluates each
//     V[s'][i] = R[k,s'] * c_{s'}(m'(i,k,s'), M'[k,s'])^-rho exactly once.
//   * Phase 1: wave w handles next states s' = w, w + 4, ... for the 64 nodes of the
//     tile, one node per lane.  Within a wave the queries m' = R a_i + W l(s') are
//     increasing in the lane and all search the same two next-period rows (the M'
//     bracket is wave-uniform), so the log-bucket index lookups and the bracket
//     searches coalesce.  V goes to LDS [s'][i].
//   * Phase 2: wave w handles current states s = w, w + 4, ...: E[s][i] =
//     beta * sum_{s'} V[s'][i] P[s,s'] (AS:1485) in NumPy's pairwise order, V read from
//     LDS (conflict-free), P[s,:] wave-uniform; then c = E^(-1/rho), m = a + c
//     (AS:1490-1499), written row-contiguous in i (coalesced).  Node 0 is the
//     (1e-7, 1e-7) point (AS:1503-1504).
//   * In solve mode the HARK distance (max |dm|, |dc|) is reduced per block and folded
//     into a per-calibration slot with a 64-bit atomicMax on the bit pattern of the
//     non-negative double.
// Splitting over (s', i) instead of one thread per node gives 4x the waves and a
// 4x shorter dependent chain per lane (measured 1.0 ms -> see profiles/).
#include "common.h"
#include "internal.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace aiy {

constexpr int kEgmBlock = 256;
// Minimum waves per SIMD the cycle kernel is compiled for (register budget); tuning builds
// override it (tools/egm_time.py).
#ifndef AIY_EGM_WAVES_PER_EU
#define AIY_EGM_WAVES_PER_EU 6   // measured: 1 (4 by registers) 195, 5: 174, 6: 161 us per cycle
#endif
constexpr int kTile = 64;                     // asset nodes per block (one per lane)
constexpr int kEgmWaves = kEgmBlock / kWave;  // 4
// Per-calibration convergence words: 3 rotating distance slots x kSub sub-slots (block b
// folds into sub-slot b % kSub, so ~2 400 blocks do not serialise on one address), then
// the sticky converged flag.
constexpr int kSub = 32;
constexpr int kFlag = 3 * kSub;
constexpr int kSlots = 3 * kSub + 4;

struct EgmDev {
  int n_cal, S, n_M, n_a;
  const double* a_grid;
  const double* M_grid;
  const double* P;
  const double* R_next;
  const double* W_next;
  const double* M_next;
  const double* lab;
  const double* beta;
  const double* crra;
};

// Phase 1: V[s'][i] for s' = wave, wave + 4, ... (LOG: CRRA == 1 at compile time --
// with a runtime select the compiler evaluated the f64 pow unconditionally, measured
// 25k VALU instructions per wave).
template <bool TERMINAL, bool LOG>
__device__ __forceinline__ void egm_phase1(const EgmDev& A, const double* __restrict__ m_next,
                                           const double* __restrict__ c_next, const int* __restrict__ idx_next,
                                           int cal, int k, double a, bool active, double* Vs) {
  const int S = A.S, n_M = A.n_M, n_a = A.n_a, n1 = n_a + 1;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const double gam = A.crra[cal];
  const double* Rk = A.R_next + ((size_t)cal * n_M + k) * S;
  const double* Wk = A.W_next + ((size_t)cal * n_M + k) * S;
  const double* Mk = A.M_next + ((size_t)cal * n_M + k) * S;
  const double* lab = A.lab + (size_t)cal * S;
  const double* Mg = A.M_grid + (size_t)cal * n_M;
  const size_t tab_cal = (size_t)cal * S * n_M * n1;
  for (int sp = wave; sp < S; sp += kEgmWaves) {
    const double R = Rk[sp];
    const double q = R * a + Wk[sp] * lab[sp];  // mNextArray (AS:1024)
    double c;
    if constexpr (TERMINAL) {
      c = q * 1.0;  // IdentityFunction (AS:898)
    } else {
      const double* bm = m_next + tab_cal + (size_t)sp * n_M * n1;
      const double* bc = c_next + tab_cal + (size_t)sp * n_M * n1;
      const int* H0 = idx_next ? idx_next + ((size_t)cal * S + sp) * n_M * kIdxRow : nullptr;
      if (n_M == 1) {
        c = interp_row_idx(bm, bc, n_a, H0, q);
      } else {
        // LinearInterpOnInterp1D: y_pos = clip(searchsorted(Mgrid, M'), 1, n_M - 1)
        const double Mp = Mk[sp];
        int j = lower_bound(Mg, 0, n_M, Mp);
        j = j > n_M - 1 ? n_M - 1 : j;
        j = j < 1 ? 1 : j;
        const double alpha = (Mp - Mg[j - 1]) / (Mg[j] - Mg[j - 1]);
        const double f0 = interp_row_idx(bm + (size_t)(j - 1) * n1, bc + (size_t)(j - 1) * n1, n_a,
                                         H0 ? H0 + (size_t)(j - 1) * kIdxRow : nullptr, q);
        const double f1 = interp_row_idx(bm + (size_t)j * n1, bc + (size_t)j * n1, n_a,
                                         H0 ? H0 + (size_t)j * kIdxRow : nullptr, q);
        c = (1 - alpha) * f0 + alpha * f1;
      }
    }
    const double vP = LOG ? 1.0 / c : pow(c, -gam);  // MargValueFuncCRRA
    Vs[sp * kTile + lane] = active ? R * vP : 0.0;   // RnextArray * vPnext
  }
}

// Phase 2: outputs of current states s = wave, wave + 4, ...; returns the block-local
// part of the HARK distance.
template <int SMAX, bool LOG>
__device__ __forceinline__ double egm_phase2(const EgmDev& A, const double* __restrict__ m_next,
                                             const double* __restrict__ c_next, double* __restrict__ m_out,
                                             double* __restrict__ c_out, int cal, int k, int i, double a,
                                             bool active, bool track, const double* Vs, const double* Pl) {
  const int S = A.S, n_M = A.n_M, n1 = A.n_a + 1;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const double gam = A.crra[cal];
  const double beta = A.beta[cal];
  const size_t tab_cal = (size_t)cal * S * n_M * n1;
  double dmax = 0.0;
  for (int s = wave; s < S; s += kEgmWaves) {
    const double* Ps = Pl + s * S;
    const double sum = np_pairwise_sum<SMAX>(S, [&](int t) { return Vs[t * kTile + lane] * Ps[t]; });
    const double E = beta * sum;                              // EndOfPrdvP (AS:1485)
    const double c = LOG ? 1.0 / E : pow(E, -1.0 / gam);      // AS:1490
    const double m = a + c;                                   // AS:1499
    const size_t row = tab_cal + ((size_t)s * n_M + k) * n1;
    if (active) {
      m_out[row + i + 1] = m;
      c_out[row + i + 1] = c;
      if (track) dmax = nan_max(dmax, nan_max(fabs(m - m_next[row + i + 1]), fabs(c - c_next[row + i + 1])));
    }
    if (i == 0) {
      m_out[row] = kBorrowNode;
      c_out[row] = kBorrowNode;
    }
  }
  return dmax;
}

// Convergence protocol (solve mode, dist_slots != nullptr), per calibration 4 words:
// three rotating distance slots and a sticky "converged" flag.  Cycle n returns at
// once if the flag is set or if cycle n-1 met !(d > tol) (HARK: go = distance >
// tolerance; it then sets the flag), folds its own distance into slot n%3 and zeroes
// slot (n+1)%3 for cycle n+1.  Nothing is written after convergence, so slot
// (last % 3) keeps the final distance for the host.
template <int SMAX, bool TERMINAL>
__global__ __launch_bounds__(kEgmBlock, SMAX <= 32 ? AIY_EGM_WAVES_PER_EU : 1) void egm_cycle_kernel(EgmDev A, const double* __restrict__ m_next,
                                                              const double* __restrict__ c_next,
                                                              double* __restrict__ m_out,
                                                              double* __restrict__ c_out,
                                                              const int* __restrict__ idx_next, int cycle,
                                                              unsigned long long* dist_slots,
                                                              int* last_cycle, double tol) {
  const int cal = blockIdx.z;
  const int k = blockIdx.y;
  if (dist_slots != nullptr && cycle >= 3) {
    unsigned long long* slots = dist_slots + cal * kSlots;
    __shared__ int s_skip;
    if (threadIdx.x < kWave) {
      const bool done = load_u64_agent(&slots[kFlag]) != 0ull;   // converged earlier (sticky flag)
      double d = 0.0;
      if (threadIdx.x < kSub)
        d = __longlong_as_double((long long)load_u64_agent(&slots[((cycle - 1) % 3) * kSub + threadIdx.x]));
      d = wave_nan_max(d);
      if (threadIdx.x == 0) {
        const bool skip = done || !(d > tol);
        s_skip = skip ? 1 : 0;
        if (skip && !done && blockIdx.x == 0 && k == 0) store_u64_agent(&slots[kFlag], 1ull);
      }
    }
    __syncthreads();
    if (s_skip) return;
  }
  __shared__ double Vs[SMAX * kTile];
  __shared__ double Pl[SMAX * SMAX];
  const int S = A.S;
  const double* Pc = A.P + (size_t)cal * S * S;
  for (int q = threadIdx.x; q < S * S; q += blockDim.x) Pl[q] = Pc[q];
  const int i = blockIdx.x * kTile + (threadIdx.x & (kWave - 1));
  const bool active = i < A.n_a;
  const double a = A.a_grid[(size_t)cal * A.n_a + (active ? i : A.n_a - 1)];
  const bool track = (dist_slots != nullptr) && cycle >= 2;
  const bool log_util = A.crra[cal] == 1.0;   // block-uniform: one of two straight-line bodies
  if (log_util) egm_phase1<TERMINAL, true>(A, m_next, c_next, idx_next, cal, k, a, active, Vs);
  else egm_phase1<TERMINAL, false>(A, m_next, c_next, idx_next, cal, k, a, active, Vs);
  __syncthreads();
  double dmax;
  if (log_util) dmax = egm_phase2<SMAX, true>(A, m_next, c_next, m_out, c_out, cal, k, i, a, active, track, Vs, Pl);
  else dmax = egm_phase2<SMAX, false>(A, m_next, c_next, m_out, c_out, cal, k, i, a, active, track, Vs, Pl);

  if (dist_slots != nullptr) {
    if (track) {
      __shared__ double red[kEgmWaves];
      dmax = wave_nan_max(dmax);
      if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = dmax;
      __syncthreads();
      if (threadIdx.x == 0) {
        double d = red[0];
        for (int w = 1; w < kEgmWaves; ++w) d = nan_max(d, red[w]);
        const int b = blockIdx.x + gridDim.x * blockIdx.y;
        atomicMax(&dist_slots[cal * kSlots + (cycle % 3) * kSub + (b % kSub)],
                  (unsigned long long)__double_as_longlong(d));
      }
    }
    if (blockIdx.x == 0 && k == 0) {
      if (threadIdx.x < kSub) store_u64_agent(&dist_slots[cal * kSlots + ((cycle + 1) % 3) * kSub + threadIdx.x], 0ull);
      if (threadIdx.x == 0) last_cycle[cal] = cycle;
    }
  }
}

// cFunc[state](m, M) for arbitrary queries (HARK LinearInterpOnInterp1D scalar-M path).
__global__ void policy_eval_kernel(int S, int n_M, int n_a, const double* __restrict__ m_tab,
                                   const double* __restrict__ c_tab, const double* __restrict__ Mg,
                                   const int* __restrict__ state, const double* __restrict__ mq,
                                   const double* __restrict__ Mq, long long n, double* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int s = state[t];
  const int n1 = n_a + 1;
  const double q = mq[t];
  if (s < 0 || s >= S) { out[t] = __builtin_nan(""); return; }
  const double* bm = m_tab + (size_t)s * n_M * n1;
  const double* bc = c_tab + (size_t)s * n_M * n1;
  if (n_M == 1) { out[t] = interp_row(bm, bc, n_a, q); return; }
  const double M = Mq[t];
  int j = lower_bound(Mg, 0, n_M, M);
  j = j > n_M - 1 ? n_M - 1 : j;
  j = j < 1 ? 1 : j;
  const double alpha = (M - Mg[j - 1]) / (Mg[j] - Mg[j - 1]);
  const double f0 = interp_row(bm + (size_t)(j - 1) * n1, bc + (size_t)(j - 1) * n1, n_a, q);
  const double f1 = interp_row(bm + (size_t)j * n1, bc + (size_t)j * n1, n_a, q);
  out[t] = (1 - alpha) * f0 + alpha * f1;
}

// Host: the distance of cycle `last` = max over its sub-slots (NaN-propagating).
static double slot_max(const unsigned long long* slots, int last) {
  double d = 0.0;
  for (int q = 0; q < kSub; ++q) {
    double v;
    unsigned long long b = slots[(last % 3) * kSub + q];
    std::memcpy(&v, &b, sizeof(v));
    d = (v != v || v > d) ? v : d;
  }
  return d;
}

static int32_t check_egm(aiy_handle* h, const aiy_egm_dims* d, const aiy_egm_inputs* in) {
  if (!h) return AIY_ERR_ARG;
  if (!d || !in) return fail(h, AIY_ERR_ARG, "null dims/inputs");
  if (d->n_cal < 1 || d->S < 1 || d->n_M < 1 || d->n_a < 2)
    return fail(h, AIY_ERR_ARG, "bad dims n_cal=%d S=%d n_M=%d n_a=%d", d->n_cal, d->S, d->n_M, d->n_a);
  if (d->S > AIY_MAX_STATES) return fail(h, AIY_ERR_UNSUPPORTED, "S=%d exceeds %d", d->S, AIY_MAX_STATES);
  if (d->n_cal > 65535 || d->n_M > 65535) return fail(h, AIY_ERR_UNSUPPORTED, "grid too large");
  if (!in->a_grid || !in->P || !in->R_next || !in->W_next || !in->lab || !in->beta || !in->crra)
    return fail(h, AIY_ERR_ARG, "null input array");
  if (d->n_M > 1 && (!in->M_grid || !in->M_next)) return fail(h, AIY_ERR_ARG, "null M_grid/M_next");
  return AIY_OK;
}

static EgmDev to_dev(const aiy_egm_dims* d, const aiy_egm_inputs* in) {
  EgmDev A;
  A.n_cal = d->n_cal; A.S = d->S; A.n_M = d->n_M; A.n_a = d->n_a;
  A.a_grid = in->a_grid; A.M_grid = in->M_grid; A.P = in->P; A.R_next = in->R_next;
  A.W_next = in->W_next; A.M_next = in->M_next; A.lab = in->lab; A.beta = in->beta; A.crra = in->crra;
  return A;
}

template <bool TERM>
static void launch_cycle_t(const EgmDev& A, const double* mn, const double* cn, double* mo, double* co,
                           const int* ix, int cycle, unsigned long long* ds, int* lc, double tol, hipStream_t st) {
  dim3 grid((A.n_a + kTile - 1) / kTile, A.n_M, A.n_cal);
  dim3 block(kEgmBlock);
  if (A.S <= 8)
    hipLaunchKernelGGL((egm_cycle_kernel<8, TERM>), grid, block, 0, st, A, mn, cn, mo, co, ix, cycle, ds, lc, tol);
  else if (A.S <= 16)
    hipLaunchKernelGGL((egm_cycle_kernel<16, TERM>), grid, block, 0, st, A, mn, cn, mo, co, ix, cycle, ds, lc, tol);
  else if (A.S <= 32)
    hipLaunchKernelGGL((egm_cycle_kernel<32, TERM>), grid, block, 0, st, A, mn, cn, mo, co, ix, cycle, ds, lc, tol);
  else
    hipLaunchKernelGGL((egm_cycle_kernel<64, TERM>), grid, block, 0, st, A, mn, cn, mo, co, ix, cycle, ds, lc, tol);
}

static void launch_cycle(const EgmDev& A, const double* mn, const double* cn, double* mo, double* co, const int* ix,
                         int cycle, unsigned long long* ds, int* lc, double tol, hipStream_t st) {
  if (mn == nullptr) launch_cycle_t<true>(A, mn, cn, mo, co, nullptr, cycle, ds, lc, tol, st);
  else launch_cycle_t<false>(A, mn, cn, mo, co, ix, cycle, ds, lc, tol, st);
}

static int32_t ensure_egm_index(aiy_handle* h, size_t ints) {
  if (ints <= h->egm_idx_cap) return AIY_OK;
  if (h->d_egm_idx) (void)hipFree(h->d_egm_idx);
  h->d_egm_idx = nullptr;
  h->egm_idx_cap = 0;
  AIY_HIP(h, hipMalloc((void**)&h->d_egm_idx, ints * sizeof(int)));
  h->egm_idx_cap = ints;
  return AIY_OK;
}

static int32_t ensure_egm_scratch(aiy_handle* h, int n_cal) {
  if ((size_t)n_cal <= h->egm_cap) return AIY_OK;
  if (h->d_dist) { (void)hipFree(h->d_dist); (void)hipFree(h->d_last); }
  if (h->h_dist) { (void)hipHostFree(h->h_dist); (void)hipHostFree(h->h_last); }
  h->d_dist = nullptr; h->d_last = nullptr; h->h_dist = nullptr; h->h_last = nullptr; h->egm_cap = 0;
  AIY_HIP(h, hipMalloc((void**)&h->d_dist, sizeof(unsigned long long) * kSlots * n_cal));
  AIY_HIP(h, hipMalloc((void**)&h->d_last, sizeof(int) * n_cal));
  AIY_HIP(h, hipHostMalloc((void**)&h->h_dist, sizeof(unsigned long long) * kSlots * n_cal, hipHostMallocDefault));
  AIY_HIP(h, hipHostMalloc((void**)&h->h_last, sizeof(int) * n_cal, hipHostMallocDefault));
  h->egm_cap = n_cal;
  return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_egm_step(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in,
                                const double* m_next, const double* c_next, double* m_out, double* c_out,
                                aiy_stream stream) {
  int32_t rc = check_egm(h, dims, in);
  if (rc) return rc;
  if ((m_next == nullptr) != (c_next == nullptr)) return fail(h, AIY_ERR_ARG, "m_next/c_next must both be set or NULL");
  if (!m_out || !c_out) return fail(h, AIY_ERR_ARG, "null output");
  AIY_HIP(h, hipSetDevice(h->device));
  EgmDev A = to_dev(dims, in);
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  const long long rows = (long long)dims->n_cal * dims->S * dims->n_M;
  const int* ix = nullptr;
  if (m_next) {
    rc = ensure_egm_index(h, (size_t)rows * kIdxRow);
    if (rc) return rc;
    rc = launch_build_index(h, m_next, rows, dims->n_a + 1, h->d_egm_idx, st);
    if (rc) return rc;
    ix = h->d_egm_idx;
  }
  launch_cycle(A, m_next, c_next, m_out, c_out, ix, 0, nullptr, nullptr, 0.0, st);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

int32_t aiy_egm_solve_impl(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in, double tol,
                              int32_t max_cycles, int32_t chunk, const double* m_init, const double* c_init,
                              double* work_m, double* work_c, double* m_out, double* c_out, int32_t* cycles_out,
                              double* dist_out, aiy_stream stream) {
  int32_t rc = check_egm(h, dims, in);
  if (rc) return rc;
  if (!work_m || !work_c || !m_out || !c_out || !cycles_out || !dist_out) return fail(h, AIY_ERR_ARG, "null buffer");
  if (max_cycles < 1) return fail(h, AIY_ERR_ARG, "max_cycles must be >= 1");
  if (chunk <= 0) chunk = 32;
  AIY_HIP(h, hipSetDevice(h->device));
  rc = ensure_egm_scratch(h, dims->n_cal);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  const int n_cal = dims->n_cal;
  const size_t per_cal = (size_t)dims->S * dims->n_M * (dims->n_a + 1);
  const size_t buf = per_cal * n_cal;
  EgmDev A = to_dev(dims, in);
  const long long rows = (long long)n_cal * dims->S * dims->n_M;
  const size_t idx_per = (size_t)rows * kIdxRow;
  rc = ensure_egm_index(h, 2 * idx_per);
  if (rc) return rc;
  AIY_HIP(h, hipMemsetAsync(h->d_dist, 0, sizeof(unsigned long long) * kSlots * n_cal, st));
  AIY_HIP(h, hipMemsetAsync(h->d_last, 0, sizeof(int) * n_cal, st));
  const bool warm = m_init != nullptr;
  if (warm) {   // cycle 0 = the caller's tables (ping-pong slot 0) and their search index
    AIY_HIP(h, hipMemcpyAsync(work_m, m_init, buf * sizeof(double), hipMemcpyDeviceToDevice, st));
    AIY_HIP(h, hipMemcpyAsync(work_c, c_init, buf * sizeof(double), hipMemcpyDeviceToDevice, st));
    rc = launch_build_index(h, work_m, rows, dims->n_a + 1, h->d_egm_idx, st);
    if (rc) return rc;
  }
  const int last_allowed = max_cycles + 1;  // HARK: go = d > tol and completed < max_cycles
  int next = 1;
  while (true) {
    const int end = std::min(next + chunk, last_allowed + 1);
    for (int cyc = next; cyc < end; ++cyc) {
      const bool term = cyc == 1 && !warm;
      const double* mn = term ? nullptr : work_m + ((cyc - 1) & 1) * buf;
      const double* cn = term ? nullptr : work_c + ((cyc - 1) & 1) * buf;
      const int* ix = term ? nullptr : h->d_egm_idx + ((cyc - 1) & 1) * idx_per;
      launch_cycle(A, mn, cn, work_m + (cyc & 1) * buf, work_c + (cyc & 1) * buf, ix, cyc, h->d_dist, h->d_last, tol,
                   st);
      rc = launch_build_index(h, work_m + (cyc & 1) * buf, rows, dims->n_a + 1, h->d_egm_idx + (cyc & 1) * idx_per, st);
      if (rc) return rc;
    }
    AIY_CHECK_LAUNCH(h);
    AIY_HIP(h, hipMemcpyAsync(h->h_last, h->d_last, sizeof(int) * n_cal, hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipMemcpyAsync(h->h_dist, h->d_dist, sizeof(unsigned long long) * kSlots * n_cal, hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipStreamSynchronize(st));
    bool all = true;
    for (int c = 0; c < n_cal; ++c) {
      const int last = h->h_last[c];
      const double d = slot_max(h->h_dist + (size_t)c * kSlots, last);
      const bool conv = (last >= 2 && !(d > tol)) || last >= last_allowed;
      all = all && conv;
    }
    next = end;
    if (all || next > last_allowed) break;
  }
  for (int c = 0; c < n_cal; ++c) {
    const int last = h->h_last[c];
    const double d = slot_max(h->h_dist + (size_t)c * kSlots, last);
    cycles_out[c] = last;
    dist_out[c] = last >= 2 ? d : 100.0;
    const size_t off = (size_t)c * per_cal;
    AIY_HIP(h, hipMemcpyAsync(m_out + off, work_m + (last & 1) * buf + off, per_cal * sizeof(double),
                              hipMemcpyDeviceToDevice, st));
    AIY_HIP(h, hipMemcpyAsync(c_out + off, work_c + (last & 1) * buf + off, per_cal * sizeof(double),
                              hipMemcpyDeviceToDevice, st));
  }
  AIY_HIP(h, hipStreamSynchronize(st));
  return AIY_OK;
}

extern "C" int32_t aiy_egm_solve(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in, double tol,
                                 int32_t max_cycles, int32_t chunk, double* work_m, double* work_c, double* m_out,
                                 double* c_out, int32_t* cycles_out, double* dist_out, aiy_stream stream) {
  return aiy_egm_solve_impl(h, dims, in, tol, max_cycles, chunk, nullptr, nullptr, work_m, work_c, m_out, c_out,
                        cycles_out, dist_out, stream);
}

extern "C" int32_t aiy_egm_solve_from(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in, double tol,
                                      int32_t max_cycles, int32_t chunk, const double* m_init, const double* c_init,
                                      double* work_m, double* work_c, double* m_out, double* c_out,
                                      int32_t* cycles_out, double* dist_out, aiy_stream stream) {
  if (h && (!m_init || !c_init)) return fail(h, AIY_ERR_ARG, "null initial tables");
  return aiy_egm_solve_impl(h, dims, in, tol, max_cycles, chunk, m_init, c_init, work_m, work_c, m_out, c_out,
                        cycles_out, dist_out, stream);
}

extern "C" int32_t aiy_policy_eval(aiy_handle* h, int32_t S, int32_t n_M, int32_t n_a, const double* m_tab,
                                   const double* c_tab, const double* M_grid, const int32_t* state, const double* m,
                                   const double* M, int64_t n, double* c_out, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (S < 1 || n_M < 1 || n_a < 2 || n < 0) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (n == 0) return AIY_OK;
  if (!m_tab || !c_tab || !state || !m || !c_out || (n_M > 1 && (!M_grid || !M)))
    return fail(h, AIY_ERR_ARG, "null pointer");
  AIY_HIP(h, hipSetDevice(h->device));
  const int tb = 256;
  const long long nb = (n + tb - 1) / tb;
  hipLaunchKernelGGL(policy_eval_kernel, dim3((unsigned)nb), dim3(tb), 0, as_stream(stream), S, n_M, n_a, m_tab,
                     c_tab, M_grid, state, m, M, (long long)n, c_out);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

// Timing hook for bench.py: n_launch launches of the EGM cycle kernel alone (the search
// index of m_next is built once, outside the timed region) between two HIP events on
// `stream`.  BLOCKING.
extern "C" int32_t aiy_egm_kernel_time(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in,
                                       const double* m_next, const double* c_next, double* m_out, double* c_out,
                                       int32_t n_launch, float* ms_out, aiy_stream stream) {
  int32_t rc = check_egm(h, dims, in);
  if (rc) return rc;
  if (!m_next || !c_next || !m_out || !c_out || !ms_out || n_launch < 1) return fail(h, AIY_ERR_ARG, "bad arguments");
  AIY_HIP(h, hipSetDevice(h->device));
  EgmDev A = to_dev(dims, in);
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  const long long rows = (long long)dims->n_cal * dims->S * dims->n_M;
  rc = ensure_egm_index(h, (size_t)rows * kIdxRow);
  if (rc) return rc;
  rc = launch_build_index(h, m_next, rows, dims->n_a + 1, h->d_egm_idx, st);
  if (rc) return rc;
  int32_t trc = time_launches(
      h, st, n_launch,
      [&] { launch_cycle(A, m_next, c_next, m_out, c_out, h->d_egm_idx, 0, nullptr, nullptr, 0.0, st); }, ms_out);
  if (trc) return trc;
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}
