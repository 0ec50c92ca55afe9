// Device-resident Young-lottery distribution iteration (build-defined row E2) for gfx950:
// a whole aiy_hist_solve in ONE launch, every iteration inside the kernel.
//
// The push/mix pair (hist.hip) costs two dependent launches per iteration (~15 us at
// Table II size, thousands of iterations per GE step).  Here each calibration gets a
// CLUSTER of G workgroups (one per CU) that iterates on its own, synchronised by a
// per-calibration counter instead of kernel boundaries:
//   * workgroup w of a cluster owns asset columns [j0, j1) of every income state: the
//     mass of those columns lives in REGISTERS for the whole solve (thread t holds column
//     j0 + t, all S states);
//   * push (sources = own columns): T_s[lo] += w m, T_s[lo + 1] += (1 - w) m, accumulated
//     with LDS f64 atomics into a per-row destination SPAN buffer: a monotone lottery maps
//     the contiguous source range to the contiguous destination range
//     [lo(j0), lo(j1 - 1) + 1] of each row;
//   * the spans are published write-through (sc1) as the workgroup's slab; one cluster
//     barrier (agent-scope counter, sc1 polls);
//   * gather (destinations = own columns): T_s[d] = sum of the slabs whose span covers d
//     (the covering workgroups are fixed for the whole solve and found once at start), in
//     ascending workgroup order, every load of a row group issued before the first use;
//   * mix: mass'[s'][d] = sum_s P[s, s'] T_s[d] (P in LDS); the sup-norm change is reduced
//     to one published value per workgroup, read by the cluster after the NEXT barrier:
//     the solve stops exactly where oracle/stationary.py stationary_hist stops (first
//     iteration with max |mass' - mass| < tol) and keeps that iteration's mass.
// Per iteration and point: lo 4 B + w 8 B (L2-resident re-reads), slab 8 B out + 8 B in
// (L2 / MALL), no HBM round trip of the mass, no global atomics, one barrier.
// Shapes that do not fit (spans beyond the LDS budget, more covering workgroups per row
// than kHcCand, a non-monotone lottery) abort before the first iteration and the host
// runs the push/mix pair instead.
#include "common.h"
#include "internal.h"

#include <algorithm>

namespace aiy {

constexpr int kHcMaxG = 128;                       // workgroups per calibration cluster
constexpr int kHcCand = 32;                        // covering workgroups per (row, workgroup)
constexpr int kHcRows = 8;                         // rows whose push loads are in flight together
// rows whose gather loads are in flight together: all (S <= 8) for one column per thread
template <int SMAX, int KC>
struct HcGather {
  static constexpr int kRows = (SMAX == 8 && KC == 1) ? 8 : 4;
};
constexpr size_t kHcLdsTotal = 160 * 1024;         // per CU
constexpr unsigned long long kHcTimeoutTicks = 200000000ull;   // 2 s of the 100 MHz clock
constexpr int kHcCtrStride = 32;                   // uints between cluster counters (128 B)

struct HcRun {
  int n_cal, cal0, S, n_a, G, nj, cap;   // cap: doubles of the span buffer / one slab
  const int* lo;          // [n_cal][S][n_a]
  const double* wlo;      // [n_cal][S][n_a]
  const double* P;        // [n_cal][S][S]
  double* mass;           // [n_cal][S][n_a] in: start, out: final
  double* slab;           // [launch cals][G][2][cap]
  int* span;              // [launch cals][G][SMAX][2] (first, len)
  unsigned* ctr;          // [launch cals][kHcCtrStride]
  unsigned long long* dist;   // [launch cals][2][G]
  int* iters_out;         // [n_cal]
  unsigned* err;          // 0 ok, 1 timeout, 2 span overflow / not monotone, 3 candidate overflow
  double tol;
  int max_iter;
};

struct HcCand {
  int w, first, len, off;
};

// Cluster barrier: lane 0 adds one to the cluster counter (after the caller's drained sc1
// stores) and waits until it reaches `target`.  False on timeout (error word set).
__device__ __forceinline__ bool hc_barrier(const HcRun& r, unsigned* ctr, unsigned target, int* s_flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kHcTimeoutTicks) {
        __hip_atomic_store(r.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *s_flag = ok;
  }
  __syncthreads();
  return *s_flag != 0;
}

#ifdef AIY_DIAG_PHASES
#define HC_PH(k)                                                        \
  do {                                                                  \
    if (tid == 0 && blockIdx.x == 0) {                                  \
      const unsigned long long tn = __builtin_amdgcn_s_memrealtime();   \
      if (k) ph[k - 1] += tn - tq;                                      \
      tq = tn;                                                          \
    }                                                                   \
  } while (0)
#else
#define HC_PH(k) \
  do {           \
  } while (0)
#endif

// Sum over the 64 lanes (DPP: row shifts, then row broadcasts), valid in lane 63.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_add_src(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROWS, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_sum_lane63(double v) {
  v += dpp_add_src<0x111, 0xF>(v);   // row_shr:1
  v += dpp_add_src<0x112, 0xF>(v);   // row_shr:2
  v += dpp_add_src<0x114, 0xF>(v);   // row_shr:4
  v += dpp_add_src<0x118, 0xF>(v);   // row_shr:8   (lane 15 of every row: the row's sum)
  v += dpp_add_src<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
  v += dpp_add_src<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3
  return v;
}

template <int SMAX, int KC, int TH>
__global__ __launch_bounds__(TH) void hist_cluster_kernel(HcRun r) {
#ifdef AIY_DIAG_PHASES
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tq = 0;
#endif
  extern __shared__ double Tacc[];                 // destination spans of this workgroup
  __shared__ double sP[SMAX * SMAX];
  __shared__ int s_first[SMAX], s_off[SMAX + 1];
  __shared__ HcCand s_cand[SMAX][kHcCand];
  __shared__ int s_ncand[SMAX];
  __shared__ double s_red[TH / kWave];
  __shared__ int s_cinfo[KC * SMAX * TH];
  __shared__ int s_flag, s_stop;

  const int tid = threadIdx.x;
  const int G = r.G, S = r.S, n_a = r.n_a, cap = r.cap;
  const int lc = blockIdx.x / G;                   // calibration within this launch
  const int w = blockIdx.x - lc * G;
  const int cal = r.cal0 + lc;
  const int j0 = w * r.nj;
  const int j1 = min(j0 + r.nj, n_a);
  unsigned* ctr = r.ctr + (size_t)lc * kHcCtrStride;
  unsigned long long* dist = r.dist + (size_t)lc * 2 * G;
  const size_t row0 = (size_t)cal * S;
  const int* LO = r.lo + row0 * n_a;
  const double* WL = r.wlo + row0 * n_a;
  double* MS = r.mass + row0 * n_a;
  double* slab_cl = r.slab + (size_t)lc * G * 2 * cap;
  int* span_cl = r.span + (size_t)lc * G * SMAX * 2;

  // ---- setup: P, own spans, mass -> registers ----
  for (int q = tid; q < S * S; q += TH) sP[q] = r.P[(size_t)cal * S * S + q];
  if (tid == 0) {
    int tot = 0;
    unsigned bad = 0;
    for (int s = 0; s < S; ++s) {
      const int f = LO[(size_t)s * n_a + j0];
      const int l = LO[(size_t)s * n_a + j1 - 1] - f + 2;   // destinations lo .. lo_last + 1
      s_first[s] = f;
      s_off[s] = tot;
      if (l < 2 || f < 0 || f + l > n_a) bad = 2u;          // not a monotone lottery of ours
      tot += l > 0 ? l : 0;
      __hip_atomic_store(&span_cl[((size_t)w * SMAX + s) * 2], f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&span_cl[((size_t)w * SMAX + s) * 2 + 1], l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_off[S] = tot;
    if (tot > cap) bad = 2u;
    if (bad) __hip_atomic_store(r.err, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  double m[KC][SMAX];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int j = j0 + tid + k * TH;
#pragma unroll
    for (int s = 0; s < SMAX; ++s) m[k][s] = (s < S && j < j1) ? MS[(size_t)s * n_a + j] : 0.0;
  }
  if (!hc_barrier(r, ctr, (unsigned)G, &s_flag)) return;
  if (tid == 0) s_stop = __hip_atomic_load(r.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return;
  // covering workgroups of every row for this workgroup's columns, ascending w
  if (tid < S) {
    const int s = tid;
    int n = 0, bad = 0;
    for (int w2 = 0; w2 < G; ++w2) {
      int off = 0;
      for (int s2 = 0; s2 < s; ++s2)
        off += __hip_atomic_load(&span_cl[((size_t)w2 * SMAX + s2) * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int f = __hip_atomic_load(&span_cl[((size_t)w2 * SMAX + s) * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int l = __hip_atomic_load(&span_cl[((size_t)w2 * SMAX + s) * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (f < j1 && f + l > j0) {
        if (n < kHcCand) s_cand[s][n] = HcCand{w2, f, l, off};
        else bad = 1;
        ++n;
      }
    }
    s_ncand[s] = n < kHcCand ? n : kHcCand;
    if (bad) {
      __hip_atomic_store(r.err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  const int total = s_off[S];
  for (int q = tid; q < total; q += TH) Tacc[q] = 0.0;
  if (!hc_barrier(r, ctr, 2u * G, &s_flag)) return;
  if (tid == 0) s_stop = __hip_atomic_load(r.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return;
  // per (column, row): first covering candidate and how many cover it (fixed for the
  // solve; kept in LDS, not registers)
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int d = j0 + tid + k * TH;
#pragma unroll
    for (int s = 0; s < SMAX; ++s) {
      int cf = 0, cn = 0;
      if (s < S && d < j1) {
        const int nc = s_ncand[s];
        for (int c = 0; c < nc; ++c) {
          const HcCand cd = s_cand[s][c];
          if (d >= cd.first && d < cd.first + cd.len) {
            if (cn == 0) cf = c;
            ++cn;
          }
        }
      }
      s_cinfo[(k * SMAX + s) * TH + tid] = cf | (cn << 8);
    }
  }

  const int lane = tid & (kWave - 1);
  double dloc = 0.0;   // this workgroup's sup-norm change of the last mix
  int final_it = 0;
  for (int it = 1; it <= r.max_iter; ++it) {
    const int par = it & 1;
    HC_PH(0);
    // ---- push own sources into the span buffer (row groups: loads in flight together) ----
#pragma unroll
    for (int s0 = 0; s0 < SMAX; s0 += kHcRows) {
      if (s0 < S) {
        int dd[KC][kHcRows];
        double ww[KC][kHcRows];
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int j = j0 + tid + k * TH;
#pragma unroll
          for (int q = 0; q < kHcRows; ++q) {
            const int s = s0 + q;
            const bool ok = s < S && j < j1;
            dd[k][q] = ok ? LO[(size_t)s * n_a + j] : -1;
            ww[k][q] = ok ? WL[(size_t)s * n_a + j] : 0.0;
          }
        }
        // one LDS f64 atomic per lane and destination: adjacent lanes hit adjacent
        // destinations (no conflict) except on the borrowing constraint, where the LDS
        // serialises same-address adds at a few cycles each -- cheaper than a wave
        // segmented scan, whose dependent cross-lane steps cost ~1.4k cycles per row
        // (measured at Table II size: 17 us per iteration for the push with the scan)
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const bool act = j0 + tid + k * TH < j1;
#pragma unroll
          for (int q = 0; q < kHcRows; ++q) {
            const int s = s0 + q;
            if (s < S) {   // wave-uniform
              const int d = dd[k][q];
              const double vlo = ww[k][q] * m[k][s];            // np.add.at(T[s], lo, wlo * mass)
              const double vhi = (1.0 - ww[k][q]) * m[k][s];    // np.add.at(T[s], lo + 1, (1 - wlo) * mass)
              const int base = s_off[s] - s_first[s];
              const int d0 = __builtin_amdgcn_readfirstlane(d);
              if (__all(act && d == d0)) {
                // one destination for the whole wave (the borrowing constraint): a DPP
                // wave sum and one atomic instead of 64 same-address LDS atomics
                const double tl = wave_sum_lane63(vlo), th = wave_sum_lane63(vhi);
                if (lane == kWave - 1) {
                  atomicAdd(&Tacc[base + d0], tl);
                  if (th != 0.0) atomicAdd(&Tacc[base + d0 + 1], th);
                }
              } else if (act) {
                if (vlo != 0.0) atomicAdd(&Tacc[base + d], vlo);
                if (vhi != 0.0) atomicAdd(&Tacc[base + d + 1], vhi);
              }
            }
          }
        }
      }
    }
    __syncthreads();
    HC_PH(1);
    // ---- publish the spans write-through, re-zero the buffer ----
    double* slab = slab_cl + ((size_t)w * 2 + par) * cap;
    for (int q = tid; q < total; q += TH) {
      store_f64_agent(&slab[q], Tacc[q]);
      Tacc[q] = 0.0;
    }
    if (tid == 0)   // the previous mix's change (iteration it - 1)
      store_u64_agent(&dist[(size_t)((it - 1) & 1) * G + w], (unsigned long long)__double_as_longlong(dloc));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HC_PH(2);
    if (!hc_barrier(r, ctr, (unsigned)(it + 2) * G, &s_flag)) return;
    HC_PH(3);
    // ---- stop where the oracle stops: max change of iteration it - 1 < tol ----
    if (it >= 2) {
      if (tid < kWave) {
        double d = 0.0;
        for (int w2 = lane; w2 < G; w2 += kWave)
          d = nan_max(d, __longlong_as_double((long long)load_u64_agent(&dist[(size_t)((it - 1) & 1) * G + w2])));
        d = wave_nan_max(d);
        if (tid == 0) s_stop = (d < r.tol) ? 1 : 0;
      }
      __syncthreads();
      if (s_stop) {
        final_it = it - 1;
        break;
      }
    }
    // ---- gather own destinations from the covering slabs (ascending w), mix ----
    double T[KC][SMAX];
#pragma unroll
    for (int s0 = 0; s0 < SMAX; s0 += (HcGather<SMAX, KC>::kRows)) {
      if (s0 < S) {
        double v0[KC][(HcGather<SMAX, KC>::kRows)], v1[KC][(HcGather<SMAX, KC>::kRows)];
        bool more = false;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int d = j0 + tid + k * TH;
#pragma unroll
          for (int q = 0; q < (HcGather<SMAX, KC>::kRows); ++q) {
            const int s = s0 + q;
            v0[k][q] = 0.0;
            v1[k][q] = 0.0;
            if (s < S) {
              const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = ci & 255, cn = ci >> 8;
              if (cn >= 1) {
                const HcCand c0 = s_cand[s][cf];
                v0[k][q] = load_f64_agent(&slab_cl[((size_t)c0.w * 2 + par) * cap + c0.off + d - c0.first]);
              }
              if (cn >= 2) {
                const HcCand c1 = s_cand[s][cf + 1];
                v1[k][q] = load_f64_agent(&slab_cl[((size_t)c1.w * 2 + par) * cap + c1.off + d - c1.first]);
              }
              more = more || cn > 2;
            }
          }
        }
        // columns covered by > 2 spans (the borrowing constraint): their extra loads are
        // issued together, before the first use
        double v2[KC][(HcGather<SMAX, KC>::kRows)], v3[KC][(HcGather<SMAX, KC>::kRows)];
        bool more4 = false;
        if (__any(more)) {
#pragma unroll
          for (int k = 0; k < KC; ++k) {
            const int d = j0 + tid + k * TH;
#pragma unroll
            for (int q = 0; q < (HcGather<SMAX, KC>::kRows); ++q) {
              const int s = s0 + q;
              v2[k][q] = 0.0;
              v3[k][q] = 0.0;
              if (s < S) {
                const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = ci & 255, cn = ci >> 8;
                if (cn >= 3) {
                  const HcCand c2 = s_cand[s][cf + 2];
                  v2[k][q] = load_f64_agent(&slab_cl[((size_t)c2.w * 2 + par) * cap + c2.off + d - c2.first]);
                }
                if (cn >= 4) {
                  const HcCand c3 = s_cand[s][cf + 3];
                  v3[k][q] = load_f64_agent(&slab_cl[((size_t)c3.w * 2 + par) * cap + c3.off + d - c3.first]);
                }
                more4 = more4 || cn > 4;
              }
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < KC; ++k)
#pragma unroll
            for (int q = 0; q < (HcGather<SMAX, KC>::kRows); ++q) v2[k][q] = v3[k][q] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
          for (int q = 0; q < (HcGather<SMAX, KC>::kRows); ++q)
            if (s0 + q < SMAX) T[k][s0 + q] = ((v0[k][q] + v1[k][q]) + v2[k][q]) + v3[k][q];
        if (more4) {   // > 4 covering spans: rare, serial
#pragma unroll
          for (int k = 0; k < KC; ++k) {
            const int d = j0 + tid + k * TH;
#pragma unroll
            for (int q = 0; q < (HcGather<SMAX, KC>::kRows); ++q) {
              const int s = s0 + q;
              if (s < S) {
                const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = ci & 255, cn = ci >> 8;
                for (int c = 4; c < cn; ++c) {
                  const HcCand cx = s_cand[s][cf + c];
                  T[k][s] += load_f64_agent(&slab_cl[((size_t)cx.w * 2 + par) * cap + cx.off + d - cx.first]);
                }
              }
            }
          }
        }
      }
    }
    HC_PH(4);
    double dmax = 0.0;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const bool act = j0 + tid + k * TH < j1;
#pragma unroll
      for (int sp = 0; sp < SMAX; ++sp) {
        if (sp < S) {
          double acc = 0.0;
#pragma unroll
          for (int s = 0; s < SMAX; ++s)
            if (s < S) acc += sP[s * S + sp] * T[k][s];   // P.T @ T
          if (act) dmax = nan_max(dmax, fabs(acc - m[k][sp]));
          m[k][sp] = acc;
        }
      }
    }
    dmax = wave_nan_max(dmax);
    if (lane == 0) s_red[tid / kWave] = dmax;
    __syncthreads();
    if (tid == 0) {
      double d = s_red[0];
      for (int q = 1; q < TH / kWave; ++q) d = nan_max(d, s_red[q]);
      dloc = d;
    }
    HC_PH(5);
    final_it = it;
  }
#ifdef AIY_DIAG_PHASES
  if (tid == 0 && blockIdx.x == 0 && final_it > 0)
    printf("[hist phases] G=%d nj=%d iters=%d us/iter: push %.2f publish %.2f barrier %.2f check+gather %.2f mix %.2f\n",
           G, r.nj, final_it, ph[0] * 0.01 / final_it, ph[1] * 0.01 / final_it, ph[2] * 0.01 / final_it,
           ph[3] * 0.01 / final_it, ph[4] * 0.01 / final_it);
#endif
  // ---- final mass of the own columns, iteration count ----
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int j = j0 + tid + k * TH;
#pragma unroll
    for (int s = 0; s < SMAX; ++s)
      if (s < S && j < j1) MS[(size_t)s * n_a + j] = m[k][s];
  }
  if (w == 0 && tid == 0) r.iters_out[cal] = final_it;
}

// Host plan of one cluster launch shape: one column per thread (KC = 1) with 512- or
// 1024-thread workgroups (the 1024 form keeps 16 waves per CU for latency hiding when a
// workgroup owns more than 512 columns).
struct HcPlan {
  int G = 0, nj = 0, th = 0, smax = 0, cals_per_launch = 0, cap = 0;
  size_t lds = 0;
  const void* fn = nullptr;
};

template <int SMAX, int TH>
static const void* hc_fn() {
  return reinterpret_cast<const void*>(hist_cluster_kernel<SMAX, 1, TH>);
}

static const void* hc_pick(int smax, int th) {
  if (smax == 8) return th == 512 ? hc_fn<8, 512>() : hc_fn<8, 1024>();
  if (smax == 16) return hc_fn<16, 512>();
  return hc_fn<32, 512>();
}

static bool hc_make_plan(aiy_handle* h, int n_cal, int S, int n_a, HcPlan& p) {
  if (S > 32 || S < 1 || n_a < 2) return false;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus < 1) return false;
  p.smax = S <= 8 ? 8 : (S <= 16 ? 16 : 32);
  const int th_max = p.smax == 8 ? 1024 : 512;
  const int g_min = (n_a + th_max - 1) / th_max;
  if (g_min > kHcMaxG || g_min > cus) return false;
  const int g_cap = h->hist_cluster_cap > 0 ? h->hist_cluster_cap : 32;
  int G = std::max(g_min, std::min(std::min(g_cap, kHcMaxG), cus / std::max(1, n_cal)));
  G = std::min(G, n_a);
  p.nj = (n_a + G - 1) / G;
  p.G = (n_a + p.nj - 1) / p.nj;                    // every workgroup owns >= 1 column
  p.th = p.nj <= 512 ? 512 : 1024;
  if (p.th > th_max) return false;
  p.cals_per_launch = std::max(1, cus / p.G);
  p.fn = hc_pick(p.smax, p.th);
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, p.fn) != hipSuccess) return false;
  const size_t stat = fa.sharedSizeBytes;
  if (stat + 4096 >= kHcLdsTotal) return false;
  p.lds = (kHcLdsTotal - stat - 1024) / 256 * 256;
  p.cap = (int)(p.lds / sizeof(double));
  return true;
}

static int32_t hc_scratch(aiy_handle* h, int cals, int G, int cap) {
  const size_t need = (size_t)cals * G * 2 * cap * sizeof(double) + (size_t)cals * G * 32 * 2 * sizeof(int) +
                      (size_t)cals * kHcCtrStride * sizeof(unsigned) + (size_t)cals * 2 * G * sizeof(unsigned long long) +
                      256;
  if (need > h->hc_cap) {
    if (h->d_hc) (void)hipFree(h->d_hc);
    h->d_hc = nullptr;
    h->hc_cap = 0;
    AIY_HIP(h, hipMalloc(&h->d_hc, need));
    h->hc_cap = need;
  }
  return AIY_OK;
}

// A whole distribution iteration of n_cal calibrations in cluster launches.  Returns
// AIY_OK; AIY_ERR_UNSUPPORTED when the shape does not fit (the caller then runs the
// push/mix pair: a calibration whose cluster had finished restarts from its converged
// mass); or an error.
int32_t hist_solve_resident(aiy_handle* h, int n_cal, int S, int n_a, const int* lo, const double* wlo,
                            const double* P, double tol, int max_iter, double* mass, int* d_iters, hipStream_t st) {
  HcPlan p;
  if (!hc_make_plan(h, n_cal, S, n_a, p)) return AIY_ERR_UNSUPPORTED;
  AIY_HIP(h, hipFuncSetAttribute(p.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds));
  int per_cu = 0;
  AIY_HIP(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, p.fn, p.th, p.lds));
  if (per_cu < 1) return AIY_ERR_UNSUPPORTED;
  const int per_launch = std::min(n_cal, p.cals_per_launch);
  int32_t rc = hc_scratch(h, per_launch, p.G, p.cap);
  if (rc) return rc;
  char* base = static_cast<char*>(h->d_hc);
  HcRun r;
  r.n_cal = n_cal; r.S = S; r.n_a = n_a; r.G = p.G; r.nj = p.nj; r.cap = p.cap;
  r.lo = lo; r.wlo = wlo; r.P = P; r.mass = mass; r.iters_out = d_iters; r.tol = tol; r.max_iter = max_iter;
  r.slab = reinterpret_cast<double*>(base);
  size_t off = (size_t)per_launch * p.G * 2 * p.cap * sizeof(double);
  r.span = reinterpret_cast<int*>(base + off);
  off += (size_t)per_launch * p.G * 32 * 2 * sizeof(int);
  r.ctr = reinterpret_cast<unsigned*>(base + off);
  const size_t ctr_bytes = (size_t)per_launch * kHcCtrStride * sizeof(unsigned);
  off += ctr_bytes;
  r.dist = reinterpret_cast<unsigned long long*>(base + off);
  off += (size_t)per_launch * 2 * p.G * sizeof(unsigned long long);
  r.err = reinterpret_cast<unsigned*>(base + off);
  for (int c0 = 0; c0 < n_cal; c0 += per_launch) {
    const int nc = std::min(per_launch, n_cal - c0);
    r.cal0 = c0;
    AIY_HIP(h, hipMemsetAsync(r.ctr, 0, ctr_bytes, st));
    AIY_HIP(h, hipMemsetAsync(r.err, 0, sizeof(unsigned), st));
    void* args[] = {&r};
    AIY_HIP(h, hipEventRecord(h->hc_ev[0], st));
    AIY_HIP(h, hipLaunchKernel(p.fn, dim3(nc * p.G), dim3(p.th), args, p.lds, st));
    AIY_HIP(h, hipEventRecord(h->hc_ev[1], st));
    unsigned err = 0;
    AIY_HIP(h, hipMemcpyAsync(&err, r.err, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipStreamSynchronize(st));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->hc_ev[0], h->hc_ev[1]) == hipSuccess) {
      h->hc_ms_sum += ms;
      h->hc_launches += 1;
    }
    if (err == 2u || err == 3u) return AIY_ERR_UNSUPPORTED;
    if (err) return fail(h, AIY_ERR_STATE, "resident histogram: cluster barrier timed out (workgroups not co-resident?)");
  }
  return AIY_OK;
}

// Plan of the resident histogram for (n_cal, S, n_a) (measurement / tests): workgroups per
// cluster, columns per workgroup, calibrations per launch; 0 when it would not run.
int32_t hist_resident_plan(aiy_handle* h, int n_cal, int S, int n_a, int* out4) {
  HcPlan p;
  if (!hc_make_plan(h, n_cal, S, n_a, p)) return 0;
  out4[0] = p.G;
  out4[1] = p.nj;
  out4[2] = p.cals_per_launch;
  out4[3] = p.cap;
  return 1;
}

}  // namespace aiy
