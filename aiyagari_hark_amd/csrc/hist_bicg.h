// The BiCGSTAB distribution solve of one calibration's cluster (build-defined row E2,
// Krylov mode) as a device function: hist_krylov.hip runs one solve per launch,
// ge_resident.hip many solves per launch inside its device-resident GE search.
// See hist_krylov.hip for the algorithm.
#pragma once

#include "common.h"
#include "hist_cluster.h"

namespace aiy {

constexpr int kHkRed = 8;   // partial sums per reduction (at most)
constexpr int kHkStall = 256;   // matvecs without a 10 % residual gain that count as a stall
constexpr double kHkStopSentinel = 1e300;   // rebalancing stop request on the max|r| partial
static_assert(2 * kHkRed <= kHcRedRec, "two granules per partial sum");
// Destinations covered by more than two spans (the borrowing constraint, the top of the grid:
// up to kHcCand covering workgroups) are summed by a whole wave, one candidate per lane, instead
// of a serial per-lane loop whose dependent slab loads put the owning workgroup ~2 us behind the
// others every matvec (tools/hist_phases.py at G = 32: its gather 4.2 vs 1.6-2.4 us).  Up to
// kHkHeavy such (column, state) entries per workgroup; more fall back to the per-lane loop.
constexpr int kHkHeavy = 31;
// only destinations with more than kHkWaveCn covering spans take a wave-parallel entry; the
// others (3 .. kHkWaveCn spans: the destinations of the lowest workgroup's range that several
// neighbours' dissaving sources reach, often hundreds of them) load their extra candidates 2
// and 3 for every state at once, one round trip instead of one per state (Table II sweep
// 60.5 -> 57.9 ms against kHkWaveCn = 2, gpurun_out r07a abt2)
#ifndef AIY_HK_WAVE_CN
#define AIY_HK_WAVE_CN 6
#endif
constexpr int kHkWaveCn = AIY_HK_WAVE_CN;
static_assert(kHcCand <= 32, "covering-span index and count packed in 5 + 6 bits");
// covering info of one (column, state): first candidate (5 bits), count (6 bits), heavy-entry
// index (5 bits; kHkHeavy = none)
__device__ __forceinline__ unsigned short hk_cinfo(int cf, int cn, int hi) {
  return (unsigned short)(cf | (cn << 5) | (hi << 11));
}
__device__ __forceinline__ int hk_cf(int ci) { return ci & 31; }
__device__ __forceinline__ int hk_cn(int ci) { return (ci >> 5) & 63; }
__device__ __forceinline__ int hk_hi(int ci) { return ci >> 11; }

// a wave-uniform double kept in SGPRs (the solve's scalars: otherwise VGPR pairs that the
// pipelined form spilled to scratch inside its loop)
__device__ __forceinline__ double hk_uni(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// shadow residual: a fixed pseudo-random value in [-1, 1) per point index q = s n_a + j
__device__ __forceinline__ double hk_rhat(unsigned q) {
  unsigned h = q * 0x9E3779B1u + 0x7F4A7C15u;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (double)(int)h * (1.0 / 2147483648.0);
}

// Phase timing (diagnostic builds, -DAIY_DIAG_PHASES=<block>: that block and the next 9,
// i.e. one calibration's cluster at Table II size): time since the previous
// mark is added to slot k: 0 push, 1 publish, 2 matvec barrier, 3 gather + mix,
// 4 reductions (partials, publish, barrier, read), 5 vector updates
#ifdef AIY_DIAG_PHASES
#define HK_PH(k)                                                        \
  do {                                                                  \
    if (tid == 0 && blockIdx.x >= AIY_DIAG_PHASES && blockIdx.x < AIY_DIAG_PHASES + 10) { \
      const unsigned long long tn = __builtin_amdgcn_s_memrealtime();   \
      if ((k) >= 0) ph[(k)] += tn - tq;                                 \
      tq = tn;                                                          \
    }                                                                   \
  } while (0)
#else
#define HK_PH(k) \
  do {           \
  } while (0)
#endif

template <int SMAX, int KC, int TH>
struct HkShared {
  double* Tacc;                    // span buffer (cap doubles); for SMAX <= 8 then v
  int* s_base;                     // [SMAX]
  int (*s_pub)[2];                 // [2 SMAX][2]
  int* s_tot;
  HcCand (*s_cand)[kHcCand];       // [SMAX][kHcCand]
  int* s_ncand;                    // [SMAX]
  unsigned short* s_cinfo;         // [KC SMAX TH]
  double* s_P;                     // [SMAX SMAX]
  double (*s_part)[TH / kWave];    // [kHkRed]
  double* s_res;                   // [kHkRed]
  int* s_flag;
  int* s_stop;
  int* s_ex;                       // [SMAX][2] pull form: exported prefix / suffix of the own sources
  int* s_nheavy;                   // heavy (column, state) entries of this workgroup
  int* s_wcnt;                     // [TH / kWave] per-wave counts while numbering them
  int (*s_heavy)[4];               // [kHkHeavy] (k, s, tid, cf | cn << 8)
  double* s_hval;                  // [kHkHeavy] their wave sums
  int* s_rok;                      // reduction riding on a matvec barrier: granules read in time
};

// One calibration's BiCGSTAB distribution solve by the workgroups of its cluster (this
// workgroup: w of G, own columns [j0, j1)); shared by hist_bicg_kernel (one solve per
// launch) and the device-resident GE search (ge_resident.hip, many solves per launch).
// (pointers typed global: hk_solve_isolated receives them as plain arguments, where the
// compiler could not infer their address space and would use flat accesses)
struct HkArgs {
  int G, S, n_a, cap, w, j0, j1;
  gptr<const int> LO;          // [S][n_a] lottery of the calibration (index)
  gptr<const double> WL;       // [S][n_a] lottery weight on lo
  gptr<double> X;              // [S][n_a] in: start, out: T x (own columns)
  gptr<double> Pg;             // [S][n_a] p scratch rows
  gptr<double> Vg;             // v block of this workgroup in HBM (SMAX > 8)
  gptr<double> slab_cl;        // [G][2][cap]
  gptr<int> span_cl;           // [G][SMAX][4]
  gptr<unsigned> ctr;          // cluster barrier counter
  gptr<unsigned long long> gran;   // [2][G][kHcRedRec] reduction granules
  gptr<const double> Pc;       // [S][S]
  double tol;
  int max_iter;
  gptr<unsigned> err;
  // rebalancing (ge_resident.hip): stop at the next iteration once *stop_ctr >= stop_at
  // (nullptr: never); the solve then returns -(2 + matvecs) with X a valid iterate
  gptr<const unsigned> stop_ctr;
  unsigned stop_at;
  // pull form of the matvec (PULL = true, hist_pull.h's lottery pull with the vectors kept in
  // registers): the matvec input staged in Qg, the inverse lottery in Ainv
  gptr<double> Qg;             // [S][n_a]
  gptr<int> Ainv;              // [S][n_a + 1]
  bool lottery_fresh;          // LO / WL written in this launch by other workgroups (sc1 loads)
};

// Returns the matvecs of the solve, or -1 when the cluster stops (error word set: a
// timeout, a span that does not fit, too many covering workgroups), or -(2 + matvecs) when
// a rebalancing stop was requested (X holds the current iterate; a later solve restarts
// from it).  nb / ne: the
// cluster barriers / reductions passed so far in this launch (counted on).
template <int SMAX, int KC, int TH, bool PULL = false, bool FUSEA = false>
__device__ __forceinline__ int hk_solve(const HkArgs& r, const HkShared<SMAX, KC, TH>& L, unsigned& nb,
                                        unsigned& ne) {
  constexpr bool kVlds = SMAX <= 8;
#ifdef AIY_DIAG_PHASES
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tq = 0;
#endif
  double* Tacc = L.Tacc;
  int* s_base = L.s_base;
  int (*s_pub)[2] = L.s_pub;
  HcCand (*s_cand)[kHcCand] = L.s_cand;
  int* s_ncand = L.s_ncand;
  unsigned short* s_cinfo = L.s_cinfo;
  double* s_P = L.s_P;
  double (*s_part)[TH / kWave] = L.s_part;
  double* s_res = L.s_res;
  int& s_flag = *L.s_flag;
  int& s_stop = *L.s_stop;
  int& s_tot = *L.s_tot;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wid = tid / kWave;
  const int G = r.G, S = r.S, n_a = r.n_a, cap = r.cap;
  const int w = r.w;
  const int j0 = r.j0;
  const int j1 = r.j1;
  unsigned* ctr = (unsigned*)r.ctr;
  unsigned long long* gran = (unsigned long long*)r.gran;
  const int* LO = (const int*)r.LO;
  const double* WL = (const double*)r.WL;
  double* X = (double*)r.X;   // x: the iterate, own columns read-modify-written
  double* slab_cl = (double*)r.slab_cl;
  const double* __restrict__ Pc = (const double*)r.Pc;
  int* span_cl = (int*)r.span_cl;
  unsigned* err = (unsigned*)r.err;

  // ---- setup (as hist_cluster_kernel): P, own spans, covering candidates ----
  for (int q = tid; q < SMAX * SMAX; q += TH) {
    const int s = q / SMAX, sp = q - s * SMAX;
    s_P[q] = (s < S && sp < S) ? Pc[s * S + sp] : 0.0;
  }
  auto barrier = [&]() -> bool {
    ++nb;
    return hc_barrier(err, ctr, (unsigned)G * nb, &s_flag);
  };
  // pull form: the inverse lottery of the own destinations, staged in LDS (Tacc's space)
  const int n_own = j1 - j0, aspan = n_own + 2;
  int* s_A = reinterpret_cast<int*>(Tacc);
  int* s_ex = L.s_ex;
  int* Ainv = (int*)r.Ainv;
  double* Qg = (double*)r.Qg;
  auto lo_at = [&](int s, int j) -> int {
    const int* p = LO + (size_t)s * n_a + j;
    return r.lottery_fresh ? __hip_atomic_load(to_global(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
  };
  if constexpr (PULL) {
    const int n1 = n_a + 1;
    unsigned bad = 0u;
    // a lottery written in this launch (the resident GE search): every workgroup's entries are
    // in memory before the neighbour's column j0 - 1 is read
    if (r.lottery_fresh) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!barrier()) return -1;
    }
    for (int q = tid; q < S * n_own; q += TH) {
      const int s = q / n_own, j = j0 + (q - s * n_own);
      const int l = lo_at(s, j);
      const int lp = j > 0 ? lo_at(s, j - 1) : -1;
      // only a monotone lottery inside the grid is scattered (anything else: error 2, the
      // caller falls back); the loops never index outside the row
      const bool ok = l >= 0 && l <= n_a - 2 && lp >= -1 && lp <= l;
      if (!ok) {
        bad = 2u;
        continue;
      }
      for (int d = lp + 1; d <= l; ++d)
        __hip_atomic_store(to_global(&Ainv[(size_t)s * n1 + d]), j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (j == n_a - 1)
        for (int d = l + 1; d <= n_a; ++d)
          __hip_atomic_store(to_global(&Ainv[(size_t)s * n1 + d]), n_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (S * aspan * (int)sizeof(int) > cap * (int)sizeof(double)) bad = 2u;
    if (bad) __hip_atomic_store(to_global(err), bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < S) {   // exported prefix [j0, ex0) (lo < j0) and suffix [ex1, j1) (lo + 1 >= j1)
      const int s = tid;
      int lo = j0, hi = j1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (lo_at(s, mid) < j0) lo = mid + 1; else hi = mid;
      }
      s_ex[2 * s] = lo;
      int lo2 = j0, hi2 = j1;
      while (lo2 < hi2) {
        const int mid = (lo2 + hi2) >> 1;
        if (lo_at(s, mid) + 1 < j1) lo2 = mid + 1; else hi2 = mid;
      }
      s_ex[2 * s + 1] = lo2;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!barrier()) return -1;
    if (tid == 0) s_stop = __hip_atomic_load(to_global(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    __syncthreads();
    if (s_stop) return -1;
    for (int q = tid; q < S * aspan; q += TH) {   // A(d) for d in [j0 - 1, j1] (A(-1) = 0)
      const int s = q / aspan, d = j0 - 1 + (q - s * aspan);
      s_A[q] = d < 0 ? 0 : __hip_atomic_load(to_global(&Ainv[(size_t)s * n1 + d]), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  if (!PULL && tid == 0) {
    int tot = 0;
    unsigned bad = 0;
    for (int s = 0; s < S; ++s) {
      const int f = LO[(size_t)s * n_a + j0];
      const int l = LO[(size_t)s * n_a + j1 - 1] - f + 2;
      if (l < 2 || f < 0 || f + l > n_a) bad = 2u;
      const int ll = l > 0 ? l : 0;
      s_base[s] = tot - f;
      s_pub[2 * s][0] = tot;
      s_pub[2 * s][1] = tot + max(0, min(ll, j0 - f));
      s_pub[2 * s + 1][0] = tot + min(ll, max(0, j1 - f));
      s_pub[2 * s + 1][1] = tot + ll;
      int* sp = &span_cl[((size_t)w * SMAX + s) * 4];
      __hip_atomic_store(to_global(&sp[0]), f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(to_global(&sp[1]), ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(to_global(&sp[2]), tot - f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tot += ll;
    }
    s_tot = tot;
    *L.s_nheavy = 0;
    if (tot > cap) bad = 2u;
    if (bad) __hip_atomic_store(to_global(err), bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (!PULL) {
  if (!barrier()) return -1;
  if (tid == 0) s_stop = __hip_atomic_load(to_global(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return -1;
  if (tid < S) {
    const int s = tid;
    int n = 0, bad = 0;
    for (int w2 = 0; w2 < G; ++w2) {
      const int* sp = &span_cl[((size_t)w2 * SMAX + s) * 4];
      const int f = __hip_atomic_load(to_global(&sp[0]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int l = __hip_atomic_load(to_global(&sp[1]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (f < j1 && f + l > j0) {
        const int base = __hip_atomic_load(to_global(&sp[2]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n < kHcCand) s_cand[s][n] = HcCand{w2, f, l, base};
        else bad = 1;
        ++n;
      }
    }
    s_ncand[s] = n < kHcCand ? n : kHcCand;
    if (bad) {
      __hip_atomic_store(to_global(err), 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  const int total = s_tot;
  for (int q = tid; q < total; q += TH) Tacc[q] = 0.0;
  if (!barrier()) return -1;
  if (tid == 0) s_stop = __hip_atomic_load(to_global(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return -1;
  }   // !PULL setup
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    if (PULL) break;
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
      // a heavy destination: a wave-parallel entry, numbered in (k, s, thread) order so that
      // which destinations get the kHkHeavy entries (and so the summation order of the
      // others) is the same in every run
      const bool heavy = cn > kHkWaveCn;
      const unsigned long long bm = __ballot(heavy);
      if (lane == 0) L.s_wcnt[wid] = __popcll(bm);
      __syncthreads();
      int base = *L.s_nheavy;
      for (int q = 0; q < wid; ++q) base += L.s_wcnt[q];
      int tot = 0;
      for (int q = 0; q < TH / kWave; ++q) tot += L.s_wcnt[q];
      const int e = base + __popcll(bm & ((1ull << lane) - 1ull));
      int hi = kHkHeavy;
      if (heavy && e < kHkHeavy) {
        hi = e;
        L.s_heavy[e][0] = k;
        L.s_heavy[e][1] = s;
        L.s_heavy[e][2] = tid;
        L.s_heavy[e][3] = cf | (cn << 8);
      }
      __syncthreads();   // every wave read s_nheavy and s_wcnt before they change
      if (tid == 0) *L.s_nheavy = base + tot;   // (thread 0: wave 0, base = the running total)
      s_cinfo[(k * SMAX + s) * TH + tid] = hk_cinfo(cf, cn, hi);
    }
  }
  // lottery in registers with one column per thread at <= 8 waves (256 VGPRs); with two columns
  // per thread, or 16 waves (128 VGPRs), the registers hold the Krylov vectors
  constexpr bool kLoReg = SMAX <= 8 && KC == 1 && TH <= 512;
  int dreg[KC][kLoReg ? SMAX : 1];
  double wreg[KC][kLoReg ? SMAX : 1];
  if constexpr (kLoReg) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int j = j0 + tid + k * TH;
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        const bool ok = s < S && j < j1;
        dreg[k][s] = ok ? LO[(size_t)s * n_a + j] : -1;
        wreg[k][s] = ok ? WL[(size_t)s * n_a + j] : 0.0;
      }
    }
  }
  const int v_base = lane < S ? s_base[lane] : 0;
  const int v_plo = lane < 2 * S ? s_pub[lane][0] : 0;
  const int v_phi = lane < 2 * S ? s_pub[lane][1] : 0;
  // the column index is re-materialised per phase through an empty asm: otherwise the
  // compiler hoists every point's address, hash and predicate out of the loop and keeps
  // them live across the gathers (hundreds of VGPRs of spills)
  const int jbase = j0 + tid;
  auto col = [&]() {
    int c = jbase;
    asm volatile("" : "+v"(c));
    return c;
  };

  // ---- the matvec pieces ----
  // push q's own sources into the LDS spans (np.add.at(T[s], lo, wlo q) and lo + 1)
  auto push = [&](const double (&q)[KC][SMAX]) {
    // lottery rows in groups whose loads (L2) are all in flight before the first atomic
    constexpr int PR = SMAX <= 8 ? SMAX : 4;
    const int jc = col();   // lottery addresses formed here, not hoisted (they spilled)
#pragma unroll
    for (int s0 = 0; s0 < SMAX; s0 += PR) {
      if (s0 < S) {
        int dd[KC][PR];
        double ww[KC][PR];
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int j = jc + k * TH;
#pragma unroll
          for (int u = 0; u < PR; ++u) {
            const int s = s0 + u;
            if constexpr (kLoReg) {
              dd[k][u] = s < SMAX ? dreg[k][s < SMAX ? s : 0] : -1;
              ww[k][u] = s < SMAX ? wreg[k][s < SMAX ? s : 0] : 0.0;
            } else {
              // unconditional loads at a clamped index (no exec-masked branch per load)
              const bool ok = s < S && j < j1;
              const int q = min(s, S - 1) * n_a + min(j, n_a - 1);
              const int dv = LO[q];
              const double wv = WL[q];
              dd[k][u] = ok ? dv : -1;
              ww[k][u] = ok ? wv : 0.0;
            }
          }
        }
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const bool act = j0 + tid + k * TH < j1;
#pragma unroll
          for (int u = 0; u < PR; ++u) {
            const int s = s0 + u;
            if (s < S) {   // wave-uniform
              const int d = dd[k][u];
              const double vlo = ww[k][u] * q[k][s];          // np.add.at(T[s], lo, wlo q)
              const double vhi = (1.0 - ww[k][u]) * q[k][s];  // np.add.at(T[s], lo + 1, (1 - wlo) q)
              const int ilo = __builtin_amdgcn_readlane(v_base, s) + d, ihi = ilo + 1;
              const int d0 = __builtin_amdgcn_readfirstlane(d);
              if (__all(act && d == d0)) {   // the whole wave on one destination (borrowing constraint)
                const double tl = wave_sum_lane63(vlo), th = wave_sum_lane63(vhi);
                if (lane == kWave - 1) {
                  atomicAdd(&Tacc[ilo], tl);
                  if (th != 0.0) atomicAdd(&Tacc[ihi], th);
                }
              } else if (act) {
                if (vlo != 0.0) atomicAdd(&Tacc[ilo], vlo);
                if (vhi != 0.0) atomicAdd(&Tacc[ihi], vhi);
              }
            }
          }
        }
      }
    }
    __syncthreads();
  };
  // publish the foreign parts of the spans write-through to slab `par`, re-zero them
  auto publish = [&](int par) {
    double* slab = slab_cl + ((size_t)w * 2 + par) * cap;
    for (int rr = 0; rr < 2 * S; ++rr) {
      const int lo = __builtin_amdgcn_readlane(v_plo, rr), hi = __builtin_amdgcn_readlane(v_phi, rr);
      for (int q = lo + tid; q < hi; q += TH) {
        store_f64_agent(&slab[q], Tacc[q]);
        Tacc[q] = 0.0;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // gather the own destinations (ascending covering workgroup) and mix: Tq[k][s'] =
  // sum_s P[s, s'] T_s[d]
  auto gather_mix = [&](int par, double (&out)[KC][SMAX]) {
    constexpr int GR = 4;
    double T[KC][SMAX];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) T[k][s] = 0.0;
    bool more = false;
#pragma unroll
    for (int s0 = 0; s0 < SMAX; s0 += GR) {
      if (s0 < S) {
        double v0[KC][GR], v1[KC][GR];
        int oq[KC][GR];
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int d = j0 + tid + k * TH;
#pragma unroll
          for (int q = 0; q < GR; ++q) {
            const int s = s0 + q;
            v0[k][q] = 0.0;
            v1[k][q] = 0.0;
            oq[k][q] = -1;
            if (s < S) {
              const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = hk_cf(ci), cn = hk_cn(ci);
              if (cn >= 1) {
                const HcCand c = s_cand[s][cf];
                if (c.w != w) v0[k][q] = load_f64_agent(&slab_cl[((size_t)c.w * 2 + par) * cap + c.base + d]);
                else oq[k][q] = c.base + d;
              }
              if (cn >= 2) {
                const HcCand c = s_cand[s][cf + 1];
                if (c.w != w) v1[k][q] = load_f64_agent(&slab_cl[((size_t)c.w * 2 + par) * cap + c.base + d]);
                else oq[k][q] = c.base + d;
              }
              more = more || (cn > 2 && hk_hi(ci) == kHkHeavy);
            }
          }
        }
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
          for (int q = 0; q < GR; ++q)
            if (oq[k][q] >= 0) {
              T[k][s0 + q] = Tacc[oq[k][q]];
              Tacc[oq[k][q]] = 0.0;
            }
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
          for (int q = 0; q < GR; ++q) T[k][s0 + q] = (v0[k][q] + v1[k][q]) + T[k][s0 + q];
      }
    }
    // heavy destinations (more than two covering spans): one wave per entry, candidate 2 + lane
    // in lane order, summed by the wave's fixed DPP tree; the owner adds the sum
    const int nh = min(*L.s_nheavy, kHkHeavy);   // block-uniform
    if (nh > 0) {
      // every entry of this wave loaded before the first sum (one round trip, not one per entry)
      constexpr int NW = TH / kWave, EPW = (kHkHeavy + NW - 1) / NW;
      double hx[EPW];
#pragma unroll
      for (int i = 0; i < EPW; ++i) {
        const int e = wid + i * NW;
        hx[i] = 0.0;
        if (e < nh) {   // wave-uniform
          const int ek = L.s_heavy[e][0], es = L.s_heavy[e][1], et = L.s_heavy[e][2], ec = L.s_heavy[e][3];
          const int c = 2 + lane;
          if (c < (ec >> 8)) hx[i] = hc_take(s_cand[es][(ec & 255) + c], w, j0 + et + ek * TH, par, cap, slab_cl, Tacc);
        }
      }
#pragma unroll
      for (int i = 0; i < EPW; ++i) {
        const int e = wid + i * NW;
        if (e < nh) {
          const double sum = wave_sum_lane63(hx[i]);
          if (lane == kWave - 1) L.s_hval[e] = sum;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s)
          if (s < S) {
            const int ci = s_cinfo[(k * SMAX + s) * TH + tid];
            if (hk_hi(ci) < kHkHeavy) T[k][s] += L.s_hval[hk_hi(ci)];
          }
    }
    if (__any(more)) {   // destinations with more than two covering spans and no wave entry
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int d = j0 + tid + k * TH;
        double e2[SMAX], e3[SMAX];   // candidates 2 and 3 of every state, all in flight
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          e2[s] = 0.0;
          e3[s] = 0.0;
          if (s < S) {
            const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = hk_cf(ci), cn = hk_cn(ci);
            if (cn > 2 && hk_hi(ci) == kHkHeavy) {
              e2[s] = hc_take(s_cand[s][cf + 2], w, d, par, cap, slab_cl, Tacc);
              if (cn > 3) e3[s] = hc_take(s_cand[s][cf + 3], w, d, par, cap, slab_cl, Tacc);
            }
          }
        }
#pragma unroll
        for (int s = 0; s < SMAX; ++s) T[k][s] += e2[s] + e3[s];
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          if (s < S) {
            const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = hk_cf(ci), cn = hk_cn(ci);
            if (hk_hi(ci) < kHkHeavy) continue;
            for (int c0 = 4; c0 < cn; c0 += 4) {   // (more than four spans and no wave entry: rare)
              double x[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int c = c0 + u;
                x[u] = 0.0;
                if (c < cn) x[u] = hc_take(s_cand[s][cf + c], w, d, par, cap, slab_cl, Tacc);
              }
              T[k][s] += ((x[0] + x[1]) + x[2]) + x[3];
            }
          }
        }
      }
    }
#pragma unroll
    for (int sp = 0; sp < SMAX; ++sp) {
      double pc[SMAX];
      asm volatile("" ::: "memory");   // one column of P at a time (else all of P is hoisted)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) pc[s] = s_P[s * SMAX + sp];
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        double acc = 0.0;
#pragma unroll
        for (int s = 0; s < SMAX; ++s) acc += pc[s] * T[k][s];
        out[k][sp] = acc;
      }
    }
  };
  // pull form: q of the own points staged in Qg (the exported entries write-through), one
  // cluster barrier, then every own destination pulls its sources (hist_pull.h)
  auto stage_q = [&](const double (&q)[KC][SMAX]) {
    const int jc = col();
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int j = jc + k * TH;
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        if (s < S && j < j1) {
          double* p = Qg + (size_t)s * n_a + j;
          if (j < s_ex[2 * s] || j >= s_ex[2 * s + 1]) store_f64_agent(p, q[k][s]);
          else *p = q[k][s];
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto w_at = [&](int s, int j) -> double {
    const double* p = WL + (size_t)s * n_a + j;
    return r.lottery_fresh ? load_f64_agent(p) : *p;
  };
  auto q_at = [&](int s, int j) -> double { return load_f64_agent(Qg + (size_t)s * n_a + j); };
  auto pull_mix = [&](double (&out)[KC][SMAX]) {
    const int jc = col();
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      asm volatile("" ::: "memory");   // one column's loads at a time (else both are hoisted: spills)
      const int d = jc + k * TH;
      const bool valid = d < j1;
      double T[SMAX];
#pragma unroll
      for (int s = 0; s < SMAX; ++s) T[s] = 0.0;
      constexpr int GRP = SMAX <= 8 ? (KC == 1 ? (SMAX + 1) / 2 : 2) : 4;
#pragma unroll
      for (int s0 = 0; s0 < SMAX; s0 += GRP) {
        if (s0 >= S) break;   // wave-uniform
        asm volatile("" ::: "memory");
        int a0[GRP], a1[GRP], a2[GRP];
        double wv[GRP][4], qv[GRP][4];
#pragma unroll
        for (int u = 0; u < GRP; ++u) {
          const int sc = min(s0 + u, S - 1);
          const int* As = s_A + sc * aspan - (j0 - 1);
          // (clamped into the row: the loops below never leave it)
          a0[u] = valid ? min(max(As[d - 1], 0), n_a) : 0;
          a1[u] = valid ? min(max(As[d], a0[u]), n_a) : 0;
          a2[u] = valid ? min(max(As[d + 1], a1[u]), n_a) : 0;
          const int i0 = min(a1[u], n_a - 1), i1 = min(a1[u] + 1, n_a - 1);
          const int i2 = min(a0[u], n_a - 1), i3 = min(a0[u] + 1, n_a - 1);
          wv[u][0] = w_at(sc, i0); qv[u][0] = q_at(sc, i0);
          wv[u][1] = w_at(sc, i1); qv[u][1] = q_at(sc, i1);
          wv[u][2] = w_at(sc, i2); qv[u][2] = q_at(sc, i2);
          wv[u][3] = w_at(sc, i3); qv[u][3] = q_at(sc, i3);
        }
#pragma unroll
        for (int u = 0; u < GRP; ++u) {
          const int sr = s0 + u;
          if (sr < S) {   // wave-uniform
            const int n1c = a2[u] - a1[u], n0c = a1[u] - a0[u];
            const bool heavy = valid && (n1c + n0c) > kWave;
            double acc = 0.0;
            if (valid && !heavy) {
              if (n1c > 0) acc += wv[u][0] * qv[u][0];                    // np.add.at(T, lo, w q), ascending j
              if (n1c > 1) acc += wv[u][1] * qv[u][1];
              for (int j = a1[u] + 2; j < a2[u]; ++j) acc += w_at(sr, j) * q_at(sr, j);
              if (n0c > 0) acc += (1.0 - wv[u][2]) * qv[u][2];            // np.add.at(T, lo + 1, (1 - w) q)
              if (n0c > 1) acc += (1.0 - wv[u][3]) * qv[u][3];
              for (int j = a0[u] + 2; j < a1[u]; ++j) acc += (1.0 - w_at(sr, j)) * q_at(sr, j);
            }
            unsigned long long hm = __ballot(heavy);
            while (hm) {   // a destination with many sources: its whole wave, fixed order
              const int h = __builtin_ctzll(hm);
              hm &= hm - 1ull;
              const int b0 = __builtin_amdgcn_readlane(a0[u], h), b1 = __builtin_amdgcn_readlane(a1[u], h),
                        b2 = __builtin_amdgcn_readlane(a2[u], h);
              double pa = 0.0, pb = 0.0;
              for (int j = b1 + lane; j < b2; j += kWave) pa += w_at(sr, j) * q_at(sr, j);
              for (int j = b0 + lane; j < b1; j += kWave) pb += (1.0 - w_at(sr, j)) * q_at(sr, j);
              const double ta = wave_sum_lane63(pa), tb = wave_sum_lane63(pb);
              const double tot = __shfl(ta, kWave - 1, kWave) + __shfl(tb, kWave - 1, kWave);
              if (lane == h) acc = tot;
            }
            T[sr] = acc;
          }
        }
      }
#pragma unroll
      for (int sp = 0; sp < SMAX; ++sp) {
        double pc[SMAX];
        asm volatile("" ::: "memory");   // one column of P at a time
#pragma unroll
        for (int s = 0; s < SMAX; ++s) pc[s] = s_P[s * SMAX + sp];
        double acc = 0.0;
#pragma unroll
        for (int s = 0; s < SMAX; ++s) acc += pc[s] * T[s];
        out[k][sp] = acc;
      }
    }
  };
  // one matvec: out = T q (the cluster exchange in the middle)
  auto matvec = [&](const double (&q)[KC][SMAX], double (&out)[KC][SMAX]) -> bool {
    if constexpr (PULL) {
      HK_PH(5);
      stage_q(q);
      HK_PH(1);
      if (!barrier()) return false;
      HK_PH(2);
      pull_mix(out);
      HK_PH(3);
      return true;
    }
    HK_PH(5);
    push(q);
    HK_PH(0);
    const int par = (int)((nb + 1) & 1);
    publish(par);
    HK_PH(1);
    if (!barrier()) return false;
    HK_PH(2);
    gather_mix(par, out);
    HK_PH(3);
    return true;
  };
  // cluster-wide reduction of NV per-thread partials (bit v of kmax: nan_max, else sum),
  // fixed order at every level, so every workgroup gets the same s_res
  // cluster-wide reduction of NV per-thread partials (bit v of kmax: nan_max, else sum),
  // fixed order at every level, so every workgroup gets the same s_res.  The workgroup's
  // values travel as tagged 8-byte granules ({epoch, 32 data bits}, two per double, sc1
  // stores; MI355X_MICROARCH.md hand-off R2): the data is its own flag, so there is no
  // counter barrier and no store drain -- wave 0 re-reads the cluster's granules until
  // every tag carries this reduction's epoch.  Epochs count up from 1 within a launch (the
  // host zeroes the granules before each launch); slots alternate by epoch parity, and a
  // matvec barrier separates any two reductions, so a slot is rewritten only after every
  // workgroup has read it.
  // the workgroup's wave partials of nv values into s_part (visible after the next barrier)
  auto wave_parts = [&](const double* vals, int nv, unsigned kmax) {
#pragma unroll
    for (int v = 0; v < kHkRed; ++v) {
      if (v < nv) {
        const double x = (kmax >> v) & 1u ? wave_nan_max(vals[v]) : wave_sum_lane63(vals[v]);
        if (lane == kWave - 1) s_part[v][wid] = x;
      }
    }
  };
  // threads < nv: the workgroup's values (waves in fixed order) as two tagged granules each
  auto store_granules = [&](unsigned long long* slot, unsigned long long tag, int nv, unsigned kmax) {
    if (tid < nv) {
      const int v = tid;
      double x = s_part[v][0];
      for (int q = 1; q < TH / kWave; ++q) x = (kmax >> v) & 1u ? nan_max(x, s_part[v][q]) : x + s_part[v][q];
      const unsigned long long b = (unsigned long long)__double_as_longlong(x);
      unsigned long long* g = slot + (size_t)w * (2 * kHkRed) + 2 * v;
      __hip_atomic_store(to_global(g), tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(to_global(g + 1), tag | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // wave 0: every workgroup's granules (until every tag carries this epoch), fixed-order sums
  // into s_res; *s_ok = 0 on timeout (error word set)
  auto sweep = [&](const unsigned long long* slot, unsigned long long tag, int nv, unsigned kmax, int* s_ok) {
    {
      double xa[kHkRed], xb[kHkRed];
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      bool ok;
      do {   // every granule load of a pass in flight before the tag test
        ok = true;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int w2 = lane + u * kWave;
#pragma unroll
          for (int v = 0; v < kHkRed; ++v) {
            double x = 0.0;
            if (v < nv && w2 < G) {
              const unsigned long long* g = slot + (size_t)w2 * (2 * kHkRed) + 2 * v;
              const unsigned long long hi = __hip_atomic_load(to_global(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const unsigned long long lo = __hip_atomic_load(to_global(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ok = ok && (hi & 0xffffffff00000000ull) == tag && (lo & 0xffffffff00000000ull) == tag;
              x = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
            }
            if (u == 0) xa[v] = x;
            else xb[v] = x;
          }
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kHcTimeoutTicks) {
          if (lane == 0) __hip_atomic_store(to_global(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      } while (true);
      if (lane == 0) *s_ok = ok ? 1 : 0;
#pragma unroll
      for (int v = 0; v < kHkRed; ++v) {
        if (v < nv) {
          const bool mx = (kmax >> v) & 1u;
          const double y = mx ? wave_nan_max(nan_max(xa[v], xb[v])) : wave_sum_lane63(xa[v] + xb[v]);
          if (lane == kWave - 1) s_res[v] = y;
        }
      }
    }
  };
  auto reduce = [&](double (&vals)[kHkRed], int nv, unsigned kmax, auto&& prefetch) -> bool {
    HK_PH(5);
    wave_parts(vals, nv, kmax);
    __syncthreads();
    ++ne;
    const unsigned long long tag = (unsigned long long)ne << 32;
    unsigned long long* slot = gran + (size_t)(ne & 1) * G * (2 * kHkRed);
    store_granules(slot, tag, nv, kmax);
    prefetch();   // loads the step after the reduction needs, in flight across the sweep
    if (wid == 0) sweep(slot, tag, nv, kmax, &s_flag);
    __syncthreads();
    HK_PH(4);
    return s_flag != 0;
  };
  // one matvec out = T q whose cluster barrier also carries a reduction of nv values computed
  // before it (pipelined BiCGSTAB): the granules are stored before the publish's store drain,
  // so every workgroup's are in memory once the barrier has passed; wave 0 reads them while
  // the other waves gather, and s_res is valid on return
  // do_push(): the push of the matvec input (ends with a workgroup barrier)
  auto matvec_rp = [&](auto&& do_push, double (&out)[KC][SMAX], const double* vals, int nv, unsigned kmax) -> bool {
    HK_PH(5);
    wave_parts(vals, nv, kmax);
    do_push();   // ends with a workgroup barrier: s_part complete
    HK_PH(0);
    ++ne;
    const unsigned long long tag = (unsigned long long)ne << 32;
    unsigned long long* slot = gran + (size_t)(ne & 1) * G * (2 * kHkRed);
    store_granules(slot, tag, nv, kmax);
    const int par = (int)((nb + 1) & 1);
    publish(par);   // every thread's s_waitcnt vmcnt(0): slabs and granules drained
    HK_PH(1);
    if (!barrier()) return false;
    HK_PH(2);
    // the sweep by the last wave: with one column per thread its lanes own no columns whenever
    // a workgroup has <= TH - 64 of them (G >= 23 at N_a = 10 000), so it overlaps the gather
    if (wid == TH / kWave - 1) sweep(slot, tag, nv, kmax, L.s_rok);
    gather_mix(par, out);
    __syncthreads();
    HK_PH(3);
    return *L.s_rok != 0;
  };
  auto matvec_r = [&](const double (&q)[KC][SMAX], double (&out)[KC][SMAX], const double* vals, int nv,
                      unsigned kmax) -> bool { return matvec_rp([&] { push(q); }, out, vals, nv, kmax); };
  // ---- BiCGSTAB ----
  // registers: r (then s), p, and the matvec result; v waits in LDS (behind the spans) and
  // p in the HBM scratch row across the second matvec, whose gather needs the registers
  double rv[KC][SMAX], pv[KC][SMAX], tv[KC][SMAX];
  // v: in LDS behind the spans when it fits (SMAX <= 8), else a per-workgroup HBM block of
  // the same [KC][SMAX][TH] layout (behind the p rows of the scratch)
  double* Vl = kVlds ? Tacc + cap : (double*)r.Vg;
  double* Pg = (double*)r.Pg;
  auto vidx = [&](int k, int s) { return (k * SMAX + s) * TH + tid; };
  double part[kHkRed];
  const double tol = r.tol;
  int mv = 0;                 // matvecs
  bool restart = true, first = true;
  double rho = 0.0, total0 = 0.0;
  auto own = [&](int jc, int k, int s) { return s < S && jc + k * TH < j1; };
  unsigned seed = 0;   // shadow-residual choice; a stagnating solve restarts with the next one
  auto rh_at = [&](int jc, int k, int s) { return hk_rhat((unsigned)(s * n_a + jc + k * TH) + seed * 0x5BD1E995u); };
  double best = __builtin_inf();   // best recursive max|r| since the last restart, and when
  int mv_best = 0;
  auto gidx = [&](int jc, int k, int s) { return (size_t)s * n_a + jc + k * TH; };
  // FUSEA (one column per thread, the resident search): alpha's reduction rides on the first
  // matvec's cluster barrier.  <rh, v> = <rh, A p> = <A^T rh, p> with A = I - T, and
  // u = A^T rh is fixed for a solve (a new shadow residual recomputes it): its own points sit in
  // the Qg rows, and <u, p> is formed when p is, before the matvec.  One cluster reduction per
  // iteration instead of two; the same recurrence otherwise.
  //   (T^T y)[s][j] = sum_s' P[s, s'] (wlo y[s'][lo] + (1 - wlo) y[s'][lo + 1])
  double* Ug = (double*)r.Qg;
  double pu = 0.0;   // this thread's part of <u, p>
  auto make_u = [&]() {   // u of the own points -> Ug; pu = <u, p> with p = r
    if constexpr (FUSEA) {
      const int jc = col();
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          if (own(jc, k, s)) {
            int d;
            double wl;
            if constexpr (kLoReg) {
              d = dreg[k][s];
              wl = wreg[k][s];
            } else {   // (two columns per thread: the own lottery from L2, once per solve)
              d = LO[gidx(jc, k, s)];
              wl = WL[gidx(jc, k, s)];
            }
            double tr = 0.0;
            for (int sp = 0; sp < S; ++sp) {
              const unsigned q = (unsigned)(sp * n_a + d) + seed * 0x5BD1E995u;
              tr += s_P[s * SMAX + sp] * (wl * hk_rhat(q) + (1.0 - wl) * hk_rhat(q + 1u));
            }
            const double u = rh_at(jc, k, s) - tr;
            Ug[gidx(jc, k, s)] = u;
            acc += u * pv[k][s];
          }
        }
      pu = acc;
    }
  };
  // FUSEA with two columns per thread: u of the own points is read back when the new p is formed
  // (AIY_FUSEA_KC2 = 1: prefetched with x and p across the second reduction; 2: loaded after it,
  // beside the new p, so it holds no registers across the reduction)
#ifndef AIY_FUSEA_KC2
#define AIY_FUSEA_KC2 0
#endif
  constexpr bool kUqPre = KC == 1 || AIY_FUSEA_KC2 == 1;
  HK_PH(-1);
  while (true) {
    if (restart) {
      // true residual of x: pv = x, tv = T x, rv = T x - x
      int jc = col();
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          const double xv = X[min(s, S - 1) * n_a + min(jc + k * TH, n_a - 1)];
          pv[k][s] = own(jc, k, s) ? xv : 0.0;
        }
      if (!matvec(pv, tv)) return -1;
      ++mv;
      jc = col();
      double rr = 0.0, rm = 0.0, xs = 0.0;
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          rv[k][s] = tv[k][s] - pv[k][s];
          if (own(jc, k, s)) {
            rr += rh_at(jc, k, s) * rv[k][s];
            rm = nan_max(rm, fabs(rv[k][s]));
            xs += pv[k][s];
          }
        }
      part[0] = rr;
      part[1] = rm;
      part[2] = xs;
      if (!reduce(part, 3, 2u, [] {})) return -1;
      rho = s_res[0];
      if (mv == 1) total0 = s_res[2];   // the starting mass's total
      if (s_res[1] < tol || mv >= r.max_iter) {   // converged (np.max(...) < tol: NaN never is)
        // T x rescaled to the start's total: the residual test cannot see the scale of x,
        // and near a breakdown (huge alpha) rounding can move sum(x) away from it; T
        // preserves totals, as the plain iteration does
        const double scale = total0 / s_res[2];
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
          for (int s = 0; s < SMAX; ++s)
            if (own(jc, k, s)) X[gidx(jc, k, s)] = mv == 1 ? tv[k][s] : tv[k][s] * scale;
        break;
      }
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) pv[k][s] = rv[k][s];
      make_u();
      restart = false;
      first = true;
    }
    // v = p - T p (to LDS); alpha = rho / <rh, v>; the previous step's max|r| rides along.
    // r waits in v's slot during this matvec (only p and the result stay in registers)
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) Vl[vidx(k, s)] = rv[k][s];
    // rebalancing stop request: polled every 8th iteration by thread 0 into LDS (the matvec's
    // barriers make it visible; the partial below carries it to every workgroup).  mv grows by
    // 2 per iteration and is odd after a restart's true-residual matvec, so the iteration
    // number is mv >> 1
    if (r.stop_ctr != nullptr && tid == 0 && ((mv >> 1) & 7) == 0)
      s_stop = __hip_atomic_load((const unsigned*)r.stop_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= r.stop_at;
    double xq[KC][SMAX];   // x of the own points, for x += alpha p
    int jc;
    if constexpr (FUSEA) {
      // <u, p> and max|r| ride on this matvec's barrier (the stop request as a sentinel on the
      // max, which no residual of a mass vector reaches); x's loads in flight across it (one
      // column per thread; with two, x is loaded after the matvec: its registers are full)
      jc = col();
      double rm = 0.0;
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          if (own(jc, k, s)) rm = nan_max(rm, fabs(Vl[vidx(k, s)]));
          if constexpr (KC == 1) xq[k][s] = X[min(s, S - 1) * n_a + min(jc + k * TH, n_a - 1)];
        }
      part[0] = pu;
      part[1] = (r.stop_ctr != nullptr && tid == 0 && s_stop) ? kHkStopSentinel : rm;
      if (!matvec_r(pv, tv, part, 2, 2u)) return -1;
      ++mv;
      jc = col();
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          const double v = pv[k][s] - tv[k][s];
          rv[k][s] = Vl[vidx(k, s)];
          Vl[vidx(k, s)] = v;
          if constexpr (KC > 1) xq[k][s] = X[min(s, S - 1) * n_a + min(jc + k * TH, n_a - 1)];
        }
    } else {
      if (!matvec(pv, tv)) return -1;
      ++mv;
      jc = col();
      double rvv = 0.0, rm = 0.0;
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          const double v = pv[k][s] - tv[k][s];
          rv[k][s] = Vl[vidx(k, s)];
          Vl[vidx(k, s)] = v;
          if (own(jc, k, s)) {
            rvv += rh_at(jc, k, s) * v;
            rm = nan_max(rm, fabs(rv[k][s]));
          }
        }
      part[0] = rvv;
      // the stop request rides on the max|r| partial as a sentinel no residual of a mass vector
      // reaches (the cluster max is the same in every workgroup)
      part[1] = (r.stop_ctr != nullptr && tid == 0 && s_stop) ? kHkStopSentinel : rm;
      if (!reduce(part, 2, 2u, [&] {
            const int jq = col();
#pragma unroll
            for (int k = 0; k < KC; ++k)
#pragma unroll
              for (int s = 0; s < SMAX; ++s) xq[k][s] = X[min(s, S - 1) * n_a + min(jq + k * TH, n_a - 1)];
          }))
        return -1;
    }
    if (s_res[1] >= kHkStopSentinel) return -(2 + mv);   // every workgroup reads the same max
    if ((!first && s_res[1] < tol) || mv >= r.max_iter) {   // recursive residual converged: verify
      restart = true;
      continue;
    }
    // stagnation (BiCGSTAB can stall for a particular shadow residual: one Table II cell
    // sat at max|r| ~ 6e-5 with the first hash): no 10 % gain in kHkStall matvecs ->
    // restart from the true residual with the next shadow residual
    if (first || s_res[1] < 0.9 * best) {
      best = first ? __builtin_inf() : s_res[1];
      mv_best = mv;
    } else if (mv - mv_best > kHkStall) {
      ++seed;
      best = __builtin_inf();
      restart = true;
      continue;
    }
    first = false;
    const double alpha = rho / s_res[0];
    if (!(fabs(alpha) < 1e300)) {   // breakdown (<rh, v> = 0) or NaN: restart from the true residual
      restart = true;
      continue;
    }
    // x += alpha p; p -> HBM scratch; s = r - alpha v (in rv); t = s - T s (in tv)
    jc = col();
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        if (own(jc, k, s)) {
          const int g = s * n_a + jc + k * TH;
          X[g] = xq[k][s] + alpha * pv[k][s];
          Pg[g] = pv[k][s];
        }
        rv[k][s] -= alpha * Vl[vidx(k, s)];
      }
    if (!matvec(rv, tv)) return -1;
    ++mv;
    jc = col();
    double ts = 0.0, tt = 0.0, rs = 0.0, rt = 0.0, sm = 0.0;
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        tv[k][s] = rv[k][s] - tv[k][s];
        if (own(jc, k, s)) {
          const double h = rh_at(jc, k, s);
          ts += tv[k][s] * rv[k][s];
          tt += tv[k][s] * tv[k][s];
          rs += h * rv[k][s];
          rt += h * tv[k][s];
          sm = nan_max(sm, fabs(rv[k][s]));
        }
      }
    part[0] = ts;
    part[1] = tt;
    part[2] = rs;
    part[3] = rt;
    part[4] = sm;
    double pq[KC][SMAX];   // x and p of the own points, for x += omega s and the new p
    double uq[FUSEA && kUqPre ? KC : 1][SMAX];   // FUSEA: u of the own points, for <u, p> of the new p
    if (!reduce(part, 5, 16u, [&] {
          const int jq = col();
#pragma unroll
          for (int k = 0; k < KC; ++k)
#pragma unroll
            for (int s = 0; s < SMAX; ++s) {
              const int g = min(s, S - 1) * n_a + min(jq + k * TH, n_a - 1);
              xq[k][s] = X[g];
              pq[k][s] = Pg[g];
              if constexpr (FUSEA && kUqPre) uq[k][s] = Ug[g];
            }
        }))
      return -1;
    double omega = (s_res[4] < tol) ? 0.0 : s_res[0] / s_res[1];
    if (!(fabs(omega) < 1e300)) omega = 0.0;
    if (omega == 0.0) {   // s already below tol (x + alpha p is the answer), or <t, t> = 0: verify
      restart = true;
      continue;
    }
    const double rho2 = s_res[2] - omega * s_res[3];
    const double beta = (rho2 / rho) * (alpha / omega);
    rho = rho2;
    // x += omega s; r = s - omega t; p = r + beta (p - omega v)
    jc = col();
    double pun = 0.0;
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        const bool ow = own(jc, k, s);
        if (ow) X[s * n_a + jc + k * TH] = xq[k][s] + omega * rv[k][s];
        const double pold = ow ? pq[k][s] : 0.0;
        rv[k][s] = rv[k][s] - omega * tv[k][s];
        pv[k][s] = rv[k][s] + beta * (pold - omega * Vl[vidx(k, s)]);
        if constexpr (FUSEA && kUqPre)
          if (ow) pun += uq[k][s] * pv[k][s];
      }
    if constexpr (FUSEA && !kUqPre) {   // u read back beside the new p (every load before the first use)
      double ul[KC][SMAX];
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s) ul[k][s] = Ug[min(s, S - 1) * n_a + min(jc + k * TH, n_a - 1)];
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int s = 0; s < SMAX; ++s)
          if (own(jc, k, s)) pun += ul[k][s] * pv[k][s];
    }
    pu = pun;
    if (!(fabs(beta) < 1e300) || rho == 0.0) restart = true;
  }
#ifdef AIY_DIAG_PHASES
  if (tid == 0 && blockIdx.x >= AIY_DIAG_PHASES && blockIdx.x < AIY_DIAG_PHASES + 10 && mv > 0)
    printf("[bicg phases] block %d G=%d nj=%d matvecs=%d us/matvec: push %.2f publish %.2f barrier %.2f gather+mix "
           "%.2f reduce %.2f vector %.2f\n",
           (int)blockIdx.x, G, j1 - j0, mv, ph[0] * 0.01 / mv, ph[1] * 0.01 / mv, ph[2] * 0.01 / mv, ph[3] * 0.01 / mv,
           ph[4] * 0.01 / mv, ph[5] * 0.01 / mv);
#endif
  return mv;
}

// hk_solve as its own (not inlined) function with its LDS declared here: a caller that
// carries a lot of live state of its own (ge_resident.hip's search loop) would otherwise
// force the solve's registers into scratch; the call costs a few register saves per
// solve.  The span buffer / v share the caller's dynamic LDS.
template <int SMAX, int KC, int TH, bool PULL = false, bool FUSEA = false>
__device__ __noinline__ int hk_solve_isolated(HkArgs a, unsigned* nb_io, unsigned* ne_io);
// the same body inlined into the caller (the pull form spilled more as a separate function)
template <int SMAX, int KC, int TH, bool PULL = false, bool FUSEA = false>
__device__ __forceinline__ int hk_solve_inlined(HkArgs a, unsigned* nb_io, unsigned* ne_io) {
  extern __shared__ double hk_dyn_in[];
  __shared__ int s_base[SMAX];
  __shared__ int s_pub[2 * SMAX][2];
  __shared__ int s_tot;
  __shared__ HcCand s_cand[SMAX][kHcCand];
  __shared__ int s_ncand[SMAX];
  __shared__ unsigned short s_cinfo[PULL ? 1 : KC * SMAX * TH];
  __shared__ double s_P[SMAX * SMAX];
  __shared__ double s_part[kHkRed][TH / kWave];
  __shared__ double s_res[kHkRed];
  __shared__ int s_flag, s_stop;
  __shared__ int s_ex[2 * SMAX];
  __shared__ int s_nheavy, s_heavy[kHkHeavy][4], s_rok, s_wcnt[TH / kWave];
  __shared__ double s_hval[kHkHeavy];
  HkShared<SMAX, KC, TH> L{hk_dyn_in, s_base, s_pub, &s_tot, s_cand, s_ncand, s_cinfo, s_P, s_part, s_res,
                                 &s_flag, &s_stop, s_ex, &s_nheavy, s_wcnt, s_heavy, s_hval, &s_rok};
  unsigned nb = *nb_io, ne = *ne_io;
  const int mv = hk_solve<SMAX, KC, TH, PULL, FUSEA>(a, L, nb, ne);
  *nb_io = nb;
  *ne_io = ne;
  return mv;
}
template <int SMAX, int KC, int TH, bool PULL, bool FUSEA>
__device__ __noinline__ int hk_solve_isolated(HkArgs a, unsigned* nb_io, unsigned* ne_io) {
  extern __shared__ double hk_dyn[];
  __shared__ int s_base[SMAX];
  __shared__ int s_pub[2 * SMAX][2];
  __shared__ int s_tot;
  __shared__ HcCand s_cand[SMAX][kHcCand];
  __shared__ int s_ncand[SMAX];
  __shared__ unsigned short s_cinfo[KC * SMAX * TH];
  __shared__ double s_P[SMAX * SMAX];
  __shared__ double s_part[kHkRed][TH / kWave];
  __shared__ double s_res[kHkRed];
  __shared__ int s_flag, s_stop;
  __shared__ int s_ex[2 * SMAX];
  __shared__ int s_nheavy, s_heavy[kHkHeavy][4], s_rok, s_wcnt[TH / kWave];
  __shared__ double s_hval[kHkHeavy];
  HkShared<SMAX, KC, TH> L{hk_dyn, s_base, s_pub, &s_tot, s_cand, s_ncand, s_cinfo, s_P, s_part, s_res,
                                 &s_flag, &s_stop, s_ex, &s_nheavy, s_wcnt, s_heavy, s_hval, &s_rok};
  unsigned nb = *nb_io, ne = *ne_io;
  const int mv = hk_solve<SMAX, KC, TH, PULL, FUSEA>(a, L, nb, ne);
  *nb_io = nb;
  *ne_io = ne;
  return mv;
}

}  // namespace aiy
