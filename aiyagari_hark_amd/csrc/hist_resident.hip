// Device-resident Young-lottery distribution iteration (build-defined row E2) for gfx950:
// a whole aiy_hist_solve in ONE launch, every iteration inside the kernel.
//
// The push/mix pair (hist.hip) costs two dependent launches per iteration (~15 us at
// Table II size, thousands of iterations per GE step).  Here each calibration gets a
// CLUSTER of G workgroups (one per CU) that iterates on its own, synchronised by a
// per-calibration counter instead of kernel boundaries:
//   * workgroup w of a cluster owns asset columns [j0, j1) of every income state: the
//     mass of those columns lives in REGISTERS for the whole solve (thread t holds columns
//     j0 + t + k * TH, all S states; with S <= 8 also their lottery);
//   * push (sources = own columns): T_s[lo] += w m, T_s[lo + 1] += (1 - w) m, accumulated
//     with LDS f64 atomics into a per-row destination SPAN buffer: a monotone lottery maps
//     the contiguous source range to the contiguous destination range
//     [lo(j0), lo(j1 - 1) + 1] of each row;
//   * the parts of the spans outside the own columns are published write-through (sc1) as
//     the workgroup's slab (the own part stays in LDS); one cluster barrier (agent-scope
//     counter, sc1 polls);
//   * gather (destinations = own columns): T_s[d] = sum of the slabs whose span covers d
//     (the covering workgroups are fixed for the whole solve and found once at start), in
//     ascending workgroup order, every load of a row group issued before the first use;
//   * mix: mass'[s'][d] = sum_s P[s, s'] T_s[d] (P broadcast from LDS); the sup-norm change is reduced
//     to one published value per workgroup, read by the cluster after the NEXT barrier:
//     the solve stops exactly where oracle/stationary.py stationary_hist stops (first
//     iteration with max |mass' - mass| < tol) and keeps that iteration's mass.
// Per iteration: the mass and (S <= 8) the lottery stay in registers, only the span
// entries that cross a workgroup boundary go through memory (write-through slab, MALL),
// no global atomics, one barrier.
// Shapes that do not fit (spans beyond the LDS budget, more covering workgroups per row
// than kHcCand, a non-monotone lottery) abort before the first iteration and the host
// runs the push/mix pair instead.
#include "common.h"
#include "internal.h"
#include "hist_cluster.h"

#include <algorithm>
#include <type_traits>

namespace aiy {

#ifdef AIY_DIAG_PHASES
#define HC_PH(k)                                                        \
  do {                                                                  \
    if (tid == 0 && blockIdx.x == AIY_DIAG_PHASES) {                    \
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

template <int SMAX, int KC, int TH>
__global__ __launch_bounds__(TH) void hist_cluster_kernel(HcRun r) {
#ifdef AIY_DIAG_PHASES
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tq = 0;
#endif
  // Span buffer (LDS Tacc and the published slab alike): row after row, destination d of
  // row s at s_base[s] + d.  Only the parts outside the own columns are published
  // (s_pub: per row the ranges below j0 and from j1 on).
  extern __shared__ double Tacc[];
  __shared__ int s_base[SMAX];
  __shared__ int s_pub[2 * SMAX][2];
  __shared__ int s_tot;
  __shared__ HcCand s_cand[SMAX][kHcCand];
  __shared__ int s_ncand[SMAX];
  __shared__ double s_red[TH / kWave];
  __shared__ int s_cinfo[KC * SMAX * TH];
  __shared__ int s_flag, s_stop;
  __shared__ unsigned s_nc;
  __shared__ double s_dot[2];
  __shared__ double s_dotw[2][TH / kWave];
  __shared__ double s_lam[2], s_fext;
  __shared__ double s_P[SMAX * SMAX];              // P[s][s'] zero-padded to SMAX x SMAX

  const int tid = threadIdx.x;
  const int G = r.G, S = r.S, n_a = r.n_a, cap = r.cap;
  const int lc = blockIdx.x / G;                   // calibration within this launch
  const int w = blockIdx.x - lc * G;
  const int cal = r.cal0 + lc;
  const int j0 = w * r.nj;
  const int j1 = min(j0 + r.nj, n_a);
  unsigned* ctr = r.ctr + (size_t)lc * kHcCtrStride;
  unsigned long long* cw = reinterpret_cast<unsigned long long*>(ctr + 2);   // [2] per-parity words
  double* dist = r.dist + (size_t)lc * 2 * G * 4;
  double* DB = r.dbuf ? r.dbuf + (size_t)cal * S * n_a : nullptr;
  const int E = r.accel;
  const size_t row0 = (size_t)cal * S;
  const int* LO = r.lo + row0 * n_a;
  const double* WL = r.wlo + row0 * n_a;
  double* MS = r.mass + row0 * n_a;
  double* slab_cl = r.slab + (size_t)lc * G * 2 * cap;
  const double* __restrict__ Pc = r.P + (size_t)cal * S * S;
  int* span_cl = r.span + (size_t)lc * G * SMAX * 4;   // per (w, s): first, len, base

  // ---- setup: P, own spans and their layout, mass -> registers ----
  for (int q = tid; q < SMAX * SMAX; q += TH) {
    const int s = q / SMAX, sp = q - s * SMAX;
    s_P[q] = (s < S && sp < S) ? Pc[s * S + sp] : 0.0;
  }
  if (tid == 0) {
    int tot = 0;
    unsigned bad = 0;
    for (int s = 0; s < S; ++s) {
      const int f = LO[(size_t)s * n_a + j0];
      const int l = LO[(size_t)s * n_a + j1 - 1] - f + 2;   // destinations lo .. lo_last + 1
      if (l < 2 || f < 0 || f + l > n_a) bad = 2u;          // not a monotone lottery of ours
      const int ll = l > 0 ? l : 0;
      s_base[s] = tot - f;
      // foreign parts of the row: destinations below j0 and from j1 on
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
    if (tot > cap) bad = 2u;
    if (bad) __hip_atomic_store(to_global(r.err), bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  if (tid == 0) s_stop = __hip_atomic_load(to_global(r.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return;
  // covering workgroups of every row for this workgroup's columns, ascending w
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
      __hip_atomic_store(to_global(r.err), 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  const int total = s_tot;
  for (int q = tid; q < total; q += TH) Tacc[q] = 0.0;
  if (!hc_barrier(r, ctr, 2u * G, &s_flag)) return;
  if (tid == 0) s_stop = __hip_atomic_load(to_global(r.err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
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
  double aloc = 0.0, bloc = 0.0;   // Aitken dot products of the last mix
  unsigned nc_prev[2] = {0u, 0u};  // thread 0: flag counts of the two parities
  int final_it = 0;
  if (tid == 0) {
    s_lam[0] = s_lam[1] = -1.0;
    s_fext = 0.0;
  }
  // the lottery (lo, weight) of the own columns is fixed for the whole solve: with S <= 8
  // it is held in registers, loaded once (larger S re-read it from L2 every iteration)
  constexpr bool kLoReg = SMAX == 8;
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
  // per-row span bases (lane s) and publish ranges (lane r: [lo, hi)) held in VGPR lanes,
  // read with v_readlane inside the loop (no LDS round trip per row)
  const int v_base = lane < S ? s_base[lane] : 0;
  const int v_plo = lane < 2 * S ? s_pub[lane][0] : 0;
  const int v_phi = lane < 2 * S ? s_pub[lane][1] : 0;
  // Aitken phases of mix `it` (it % E): E - 2 store the difference; E - 1 and 0 form the
  // dot products <d_it, d_it-1>, |d_it-1|^2 of two consecutive ratio estimates; at 1 the
  // cluster may extrapolate along d_it (s_fext, decided from those two estimates)
  auto is_dot = [&](int i) { return E > 0 && i >= E - 1 && (i % E == E - 1 || i % E == 0); };
  for (int it = 1; it <= r.max_iter; ++it) {
    const int par = it & 1;
    HC_PH(0);
    // ---- push own sources into the span buffer ----
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
            if constexpr (kLoReg) {
              dd[k][q] = dreg[k][s];
              ww[k][q] = wreg[k][s];
            } else {
              const bool ok = s < S && j < j1;
              dd[k][q] = ok ? LO[(size_t)s * n_a + j] : -1;
              ww[k][q] = ok ? WL[(size_t)s * n_a + j] : 0.0;
            }
          }
        }
        // one LDS f64 atomic per lane and destination: adjacent lanes hit adjacent
        // destinations (no conflict) except on the borrowing constraint, where the whole
        // wave shares one destination and a DPP wave sum replaces 64 same-address atomics
        // (a general segmented scan costs ~1.4k cycles of dependent cross-lane steps per
        // row: measured 17 us per iteration for the push at Table II size)
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
              const int ilo = __builtin_amdgcn_readlane(v_base, s) + d, ihi = ilo + 1;
              const int d0 = __builtin_amdgcn_readfirstlane(d);
              if (__all(act && d == d0)) {
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
    HC_PH(1);
    // ---- publish the parts of the spans outside the own columns write-through and re-zero
    // them; the own part stays in LDS for the own gather ----
    double* slab = slab_cl + ((size_t)w * 2 + par) * cap;
    for (int rr = 0; rr < 2 * S; ++rr) {
      const int lo = __builtin_amdgcn_readlane(v_plo, rr), hi = __builtin_amdgcn_readlane(v_phi, rr);
      for (int q = lo + tid; q < hi; q += TH) {
        store_f64_agent(&slab[q], Tacc[q]);
        Tacc[q] = 0.0;
      }
    }
    const bool dot_prev = is_dot(it - 1);   // mix it - 1 formed Aitken dot products
    if (tid == 0 && dot_prev) {
      double* dp = &dist[((size_t)((it - 1) & 1) * G + w) * 4];
      store_f64_agent(&dp[1], aloc);
      store_f64_agent(&dp[2], bloc);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HC_PH(2);
    // the barrier carries the stop test: flag = change of mix it - 1 not below tol (NaN
    // included, as np.max(...) < tol is False for NaN)
    const unsigned flag = (it >= 2 && dloc < r.tol) ? 0u : 1u;
    if (!hc_barrier_count(r.err, &cw[par], (unsigned)G * (unsigned)((it + par) / 2), flag, &s_nc, &s_flag)) return;
    HC_PH(3);
    // ---- gather own destinations from the covering spans (ascending w): foreign ones from
    // their slabs, the own one from LDS ----
    constexpr int GR = HcGather<SMAX, KC, TH>::kRows;
    double T[KC][SMAX];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int s = 0; s < SMAX; ++s) T[k][s] = 0.0;   // rows beyond S stay 0 (padded mix)
    bool more = false;
#pragma unroll
    for (int s0 = 0; s0 < SMAX; s0 += GR) {
      if (s0 < S) {
        double v0[KC][GR], v1[KC][GR];
        int oq[KC][GR];   // LDS index of the own span's share, -1: none among the first two
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
              const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = ci & 255, cn = ci >> 8;
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
              more = more || cn > 2;
            }
          }
        }
        // the own span's share once every slab load of the group is in flight (with two
        // covering spans the sum does not depend on their order)
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
    // stop where the oracle stops: the first iteration whose max change is < tol, keeping
    // that iteration's mass (no flag of this barrier's parity was added)
    if (it >= 2 && s_nc == nc_prev[par]) {
      final_it = it - 1;
      break;
    }
    nc_prev[par] = s_nc;
    if (dot_prev) {   // Aitken: the cluster's dot products of mix it - 1
      if (tid < kWave) {
        const double* dq = &dist[(size_t)((it - 1) & 1) * G * 4];
        double xa[2], xb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int w2 = lane + u * kWave;
          const bool ok = w2 < G;
          xa[u] = ok ? load_f64_agent(&dq[w2 * 4 + 1]) : 0.0;
          xb[u] = ok ? load_f64_agent(&dq[w2 * 4 + 2]) : 0.0;
        }
        // fixed-order sums over the workgroups (lane pairs, then the DPP tree)
        const double asum = wave_sum_lane63(xa[0] + xa[1]);
        const double bsum = wave_sum_lane63(xb[0] + xb[1]);
        if (lane == kWave - 1) {
          s_dot[0] = asum;
          s_dot[1] = bsum;
        }
      }
      __syncthreads();
      if (tid == 0) {
        const double a = s_dot[0], b = s_dot[1];
        const int ph = (it - 1) % E;           // E - 1: first estimate, 0: second
        s_lam[ph == 0 ? 1 : 0] = b > 0.0 ? a / b : -1.0;
        if (it > E && it % E == 1) {
          const double l0 = s_lam[0], l1 = s_lam[1];
          if (l1 > 0.5 && l1 < 1.0 - 1e-9 && fabs(l1 - l0) < 1e-3 * (1.0 - l1)) s_fext = l1 / (1.0 - l1);
          s_lam[0] = s_lam[1] = -1.0;
        }
      }
      __syncthreads();
    }
    HC_PH(4);
    if (__any(more)) {   // columns covered by > 2 spans (the borrowing constraint)
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int d = j0 + tid + k * TH;
#pragma unroll
        for (int s = 0; s < SMAX; ++s) {
          if (s < S) {
            const int ci = s_cinfo[(k * SMAX + s) * TH + tid], cf = ci & 255, cn = ci >> 8;
            for (int c0 = 2; c0 < cn; c0 += 4) {   // four loads in flight per step
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
    HC_PH(5);
    const int aph = E > 0 ? it % E : -1;
    const bool a_store = E > 0 && (aph == E - 2 || aph == E - 1);
    const bool a_dot = is_dot(it);
    const double fext = s_fext;
    double dmax = 0.0, ap = 0.0, bp = 0.0;
    // branch-free over the padded SMAX x SMAX block (rows and columns beyond S and the
    // columns beyond j1 carry zeros), one column of P in registers at a time (the next
    // one's LDS reads in flight; the empty asm keeps the compiler from hoisting all of P
    // into registers), the Aitken bookkeeping (2-3 of every E iterations) in its own copy
    auto mix = [&](auto aitken) {
      double pc[SMAX], pn[SMAX];
#pragma unroll
      for (int s = 0; s < SMAX; ++s) pc[s] = s_P[s * SMAX];
#pragma unroll
      for (int sp = 0; sp < SMAX; ++sp) {
        if (sp + 1 < SMAX) {
#pragma unroll
          for (int s = 0; s < SMAX; ++s) pn[s] = s_P[s * SMAX + sp + 1];
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int j = j0 + tid + k * TH;
          double acc = 0.0;
#pragma unroll
          for (int s = 0; s < SMAX; ++s) acc += pc[s] * T[k][s];   // P.T @ T
          const double dnew = acc - m[k][sp];
          dmax = nan_max(dmax, fabs(dnew));
          if constexpr (decltype(aitken)::value) {
            if (j < j1 && sp < S) {
              if (a_dot) {
                const double dprev = DB[(size_t)sp * n_a + j];
                ap += dnew * dprev;
                bp += dprev * dprev;
              }
              if (a_store) DB[(size_t)sp * n_a + j] = dnew;
            }
          }
          m[k][sp] = acc + fext * dnew;   // fext = 0: acc; else x* ~ x + d lambda / (1 - lambda)
        }
#pragma unroll
        for (int s = 0; s < SMAX; ++s) pc[s] = pn[s];
      }
    };
    if (a_dot || a_store) mix(std::true_type{});
    else mix(std::false_type{});
    HC_PH(6);
    dmax = wave_nan_max(dmax);
    if (lane == 0) s_red[tid / kWave] = dmax;
    if (a_dot) {
      ap = wave_sum_lane63(ap);
      bp = wave_sum_lane63(bp);
      if (lane == kWave - 1) {
        s_dotw[0][tid / kWave] = ap;
        s_dotw[1][tid / kWave] = bp;
      }
    }
    __syncthreads();
    if (tid == 0) {
      double d = s_red[0];
      for (int q = 1; q < TH / kWave; ++q) d = nan_max(d, s_red[q]);
      dloc = d;
      aloc = bloc = 0.0;
      if (a_dot)
        for (int q = 0; q < TH / kWave; ++q) {
          aloc += s_dotw[0][q];
          bloc += s_dotw[1][q];
        }
      s_fext = 0.0;
    }
    HC_PH(7);
    final_it = it;
  }
#ifdef AIY_DIAG_PHASES
  if (tid == 0 && blockIdx.x == AIY_DIAG_PHASES && final_it > 0)
    printf("[hist phases] block %d G=%d nj=%d iters=%d us/iter: push %.2f publish %.2f barrier %.2f gather %.2f "
           "heavy %.2f mix %.2f reduce %.2f\n",
           (int)blockIdx.x, G, r.nj, final_it, ph[0] * 0.01 / final_it, ph[1] * 0.01 / final_it,
           ph[2] * 0.01 / final_it, ph[3] * 0.01 / final_it, ph[4] * 0.01 / final_it, ph[5] * 0.01 / final_it,
           ph[6] * 0.01 / final_it);
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

// Host plan of one cluster launch shape: 512-thread workgroups, one or two columns per
// thread (two only with S <= 8, where the lottery and the mass stay in registers).
struct HcPlan {
  int G = 0, nj = 0, th = 0, kc = 0, smax = 0, cals_per_launch = 0, cap = 0, cw = 0;
  size_t vblock = 0;
  size_t lds = 0;
  const void* fn = nullptr;
  bool pull = false;   // hist_pull.h form (S > 8 BiCGSTAB)
  bool pull_small = false;   // hk_solve's pull matvec (S <= 8, AIY_OPT_HIST_PULL)
};

template <int SMAX, int KC, int TH>
static const void* hc_fn() {
  return reinterpret_cast<const void*>(hist_cluster_kernel<SMAX, KC, TH>);
}

static const void* hc_pick(int smax, int kc) {
  if (smax == 8) return kc == 1 ? hc_fn<8, 1, 512>() : hc_fn<8, 2, 512>();
  if (smax == 16) return hc_fn<16, 1, 512>();
  return hc_fn<32, 1, 512>();
}

static bool hc_make_plan(aiy_handle* h, int n_cal, int S, int n_a, HcPlan& p, bool krylov = false) {
  // the push forms hold up to 32 states, the pull form (BiCGSTAB, S > 8) up to 64
  if (S < 1 || n_a < 2 || S > (krylov ? 64 : 32)) return false;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus < 1) return false;
  if (krylov && S > 8) {   // pull form (hist_pull.h): vectors in HBM, every calibration at once
    p.pull = true;
    p.smax = 32;
    p.th = kHpTH;
    p.kc = 1;
    p.cap = 0;
    p.vblock = 0;
    p.fn = hist_pull_pick(S);
    if (!p.fn) return false;
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, p.fn) != hipSuccess) return false;
    int lds_dev = 0;
    if (hipDeviceGetAttribute(&lds_dev, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device) != hipSuccess)
      return false;
    const size_t lds_total = std::min<size_t>(kHcLdsTotal, (size_t)lds_dev);
    if (fa.sharedSizeBytes + 4096 >= lds_total) return false;
    const size_t budget = lds_total - fa.sharedSizeBytes - 1024;
    // the staged inverse lottery plus room for a 64-column chunk of row sums
    if (budget <= (size_t)S * 64 * sizeof(double)) return false;
    const int max_own = (int)((budget - (size_t)S * 64 * sizeof(double)) / (sizeof(int) * (size_t)S)) - 2;
    if (max_own < 1) return false;
    const int g_min = (n_a + max_own - 1) / max_own;
    if (g_min > kHcMaxG || g_min > cus) return false;
    const int g_cap = h->hist_cluster_cap > 0 ? h->hist_cluster_cap : kHcMaxG;
    int G = std::max(g_min, std::min(std::min(g_cap, kHcMaxG), cus / std::max(1, n_cal)));
    G = std::min(G, n_a);
    p.nj = (n_a + G - 1) / G;
    p.G = (n_a + p.nj - 1) / p.nj;
    p.cals_per_launch = std::max(1, cus / p.G);
    return hist_pull_plan(S, p.nj, budget, &p.cw, &p.lds);
  }
  if (S > 32) return false;   // (the push forms)
  p.smax = S <= 8 ? 8 : (S <= 16 ? 16 : 32);
  const int kc_max = p.smax == 8 ? 2 : 1;
  p.th = 512;
  const int g_min = (n_a + p.th * kc_max - 1) / (p.th * kc_max);
  if (g_min > kHcMaxG || g_min > cus) return false;
  const int g_cap = h->hist_cluster_cap > 0 ? h->hist_cluster_cap : 32;
  int G = std::max(g_min, std::min(std::min(g_cap, kHcMaxG), cus / std::max(1, n_cal)));
  G = std::min(G, n_a);
  p.nj = (n_a + G - 1) / G;
  p.G = (n_a + p.nj - 1) / p.nj;                    // every workgroup owns >= 1 column
  p.kc = p.nj <= p.th ? 1 : 2;
  if (p.kc > kc_max) return false;
  p.cals_per_launch = std::max(1, cus / p.G);
  int smax_k = p.smax;
  p.fn = krylov ? hist_bicg_pick(S, p.smax, p.kc, &smax_k, h->hist_pull != 0) : hc_pick(p.smax, p.kc);
  p.pull_small = krylov && h->hist_pull != 0 && p.smax == 8;
  if (!p.fn) return false;
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, p.fn) != hipSuccess) return false;
  const size_t stat = fa.sharedSizeBytes;
  // the LDS budget is the device's own (160 KB per CU on gfx950; an arch override with
  // less LDS makes the plan not fit instead of failing the attribute call below)
  int lds_dev = 0;
  if (hipDeviceGetAttribute(&lds_dev, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device) != hipSuccess)
    return false;
  const size_t lds_total = std::min<size_t>(kHcLdsTotal, (size_t)lds_dev);
  if (stat + 4096 >= lds_total) return false;
  p.lds = (lds_total - stat - 1024) / 256 * 256;
  // BiCGSTAB: one resident vector (v, [KC][SMAX][TH] doubles) behind the span buffer
  const size_t vbytes = krylov && smax_k <= 8 ? (size_t)p.kc * smax_k * p.th * sizeof(double) : 0;
  p.vblock = krylov && smax_k > 8 ? (size_t)p.kc * smax_k * p.th : 0;   // v in HBM, doubles per workgroup
  if (p.lds <= vbytes + 4096) return false;
  p.cap = (int)((p.lds - vbytes) / sizeof(double));
  return true;
}

static int32_t hc_scratch(aiy_handle* h, int cals, int G, int cap) {
  const size_t need = (size_t)cals * G * 2 * cap * sizeof(double) + (size_t)cals * G * 32 * 4 * sizeof(int) +
                      (size_t)cals * kHcCtrStride * sizeof(unsigned) + (size_t)cals * 2 * G * kHcRedRec * sizeof(double) +
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
  const bool krylov = h->hist_krylov != 0;
  if (!hc_make_plan(h, n_cal, S, n_a, p, krylov)) return AIY_ERR_UNSUPPORTED;
  // a launch shape the device does not admit is "unsupported" (the caller's push/mix
  // fallback runs), not a hard error
  if (hipFuncSetAttribute(p.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess) {
    (void)hipGetLastError();
    return AIY_ERR_UNSUPPORTED;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, p.fn, p.th, p.lds) != hipSuccess) {
    (void)hipGetLastError();
    return AIY_ERR_UNSUPPORTED;
  }
  if (per_cu < 1) return AIY_ERR_UNSUPPORTED;
  const int per_launch = std::min(n_cal, p.cals_per_launch);
  int32_t rc = hc_scratch(h, per_launch, p.G, p.cap);
  if (rc) return rc;
  char* base = static_cast<char*>(h->d_hc);
  HcRun r;
  r.n_cal = n_cal; r.S = S; r.n_a = n_a; r.G = p.G; r.nj = p.nj; r.cap = p.cap; r.cw = p.cw;
  r.lo = lo; r.wlo = wlo; r.P = P; r.mass = mass; r.iters_out = d_iters; r.tol = tol; r.max_iter = max_iter;
  r.tolv = krylov ? h->hist_tolv : nullptr;   // per-calibration tolerances (BiCGSTAB form)
  r.slab = reinterpret_cast<double*>(base);
  size_t off = (size_t)per_launch * p.G * 2 * p.cap * sizeof(double);
  r.span = reinterpret_cast<int*>(base + off);
  off += (size_t)per_launch * p.G * 32 * 4 * sizeof(int);
  r.ctr = reinterpret_cast<unsigned*>(base + off);
  const size_t ctr_bytes = (size_t)per_launch * kHcCtrStride * sizeof(unsigned);
  off += ctr_bytes;
  r.dist = reinterpret_cast<double*>(base + off);
  off += (size_t)per_launch * 2 * p.G * kHcRedRec * sizeof(double);
  r.accel = krylov ? 0 : h->hist_accel;
  r.dbuf = nullptr;
  r.ainv = nullptr;
  if (p.pull) {   // pull form: four [S][n_a] vectors per calibration + the inverse lottery
    const size_t vb = (size_t)n_cal * 4 * S * n_a * sizeof(double);
    const size_t db = vb + (size_t)n_cal * S * (n_a + 1) * sizeof(int);
    if (db > h->hc_dcap) {
      if (h->d_hcd) (void)hipFree(h->d_hcd);
      h->d_hcd = nullptr;
      h->hc_dcap = 0;
      AIY_HIP(h, hipMalloc(&h->d_hcd, db));
      h->hc_dcap = db;
    }
    r.dbuf = static_cast<double*>(h->d_hcd);
    r.ainv = reinterpret_cast<int*>(static_cast<char*>(h->d_hcd) + vb);
  } else if (r.accel > 0 || krylov) {   // Aitken: stored differences; BiCGSTAB: the p scratch rows
    if (r.accel > 0 && r.accel < 4) r.accel = 4;
    // p rows (+ v blocks); pull form: + the matvec input rows and the inverse lottery
    const size_t dvec = ((size_t)n_cal * S * n_a * (p.pull_small ? 2 : 1) + (size_t)per_launch * p.G * p.vblock) *
                        sizeof(double);
    const size_t db = dvec + (p.pull_small ? (size_t)n_cal * S * (n_a + 1) * sizeof(int) : 0);
    if (db > h->hc_dcap) {
      if (h->d_hcd) (void)hipFree(h->d_hcd);
      h->d_hcd = nullptr;
      h->hc_dcap = 0;
      AIY_HIP(h, hipMalloc(&h->d_hcd, db));
      h->hc_dcap = db;
    }
    r.dbuf = static_cast<double*>(h->d_hcd);
    if (p.pull_small) r.ainv = reinterpret_cast<int*>(static_cast<char*>(h->d_hcd) + dvec);
  }
  r.err = reinterpret_cast<unsigned*>(base + off);
  for (int c0 = 0; c0 < n_cal; c0 += per_launch) {
    const int nc = std::min(per_launch, n_cal - c0);
    r.cal0 = c0;
    AIY_HIP(h, hipMemsetAsync(r.ctr, 0, ctr_bytes, st));
    if (krylov)   // reduction granules: epochs count from 1 in every launch
      AIY_HIP(h, hipMemsetAsync(r.dist, 0, (size_t)per_launch * 2 * p.G * kHcRedRec * sizeof(double), st));
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
