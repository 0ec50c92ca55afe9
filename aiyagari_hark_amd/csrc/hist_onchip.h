// Pull-form BiCGSTAB distribution solve with the Krylov vectors ON CHIP (build-defined row
// E2, configs[4]: 25-state Rouwenhorst at N_a = 50 000), one calibration per launch on every
// CU of the device.
//
// hist_pull.h keeps r, p, v, t and x in HBM because three calibrations share the device
// (85 workgroups and 589 columns x 25 states each); every matvec and every elementwise
// update then streams those vectors, ~170 us per matvec of the three (phase build:
// pull + mix ~100, updates ~27, barrier ~8, reductions).  With ONE calibration on 256
// workgroups a workgroup owns <= 196 columns x 25 states = 4 900 points, and a thread's
// <= PPT points of each vector fit in registers.  A matvec then moves only what crosses a
// workgroup boundary:
//   1. the input vector's own points go to LDS (point q of the workgroup at LDS index q), its
//      exported entries (sources another workgroup pulls, hist_pull.h) to HBM write-through;
//   2. cluster barrier;
//   3. pull: T_s[d] for (own destination d, half of the states) -- sources from LDS when own,
//      from HBM (sc1) when foreign -- into LDS (the same sums in the same order as hist_pull.h);
//   4. mix: out[s'][d] = sum_s P[s, s'] T_s[d] for (d, half of s') back into the input's LDS;
//   5. every thread reads its own points' outputs; the BiCGSTAB updates stay in registers.
// The recurrences, stopping rule and restarts are hp_solve's; only the partial dot products
// are summed in a different (fixed) order.
#pragma once

#include "common.h"
#include "hist_bicg.h"
#include "hist_cluster.h"
#include "hist_pull.h"

namespace aiy {

constexpr int kHoMaxG = 256;   // workgroups of the cluster (reductions read up to 4 granules per lane)
constexpr int kHoPPT = 10;     // own points per thread (S x columns <= kHoPPT x threads)

// Dynamic LDS of the on-chip solve for n_own columns and S states: staged inverse lottery
// [S][n_own + 2] ints, then three [S][n_own] double planes (the own lottery weights; the
// matvec input / output; the pull sums).
__host__ __device__ inline size_t ho_lds_bytes(int S, int n_own) {
  const size_t a = ((size_t)S * (n_own + 2) * sizeof(int) + 15) / 16 * 16;
  return a + 3 * (size_t)S * n_own * sizeof(double);
}

template <int SMAX, int TH>
__device__ __forceinline__ int ho_solve(const HpArgs& r, char* dyn, unsigned& nb, unsigned& ne) {
  constexpr int PPT = kHoPPT;
  __shared__ double s_P[SMAX * SMAX];
  __shared__ int s_ex[2 * SMAX];
  __shared__ double s_part[kHkRed][TH / kWave];
  __shared__ double s_res[kHkRed];
  __shared__ int s_flag, s_stop;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int G = r.G, S = r.S, n_a = r.n_a, w = r.w, j0 = r.j0, j1 = r.j1;
  const int n_own = j1 - j0, span = n_own + 2, np = S * n_own;
  const int* LO = (const int*)r.LO;
  const double* WL = (const double*)r.WL;
  int* A = (int*)r.A;
  double* Xg = (double*)r.X;   // in: start, out: the solution; exported x of restarts
  double* Rg = (double*)r.R;   // exported entries of s (the second matvec's input)
  double* Pg = (double*)r.P;   // exported entries of p
  unsigned* ctr = (unsigned*)r.ctr;
  unsigned long long* gran = (unsigned long long*)r.gran;
  unsigned* err = (unsigned*)r.err;
  const int n1 = n_a + 1;
  int* s_A = reinterpret_cast<int*>(dyn);
  double* s_Q = reinterpret_cast<double*>(dyn + ((size_t)S * span * sizeof(int) + 15) / 16 * 16);
  double* s_T = s_Q + np;
  double* s_W = s_T + np;

#ifdef AIY_DIAG_PHASES
  // diagnostic build: 100 MHz ticks -- 0 stage + barrier, 1 pull, 2 mix, 3 reductions, 4 updates
  unsigned long long oph[5] = {0, 0, 0, 0, 0}, otq = __builtin_amdgcn_s_memrealtime();
#define HO_PH(k)                                                        \
  do {                                                                  \
    if (tid == 0) {                                                     \
      const unsigned long long tn = __builtin_amdgcn_s_memrealtime();   \
      oph[(k)] += tn - otq;                                             \
      otq = tn;                                                         \
    }                                                                   \
  } while (0)
#else
#define HO_PH(k) \
  do {           \
  } while (0)
#endif
  auto barrier = [&]() -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's sc1 stores have left
    ++nb;
    return hc_barrier(err, ctr, (unsigned)G * nb, &s_flag);
  };

  // ---- setup (hist_pull.h): P; inverse lottery scatter of the own sources; exported bounds ----
  for (int q = tid; q < SMAX * SMAX; q += TH) {
    const int s = q / SMAX, sp = q - s * SMAX;
    s_P[q] = (s < S && sp < S) ? ((const double*)r.Pc)[s * S + sp] : 0.0;
  }
  unsigned bad = 0u;
  for (int q = tid; q < np; q += TH) {
    const int s = q / n_own, j = j0 + (q - s * n_own);
    const int l = LO[(size_t)s * n_a + j];
    const int lp = j > 0 ? LO[(size_t)s * n_a + j - 1] : -1;
    const bool ok = l >= 0 && l <= n_a - 2 && lp >= -1 && lp <= l;
    if (!ok) {
      bad = 2u;
      continue;
    }
    for (int d = lp + 1; d <= l; ++d)
      __hip_atomic_store(to_global(&A[(size_t)s * n1 + d]), j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (j == n_a - 1)
      for (int d = l + 1; d <= n_a; ++d)
        __hip_atomic_store(to_global(&A[(size_t)s * n1 + d]), n_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (bad) __hip_atomic_store(to_global(err), bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < S) {   // exported prefix [j0, ex0) (lo < j0) and suffix [ex1, j1) (lo + 1 >= j1)
    const int s = tid;
    const int* Ls = LO + (size_t)s * n_a;
    int lo = j0, hi = j1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (Ls[mid] < j0) lo = mid + 1; else hi = mid;
    }
    s_ex[2 * s] = lo;
    int lo2 = j0, hi2 = j1;
    while (lo2 < hi2) {
      const int mid = (lo2 + hi2) >> 1;
      if (Ls[mid] + 1 < j1) lo2 = mid + 1; else hi2 = mid;
    }
    s_ex[2 * s + 1] = lo2;
  }
  if (!barrier()) return -1;
  if (tid == 0) s_stop = __hip_atomic_load(to_global(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return -1;
  for (int q = tid; q < S * span; q += TH) {   // A(d) for d in [j0 - 1, j1] (A(-1) = 0)
    const int s = q / span, d = j0 - 1 + (q - s * span);
    s_A[q] = d < 0 ? 0 : __hip_atomic_load(to_global(&A[(size_t)s * n1 + d]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int q = tid; q < np; q += TH) {   // the own sources' lottery weights
    const int s = q / n_own, j = j0 + (q - s * n_own);
    s_W[q] = WL[(size_t)s * n_a + j];
  }

  // own points of this thread: q = tid + k TH (the LDS plane index), k < PPT
  auto pt_s = [&](int k) { return (tid + k * TH) / n_own; };
  auto pt_j = [&](int k) { const int q = tid + k * TH; return j0 + (q - (q / n_own) * n_own); };
  auto pt_ok = [&](int k) { return tid + k * TH < np; };
  auto exported = [&](int s, int j) { return j < s_ex[2 * s] || j >= s_ex[2 * s + 1]; };

  double xv[PPT], rv[PPT], pv[PPT], vv[PPT], tv[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    xv[k] = pt_ok(k) ? Xg[(size_t)pt_s(k) * n_a + pt_j(k)] : 0.0;
    rv[k] = pv[k] = vv[k] = tv[k] = 0.0;
  }
  __syncthreads();

  // pull sums of destination d for states [sa, sb): sources from the staged plane when own,
  // from Qg (sc1) when foreign; ascending j as np.add.at (hist_pull.h pull_group)
  // a source's weight w and value q: the staged planes when own, global memory when foreign
  auto src = [&](const double* Qg, int s, int j, double& wj) -> double {
    if (j >= j0 && j < j1) {
      wj = s_W[s * n_own + (j - j0)];
      return s_Q[s * n_own + (j - j0)];
    }
    wj = WL[(size_t)s * n_a + j];
    return load_f64_agent(Qg + (size_t)s * n_a + j);
  };
  auto pull_states = [&](const double* Qg, int d, bool valid, int sa, int sb) {
    for (int s = sa; s < sb; ++s) {
      const int* As = s_A + s * span - (j0 - 1);
      const int a0 = valid ? min(max(As[d - 1], 0), n_a) : 0;
      const int a1 = valid ? min(max(As[d], a0), n_a) : 0;
      const int a2 = valid ? min(max(As[d + 1], a1), n_a) : 0;
      const int n1c = a2 - a1, n0c = a1 - a0;
      const bool heavy = valid && (n1c + n0c) > kHpHeavy;
      double acc = 0.0;
      if (valid && !heavy) {
        double wj;
        for (int j = a1; j < a2; ++j) {   // np.add.at(T, lo, w q)
          const double qj = src(Qg, s, j, wj);
          acc += wj * qj;
        }
        for (int j = a0; j < a1; ++j) {   // np.add.at(T, lo + 1, (1 - w) q)
          const double qj = src(Qg, s, j, wj);
          acc += (1.0 - wj) * qj;
        }
      }
      unsigned long long hm = __ballot(heavy);
      while (hm) {   // wave-uniform: a destination with many sources, summed by the whole wave
        const int h = __builtin_ctzll(hm);
        hm &= hm - 1ull;
        const int b0 = __builtin_amdgcn_readlane(a0, h), b1 = __builtin_amdgcn_readlane(a1, h),
                  b2 = __builtin_amdgcn_readlane(a2, h);
        double pa = 0.0, pb = 0.0;
        for (int j = b1 + lane; j < b2; j += kHpUnroll * kWave) {
          double wj[kHpUnroll], qj[kHpUnroll];
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e) qj[e] = src(Qg, s, min(j + e * kWave, b2 - 1), wj[e]);
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e)
            if (j + e * kWave < b2) pa += wj[e] * qj[e];
        }
        for (int j = b0 + lane; j < b1; j += kHpUnroll * kWave) {
          double wj[kHpUnroll], qj[kHpUnroll];
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e) qj[e] = src(Qg, s, min(j + e * kWave, b1 - 1), wj[e]);
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e)
            if (j + e * kWave < b1) pb += (1.0 - wj[e]) * qj[e];
        }
        const double ta = wave_sum_lane63(pa), tb = wave_sum_lane63(pb);
        const double tot = __shfl(ta, kWave - 1, kWave) + __shfl(tb, kWave - 1, kWave);
        if (lane == h) acc = tot;
      }
      if (valid) s_T[s * n_own + (d - j0)] = acc;
    }
  };
  const int Sh = (S + 1) / 2;   // the two halves of the states
  // out = T q: stage q (registers -> LDS plane; exported entries -> Qg), barrier, pull, mix;
  // afterwards out[k] of every own point
  auto matvec = [&](const double (&qv)[PPT], double* Qg, double (&out)[PPT]) -> bool {
    HO_PH(4);
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      if (pt_ok(k)) {
        const int q = tid + k * TH, s = pt_s(k), j = pt_j(k);
        s_Q[q] = qv[k];
        if (exported(s, j)) store_f64_agent(Qg + (size_t)s * n_a + j, qv[k]);
      }
    }
    if (!barrier()) return false;   // every workgroup's exported q is in memory (and s_Q is complete)
    HO_PH(0);
    // pull: the first half of the waves takes states [0, Sh), the second [Sh, S), each lane a
    // destination; the half is wave-uniform and every lane of a wave runs every state (the
    // heavy sums need the whole wave on one state)
    {
      constexpr int HL = TH / 2;
      const int half = tid / HL;   // wave-uniform (HL a multiple of the wave)
      for (int b = 0; b < n_own; b += HL) {
        const int dl = b + (tid - half * HL);
        const bool valid = dl < n_own;
        pull_states(Qg, valid ? j0 + dl : j0, valid, half == 0 ? 0 : Sh, half == 0 ? Sh : S);
      }
    }
    __syncthreads();
    HO_PH(1);
    // mix into the input plane (free now): out[s'][d] = sum_s P[s, s'] T_s[d]
    for (int t = tid; t < 2 * n_own; t += TH) {
      const int half = t / n_own, dl = t - half * n_own;
      double Tq[SMAX];
#pragma unroll
      for (int s = 0; s < SMAX; ++s) Tq[s] = s < S ? s_T[s * n_own + dl] : 0.0;
      const int sa = half == 0 ? 0 : Sh, sb = half == 0 ? Sh : S;
      for (int sp = sa; sp < sb; ++sp) {
        double acc = 0.0;
#pragma unroll
        for (int s = 0; s < SMAX; ++s) acc += s_P[s * SMAX + sp] * Tq[s];   // (P.T @ T)[sp, d]
        s_Q[sp * n_own + dl] = acc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PPT; ++k) out[k] = pt_ok(k) ? s_Q[tid + k * TH] : 0.0;
    __syncthreads();   // the plane is restaged by the next matvec
    HO_PH(2);
    return true;
  };
  // cluster-wide reduction (hist_bicg.h's protocol) over up to kHoMaxG workgroups
  auto reduce = [&](double (&vals)[kHkRed], int nv, unsigned kmax) -> bool {
    HO_PH(4);
#pragma unroll
    for (int v = 0; v < kHkRed; ++v) {
      if (v < nv) {
        const double x = (kmax >> v) & 1u ? wave_nan_max(vals[v]) : wave_sum_lane63(vals[v]);
        if (lane == kWave - 1) s_part[v][wid] = x;
      }
    }
    __syncthreads();
    ++ne;
    const unsigned long long tag = (unsigned long long)ne << 32;
    unsigned long long* slot = gran + (size_t)(ne & 1) * G * (2 * kHkRed);
    if (tid < nv) {
      const int v = tid;
      double x = s_part[v][0];
      for (int q = 1; q < TH / kWave; ++q) x = (kmax >> v) & 1u ? nan_max(x, s_part[v][q]) : x + s_part[v][q];
      const unsigned long long b = (unsigned long long)__double_as_longlong(x);
      unsigned long long* g = slot + (size_t)w * (2 * kHkRed) + 2 * v;
      __hip_atomic_store(to_global(g), tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(to_global(g + 1), tag | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wid == 0) {
      constexpr int U = kHoMaxG / kWave;
      // the lane's granules of every pass folded at once (fixed order u = 0 .. U - 1); the pass
      // whose tags all match is the one kept
      double xs[kHkRed];
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      bool ok;
      do {
        ok = true;
#pragma unroll
        for (int v = 0; v < kHkRed; ++v) {
          double a = 0.0;
          if (v < nv) {
            const bool mx = (kmax >> v) & 1u;
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int w2 = lane + u * kWave;
              double x = 0.0;
              if (w2 < G) {
                const unsigned long long* g = slot + (size_t)w2 * (2 * kHkRed) + 2 * v;
                const unsigned long long hi = __hip_atomic_load(to_global(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long lo = __hip_atomic_load(to_global(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = ok && (hi & 0xffffffff00000000ull) == tag && (lo & 0xffffffff00000000ull) == tag;
                x = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
              }
              a = u == 0 ? x : (mx ? nan_max(a, x) : a + x);
            }
          }
          xs[v] = a;
        }
        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kHcTimeoutTicks) {
          if (lane == 0) __hip_atomic_store(to_global(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      } while (true);
      if (lane == 0) s_flag = ok ? 1 : 0;
#pragma unroll
      for (int v = 0; v < kHkRed; ++v) {
        if (v < nv) {
          const bool mx = (kmax >> v) & 1u;
          const double y = mx ? wave_nan_max(xs[v]) : wave_sum_lane63(xs[v]);
          if (lane == kWave - 1) s_res[v] = y;
        }
      }
    }
    __syncthreads();
    HO_PH(3);
    return s_flag != 0;
  };

  // ---- BiCGSTAB on (I - T) x = 0 (hp_solve's recurrences and stopping rule) ----
  double part[kHkRed];
  const double tol = r.tol;
  int mv = 0;
  bool restart = true, first = true;
  double rho = 0.0, total0 = 0.0;
  unsigned seed = 0;
  auto rh_at = [&](int k) { return hk_rhat((unsigned)(pt_s(k) * n_a + pt_j(k)) + seed * 0x5BD1E995u); };
  double best = __builtin_inf();
  int mv_best = 0;
  double rm_cur = 0.0;
  double alpha = 0.0;
  double out[PPT];
  while (true) {
    if (restart) {
      // t = T x, r = t - x (p = r); the converged answer is t
      if (!matvec(xv, Xg, out)) return -1;
      ++mv;
      double rr = 0.0, rm = 0.0, xs = 0.0;
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        if (pt_ok(k)) {
          tv[k] = out[k];
          rv[k] = out[k] - xv[k];
          pv[k] = rv[k];
          rr += rh_at(k) * rv[k];
          rm = nan_max(rm, fabs(rv[k]));
          xs += xv[k];
        }
      }
      part[0] = rr;
      part[1] = rm;
      part[2] = xs;
      if (!reduce(part, 3, 2u)) return -1;
      rho = s_res[0];
      rm_cur = rm;
      if (mv == 1) total0 = s_res[2];
      if (s_res[1] < tol || mv >= r.max_iter) {
        const double scale = total0 / s_res[2];
        const bool one = mv == 1;
#pragma unroll
        for (int k = 0; k < PPT; ++k)
          if (pt_ok(k)) Xg[(size_t)pt_s(k) * n_a + pt_j(k)] = one ? tv[k] : tv[k] * scale;
        break;
      }
      restart = false;
      first = true;
    }
    // v = p - T p; alpha = rho / <rh, v>; max|r| rides along
    if (!matvec(pv, Pg, out)) return -1;
    ++mv;
    double rvv = 0.0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      vv[k] = pv[k] - out[k];
      if (pt_ok(k)) rvv += rh_at(k) * vv[k];
    }
    part[0] = rvv;
    part[1] = rm_cur;
    if (!reduce(part, 2, 2u)) return -1;
    if ((!first && s_res[1] < tol) || mv >= r.max_iter) {
      restart = true;
      continue;
    }
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
    alpha = rho / s_res[0];
    if (!(fabs(alpha) < 1e300)) {
      restart = true;
      continue;
    }
    // s = r - alpha v (in rv); t = s - T s; omega = <t, s> / <t, t>
#pragma unroll
    for (int k = 0; k < PPT; ++k) rv[k] -= alpha * vv[k];
    if (!matvec(rv, Rg, out)) return -1;
    ++mv;
    double ts = 0.0, tt = 0.0, rs = 0.0, rt = 0.0, sm = 0.0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      tv[k] = rv[k] - out[k];
      if (pt_ok(k)) {
        const double h = rh_at(k);
        ts += tv[k] * rv[k];
        tt += tv[k] * tv[k];
        rs += h * rv[k];
        rt += h * tv[k];
        sm = nan_max(sm, fabs(rv[k]));
      }
    }
    part[0] = ts;
    part[1] = tt;
    part[2] = rs;
    part[3] = rt;
    part[4] = sm;
    if (!reduce(part, 5, 16u)) return -1;
    double omega = (s_res[4] < tol) ? 0.0 : s_res[0] / s_res[1];
    if (!(fabs(omega) < 1e300)) omega = 0.0;
    if (omega == 0.0) {   // x + alpha p is the answer (or <t, t> = 0): verify
#pragma unroll
      for (int k = 0; k < PPT; ++k) xv[k] += alpha * pv[k];
      restart = true;
      continue;
    }
    const double rho2 = s_res[2] - omega * s_res[3];
    const double beta = (rho2 / rho) * (alpha / omega);
    rho = rho2;
    // x += alpha p + omega s; r = s - omega t; p = r + beta (p - omega v)
    double rmn = 0.0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      xv[k] = (xv[k] + alpha * pv[k]) + omega * rv[k];
      const double rn = rv[k] - omega * tv[k];
      pv[k] = rn + beta * (pv[k] - omega * vv[k]);
      rv[k] = rn;
      if (pt_ok(k)) rmn = nan_max(rmn, fabs(rn));
    }
    rm_cur = rmn;
    if (!(fabs(beta) < 1e300) || rho == 0.0) restart = true;
  }
#ifdef AIY_DIAG_PHASES
  if (tid == 0 && (w == 0 || w == G / 2 || w == G - 1) && mv > 0)
    printf("[onchip phases] wg %d/%d cols %d matvecs %d us/matvec: stage+barrier %.2f pull %.2f mix %.2f reduce %.2f "
           "updates %.2f\n", w, G, n_own, mv, oph[0] * 0.01 / mv, oph[1] * 0.01 / mv, oph[2] * 0.01 / mv,
           oph[3] * 0.01 / mv, oph[4] * 0.01 / mv);
#endif
#undef HO_PH
  return mv;
}

}  // namespace aiy
