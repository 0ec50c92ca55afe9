// Pull-form BiCGSTAB distribution solve of one calibration's cluster (build-defined row E2)
// for many income states (configs[4]: 25-state Rouwenhorst at N_a = 50 000).
//
// The push form (hist_bicg.h) keeps r, p and the matvec result of every own point in
// registers (3 S doubles per column) and scatters the lottery into LDS spans with atomics.
// At S = 25 those registers do not fit (the kernel spilled ~1.1 KB per lane to scratch:
// ~300 us per matvec) and the spans would need 25 rows of LDS.  Here the Krylov vectors live
// in HBM ([S][n_a] rows per calibration, the calibration's 3 x 10 MB stay in the MALL) and a
// matvec PULLS: a monotone lottery maps the sources of destination d of row s to contiguous
// ranges, with A_s(d) = the first source j whose lottery index lo_j >= d,
//
//   T_s[d] = sum_{j in [A(d), A(d+1))} w_j q_j  +  sum_{j in [A(d-1), A(d))} (1 - w_j) q_j
//
// summed in ascending j: exactly np.add.at(T[s], lo, w q) followed by np.add.at(T[s],
// lo + 1, (1 - w) q) of oracle/stationary.py hist_step -- no atomics, so every matvec is
// deterministic run to run.  A destination with more than kHpHeavy sources (the borrowing
// constraint, the top of the grid) is summed by its whole wave: lane-strided partials and a
// fixed-order wave reduction.  Then mix: mass'[s'][d] = sum_s P[s, s'] T_s[d].
//
// Cross-workgroup data: only sources in an own column's "exported" prefix / suffix (whose
// lo or lo + 1 falls outside the own columns) are read by other workgroups; they are stored
// write-through (sc1) and drained before the cluster barrier, and foreign sources are read
// with sc1 loads (MI355X_MICROARCH.md hand-off rules); everything else is plain.  The inverse
// lottery A is built once per solve by a scatter over the own sources (sc1) and staged in LDS
// for the own destinations.
#pragma once

#include "common.h"
#include "hist_bicg.h"
#include "hist_cluster.h"

namespace aiy {

constexpr int kHpHeavy = 64;   // sources of one destination above which its wave sums them
constexpr int kHpUnroll = 4;   // wave strides of a heavy sum with their loads in flight together
constexpr int kHpRunLane = 32;   // inverse-lottery runs longer than this are stored by the whole wave
#ifdef AIY_HP_GRP
constexpr int kHpGrp = AIY_HP_GRP;   // tuning builds only
#else
constexpr int kHpGrp = 5;      // income states of one pull item
#endif

struct HpArgs {
  int G, S, n_a, w, j0, j1;
  int cw;                     // columns of one matvec chunk (the row sums of a chunk sit in LDS)
  gptr<const int> LO;         // [S][n_a] lottery index
  gptr<const double> WL;      // [S][n_a] lottery weight on lo
  bool lottery_fresh;         // LO / WL written in this launch by other workgroups (sc1 loads)
  gptr<int> A;                // [S][n_a + 1] inverse lottery (scratch)
  gptr<double> X;             // [S][n_a] in: start, out: T x (own columns)
  gptr<double> R, P, V, T;    // [S][n_a] BiCGSTAB vectors
  gptr<unsigned> ctr;         // cluster barrier counter
  gptr<unsigned long long> gran;   // [2][G][kHcRedRec] reduction granules
  gptr<const double> Pc;      // [S][S]
  double tol;
  int max_iter;
  gptr<unsigned> err;
  gptr<const unsigned> stop_ctr;   // rebalancing stop (nullptr: never), as HkArgs
  unsigned stop_at;
};

// LDS of the solve: P, the staged inverse lottery of the own destinations d in [j0 - 1, j1]
// (row stride n_own + 2) followed by a chunk's row sums ([S][cw] doubles, hp_lds_bytes), the
// exported prefix / suffix bounds, reduction partials.
template <int SMAX, int TH>
struct HpShared {
  double* s_P;                     // [SMAX][SMAX]
  int* s_A;                        // [SMAX][span]
  int* s_ex;                       // [SMAX][2]
  double (*s_part)[TH / kWave];    // [kHkRed]
  double* s_res;                   // [kHkRed]
  int* s_flag;
  int* s_stop;
};
__host__ __device__ constexpr size_t hp_lds_a_ints(int S, int n_own) {   // s_A, padded to 8 B
  return ((size_t)S * (size_t)(n_own + 2) + 1) / 2 * 2;
}
__host__ __device__ constexpr size_t hp_lds_bytes(int S, int n_own, int cw) {
  return hp_lds_a_ints(S, n_own) * sizeof(int) + (size_t)S * (size_t)cw * sizeof(double);
}

// Returns the matvecs of the solve, -1 when the cluster stops (error word: 1 timeout, 2 a
// non-monotone lottery), or -(2 + matvecs) on a rebalancing stop (X holds the iterate).
template <int SMAX, int TH>
__device__ __forceinline__ int hp_solve(const HpArgs& r, const HpShared<SMAX, TH>& L, unsigned& nb, unsigned& ne) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int G = r.G, S = r.S, n_a = r.n_a, w = r.w, j0 = r.j0, j1 = r.j1;
  const int n_own = j1 - j0, span = n_own + 2;
  const int* LO = (const int*)r.LO;
  const double* WL = (const double*)r.WL;
  int* A = (int*)r.A;
  double* X = (double*)r.X;
  double* Rv = (double*)r.R;
  double* Pv = (double*)r.P;
  double* Vv = (double*)r.V;
  double* Tv = (double*)r.T;
  unsigned* ctr = (unsigned*)r.ctr;
  unsigned long long* gran = (unsigned long long*)r.gran;
  unsigned* err = (unsigned*)r.err;
  double* s_P = L.s_P;
  int* s_A = L.s_A;
  int* s_ex = L.s_ex;
  int& s_flag = *L.s_flag;
  int& s_stop = *L.s_stop;
  const int n1 = n_a + 1;
  // a matvec runs in column chunks of cw: the chunk's pull items (a group of kHpGrp states x
  // a column) packed over all lanes, the row sums in LDS, then a column per thread mixes
  const int cw = r.cw;
  const int ng = (S + kHpGrp - 1) / kHpGrp;
  double* s_T = reinterpret_cast<double*>(s_A + hp_lds_a_ints(S, n_own));   // [S][cw]
#ifdef AIY_DIAG_PHASES
  // diagnostic build: 100 MHz ticks per phase -- 0 pull + mix + fuse, 1 matvec barrier,
  // 2 reductions, 3 elementwise updates, 4 setup
  unsigned long long hph[5] = {0, 0, 0, 0, 0}, htq = __builtin_amdgcn_s_memrealtime();
#define HP_PH(k)                                                          \
  do {                                                                    \
    if (tid == 0) {                                                       \
      const unsigned long long tn = __builtin_amdgcn_s_memrealtime();     \
      hph[(k)] += tn - htq;                                               \
      htq = tn;                                                           \
    }                                                                     \
  } while (0)
#else
#define HP_PH(k) \
  do {           \
  } while (0)
#endif

  auto barrier = [&]() -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's sc1 stores have left
    ++nb;
    return hc_barrier(err, ctr, (unsigned)G * nb, &s_flag);
  };
  auto lo_at = [&](int s, int j) -> int {
    const int* p = LO + (size_t)s * n_a + j;
    return r.lottery_fresh ? __hip_atomic_load(to_global(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
  };

  // ---- setup: P; inverse lottery scatter of the own sources; exported bounds ----
  for (int q = tid; q < SMAX * SMAX; q += TH) {
    const int s = q / SMAX, sp = q - s * SMAX;
    s_P[q] = (s < S && sp < S) ? ((const double*)r.Pc)[s * S + sp] : 0.0;
  }
  unsigned bad = 0u;
  // a lottery written in this launch (the resident GE search): every workgroup's entries are
  // in memory before the neighbour's column j0 - 1 is read
  if (r.lottery_fresh && !barrier()) return -1;
  // A(d) = j for d in (lo_{j-1}, lo_j], and n_a past lo_{n_a-1}: a run per source.  A source
  // can own a long run (the borrowing-constrained agent of a high income state saves past
  // ~30 000 of 50 000 nodes at configs[4]), which one lane stored serially in ~1.3 ms: runs
  // longer than kHpRunLane are stored by the lane's whole wave
  auto fill_run = [&](int s, int b, int e, int v) {   // A(d) = v for d in [b, e] of row s
    const bool wide = e - b >= kHpRunLane;
    if (!wide)
      for (int d = b; d <= e; ++d)
        __hip_atomic_store(to_global(&A[(size_t)s * n1 + d]), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long wm = __ballot(wide);
    while (wm) {   // wave-uniform
      const int h = __builtin_ctzll(wm);
      wm &= wm - 1ull;
      const int sh = __builtin_amdgcn_readlane(s, h), bh = __builtin_amdgcn_readlane(b, h),
                eh = __builtin_amdgcn_readlane(e, h), vh = __builtin_amdgcn_readlane(v, h);
      for (int d = bh + lane; d <= eh; d += kWave)
        __hip_atomic_store(to_global(&A[(size_t)sh * n1 + d]), vh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  for (int q0 = 0; q0 < S * n_own; q0 += TH) {   // uniform trip count (the wave fills need every lane)
    const int q = q0 + tid;
    int s = 0, rb = 0, re = -1, rv = 0, tb = 0, te = -1;   // empty runs
    if (q < S * n_own) {
      s = q / n_own;
      const int j = j0 + (q - s * n_own);
      const int l = lo_at(s, j);
      const int lp = j > 0 ? lo_at(s, j - 1) : -1;
      // only a monotone lottery inside the grid is scattered (anything else: error 2, the caller
      // falls back); the runs never leave the row
      const bool ok = l >= 0 && l <= n_a - 2 && lp >= -1 && lp <= l;
      if (!ok) {
        bad = 2u;
      } else {
        rb = lp + 1;
        re = l;
        rv = j;
        if (j == n_a - 1) {
          tb = l + 1;
          te = n_a;
        }
      }
    }
    fill_run(s, rb, re, rv);
    fill_run(s, tb, te, n_a);
  }
  if (bad) __hip_atomic_store(to_global(err), bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // exported prefix [j0, ex0) (lo < j0) and suffix [ex1, j1) (lo + 1 >= j1) of each row
  if (tid < S) {
    const int s = tid;
    int lo = j0, hi = j1;   // first own j with lo_j >= j0
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lo_at(s, mid) < j0) lo = mid + 1; else hi = mid;
    }
    s_ex[2 * s] = lo;
    int lo2 = j0, hi2 = j1;   // first own j with lo_j + 1 >= j1
    while (lo2 < hi2) {
      const int mid = (lo2 + hi2) >> 1;
      if (lo_at(s, mid) + 1 < j1) lo2 = mid + 1; else hi2 = mid;
    }
    s_ex[2 * s + 1] = lo2;
  }
  if (!barrier()) return -1;
  if (tid == 0) s_stop = __hip_atomic_load(to_global(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  __syncthreads();
  if (s_stop) return -1;
  for (int q = tid; q < S * span; q += TH) {   // A(d) for d in [j0 - 1, j1] (A(-1) = 0)
    const int s = q / span, d = j0 - 1 + (q - s * span);
    s_A[s * span + (d - j0 + 1)] =
        d < 0 ? 0 : __hip_atomic_load(to_global(&A[(size_t)s * n1 + d]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the start x may have been stored plain by its owner in this launch (the GE search's warm
  // start): its exported entries are written through before the first matvec's barrier
  for (int q = tid; q < S * n_own; q += TH) {
    const int s = q / n_own, j = j0 + (q - s * n_own);
    if (j < s_ex[2 * s] || j >= s_ex[2 * s + 1]) {
      double* p = X + (size_t)s * n_a + j;
      store_f64_agent(p, *p);
    }
  }
  __syncthreads();

  // stores of the vectors a matvec reads: write-through where another workgroup pulls them
  auto put = [&](double* V, int s, int j, double v) {
    double* p = V + (size_t)s * n_a + j;
    if (j < s_ex[2 * s] || j >= s_ex[2 * s + 1]) store_f64_agent(p, v);
    else *p = v;
  };
  // source loads: sc1 (L2-served) for every source, own or foreign -- own plain stores are in
  // the own L2, foreign ones were written through (no per-lane branch between load kinds)
  auto q_at = [&](const double* Q, int s, int j) -> double { return load_f64_agent(Q + (size_t)s * n_a + j); };
  auto w_at = [&](int s, int j) -> double {
    const double* p = WL + (size_t)s * n_a + j;
    return r.lottery_fresh ? load_f64_agent(p) : *p;
  };
  // T_s[d] for the rows s0 .. s0 + GRP of this lane's destination d, into s_T[s][c]: the
  // first two sources of each part (lo = d: w q; lo = d - 1: (1 - w) q) loaded for all rows of
  // the group at once (clamped indices, unconditional), further sources in a loop (rare), a
  // destination with more than kHpHeavy sources by its whole wave.  s0 may differ between the
  // lanes of a wave (an item round can straddle two groups); `live`: the lane holds an item.
  constexpr int GRP = kHpGrp;
  auto pull_item = [&](const double* Q, int s0, int d, int c, bool live) {
    int a0[GRP], a1[GRP], a2[GRP];
    double wv[GRP][4], qv[GRP][4];
#pragma unroll
    for (int u = 0; u < GRP; ++u) {
      const int s = s0 + u < S ? s0 + u : S - 1;
      const int* As = s_A + s * span - (j0 - 1);
      // (clamped into the row: the loops below never leave it)
      const bool valid = live && s0 + u < S;
      a0[u] = valid ? min(max(As[d - 1], 0), n_a) : 0;
      a1[u] = valid ? min(max(As[d], a0[u]), n_a) : 0;
      a2[u] = valid ? min(max(As[d + 1], a1[u]), n_a) : 0;
      const int i0 = min(a1[u], n_a - 1), i1 = min(a1[u] + 1, n_a - 1);
      const int i2 = min(a0[u], n_a - 1), i3 = min(a0[u] + 1, n_a - 1);
      wv[u][0] = w_at(s, i0); qv[u][0] = q_at(Q, s, i0);
      wv[u][1] = w_at(s, i1); qv[u][1] = q_at(Q, s, i1);
      wv[u][2] = w_at(s, i2); qv[u][2] = q_at(Q, s, i2);
      wv[u][3] = w_at(s, i3); qv[u][3] = q_at(Q, s, i3);
    }
#pragma unroll
    for (int u = 0; u < GRP; ++u) {
      const int s = s0 + u < S ? s0 + u : S - 1;
      const bool valid = live && s0 + u < S;
      const int n1c = a2[u] - a1[u], n0c = a1[u] - a0[u];
      const bool heavy = valid && (n1c + n0c) > kHpHeavy;
      double acc = 0.0;
      if (valid && !heavy) {
        if (n1c > 0) acc += wv[u][0] * qv[u][0];                     // np.add.at(T, lo, w q), ascending j
        if (n1c > 1) acc += wv[u][1] * qv[u][1];
        for (int j = a1[u] + 2; j < a2[u]; ++j) acc += w_at(s, j) * q_at(Q, s, j);
        if (n0c > 0) acc += (1.0 - wv[u][2]) * qv[u][2];             // np.add.at(T, lo + 1, (1 - w) q)
        if (n0c > 1) acc += (1.0 - wv[u][3]) * qv[u][3];
        for (int j = a0[u] + 2; j < a1[u]; ++j) acc += (1.0 - w_at(s, j)) * q_at(Q, s, j);
      }
      unsigned long long hm = __ballot(heavy);
      while (hm) {   // wave-uniform
        const int h = __builtin_ctzll(hm);
        hm &= hm - 1ull;
        const int b0 = __builtin_amdgcn_readlane(a0[u], h), b1 = __builtin_amdgcn_readlane(a1[u], h),
                  b2 = __builtin_amdgcn_readlane(a2[u], h), sh = __builtin_amdgcn_readlane(s, h);
        // lane-strided partials, kHpUnroll strides' loads in flight at once (the same order)
        double pa = 0.0, pb = 0.0;
        for (int j = b1 + lane; j < b2; j += kHpUnroll * kWave) {
          double wj[kHpUnroll], qj[kHpUnroll];
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e) {
            const int jc = min(j + e * kWave, b2 - 1);
            wj[e] = w_at(sh, jc);
            qj[e] = q_at(Q, sh, jc);
          }
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e)
            if (j + e * kWave < b2) pa += wj[e] * qj[e];
        }
        for (int j = b0 + lane; j < b1; j += kHpUnroll * kWave) {
          double wj[kHpUnroll], qj[kHpUnroll];
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e) {
            const int jc = min(j + e * kWave, b1 - 1);
            wj[e] = w_at(sh, jc);
            qj[e] = q_at(Q, sh, jc);
          }
#pragma unroll
          for (int e = 0; e < kHpUnroll; ++e)
            if (j + e * kWave < b1) pb += (1.0 - wj[e]) * qj[e];
        }
        const double ta = wave_sum_lane63(pa), tb = wave_sum_lane63(pb);
        const double tot = __shfl(ta, kWave - 1, kWave) + __shfl(tb, kWave - 1, kWave);
        if (lane == h) acc = tot;
      }
      if (valid) s_T[s * cw + c] = acc;
    }
  };
  // out = T Q on every own point, handed to fuse(s', d, out) in column order
  auto matvec = [&](const double* Q, auto&& fuse) -> bool {
    HP_PH(3);
    if (!barrier()) return false;   // every workgroup's Q is in memory
    HP_PH(1);
    for (int c0 = j0; c0 < j1; c0 += cw) {
      const int cn = min(cw, j1 - c0);
      // pull: items (state group, column) group-major (a wave's lanes: consecutive columns of
      // one group), every lane of every wave in every round (the heavy sums need the wave)
      const int items = ng * cn;
      for (int i0 = 0; i0 < items; i0 += TH) {
        const int i = i0 + tid;
        const bool live = i < items;
        const int g = live ? i / cn : 0;
        const int c = live ? i - g * cn : 0;
        pull_item(Q, g * GRP, c0 + c, c, live);
      }
      __syncthreads();
      for (int c = tid; c < cn; c += TH) {
        // P's LDS entries are loop-invariant: without this fence they were all hoisted out of
        // the chunk loop (800 values live: 1.5 KB/lane of spills)
        asm volatile("" ::: "memory");
        const int d = c0 + c;
        // the own values Q[sp][d] the fused updates need, a chunk of states at a time, loaded
        // together ahead of the chunk's stores (a load after a store to another vector is not
        // hoisted past it: one load round trip per state otherwise)
        constexpr int CH = 8;
#pragma unroll
        for (int sp0 = 0; sp0 < SMAX; sp0 += CH) {
          if (sp0 < S) {   // wave-uniform
            double qo[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) qo[u] = sp0 + u < S ? Q[(size_t)(sp0 + u) * n_a + d] : 0.0;
            // (P.T @ T)[sp, d] for the chunk's CH outputs at once, s ascending (the same sums):
            // each row sum read from LDS once per chunk, P's row segment as wide LDS reads
            double acc[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) acc[u] = 0.0;
#pragma unroll
            for (int s = 0; s < SMAX; ++s) {
              if (s < S) {   // wave-uniform
                const double t = s_T[s * cw + c];
#pragma unroll
                for (int u = 0; u < CH; ++u) acc[u] += s_P[s * SMAX + sp0 + u] * t;
              }
            }
#pragma unroll
            for (int u = 0; u < CH; ++u)
              if (sp0 + u < S) fuse(sp0 + u, d, acc[u], qo[u]);
          }
        }
      }
      __syncthreads();   // the chunk's row sums are read before the next chunk's pulls
    }
    HP_PH(0);
    return true;
  };
  // cluster-wide reduction (hist_bicg.h's protocol: tagged granules, fixed order)
  auto reduce = [&](double (&vals)[kHkRed], int nv, unsigned kmax) -> bool {
    HP_PH(3);
#pragma unroll
    for (int v = 0; v < kHkRed; ++v) {
      if (v < nv) {
        const double x = (kmax >> v) & 1u ? wave_nan_max(vals[v]) : wave_sum_lane63(vals[v]);
        if (lane == kWave - 1) L.s_part[v][wid] = x;
      }
    }
    __syncthreads();
    ++ne;
    const unsigned long long tag = (unsigned long long)ne << 32;
    unsigned long long* slot = gran + (size_t)(ne & 1) * G * (2 * kHkRed);
    if (tid < nv) {
      const int v = tid;
      double x = L.s_part[v][0];
      for (int q = 1; q < TH / kWave; ++q) x = (kmax >> v) & 1u ? nan_max(x, L.s_part[v][q]) : x + L.s_part[v][q];
      const unsigned long long b = (unsigned long long)__double_as_longlong(x);
      unsigned long long* g = slot + (size_t)w * (2 * kHkRed) + 2 * v;
      __hip_atomic_store(to_global(g), tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(to_global(g + 1), tag | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wid == 0) {
      double xa[kHkRed], xb[kHkRed];
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      bool ok;
      do {
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
      if (lane == 0) s_flag = ok ? 1 : 0;
#pragma unroll
      for (int v = 0; v < kHkRed; ++v) {
        if (v < nv) {
          const bool mx = (kmax >> v) & 1u;
          const double y = mx ? wave_nan_max(nan_max(xa[v], xb[v])) : wave_sum_lane63(xa[v] + xb[v]);
          if (lane == kWave - 1) L.s_res[v] = y;
        }
      }
    }
    __syncthreads();
    HP_PH(2);
    return s_flag != 0;
  };
  // every own point once (elementwise updates between the matvecs)
  // every own point once (elementwise updates between the matvecs), UP points per thread at a
  // time: ld(g) -> the point's inputs for all UP points first, then st(s, j, g, inputs) (the
  // next points' loads are not hoisted past this point's stores otherwise)
  auto own_points = [&](auto&& ld, auto&& st) {
#ifdef AIY_HP_UP
    constexpr int UP = AIY_HP_UP;   // tuning builds only
#else
    constexpr int UP = 8;   // (4: 13.44, 8: 13.13, 16: 13.20 ms per configs[4] solve launch)
#endif
    const int np = S * n_own;
    for (int q0 = tid; q0 < np; q0 += UP * TH) {
      decltype(ld((size_t)0)) in[UP];
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const int q = min(q0 + u * TH, np - 1);
        const int s = q / n_own, j = j0 + (q - s * n_own);
        in[u] = ld((size_t)s * n_a + j);
      }
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const int q = q0 + u * TH;
        if (q < np) {
          const int s = q / n_own, j = j0 + (q - s * n_own);
          st(s, j, (size_t)s * n_a + j, in[u]);
        }
      }
    }
  };

  // ---- BiCGSTAB on (I - T) x = 0 (hist_bicg.h, the same recurrences and stopping rule) ----
  double part[kHkRed];
  const double tol = r.tol;
  int mv = 0;
  bool restart = true, first = true;
  double rho = 0.0, total0 = 0.0;
  unsigned seed = 0;
  auto rh_at = [&](int s, int j) { return hk_rhat((unsigned)(s * n_a + j) + seed * 0x5BD1E995u); };
  double best = __builtin_inf();
  int mv_best = 0;
  double rm_cur = 0.0;   // this thread's part of max|r| of the current r (kept from where r was written)
  double alpha = 0.0;
  HP_PH(4);
  while (true) {
    if (restart) {
      // t = T x, r = t - x (p = r); the converged answer is t
      double rr = 0.0, rm = 0.0, xs = 0.0;
      if (!matvec(X, [&](int s, int j, double out, double x) {
            const size_t g = (size_t)s * n_a + j;
            const double rv = out - x;
            Tv[g] = out;
            put(Rv, s, j, rv);
            put(Pv, s, j, rv);
            rr += rh_at(s, j) * rv;
            rm = nan_max(rm, fabs(rv));
            xs += x;
          }))
        return -1;
      ++mv;
      part[0] = rr;
      part[1] = rm;
      part[2] = xs;
      if (!reduce(part, 3, 2u)) return -1;
      rho = L.s_res[0];
      rm_cur = rm;
      if (mv == 1) total0 = L.s_res[2];
      if (L.s_res[1] < tol || mv >= r.max_iter) {
        const double scale = total0 / L.s_res[2];
        const bool one = mv == 1;
        own_points([&](size_t g) { return Tv[g]; },
                   [&](int s, int j, size_t, double t) { put(X, s, j, one ? t : t * scale); });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        break;
      }
      restart = false;
      first = true;
    }
    if (r.stop_ctr != nullptr && tid == 0 && ((mv >> 1) & 7) == 0)
      s_stop = __hip_atomic_load((const unsigned*)r.stop_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= r.stop_at;
    // v = p - T p; alpha = rho / <rh, v>; max|r| rides along
    double rvv = 0.0;
    if (!matvec(Pv, [&](int s, int j, double out, double pq) {
          const size_t g = (size_t)s * n_a + j;
          const double v = pq - out;
          Vv[g] = v;
          rvv += rh_at(s, j) * v;
        }))
      return -1;
    ++mv;
    part[0] = rvv;
    part[1] = (r.stop_ctr != nullptr && tid == 0 && s_stop) ? kHkStopSentinel : rm_cur;
    if (!reduce(part, 2, 2u)) return -1;
    if (L.s_res[1] >= kHkStopSentinel) return -(2 + mv);
    if ((!first && L.s_res[1] < tol) || mv >= r.max_iter) {
      restart = true;
      continue;
    }
    if (first || L.s_res[1] < 0.9 * best) {
      best = first ? __builtin_inf() : L.s_res[1];
      mv_best = mv;
    } else if (mv - mv_best > kHkStall) {
      ++seed;
      best = __builtin_inf();
      restart = true;
      continue;
    }
    first = false;
    alpha = rho / L.s_res[0];
    if (!(fabs(alpha) < 1e300)) {
      restart = true;
      continue;
    }
    // s = r - alpha v (into R); x += alpha p waits for the omega step (one pass over x)
    own_points([&](size_t g) { return Rv[g] - alpha * Vv[g]; }, [&](int s, int j, size_t, double v) { put(Rv, s, j, v); });
    // t = s - T s; omega = <t, s> / <t, t>
    double ts = 0.0, tt = 0.0, rs = 0.0, rt = 0.0, sm = 0.0;
    if (!matvec(Rv, [&](int s, int j, double out, double sv) {
          const size_t g = (size_t)s * n_a + j;
          const double t = sv - out;
          Tv[g] = t;
          const double h = rh_at(s, j);
          ts += t * sv;
          tt += t * t;
          rs += h * sv;
          rt += h * t;
          sm = nan_max(sm, fabs(sv));
        }))
      return -1;
    ++mv;
    part[0] = ts;
    part[1] = tt;
    part[2] = rs;
    part[3] = rt;
    part[4] = sm;
    if (!reduce(part, 5, 16u)) return -1;
    double omega = (L.s_res[4] < tol) ? 0.0 : L.s_res[0] / L.s_res[1];
    if (!(fabs(omega) < 1e300)) omega = 0.0;
    if (omega == 0.0) {   // x + alpha p is the answer (or <t, t> = 0): verify
      own_points([&](size_t g) { return X[g] + alpha * Pv[g]; }, [&](int s, int j, size_t, double v) { put(X, s, j, v); });
      restart = true;
      continue;
    }
    const double rho2 = L.s_res[2] - omega * L.s_res[3];
    const double beta = (rho2 / rho) * (alpha / omega);
    rho = rho2;
    // x += alpha p + omega s (the p of this step, before its update); r = s - omega t;
    // p = r + beta (p - omega v); max|r| for the next step's check
    double rmn = 0.0;
    struct Up2 {
      double sv, t, pold, x, v;
    };
    own_points([&](size_t g) { return Up2{Rv[g], Tv[g], Pv[g], X[g], Vv[g]}; },
               [&](int s, int j, size_t, const Up2& u) {
                 put(X, s, j, (u.x + alpha * u.pold) + omega * u.sv);
                 const double rn = u.sv - omega * u.t;
                 put(Rv, s, j, rn);
                 put(Pv, s, j, rn + beta * (u.pold - omega * u.v));
                 rmn = nan_max(rmn, fabs(rn));
               });
    rm_cur = rmn;
    if (!(fabs(beta) < 1e300) || rho == 0.0) restart = true;
  }
#ifdef AIY_DIAG_PHASES
  if (tid == 0 && (w == 0 || w == G / 2 || w == G - 1) && mv > 0)
    printf("[pull phases] wg %d/%d cols %d chunk %d matvecs %d us/matvec: pull+mix %.2f barrier %.2f reduce %.2f "
           "updates %.2f (setup %.1f us)\n", w, G, n_own, cw, mv, hph[0] * 0.01 / mv, hph[1] * 0.01 / mv,
           hph[2] * 0.01 / mv, hph[3] * 0.01 / mv, hph[4] * 0.01);
#endif
#undef HP_PH
  return mv;
}

}  // namespace aiy
