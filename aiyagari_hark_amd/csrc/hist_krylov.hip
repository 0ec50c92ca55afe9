// Device-resident stationary distribution by BiCGSTAB (build-defined row E2, Krylov mode).
//
// The distribution iteration mass' = T mass (Young lottery push, then the income mix;
// hist_resident.hip) converges at the rate of T's second eigenvalue.  For the Table II
// cells near r = 1/beta - 1 T has a dense cluster of eigenvalues just below 1 (rho = 0,
// sigma = 0.2, CRRA = 1: 0.99916, 0.99859, 0.99801, ...), so the plain iteration needs
// ~16 000 sweeps from the uniform start and single-mode Aitken extrapolation removes only
// one of those modes.  Here each calibration's cluster solves (I - T) x = 0 by BiCGSTAB
// (van der Vorst 1992) started from the given mass: every Krylov step is one matvec T q
// with exactly the cluster machinery of the plain kernel (push into LDS spans, publish
// the foreign parts write-through, cluster barrier, gather, mix), plus cluster-wide dot
// products carried on a light barrier.  Measured on the CPU restatement (scratch study,
// DESIGN.md §4b): 1 066 matvecs instead of 15 828 plain sweeps cold, 602 instead of
// 10 199 warm.
//
//   restart:  r = T x - x;  rho = <rh, r>;  stop if max|r| < tol (mass = T x)
//             p = r
//   loop:     v = p - T p;                   alpha = rho / <rh, v>   (max|r| checked here)
//             s = r - alpha v;  t = s - T s; omega = <t, s> / <t, t>
//             x += alpha p + omega s;  r = s - omega t
//             rho' = <rh, s> - omega <rh, t>;  beta = (rho' / rho) (alpha / omega)
//             p = r + beta (p - omega v)
//   when the recursive residual is below tol (or a scalar breaks down) the true residual
//   is formed again (restart), so the returned mass is T x for an x with
//   max|T x - x| < tol: the stopping rule of oracle/stationary.py stationary_hist.
//
// Every workgroup reads the same published partial sums and adds them in the same order,
// so all workgroups of a cluster compute bit-identical scalars and take the same branches
// (the barrier counts stay in step).  T is column-stochastic, so sum(x) is preserved by
// every update (sum(r) = sum(v) = sum(p) = 0).  The shadow residual rh is a fixed hash
// of the point index (rh = r0 would need one more resident vector); rh has no mean, so
// <rh, r> does not vanish on the zero-sum residuals.  x lives in `mass` (HBM, own columns
// only, read-modify-written twice per step); r, p and the matvec result in registers, v in
// LDS behind the spans and p in an HBM scratch row across the second matvec.
#include "common.h"
#include "internal.h"
#include "hist_cluster.h"
#include "hist_bicg.h"
#include "hist_pull.h"

namespace aiy {

template <int SMAX, int KC, int TH, bool PULL>
__global__ __launch_bounds__(TH) void hist_bicg_kernel(HcRun r) {
  extern __shared__ double Tacc[];
  __shared__ int s_base[SMAX];
  __shared__ int s_pub[2 * SMAX][2];
  __shared__ int s_tot;
  __shared__ HcCand s_cand[SMAX][kHcCand];
  __shared__ int s_ncand[SMAX];
  __shared__ unsigned short s_cinfo[KC * SMAX * TH];   // hk_cinfo(cf, cn, heavy index)
  __shared__ double s_P[SMAX * SMAX];
  __shared__ double s_part[kHkRed][TH / kWave];
  __shared__ double s_res[kHkRed];
  __shared__ int s_flag, s_stop;
  __shared__ int s_ex[2 * SMAX];
  __shared__ int s_nheavy, s_heavy[kHkHeavy][4], s_rok, s_wcnt[TH / kWave];
  __shared__ double s_hval[kHkHeavy];
  HkShared<SMAX, KC, TH> L{Tacc, s_base, s_pub, &s_tot, s_cand, s_ncand, s_cinfo, s_P, s_part, s_res,
                                 &s_flag, &s_stop, s_ex, &s_nheavy, s_wcnt, s_heavy, s_hval, &s_rok};
  const int G = r.G, S = r.S, n_a = r.n_a;
  const int lc = blockIdx.x / G;
  const int w = blockIdx.x - lc * G;
  const int cal = r.cal0 + lc;
  const size_t row0 = (size_t)cal * S;
  HkArgs a;
  a.G = G; a.S = S; a.n_a = n_a; a.cap = r.cap; a.w = w;
  a.j0 = w * r.nj;
  a.j1 = min(a.j0 + r.nj, n_a);
  a.LO = to_global(r.lo + row0 * n_a);
  a.WL = to_global(r.wlo + row0 * n_a);
  a.X = to_global(r.mass + row0 * n_a);
  a.Pg = to_global(r.dbuf + row0 * n_a);
  a.Vg = to_global(SMAX <= 8 ? nullptr : r.dbuf + (size_t)r.n_cal * S * n_a + (size_t)blockIdx.x * (KC * SMAX * TH));
  a.slab_cl = to_global(r.slab + (size_t)lc * G * 2 * r.cap);
  a.span_cl = to_global(r.span + (size_t)lc * G * SMAX * 4);
  a.ctr = to_global(r.ctr + (size_t)lc * kHcCtrStride);
  a.gran = to_global(reinterpret_cast<unsigned long long*>(r.dist) + (size_t)lc * 2 * G * kHcRedRec);
  a.Pc = to_global(r.P + (size_t)cal * S * S);
  a.tol = r.tolv ? r.tolv[cal] : r.tol;
  a.max_iter = r.max_iter;
  a.err = to_global(r.err);
  a.stop_ctr = to_global((const unsigned*)nullptr);
  a.stop_at = 0u;
  // pull form: the matvec input rows and the inverse lottery behind the p rows
  a.Qg = to_global(PULL ? r.dbuf + (size_t)r.n_cal * S * n_a + row0 * n_a : (double*)nullptr);
  a.Ainv = to_global(PULL ? r.ainv + (size_t)cal * S * (n_a + 1) : (int*)nullptr);
  a.lottery_fresh = false;   // the lottery launch ran before this one
  unsigned nb = 0, ne = 0;
  const int mv = hk_solve<SMAX, KC, TH, PULL>(a, L, nb, ne);
  if (mv >= 0 && w == 0 && threadIdx.x == 0) r.iters_out[cal] = mv;
}

// The pull form for many income states (hist_pull.h): one solve per launch, vectors in HBM.
template <int SMAX, int TH>
__global__ __launch_bounds__(TH) void hist_pull_kernel(HcRun r) {
  extern __shared__ int hp_dyn[];   // staged inverse lottery
  __shared__ double s_P[SMAX * SMAX];
  __shared__ int s_ex[2 * SMAX];
  __shared__ double s_part[kHkRed][TH / kWave];
  __shared__ double s_res[kHkRed];
  __shared__ int s_flag, s_stop;
  const HpShared<SMAX, TH> L{s_P, hp_dyn, s_ex, s_part, s_res, &s_flag, &s_stop};
  const int G = r.G, S = r.S, n_a = r.n_a;
  const int lc = blockIdx.x / G;
  const int w = blockIdx.x - lc * G;
  const int cal = r.cal0 + lc;
  const size_t row0 = (size_t)cal * S;
  const size_t pts = (size_t)S * n_a;
  double* vec = r.dbuf + (size_t)cal * 4 * pts;
  HpArgs a;
  a.G = G; a.S = S; a.n_a = n_a; a.w = w;
  a.j0 = w * r.nj;
  a.j1 = min(a.j0 + r.nj, n_a);
  a.cw = r.cw;
  a.LO = to_global(r.lo + row0 * n_a);
  a.WL = to_global(r.wlo + row0 * n_a);
  a.lottery_fresh = false;   // written by the lottery launch before this one
  a.A = to_global(r.ainv + (size_t)cal * S * (n_a + 1));
  a.X = to_global(r.mass + row0 * n_a);
  a.R = to_global(vec);
  a.P = to_global(vec + pts);
  a.V = to_global(vec + 2 * pts);
  a.T = to_global(vec + 3 * pts);
  a.ctr = to_global(r.ctr + (size_t)lc * kHcCtrStride);
  a.gran = to_global(reinterpret_cast<unsigned long long*>(r.dist) + (size_t)lc * 2 * G * kHcRedRec);
  a.Pc = to_global(r.P + (size_t)cal * S * S);
  a.tol = r.tolv ? r.tolv[cal] : r.tol;
  a.max_iter = r.max_iter;
  a.err = to_global(r.err);
  a.stop_ctr = to_global((const unsigned*)nullptr);
  a.stop_at = 0u;
  unsigned nb = 0, ne = 0;
  const int mv = hp_solve<SMAX, TH>(a, L, nb, ne);
  if (mv >= 0 && w == 0 && threadIdx.x == 0) r.iters_out[cal] = mv;
}

const void* hist_pull_pick(int S) {
  // by padded state count: P and a chunk's row sums sit in LDS, the state loops are unrolled
  // to SMAX (SMAX = 16 unrolled worse and spilled when the row sums were registers)
  if (S <= 32) return reinterpret_cast<const void*>(hist_pull_kernel<32, kHpTH>);
  if (S <= 64) return reinterpret_cast<const void*>(hist_pull_kernel<64, kHpTH>);   // (up to AIY_MAX_STATES)
  return nullptr;
}
bool hist_pull_plan(int S, int n_own, size_t budget, int* cw, size_t* lds) {
  const int ng = (S + kHpGrp - 1) / kHpGrp;
  long best = -1;
  for (int nch = 1; nch <= n_own; ++nch) {
    const int c = (n_own + nch - 1) / nch;
    const size_t b = (hp_lds_bytes(S, n_own, c) + 255) / 256 * 256;
    if (b > budget) continue;
    // latency rounds per matvec: the chunks' item rounds and mix passes
    const long cost = (long)nch * (((long)ng * c + kHpTH - 1) / kHpTH + (c + kHpTH - 1) / kHpTH);
    if (best < 0 || cost < best) {
      best = cost;
      *cw = c;
      *lds = b;
    }
    if (best >= 0 && (long)(nch + 1) * 2 > best) break;   // every chunk costs >= 2 rounds
  }
  return best >= 0;
}

template <int SMAX, int KC, int TH, bool PULL = false>
static const void* hk_fn() {
  return reinterpret_cast<const void*>(hist_bicg_kernel<SMAX, KC, TH, PULL>);
}

// kernel for the plan's (S, padded S, columns per thread) and its state count SMAX
// (*smax_k); nullptr when there is no instantiation.  pull: the lottery-pull matvec (S <= 8)
const void* hist_bicg_pick(int S, int smax, int kc, int* smax_k, bool pull) {
  *smax_k = smax;
  if (pull && smax == 8) {
    if (S == 7) return *smax_k = 7, (kc == 1 ? hk_fn<7, 1, 512, true>() : hk_fn<7, 2, 512, true>());
    return kc == 1 ? hk_fn<8, 1, 512, true>() : hk_fn<8, 2, 512, true>();
  }
  if (S == 7 && kc == 2) return *smax_k = 7, hk_fn<7, 2, 512>();
  if (smax == 8) return kc == 1 ? hk_fn<8, 1, 512>() : hk_fn<8, 2, 512>();
  return nullptr;   // S > 8: the pull form (hist_pull_kernel, hc_make_plan)
}

}  // namespace aiy
