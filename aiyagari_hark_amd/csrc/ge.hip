// General equilibrium of the stationary Aiyagari household (build-defined row E1) as ONE
// library call: the root search on r of K_s(r) = K_d(r) for every calibration of a batch,
// each K_s(r) evaluated on device (stationary EGM -> Young lottery -> device-resident
// distribution iteration -> K reduction), the brackets moved on the host between the
// evaluations (a handful of doubles per calibration and step).
//
//   w(r) = (1 - alpha) (alpha / (r + delta))^(alpha / (1 - alpha)),  R = 1 + r
//   K_d(r) = (alpha / (r + delta))^(1 / (1 - alpha))           (calc_R_and_W's firm, L = 1)
//
// Methods: 0 = bisection (oracle/stationary.py ge_bisect, step for step); 1 = bisection
// until both signs of K_s - K_d are evaluated, then Brent's method per calibration (the
// scipy.optimize.brentq algorithm; aiyagari_hark_amd/stationary.py _Brent is the same
// coroutine in Python).
#include "common.h"
#include "ge_search.h"
#include "internal.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

namespace aiy {

// EGM cycles launched between two host checks of the household solves (convergence,
// extrapolation); tuning builds override it
#ifndef AIY_GE_EGM_CHUNK
#define AIY_GE_EGM_CHUNK 32
#endif
constexpr int kGeEgmChunk = AIY_GE_EGM_CHUNK;
__global__ void fill_prices_kernel(int n_cal, int S, const double* __restrict__ R, const double* __restrict__ w,
                                   double* __restrict__ Rn, double* __restrict__ Wn, double* __restrict__ Mn) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_cal * S) return;
  const int c = q / S;
  Rn[q] = R[c];
  Wn[q] = w[c];
  Mn[q] = 0.0;
}

__global__ void fill_value_kernel(double* x, long long n, double v) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) x[q] = v;
}

// Secant start of the next K_s(r) evaluation from the last two (per calibration):
// x0 = cur + theta_c (cur - prev), theta_c = (r_next - r_cur) / (r_cur - r_prev) (clamped
// to [-1, 1]; 0 without a history), over `per` values per calibration.  The household
// solve and the distribution solve then start O(dr^2) from their fixed points instead of
// O(dr); the fixed points, and the stopping rules that certify them, are unchanged.
__global__ void secant_start_kernel(long long per, int n_cal, const double* __restrict__ theta,
                                    const double* __restrict__ cur, const double* __restrict__ prev,
                                    double* __restrict__ out) {
  const long long n = per * n_cal;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const double th = theta[q / per];
    const double c = cur[q];
    out[q] = th == 0.0 ? c : c + th * (c - prev[q]);
  }
}

struct GeLayout {
  size_t Rn, Wn, Mn, Mg, Rc, wc, tm, tc, wm, wc2, lo, wlo, mass, hw, pm, pc, im, ic, pmass, th, etol, htol, bytes;
};
static GeLayout ge_layout(int n_cal, int S, int n_a) {
  GeLayout L;
  const size_t ns = (size_t)n_cal * S, tab = ns * (n_a + 1), pts = ns * n_a;
  size_t o = 0;
  auto take = [&](size_t bytes) { const size_t at = o; o += (bytes + 255) / 256 * 256; return at; };
  L.Rn = take(ns * 8); L.Wn = take(ns * 8); L.Mn = take(ns * 8); L.Mg = take((size_t)n_cal * 8);
  L.Rc = take((size_t)n_cal * 8); L.wc = take((size_t)n_cal * 8);
  L.tm = take(tab * 8); L.tc = take(tab * 8); L.wm = take(2 * tab * 8); L.wc2 = take(2 * tab * 8);
  L.lo = take(pts * 4); L.wlo = take(pts * 8); L.mass = take(pts * 8); L.hw = take(2 * pts * 8);
  L.pm = take(tab * 8); L.pc = take(tab * 8); L.im = take(tab * 8); L.ic = take(tab * 8);
  L.pmass = take(pts * 8); L.th = take((size_t)n_cal * 8);
  L.etol = take((size_t)n_cal * 8); L.htol = take((size_t)n_cal * 8);
  L.bytes = o;
  return L;
}

}  // namespace aiy

using namespace aiy;

extern "C" int64_t aiy_ge_stationary_work_bytes(int32_t n_cal, int32_t S, int32_t n_a) {
  if (n_cal < 1 || S < 1 || n_a < 2) return -1;
  return (int64_t)ge_layout(n_cal, S, n_a).bytes;
}

extern "C" int32_t aiy_ge_stationary(aiy_handle* h, const aiy_stationary_model* M, const aiy_ge_options* o,
                                     void* work, double* r_out, double* K_out, double* Ks_out, int32_t* steps_out,
                                     int32_t* egm_cycles_out, int32_t* hist_iters_out, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!M || !o || !work || !r_out || !K_out) return fail(h, AIY_ERR_ARG, "null argument");
  const int n_cal = M->n_cal, S = M->S, n_a = M->n_a;
  if (n_cal < 1 || S < 1 || S > AIY_MAX_STATES || n_a < 2) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (!M->a_grid || !M->P || !M->lab || !M->beta || !M->crra || !M->alpha || !M->delta || !M->disc)
    return fail(h, AIY_ERR_ARG, "null model array");
  if (o->method != 0 && o->method != 1) return fail(h, AIY_ERR_ARG, "method must be 0 (bisect) or 1 (brent)");
  if (!(o->r_tol > 0) || o->max_steps < 1) return fail(h, AIY_ERR_ARG, "bad r_tol / max_steps");
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  {   // the whole search in one device-resident launch where the shape allows (ge_resident.hip)
    const int32_t rr = ge_stationary_resident(h, M, o, r_out, K_out, Ks_out, steps_out, egm_cycles_out,
                                              hist_iters_out, o->status_out, st);
    if (rr < 0) return rr;
    if (rr == 1) return AIY_OK;
  }
  const GeLayout L = ge_layout(n_cal, S, n_a);
  char* base = static_cast<char*>(work);
  double* Rn = reinterpret_cast<double*>(base + L.Rn);
  double* Wn = reinterpret_cast<double*>(base + L.Wn);
  double* Mn = reinterpret_cast<double*>(base + L.Mn);
  double* Mg = reinterpret_cast<double*>(base + L.Mg);
  double* Rc = reinterpret_cast<double*>(base + L.Rc);
  double* wc = reinterpret_cast<double*>(base + L.wc);
  double* tm = reinterpret_cast<double*>(base + L.tm);
  double* tc = reinterpret_cast<double*>(base + L.tc);
  double* wm = reinterpret_cast<double*>(base + L.wm);
  double* wc2 = reinterpret_cast<double*>(base + L.wc2);
  int32_t* lo = reinterpret_cast<int32_t*>(base + L.lo);
  double* wlo = reinterpret_cast<double*>(base + L.wlo);
  double* mass = reinterpret_cast<double*>(base + L.mass);
  double* hw = reinterpret_cast<double*>(base + L.hw);
  double* pm = reinterpret_cast<double*>(base + L.pm);      // previous evaluation's tables
  double* pc = reinterpret_cast<double*>(base + L.pc);
  double* im = reinterpret_cast<double*>(base + L.im);      // secant starts
  double* ic = reinterpret_cast<double*>(base + L.ic);
  double* pmass = reinterpret_cast<double*>(base + L.pmass);
  double* d_th = reinterpret_cast<double*>(base + L.th);
  const long long tab_per = (long long)S * (n_a + 1), pts_per = (long long)S * n_a;
  std::vector<double> r_cur(n_cal, 0.0), r_prev(n_cal, 0.0), theta(n_cal, 0.0);
  // loose bracketing: per-calibration tolerances of this step, and the calibrations whose
  // last (loose) evaluation was too close to the root to trust its sign
  double* d_etol = reinterpret_cast<double*>(base + L.etol);
  double* d_htol = reinterpret_cast<double*>(base + L.htol);
  std::vector<double> etol(n_cal, o->egm_tol), htol(n_cal, o->hist_tol);
  std::vector<char> loose(n_cal, 0), refine(n_cal, 0), adapt(n_cal, 0);
  std::vector<double> fmin_rel(n_cal, HUGE_VAL);   // smallest accepted |K_s - K_d| / K_d (ge_search.h)
  const bool loose_on = o->loose_bracket && o->method == 1;
  const double kLooseEgm = std::max(o->egm_tol, AIY_GE_LOOSE_EGM), kLooseHist = std::max(o->hist_tol, std::pow(10.0, -(double)h->ge_loose_hist));
  const unsigned sec_blocks = 1024;
  AIY_HIP(h, hipMemsetAsync(Mg, 0, sizeof(double) * n_cal, st));

  std::vector<int32_t> status(n_cal, 0);   // aiy_ge_options.status_out bits
  const int max_cyc = o->max_egm_cycles > 0 ? o->max_egm_cycles : 5000;
  const int max_hist = o->max_hist_iter > 0 ? o->max_hist_iter : 200000;
  std::vector<RootSearch> rs(n_cal);
  for (int c = 0; c < n_cal; ++c) {
    const double lo0 = o->r_lo ? o->r_lo[c] : -0.5 * M->delta[c];
    const double hi0 = o->r_hi ? o->r_hi[c] : 1.0 / M->disc[c] - 1.0 - 1e-9;
    rs[c].init(lo0, hi0, o->r_tol, o->method, o->loose_bracket != 0 ? h->ge_logsec : 0);
  }
  std::vector<double> R(n_cal), w(n_cal), Kd(n_cal), Ks(n_cal, 0.0), Ks_fin(n_cal, 0.0);
  std::vector<int32_t> cyc(n_cal), its(n_cal);
  std::vector<double> dist(n_cal);
  aiy_egm_dims dims{n_cal, S, 1, n_a};
  aiy_egm_inputs in{M->a_grid, Mg, M->P, Rn, Wn, Mn, M->lab, M->beta, M->crra};
  const int saved_accel = h->hist_accel, saved_krylov = h->hist_krylov;
  int steps = 0;
  int32_t rc = AIY_OK;
  long long cyc_sum = 0, it_sum = 0;
  // a calibration whose search ends on an evaluation at looser tolerances (loose
  // bracketing, or Brent's adaptive distribution tolerance) has that r evaluated once more at
  // egm_tol / hist_tol (warm: a few cycles and matvecs) before its K_s is reported; fin[c] marks
  // it for that final pass, which evaluates r_cur[c] (the others re-evaluate their rs.x as every
  // step does for finished calibrations)
  std::vector<char> fin(n_cal, 0);
  bool final_pass = false;
  while (steps < o->max_steps || final_pass) {
    bool all_done = true;
    for (int c = 0; c < n_cal; ++c) all_done = all_done && rs[c].done;
    if (all_done && !final_pass) {
      for (int c = 0; c < n_cal; ++c) final_pass = final_pass || fin[c];
      if (!final_pass) break;
    }
    for (int c = 0; c < n_cal; ++c) {
      const double r = fin[c] ? r_cur[c] : rs[c].x, a = M->alpha[c], d = M->delta[c];
      const double KtoL = std::pow(a / (r + d), 1.0 / (1.0 - a));
      R[c] = 1.0 + r;
      w[c] = (1.0 - a) * std::pow(KtoL, a);
      Kd[c] = KtoL;
    }
    AIY_HIP(h, hipMemcpyAsync(Rc, R.data(), sizeof(double) * n_cal, hipMemcpyHostToDevice, st));
    AIY_HIP(h, hipMemcpyAsync(wc, w.data(), sizeof(double) * n_cal, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(fill_prices_kernel, dim3((n_cal * S + 255) / 256), dim3(256), 0, st, n_cal, S, Rc, wc, Rn, Wn,
                       Mn);
    AIY_CHECK_LAUNCH(h);
    if (loose_on) {
      for (int c = 0; c < n_cal; ++c) {
        // bracketing evaluations run loose (Brent's at the full tolerances)
        loose[c] = !rs[c].brent && !rs[c].done && !refine[c];
        etol[c] = loose[c] ? kLooseEgm : o->egm_tol;
        htol[c] = loose[c] ? kLooseHist : o->hist_tol;
        // Brent's evaluations at the adaptive tolerance, refined ones at the full one
        adapt[c] = 0;
        if (kGeAdapt && rs[c].brent && !rs[c].done && !refine[c]) {
          htol[c] = ge_adapt_htol(fmin_rel[c], o->hist_tol, kLooseHist);
          adapt[c] = htol[c] > o->hist_tol;
        }
      }
      AIY_HIP(h, hipMemcpyAsync(d_etol, etol.data(), sizeof(double) * n_cal, hipMemcpyHostToDevice, st));
      AIY_HIP(h, hipMemcpyAsync(d_htol, htol.data(), sizeof(double) * n_cal, hipMemcpyHostToDevice, st));
      h->egm_tolv = d_etol;
      h->egm_tolh = etol.data();
      h->hist_tolv = d_htol;
    }
    const bool warm_egm = o->warm_egm && steps > 0;
    // secant starts (steps >= 2, warm): x0 = cur + theta (cur - prev); the current
    // evaluation's tables / mass become the previous ones (pointer swap)
    const bool secant = o->secant_start && o->warm_egm && o->warm_hist && steps >= 2;
    if (secant) {
      for (int c = 0; c < n_cal; ++c) {
        const double den = r_cur[c] - r_prev[c];
        double th = den != 0.0 && !fin[c] ? (rs[c].x - r_cur[c]) / den : 0.0;
        theta[c] = std::isfinite(th) ? std::max(-1.0, std::min(1.0, th)) : 0.0;
      }
      AIY_HIP(h, hipMemcpyAsync(d_th, theta.data(), sizeof(double) * n_cal, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(secant_start_kernel, dim3(sec_blocks), dim3(256), 0, st, tab_per, n_cal, d_th, tm, pm, im);
      hipLaunchKernelGGL(secant_start_kernel, dim3(sec_blocks), dim3(256), 0, st, tab_per, n_cal, d_th, tc, pc, ic);
      AIY_CHECK_LAUNCH(h);
    }
    if (warm_egm) {
      std::swap(tm, pm);   // pm: the current evaluation's tables (next step's "previous")
      std::swap(tc, pc);
    }
    const double* init_m = secant ? im : pm;
    const double* init_c = secant ? ic : pc;
    h->egm_extrap = o->egm_extrapolate != 0;
    rc = aiy_egm_solve_impl(h, &dims, &in, o->egm_tol, max_cyc, kGeEgmChunk,
                            warm_egm ? init_m : nullptr, warm_egm ? init_c : nullptr, wm, wc2, tm, tc, cyc.data(),
                            dist.data(), stream);
    h->egm_extrap = 0;
    if (rc) {
      h->egm_tolv = h->egm_tolh = h->hist_tolv = nullptr;
      break;
    }
    rc = aiy_hist_lottery(h, n_cal, S, n_a, tm, tc, M->a_grid, Rc, wc, M->lab, lo, wlo, stream);
    if (rc) break;
    if (!(o->warm_hist && steps > 0)) {
      const long long n = (long long)n_cal * S * n_a;
      hipLaunchKernelGGL(fill_value_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, mass, n,
                         1.0 / ((double)S * n_a));
      AIY_CHECK_LAUNCH(h);
    } else if (o->warm_egm) {
      // mass <- secant start from (mass, pmass); pmass <- the current evaluation's mass
      const size_t mb = sizeof(double) * pts_per * n_cal;
      if (secant) {
        hipLaunchKernelGGL(secant_start_kernel, dim3(sec_blocks), dim3(256), 0, st, pts_per, n_cal, d_th, mass, pmass,
                           hw);
        AIY_CHECK_LAUNCH(h);
        std::swap(mass, pmass);
        AIY_HIP(h, hipMemcpyAsync(mass, hw, mb, hipMemcpyDeviceToDevice, st));
      } else {
        AIY_HIP(h, hipMemcpyAsync(pmass, mass, mb, hipMemcpyDeviceToDevice, st));
      }
    }
    h->hist_accel = o->accel > 0 ? o->accel : 0;   // accel < 0: BiCGSTAB (AIY_OPT_HIST_KRYLOV)
    h->hist_krylov = o->accel < 0;
    rc = aiy_hist_solve(h, n_cal, S, n_a, lo, wlo, M->P, M->a_grid, o->hist_tol, max_hist, 64, mass, hw, Ks.data(),
                        its.data(), stream);
    h->hist_accel = saved_accel;
    h->hist_krylov = saved_krylov;
    h->egm_tolv = h->egm_tolh = h->hist_tolv = nullptr;
    if (rc) break;
    if (final_pass) {   // K_s of the marked calibrations at the full tolerances; the search is over
      for (int c = 0; c < n_cal; ++c)
        if (fin[c]) {
          cyc_sum += cyc[c];
          it_sum += its[c];
          if (cyc[c] > max_cyc && !(dist[c] <= etol[c])) status[c] |= 1;
          if (its[c] >= max_hist) status[c] |= 2;
          Ks_fin[c] = Ks[c];
        }
      break;
    }
    for (int c = 0; c < n_cal; ++c) {
      const bool was_done = rs[c].done;
      cyc_sum += cyc[c];
      it_sum += its[c];
      // an evaluation that stopped at an iteration cap still moves the bracket by its sign;
      // the caller learns of it through status_out
      if (!rs[c].done && cyc[c] > max_cyc && !(dist[c] <= etol[c])) status[c] |= 1;
      if (!rs[c].done && its[c] >= max_hist) status[c] |= 2;
      r_prev[c] = r_cur[c];
      r_cur[c] = rs[c].x;
      const double f = Ks[c] - Kd[c];
      refine[c] = (loose[c] && !(std::fabs(f) >= kGeSignMargin * Kd[c])) ||   // NaN: refine
                  (adapt[c] && !(std::fabs(f) >= kGeAdaptMargin * htol[c] * Kd[c]));
      if (!refine[c]) {
        rs[c].update(f, Kd[c]);
        fmin_rel[c] = std::min(fmin_rel[c], std::fabs(f) / Kd[c]);
      }
      if (!was_done && rs[c].done) fin[c] = loose[c] || adapt[c];
      Ks_fin[c] = Ks[c];
    }
    ++steps;
  }
  h->hist_accel = saved_accel;
  h->hist_krylov = saved_krylov;
  h->egm_tolv = h->egm_tolh = h->hist_tolv = nullptr;
  if (rc) return rc;
  for (int c = 0; c < n_cal; ++c) {
    const double r = rs[c].x, a = M->alpha[c], d = M->delta[c];
    r_out[c] = r;
    K_out[c] = std::pow(a / (r + d), 1.0 / (1.0 - a));
    if (Ks_out) Ks_out[c] = Ks_fin[c];
  }
  for (int c = 0; c < n_cal; ++c)
    if (!rs[c].done) status[c] |= 4;
  if (o->status_out)
    for (int c = 0; c < n_cal; ++c) o->status_out[c] = status[c];
  if (steps_out) *steps_out = steps;
  if (egm_cycles_out) *egm_cycles_out = (int32_t)std::min<long long>(cyc_sum, 0x7fffffff);
  if (hist_iters_out) *hist_iters_out = (int32_t)std::min<long long>(it_sum, 0x7fffffff);
  return AIY_OK;
}
