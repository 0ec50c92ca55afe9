// One calibration's root search on f(r) = K_s(r) - K_d(r) (build-defined row E1), shared
// by the host-driven search (ge.hip) and the device-resident one (ge_resident.hip):
// method 0 = bisection (oracle/stationary.py ge_bisect, step for step); method 1 =
// bisection until both signs of f are evaluated, then Brent's method (the
// scipy.optimize.brentq algorithm; aiyagari_hark_amd/stationary.py _Brent is the same
// coroutine in Python).  Every workgroup of a device cluster runs its own copy on
// bit-identical inputs, so all copies take the same steps.
#pragma once

#include <hip/hip_runtime.h>

namespace aiy {

struct RootSearch {
  double lo, hi, xtol;
  bool have_lo, have_hi, brent, done;
  double flo, fhi, x;
  double xpre, fpre, xcur, fcur, xblk, fblk, spre, scur;
  double xprev_eval, fprev_eval;
  int method;

  __host__ __device__ static double fabs_(double v) { return v < 0 ? -v : v; }
  __host__ __device__ static double fmin_(double a, double b) { return (b < a) ? b : a; }   // std::min

  __host__ __device__ void init(double l, double h, double tol, int meth) {
    lo = l; hi = h; xtol = tol; method = meth;
    have_lo = have_hi = brent = false;
    flo = fhi = 0.0;
    xpre = fpre = xcur = fcur = xblk = fblk = spre = scur = 0.0;
    xprev_eval = fprev_eval = 0.0;
    x = 0.5 * (lo + hi);
    done = !(hi - lo > xtol);
  }
  __host__ __device__ void update(double f) {
    if (done) return;
    if (method == 0) {   // oracle ge_bisect: Ks > Kd -> hi = mid
      if (f > 0) hi = x; else lo = x;
      if (!(hi - lo > xtol)) { done = true; x = 0.5 * (lo + hi); return; }
      x = 0.5 * (lo + hi);
      return;
    }
    if (!brent) {
      if (f > 0) { hi = x; fhi = f; have_hi = true; } else { lo = x; flo = f; have_lo = true; }
      if (hi - lo <= xtol) { done = true; x = 0.5 * (lo + hi); return; }
      if (!have_lo || !have_hi) { x = 0.5 * (lo + hi); return; }
      brent = true;
      xpre = lo; fpre = flo; xcur = hi; fcur = fhi;
      xblk = fblk = spre = scur = 0.0;
      step();
      return;
    }
    xpre = xprev_eval; fpre = fprev_eval; fcur = f;
    step();
  }
  __host__ __device__ void step() {
    const double kEps = 2.220446049250313e-16;   // DBL_EPSILON
    if (fpre * fcur < 0) { xblk = xpre; fblk = fpre; spre = scur = xcur - xpre; }
    if (fabs_(fblk) < fabs_(fcur)) {
      const double xp = xcur, xc = xblk, fp = fcur, fc = fblk;
      xpre = xp; xcur = xc; xblk = xp;
      fpre = fp; fcur = fc; fblk = fp;
    }
    const double delta = 0.5 * (xtol + 4 * kEps * fabs_(xcur));
    const double sbis = 0.5 * (xblk - xcur);
    if (fcur == 0 || fabs_(sbis) < delta) { done = true; x = xcur; return; }
    if (fabs_(spre) > delta && fabs_(fcur) < fabs_(fpre)) {
      double stry;
      if (xpre == xblk) {
        stry = -fcur * (xcur - xpre) / (fcur - fpre);
      } else {
        const double dpre = (fpre - fcur) / (xpre - xcur);
        const double dblk = (fblk - fcur) / (xblk - xcur);
        stry = -fcur * (fblk * dblk - fpre * dpre) / (dblk * dpre * (fblk - fpre));
      }
      if (2 * fabs_(stry) < fmin_(fabs_(spre), 3 * fabs_(sbis) - delta)) { spre = scur; scur = stry; }
      else { spre = sbis; scur = sbis; }
    } else {
      spre = sbis; scur = sbis;
    }
    xprev_eval = xcur; fprev_eval = fcur;
    xcur += fabs_(scur) > delta ? scur : (sbis > 0 ? delta : -delta);
    x = xcur;
  }
};

// loose-bracketing tolerances (aiy_ge_options.loose_bracket) and the sign margin a loose
// evaluation's K_s - K_d needs (|f| >= kGeSignMargin K_d)
#ifndef AIY_GE_LOOSE_EGM
#define AIY_GE_LOOSE_EGM 1e-6
#endif
#ifndef AIY_GE_LOOSE_HIST
#define AIY_GE_LOOSE_HIST 1e-10
#endif
constexpr double kGeSignMargin = 0.05;

}  // namespace aiy
