// One calibration's root search on f(r) = K_s(r) - K_d(r) (build-defined row E1), shared
// by the host-driven search (ge.hip) and the device-resident one (ge_resident.hip):
// method 0 = bisection (oracle/stationary.py ge_bisect, step for step); method 1 =
// bisection until both signs of f are evaluated, then Brent's method (the
// scipy.optimize.brentq algorithm; aiyagari_hark_amd/stationary.py _Brent is the same
// coroutine in Python), or -- with loose bracketing -- the log-coordinate bracketing and
// Brent described at `logsec` below (no Python mirror: the Python engine runs without loose
// bracketing).  Every workgroup of a device cluster runs its own copy on bit-identical
// inputs, so all copies take the same steps.
#pragma once

#include <hip/hip_runtime.h>

namespace aiy {


struct RootSearch {
  double lo, hi, xtol;
  bool have_lo, have_hi, brent, done;
  // log-secant bracketing (with loose bracketing): while only K_s < K_d has been seen, the
  // next point comes from a secant of g = log(K_s / K_d) against u = log(rtop - r) through
  // the last two such points -- near 1/beta - 1 the excess supply grows about exponentially
  // in u -- aimed 20 % past the predicted root, its distance to rtop kept within [1/16, 1/2]
  // of the current one (1/2: bisection toward rtop)
  // ... and Brent's method then runs in the same coordinates (u, g), where the root is nearly
  // linear, with the tolerance xtol / (rtop - lo) in u (so the bracket in r is <= xtol)
  bool logsec, logsec1;   // logsec1: also the one-point step (log_secant == 2)
  int nneg;
  double rtop, ua, ga, ub, gb, glo, ghi;
  bool logb;   // Brent runs in (u, g)
  double flo, fhi, x;
  double xpre, fpre, xcur, fcur, xblk, fblk, spre, scur;
  double xprev_eval, fprev_eval;
  int method;

  __host__ __device__ static double fabs_(double v) { return v < 0 ? -v : v; }
  __host__ __device__ static double fmin_(double a, double b) { return (b < a) ? b : a; }   // std::min

  __host__ __device__ void init(double l, double h, double tol, int meth, int log_secant = 0) {
    lo = l; hi = h; xtol = tol; method = meth;
    logsec = log_secant > 0 && meth == 1;
    logsec1 = logsec && log_secant >= 2;
    nneg = 0;
    rtop = h;
    ua = ga = ub = gb = glo = ghi = 0.0;
    logb = false;
    have_lo = have_hi = brent = false;
    flo = fhi = 0.0;
    xpre = fpre = xcur = fcur = xblk = fblk = spre = scur = 0.0;
    xprev_eval = fprev_eval = 0.0;
    x = 0.5 * (lo + hi);
    done = !(hi - lo > xtol);
  }
  __host__ __device__ void update(double f, double Kd = 0.0) {
    if (done) return;
    if (method == 0) {   // oracle ge_bisect: Ks > Kd -> hi = mid
      if (f > 0) hi = x; else lo = x;
      if (!(hi - lo > xtol)) { done = true; x = 0.5 * (lo + hi); return; }
      x = 0.5 * (lo + hi);
      return;
    }
    const bool tr = logsec && Kd > 0 && f > -Kd;   // transformed coordinates available
    if (!brent) {
      if (f > 0) { hi = x; fhi = f; have_hi = true; } else { lo = x; flo = f; have_lo = true; }
      if (tr) (f > 0 ? ghi : glo) = log1p(f / Kd);
      if (hi - lo <= xtol) { done = true; x = 0.5 * (lo + hi); return; }
      if (!have_lo || !have_hi) {
        const double xe = x;
        x = 0.5 * (lo + hi);
        if (logsec1 && !have_lo && tr && f > 0 && xe < rtop) {
          // only K_s > K_d seen (the first point was above the root): the same unit-slope
          // prediction from the latest point, aimed 25 % beyond the root (away from rtop),
          // the distance to rtop grown 2 .. 16 times; bisection if that leaves the bracket
          const double dc = rtop - xe;
          double dn = 1.25 * exp(log(dc) + log1p(f / Kd));
          dn = dn < 2 * dc ? 2 * dc : (dn > 16 * dc ? 16 * dc : dn);
          const double xn = rtop - dn;
          if (xn > lo && xn < hi) x = xn;
        }
        if (logsec && !have_hi && Kd > 0 && f > -Kd && xe < rtop) {
          ua = ub; ga = gb;
          ub = log(rtop - xe); gb = log1p(f / Kd);
          ++nneg;
          // one point: the slope dg/du = -1 the Table II cells show far from 1/beta - 1
          // (K_s / K_d - 1 about doubles per halving of the distance); two: their secant
          const bool two = nneg >= 2 && gb > ga && ub < ua;
          // (the one-point prediction only where it lies well toward rtop, < 1/4 of the current
          // distance: the slope is steeper where the root is far below 1/beta - 1)
          const double us = two ? ub - gb * (ub - ua) / (gb - ga) : ub + gb;   // predicted root in u
          const double dc = rtop - xe;
          if (two || (nneg == 1 && logsec1 && exp(us) < dc / 4)) {
            double dn = 0.8 * exp(us);
            dn = dn < dc / 16 ? dc / 16 : (dn > dc / 2 ? dc / 2 : dn);
            const double xn = rtop - dn;
            if (xn > lo && xn < hi) x = xn;
          }
        }
        return;
      }
      brent = true;
      if (logsec && tr && hi < rtop) {   // Brent in (u, g); xtol in u keeps the r bracket <= xtol
        logb = true;
        xtol = xtol / (rtop - lo);
        xpre = log(rtop - lo); fpre = glo; xcur = log(rtop - hi); fcur = ghi;
      } else {
        xpre = lo; fpre = flo; xcur = hi; fcur = fhi;
      }
      xblk = fblk = spre = scur = 0.0;
      step();
      if (logb) x = rtop - exp(x);
      return;
    }
    xpre = xprev_eval; fpre = fprev_eval; fcur = logb ? (tr ? log1p(f / Kd) : (f > 0 ? 1e300 : -1e300)) : f;
    step();
    if (logb) x = rtop - exp(x);
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
// (the histogram's loose tolerance is the handle option AIY_OPT_GE_LOOSE_HIST: 10^-8 by default
// since round 4, 10^-10 before; the full-size Table II / stress parity tests pass at both)
constexpr double kGeSignMargin = 0.05;

// Adaptive distribution tolerance of Brent's evaluations (with loose bracketing).  A BiCGSTAB
// solve stopped at max|T x - x| < tol leaves K_s about 4e5 tol off relative (DESIGN.md §4c:
// 4e-7 at 1e-12), and Brent's next |f| is rarely below 1/100 of the smallest |f| seen so far
// (the Table II searches: 20-80x per step), so an evaluation at tol = kGeAdaptC |f|_min / K_d
// already resolves f to well inside its expected size; its sign and value are trusted when
// |f| >= kGeAdaptMargin tol K_d (5 % at 1e-8, the bracketing margin: 12x the error estimate),
// else the same r is evaluated again at the full tolerance (continuing from its mass: the
// stopping rule of the final bracket is unchanged).  -DAIY_DIAG_NO_ADAPT turns it off.
constexpr double kGeAdaptC = 1e-9;
constexpr double kGeAdaptMargin = 5e6;
#ifdef AIY_DIAG_NO_ADAPT
constexpr bool kGeAdapt = false;
#else
constexpr bool kGeAdapt = true;
#endif
__host__ __device__ inline double ge_adapt_htol(double fmin_rel, double hist_tol, double loose_hist) {
  const double t = kGeAdaptC * fmin_rel;
  return t > loose_hist ? loose_hist : (t < hist_tol ? hist_tol : t);   // NaN: hist_tol
}

}  // namespace aiy
