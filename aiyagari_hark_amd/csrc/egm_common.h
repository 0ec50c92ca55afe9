// EGM device helpers shared by the cycle kernel (egm.hip) and the device-resident GE
// search (ge_resident.hip): wavefront-cooperative window interpolation of HARK's
// LinearInterp (Aiyagari_Support.py:1478-1482), NumPy's pairwise order for the expectation
// (AS:1485) and the CRRA power kinds (AS:1479-1490).
#pragma once

#include "common.h"

namespace aiy {

constexpr int kEgmBlock = 256;
constexpr int kTile = 64;                     // asset nodes per block (one per lane)
constexpr int kEgmWaves = kEgmBlock / kWave;  // 4
// Per-calibration convergence words: 3 rotating distance slots x kSub sub-slots (block w
// folds into sub-slot w % kSub, so ~2 400 blocks do not serialise on one address), then
// the sticky converged flag.
constexpr int kSub = 32;
constexpr int kFlag = 3 * kSub;
constexpr int kSlots = 3 * kSub + 4;
// Node window of one next-period row staged in LDS per wave: kWin nodes starting
// kHintBack below the lower bound the previous cycle found for the tile's first query
// (the 64 queries of a tile span <= 86 nodes at configs[1], tools/egm_windows.py).
constexpr int kWin = 2 * kWave;

constexpr int kHintBack = 8;


// Window loads: plain (egm.hip: tables from the previous launch) or agent-scope `sc1`
// (ge_resident.hip: rows another workgroup of the cluster wrote this launch).
template <bool AGENT>
__device__ __forceinline__ double ld_f64(const double* p) {
  if constexpr (AGENT) return load_f64_agent(p);
  else return *p;
}

// A wave-uniform double moved to SGPRs (P[s, t] read from LDS by every lane): keeps the
// S transition weights of a state out of the VGPR budget.
__device__ __forceinline__ double uniform_f64(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// sum_t V[t] * P[t] for a compile-time count N in NumPy's pairwise order (the
// np_pairwise_sum structure: 8 running partials over the first N - N % 8 terms, then
// the tail), V[t] at stride kTile in LDS, P wave-uniform.  The terms are read and
// accumulated 8 at a time behind scheduling barriers: one straight-line block over all
// N terms let the scheduler hoist every LDS read (~150 VGPRs, occupancy 2).
template <int N>
__device__ __forceinline__ double pairwise_dot(const double* V, const double* P) {
  auto f = [&](int t) { return V[t * kTile] * P[t]; };
  if constexpr (N < 8) {
    double res = 0.0;
#pragma unroll
    for (int t = 0; t < N; ++t) res += f(t);
    return res;
  } else {
    constexpr int nfull = N - N % 8;
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f(j);
#pragma unroll
    for (int g = 8; g < nfull; g += 8) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += f(g + j);
    }
    __builtin_amdgcn_sched_barrier(0);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int t = nfull; t < N; ++t) res += f(t);
    return res;
  }
}

// One next-period row's node window, one register pair per lane: nodes base + lane and
// base + 64 + lane of x (m nodes) and y (c nodes).  base < 0: no window (no hint yet).
struct RowWin {
  double x0, x1, y0, y1;
  int base;
};

template <bool AGENT = false>
__device__ __forceinline__ void load_win(const double* __restrict__ xr, const double* __restrict__ yr, int n,
                                         int base, int lane, RowWin& C) {
  // branch-free and untouched until use (every lane loads, indices clamped into the
  // row; nodes past x[n] are masked when the window is written to LDS): a window load
  // is never behind a branch or an early use, so its wait can count the loads issued
  // after it.  32-bit unsigned offsets from the wave-uniform row pointer.
  C.base = base;
  const unsigned b = base < 0 ? 0u : (unsigned)base;
  const unsigned t0 = b + (unsigned)lane, t1 = t0 + kWave;
  const unsigned un = (unsigned)n;
  const unsigned u0 = t0 <= un ? t0 : un, u1 = t1 <= un ? t1 : un;
  // byte offsets as 32-bit values: global_load with the SGPR row base + a VGPR offset
  const unsigned o0 = u0 << 3, o1 = u1 << 3;
  C.x0 = ld_f64<AGENT>(reinterpret_cast<const double*>(reinterpret_cast<const char*>(xr) + o0));
  C.y0 = ld_f64<AGENT>(reinterpret_cast<const double*>(reinterpret_cast<const char*>(yr) + o0));
  C.x1 = ld_f64<AGENT>(reinterpret_cast<const double*>(reinterpret_cast<const char*>(xr) + o1));
  C.y1 = ld_f64<AGENT>(reinterpret_cast<const double*>(reinterpret_cast<const char*>(yr) + o1));
}

// Window start from the hint (the lower bound of the tile's first query in this row
// last cycle): kHintBack nodes below it, clamped so the window stays inside the row.
__device__ __forceinline__ int win_base(int hint, int n1) {
  if (hint < 0) return -1;
  int b = hint - kHintBack;
  const int bmax = n1 - kWin > 0 ? n1 - kWin : 0;
  b = b > bmax ? bmax : b;
  return b < 0 ? 0 : b;
}

// HARK 0.12 LinearInterp of a row (n + 1 nodes, bracket i = max(searchsorted(x[:-1], q),
// 1), NaN below x[0]) at the lane's query q, wave-cooperatively from a staged window, in
// two steps so a wave can run two rows' searches side by side:
//   stage_win:  the window into the wave's LDS slice (X, Y); true where a node is NaN;
//   search_win: (after a wave fence) the lane's lower bound by a 7-step branch-free
//               search in LDS, the bracket from LDS, the interpolated value.
// ok: the window holds the lane's bracket (a hint, no NaN node, not stale); lanes without
// it are redone from global memory (interp_row_global) -- the same lower bound, so the
// result never depends on the hint.  lb: the lane's lower bound.
__device__ __forceinline__ bool stage_win(const RowWin& C, int n, double* X, double* Y, int lane) {
  const int base = C.base < 0 ? 0 : C.base;
  const double inf = __builtin_inf();
  const double x0 = base + lane <= n ? C.x0 : inf;
  const double x1 = base + lane + kWave <= n ? C.x1 : inf;
  X[lane] = x0;
  X[lane + kWave] = x1;
  Y[lane] = C.y0;
  Y[lane + kWave] = C.y1;
  return (x0 != x0) || (x1 != x1);
}

__device__ __forceinline__ double search_win(int hint_base, bool nan_nodes, int n, double q, const double* X,
                                             const double* Y, int& lb, bool& ok) {
  const int base = hint_base < 0 ? 0 : hint_base;
  const double inf = __builtin_inf();
  const int L = n - base < kWin ? n - base : kWin;   // searchable nodes (x[:-1]) in the window
  const double xf = X[0], xlast = X[kWin - 1];
  // no short-circuit: a branch here would keep two rows' searches from interleaving
  const bool lo_ok = (base == 0) | (xf < q);
  const bool hi_ok = (base + kWin - 1 >= n) | (q <= xlast);
  ok = (hint_base >= 0) & !nan_nodes & lo_ok & hi_ok;
  // branch-free search over the whole window (nodes past x[n] are +inf); counting x[n]
  // too is undone by the clamp to L (lower_bound over x[:-1], sorted rows)
  int pos = 0;
#pragma unroll
  for (int step = kWin / 2; step > 0; step >>= 1) pos = X[pos + step - 1] < q ? pos + step : pos;
  pos = pos < L ? pos : L;
  lb = base + pos;
  int ii = (lb < 1 ? 1 : lb) - base;   // in [1, kWin - 1] when ok
  ii = ok ? ii : 1;
  const double xl = X[ii - 1], xh = X[ii], yl = Y[ii - 1], yh = Y[ii];
  const double xz = base == 0 ? xf : -inf;   // x[0] <= x[base] < q otherwise (sorted rows)
  const double alpha = (q - xl) / (xh - xl);
  const double v = (1.0 - alpha) * yl + alpha * yh;
  return (q < xz) ? __builtin_nan("") : v;
}

// The same interpolation with the lower bound searched in global memory (rows without a
// usable window).
__device__ __forceinline__ double interp_row_global(const double* __restrict__ xr, const double* __restrict__ yr,
                                                    int n, double q, int& lb) {
  lb = lower_bound(xr, 0, n, q);
  const int i = lb < 1 ? 1 : lb;
  return lerp_at(xr, yr, i, q, xr[0]);
}

// interp_row_global over agent-scope (`sc1`) loads: a row another workgroup of the
// cluster wrote in this launch (ge_resident.hip); the same lower bound and arithmetic.
__device__ __forceinline__ double interp_row_global_agent(const double* __restrict__ xr,
                                                          const double* __restrict__ yr, int n, double q, int& lb) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = lo + ((hi - lo) >> 1);
    if (load_f64_agent(&xr[mid]) < q) lo = mid + 1; else hi = mid;
  }
  lb = lo;
  const int i = lb < 1 ? 1 : lb;
  const double xl = load_f64_agent(&xr[i - 1]), xh = load_f64_agent(&xr[i]);
  const double yl = load_f64_agent(&yr[i - 1]), yh = load_f64_agent(&yr[i]);
  const double alpha = (q - xl) / (xh - xl);
  const double v = (1.0 - alpha) * yl + alpha * yh;
  return (q < load_f64_agent(&xr[0])) ? __builtin_nan("") : v;
}

// CRRA powers by a compile-time kind PK of the calibration's CRRA: 1 (log utility), 3,
// 5 (the Table II values; integer powers and a root refined in f64) or 0 (any CRRA: the
// device pow).  The Table II forms differ from the correctly rounded pow by a few ulp
// (vs NumPy's pow: 1e-12 relative parity on converged tables, tests/test_gpu_parity.py);
// the ocml f64 pow was ~40 % of a stationary 24-calibration cycle.
//   marg_u:   c^-rho          (MargValueFuncCRRA, AS:1479-1482)
//   inv_marg: E^(-1/rho)      (AS:1490)
template <int PK>
__device__ __forceinline__ double marg_u(double c, double gam) {
  if constexpr (PK == 1) return 1.0 / c;
  else if constexpr (PK == 3) return 1.0 / ((c * c) * c);
  else if constexpr (PK == 5) {
    const double c2 = c * c;
    return 1.0 / ((c2 * c2) * c);
  } else return pow(c, -gam);
}
template <int PK>
__device__ __forceinline__ double inv_marg(double E, double gam) {
  if constexpr (PK == 1) return 1.0 / E;
  else if constexpr (PK == 3) return rcbrt(E);
  else if constexpr (PK == 5) {
    // y = E^(-1/5): f32 estimate, two Newton steps on y^-5 = E (y += y (1 - E y^5) / 5);
    // outside the f32 range (or NaN) the f64 pow
    if (!(E > 1e-30 && E < 1e30)) return pow(E, -0.2);
    double y = (double)powf((float)E, -0.2f);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const double y2 = y * y;
      const double e = 1.0 - E * ((y2 * y2) * y);
      y = y + y * (e * 0.2);
    }
    return y;
  } else return pow(E, -1.0 / gam);
}

}  // namespace aiy
