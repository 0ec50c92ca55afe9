// Device helpers shared by the panel kernels (panel.hip, panel_block.hip).
#pragma once

#include "common.h"

namespace aiy {

// calc_R_and_W (AS:1839-1894) prices from aggregate capital K (= mean of a).
struct Prices {
  double Mnow, Aprev, Rnow, Wnow;
  int Mrkv;
};
__device__ __forceinline__ Prices calc_prices(const aiy_market& mk, int Mrkv, double Aprev) {
  const double AggK = Aprev;
  const double Prod = mk.prod[Mrkv ? 1 : 0];
  const double AggL = mk.agg_L[Mrkv ? 1 : 0];
  const double KtoL = AggK / AggL;
  const double al = mk.cap_share;
  Prices p;
  p.Rnow = 1.0 + Prod * (al * pow(KtoL, al - 1.0)) - mk.depr_fac;
  p.Wnow = Prod * ((1.0 - al) * pow(KtoL, al));
  p.Mnow = p.Rnow * AggK + p.Wnow * AggL;
  p.Aprev = Aprev;
  p.Mrkv = Mrkv;
  return p;
}

// index_window with the row header (base, last bucket) already in registers.
template <class I>
__device__ __forceinline__ void index_window_hdr(const int* __restrict__ H, int base, int last, int n, double q, int& lo,
                                                 int& hi) {
  lo = 0;
  hi = n;
  if (base == kIdxNoBase) return;
  const long long key = idx_key<I>(q) - (long long)base;
  if (!(q > 0.0) || key < 0) { lo = 0; hi = H[0]; }
  else if (key >= I::kBuckets - 1) {
    if (last == I::kBuckets - 1) { lo = H[I::kBuckets - 1]; hi = n; } else { lo = n; hi = n; }
  }
  else if (key > last) { lo = n; hi = n; }
  else { lo = H[key]; hi = H[key + 1]; }
  if (lo < 0 || hi > n || lo > hi) { lo = 0; hi = n; }
}

__device__ __forceinline__ double lerp_pair(const double2* __restrict__ p, int i, double q, double x0) {
  const double2 lo = p[i - 1], hi = p[i];
  const double alpha = (q - lo.x) / (hi.x - lo.x);
  const double v = (1.0 - alpha) * lo.y + alpha * hi.y;
  return (q < x0) ? __builtin_nan("") : v;
}

constexpr int kLdsLab = 16;   // labour states (the KS form has S = 4 n_lab <= 64)
constexpr int kPairs = 2;     // agent pairs per lane per pass
constexpr int kAgents = 2 * kPairs;

__device__ __forceinline__ double kBorrowNodeOf(const double2* p) { return p[0].x; }


}  // namespace aiy
