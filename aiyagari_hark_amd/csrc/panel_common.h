// Device helpers shared by the panel kernels (panel.hip, panel_block.hip).
#pragma once

#include "common.h"
#include "internal.h"

namespace aiy {

// One calibration's panel model on device (aiy_panel_model).
struct PanelDev {
  int S, n_M, n_a, n_lab;
  const double* M_grid;
  const double* lab_level;
  const double* lab_cdf;
  const int* mrkv_hist;
  const int* pol_index;     // BrkIdx rows (aiy_panel_prepare), int32 words
  const double2* pol_pairs; // (m, c) interleaved rows (aiy_panel_prepare)
};

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
  // KtoL ** al and KtoL ** (al - 1) from ONE log and ONE exp (the price update sits on
  // every period's critical path; pow twice costs ~2x).  Differs from two pow calls by
  // a few ulp.
  const double ka = exp(al * log(KtoL));
  p.Rnow = 1.0 + Prod * (al * (ka / KtoL)) - mk.depr_fac;
  p.Wnow = Prod * ((1.0 - al) * ka);
  p.Mnow = p.Rnow * AggK + p.Wnow * AggL;
  p.Aprev = Aprev;
  p.Mrkv = Mrkv;
  return p;
}

// Bracket-index window of one policy row with its header (base, last bucket) already in
// registers (brk_window, common.h).
__device__ __forceinline__ void panel_window(const int* __restrict__ row, int base, int last, int n, double q, int& lo,
                                             int& hi) {
  brk_window(row, base, last, n, q, lo, hi);
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

// Persistent panel (panel_resident.hip), used by aiy_sim_periods on a single rank.
int32_t launch_resident(aiy_handle* h, const PanelDev& P, const aiy_market& mk, long long n, double* a, uint8_t* lab,
                        const double* u, long long u_ld, unsigned long long seed, unsigned ge_iter, int t0,
                        int n_periods, double* sow, double* hist_A, double* hist_M, hipStream_t st);
int32_t resident_status(aiy_handle* h, hipStream_t st);
bool resident_supported(const PanelDev& P);
constexpr long long kResMinAgents = 65536;

}  // namespace aiy
