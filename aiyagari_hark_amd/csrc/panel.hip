// Monte Carlo panel for gfx950.
//
// One period of Market.make_history ([HARK] sow -> cultivate -> reap -> mill) becomes
//   sim_period_kernel    every agent: labour draw (np.random.choice inverse CDF,
//                        Aiyagari_Support.py:1253-1254), m = R a + W l
//                        (AS:1283), c = cFunc[4l + 2 Mrkv + emp](m, M) (AS:1326-1408),
//                        a = m - c (AS:1415); per-block partial sums of a;
//   period_sum_kernel    fixed-order sum of the block partials (deterministic);
//   [ncclAllReduce]      when agents are sharded over ranks;
//   period_price_kernel  calc_R_and_W (AS:1867-1894): K = mean a, prices, history.
// The market state ("sow_state") never leaves the device; the host only enqueues.
// Agents are processed one per lane with a grid-stride loop whose grid depends only on
// the local agent count, so the summation order -- and hence every bit of the
// history -- is independent of the device and of timing.
#include "common.h"
#include "internal.h"

#include <algorithm>

namespace aiy {

constexpr int kSimBlock = 256;
constexpr int kSimMaxBlocks = 8192;

struct PanelDev {
  int S, n_M, n_a, n_lab;
  const double* m_pol;
  const double* c_pol;
  const double* M_grid;
  const double* lab_level;
  const double* lab_cdf;
  const int* mrkv_hist;
};

__global__ __launch_bounds__(kSimBlock) void sim_period_kernel(PanelDev P, long long n, long long offset,
                                                               double* __restrict__ a, uint8_t* __restrict__ lab,
                                                               const double* __restrict__ u, unsigned long long seed,
                                                               unsigned ctr0, const double* __restrict__ sow,
                                                               double* __restrict__ partials) {
  const double Mnow = load_f64_agent(&sow[0]);
  const int Mrkv = (int)load_f64_agent(&sow[2]);
  const double Rnow = load_f64_agent(&sow[3]);
  const double Wnow = load_f64_agent(&sow[4]);
  const int n_M = P.n_M, n1 = P.n_a + 1, n_lab = P.n_lab;
  // LinearInterpOnInterp1D bracket in M: the same for every agent of the period.
  int j = 1;
  double alpha = 0.0;
  if (n_M > 1) {
    j = lower_bound(P.M_grid, 0, n_M, Mnow);
    j = j > n_M - 1 ? n_M - 1 : j;
    j = j < 1 ? 1 : j;
    alpha = (Mnow - P.M_grid[j - 1]) / (P.M_grid[j] - P.M_grid[j - 1]);
  }
  double local = 0.0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += stride) {
    const int lp = lab[idx];
    const double uu = u ? u[idx] : philox_uniform(ctr0, (uint64_t)(offset + idx), seed, 0u);
    const double* cdf = P.lab_cdf + (size_t)lp * n_lab;
    int ln = 0;
    for (int t = 0; t < n_lab; ++t) ln += (cdf[t] <= uu) ? 1 : 0;  // searchsorted(cdf, u, 'right')
    const double m = Rnow * a[idx] + Wnow * (P.lab_level[ln] * 1.0);
    const int s = 4 * ln + 2 * Mrkv + 1;                                // employed (Urate = 0)
    const double* bm = P.m_pol + (size_t)s * n_M * n1;
    const double* bc = P.c_pol + (size_t)s * n_M * n1;
    double c;
    if (n_M == 1) {
      c = interp_row(bm, bc, P.n_a, m);
    } else {
      const double f0 = interp_row(bm + (size_t)(j - 1) * n1, bc + (size_t)(j - 1) * n1, P.n_a, m);
      const double f1 = interp_row(bm + (size_t)j * n1, bc + (size_t)j * n1, P.n_a, m);
      c = (1 - alpha) * f0 + alpha * f1;
    }
    const double an = m - c;
    a[idx] = an;
    lab[idx] = (uint8_t)ln;
    local += an;
  }
  __shared__ double red[kSimBlock / kWave];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) local += __shfl_down(local, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = red[0];
    for (int w = 1; w < kSimBlock / kWave; ++w) s += red[w];
    partials[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(256) void period_sum_kernel(const double* __restrict__ partials, int nb, double* sow) {
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += partials[b];
  __shared__ double red[256 / kWave];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) store_f64_agent(&sow[6], (red[0] + red[1]) + (red[2] + red[3]));
}

// calc_R_and_W (AS:1839-1894) from the (all-reduced) sum in sow[6].
__global__ void period_price_kernel(aiy_market mk, const int* __restrict__ mrkv_hist, long long n_total, int t,
                                    double* sow, double* hist_A, double* hist_M) {
  if (threadIdx.x != 0) return;
  const double Aprev = load_f64_agent(&sow[6]) / (double)n_total;   // np.mean(np.array(aNow))
  const double AggK = Aprev;
  const int Mrkv = mrkv_hist[t];
  const double Prod = mk.prod[Mrkv ? 1 : 0];
  const double AggL = mk.agg_L[Mrkv ? 1 : 0];
  const double KtoL = AggK / AggL;
  const double al = mk.cap_share;
  const double Rnow = 1.0 + Prod * (al * pow(KtoL, al - 1.0)) - mk.depr_fac;
  const double Wnow = Prod * ((1.0 - al) * pow(KtoL, al));
  const double Mnow = Rnow * AggK + Wnow * AggL;
  store_f64_agent(&sow[0], Mnow);
  store_f64_agent(&sow[1], Aprev);
  store_f64_agent(&sow[2], (double)Mrkv);
  store_f64_agent(&sow[3], Rnow);
  store_f64_agent(&sow[4], Wnow);
  store_f64_agent(&sow[5], 0.0);  // Urate: everyone employed at UrateB = UrateG = 0
  if (hist_A) hist_A[t] = Aprev;
  if (hist_M) hist_M[t] = Mnow;
}

static int sim_blocks(long long n) {
  long long nb = (n + kSimBlock - 1) / kSimBlock;
  return (int)std::max(1LL, std::min<long long>(nb, kSimMaxBlocks));
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_sim_periods(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                                   int64_t n_local, int64_t agent_offset, int64_t n_total, double* a, uint8_t* lab,
                                   const double* u, int64_t u_ld, uint64_t seed, uint32_t ge_iter, int32_t t0,
                                   int32_t n_periods, double* sow, double* hist_A, double* hist_M,
                                   aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!model || !mkt || !sow) return fail(h, AIY_ERR_ARG, "null model/market/sow");
  if (model->S < 1 || model->n_M < 1 || model->n_a < 2 || model->n_lab < 1 || model->n_lab > 255)
    return fail(h, AIY_ERR_ARG, "bad model sizes");
  if (model->S < 4 * model->n_lab) return fail(h, AIY_ERR_ARG, "S must be 4 * n_lab (KS form)");
  if (!model->m_pol || !model->c_pol || !model->lab_level || !model->lab_cdf || !model->mrkv_hist)
    return fail(h, AIY_ERR_ARG, "null model array");
  if (model->n_M > 1 && !model->M_grid) return fail(h, AIY_ERR_ARG, "null M_grid");
  if (n_local < 0 || n_total < 1 || agent_offset < 0) return fail(h, AIY_ERR_ARG, "bad agent counts");
  if (n_local > 0 && (!a || !lab)) return fail(h, AIY_ERR_ARG, "null agent arrays");
  if (u && u_ld < n_local) return fail(h, AIY_ERR_ARG, "u_ld < n_local");
  if (t0 < 0 || n_periods < 0 || t0 + (int64_t)n_periods > (1 << 20)) return fail(h, AIY_ERR_ARG, "bad period range");
  if (ge_iter >= (1u << 12)) return fail(h, AIY_ERR_ARG, "ge_iter too large for the Philox counter");
  if (n_periods == 0) return AIY_OK;
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  const int nb = sim_blocks(n_local);
  if ((size_t)nb > h->partials_cap) {
    if (h->d_partials) (void)hipFree(h->d_partials);
    h->d_partials = nullptr;
    AIY_HIP(h, hipMalloc((void**)&h->d_partials, sizeof(double) * kSimMaxBlocks));
    h->partials_cap = kSimMaxBlocks;
  }
  PanelDev P;
  P.S = model->S; P.n_M = model->n_M; P.n_a = model->n_a; P.n_lab = model->n_lab;
  P.m_pol = model->m_pol; P.c_pol = model->c_pol; P.M_grid = model->M_grid;
  P.lab_level = model->lab_level; P.lab_cdf = model->lab_cdf; P.mrkv_hist = model->mrkv_hist;
  for (int p = 0; p < n_periods; ++p) {
    const int t = t0 + p;
    const unsigned ctr0 = (ge_iter << 20) | (unsigned)t;
    const double* up = u ? u + (size_t)p * u_ld : nullptr;
    if (n_local > 0) {
      hipLaunchKernelGGL(sim_period_kernel, dim3(nb), dim3(kSimBlock), 0, st, P, (long long)n_local,
                         (long long)agent_offset, a, lab, up, (unsigned long long)seed, ctr0, sow, h->d_partials);
      hipLaunchKernelGGL(period_sum_kernel, dim3(1), dim3(256), 0, st, h->d_partials, nb, sow);
    } else {
      AIY_HIP(h, hipMemsetAsync(sow + 6, 0, sizeof(double), st));
    }
    if (h->comm) {
      ncclResult_t r = ncclAllReduce(sow + 6, sow + 6, 1, ncclDouble, ncclSum, h->comm, st);
      if (r != ncclSuccess) return fail(h, AIY_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    }
    hipLaunchKernelGGL(period_price_kernel, dim3(1), dim3(64), 0, st, *mkt, model->mrkv_hist, (long long)n_total, t,
                       sow, hist_A, hist_M);
  }
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}
