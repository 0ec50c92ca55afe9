// The reference's simulation hooks one at a time (AiyagariType.get_shocks / get_states /
// get_controls / get_poststates, Aiyagari_Support.py:1217-1415) and the panel mean the
// market's mill takes (calc_R_and_W, AS:1868), for drivers that step [HARK]
// Market.make_history period by period (sow -> cultivate -> reap -> mill -> store) through
// the drop-in surface.  Each hook is one small launch over the agents; the fused kernels
// (panel.hip, panel_resident.hip, panel_block.hip) remain the fast path for whole
// histories and give the same per-agent results (labour draws bit for bit: same inverse
// CDF, same Philox counter; assets up to the summation order of the mean).
#include "common.h"
#include "internal.h"
#include "panel_common.h"

namespace aiy {

constexpr int kHookBlock = 256;

// get_shocks (AS:1244-1256): l' = searchsorted(cumsum(P[l]) / sum, u, 'right') with u the
// host uniform (np.random.choice on the global RNG) or Philox keyed by (ge_iter, t, global
// agent index) exactly as the fused kernels draw it.
__global__ void hook_shocks_kernel(int n_lab, const double* __restrict__ cdf, long long n, long long offset,
                                   uint8_t* __restrict__ lab, const double* __restrict__ u, unsigned long long seed,
                                   unsigned ctr0) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double uu = u ? u[i] : philox_uniform(ctr0, (uint64_t)(offset + i), seed, 0u);
  const int l0 = lab[i];
  int l = 0;
  for (int q = 0; q < n_lab; ++q) l += (cdf[l0 * n_lab + q] <= uu) ? 1 : 0;
  lab[i] = (uint8_t)l;
}

// get_states (AS:1276-1283): m = Rnow a_prev + Wnow LSStates[l] Emp
__global__ void hook_states_kernel(const double* __restrict__ lvl, long long n, double R, double W,
                                   const double* __restrict__ a_prev, const uint8_t* __restrict__ lab,
                                   const uint8_t* __restrict__ emp, double* __restrict__ m_out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double e = emp ? (double)emp[i] : 1.0;
  m_out[i] = R * a_prev[i] + W * (lvl[lab[i]] * e);
}

// get_controls (AS:1295-1408): c = cFunc[4 l + 2 Mrkv + Emp](m, Mnow), HARK's
// LinearInterpOnInterp1D over the raw policy tables (the M bracket is the period's).
__global__ void hook_controls_kernel(int n_M, int n_a, const double* __restrict__ m_tab,
                                     const double* __restrict__ c_tab, int jc, double alpha, int Mrkv, long long n,
                                     const double* __restrict__ m, const uint8_t* __restrict__ lab,
                                     const uint8_t* __restrict__ emp, double* __restrict__ c_out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = emp ? (int)emp[i] : 1;
  const int s = 4 * (int)lab[i] + 2 * Mrkv + e;
  const int n1 = n_a + 1;
  const double* bm = m_tab + (size_t)s * n_M * n1;
  const double* bc = c_tab + (size_t)s * n_M * n1;
  const double q = m[i];
  if (n_M == 1) {
    c_out[i] = interp_row(bm, bc, n_a, q);
    return;
  }
  const double f0 = interp_row(bm + (size_t)jc * n1, bc + (size_t)jc * n1, n_a, q);
  const double f1 = interp_row(bm + (size_t)(jc + 1) * n1, bc + (size_t)(jc + 1) * n1, n_a, q);
  c_out[i] = (1 - alpha) * f0 + alpha * f1;
}

// get_poststates (AS:1415): a = m - c
__global__ void hook_poststates_kernel(long long n, const double* __restrict__ m, const double* __restrict__ c,
                                       double* __restrict__ a_out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a_out[i] = m[i] - c[i];
}

// Fixed-order sum of n doubles into out[0] (single workgroup: deterministic).
__global__ __launch_bounds__(1024) void hook_sum_kernel(long long n, const double* __restrict__ x,
                                                        double* __restrict__ out) {
  __shared__ double red[1024 / kWave];
  double acc = 0.0;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) acc += x[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) s += red[w];
    out[0] = s;
  }
}

static unsigned hook_blocks(long long n) { return (unsigned)((n + kHookBlock - 1) / kHookBlock); }

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_get_shocks(aiy_handle* h, int32_t n_lab, const double* lab_cdf, int64_t n, int64_t agent_offset,
                                  uint8_t* lab, const double* u, uint64_t seed, uint32_t ge_iter, int32_t t,
                                  aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_lab < 1 || n_lab > 255 || n < 0 || agent_offset < 0 || t < 0 || t >= (1 << 20))
    return fail(h, AIY_ERR_ARG, "bad sizes");
  if (ge_iter >= (1u << 12)) return fail(h, AIY_ERR_ARG, "ge_iter too large for the Philox counter");
  if (n == 0) return AIY_OK;
  if (!lab_cdf || !lab) return fail(h, AIY_ERR_ARG, "null pointer");
  AIY_HIP(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(hook_shocks_kernel, dim3(hook_blocks(n)), dim3(kHookBlock), 0, as_stream(stream), n_lab, lab_cdf,
                     (long long)n, (long long)agent_offset, lab, u, (unsigned long long)seed,
                     (ge_iter << 20) | (unsigned)t);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_get_states(aiy_handle* h, const double* lab_level, int64_t n, double Rnow, double Wnow,
                                  const double* a_prev, const uint8_t* lab, const uint8_t* emp, double* m_out,
                                  aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n < 0) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (n == 0) return AIY_OK;
  if (!lab_level || !a_prev || !lab || !m_out) return fail(h, AIY_ERR_ARG, "null pointer");
  AIY_HIP(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(hook_states_kernel, dim3(hook_blocks(n)), dim3(kHookBlock), 0, as_stream(stream), lab_level,
                     (long long)n, Rnow, Wnow, a_prev, lab, emp, m_out);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_get_controls(aiy_handle* h, int32_t S, int32_t n_M, int32_t n_a, const double* m_tab,
                                    const double* c_tab, const double* M_grid_host, int32_t Mrkv, double Mnow,
                                    int64_t n, const double* m, const uint8_t* lab, const uint8_t* emp, double* c_out,
                                    aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (S < 4 || S % 4 || n_M < 1 || n_a < 2 || n < 0 || Mrkv < 0 || Mrkv > 1) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (n == 0) return AIY_OK;
  if (!m_tab || !c_tab || !m || !lab || !c_out || (n_M > 1 && !M_grid_host)) return fail(h, AIY_ERR_ARG, "null pointer");
  // LinearInterpOnInterp1D's M bracket (clip(searchsorted(Mgrid, Mnow), 1, n_M - 1)) on the host
  int jc = 0;
  double alpha = 0.0;
  if (n_M > 1) {
    int j = 0;
    while (j < n_M && M_grid_host[j] < Mnow) ++j;
    j = j > n_M - 1 ? n_M - 1 : (j < 1 ? 1 : j);
    alpha = (Mnow - M_grid_host[j - 1]) / (M_grid_host[j] - M_grid_host[j - 1]);
    jc = j - 1;
  }
  AIY_HIP(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(hook_controls_kernel, dim3(hook_blocks(n)), dim3(kHookBlock), 0, as_stream(stream), n_M, n_a,
                     m_tab, c_tab, jc, alpha, Mrkv, (long long)n, m, lab, emp, c_out);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_get_poststates(aiy_handle* h, int64_t n, const double* m, const double* c, double* a_out,
                                      aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n < 0) return fail(h, AIY_ERR_ARG, "bad sizes");
  if (n == 0) return AIY_OK;
  if (!m || !c || !a_out) return fail(h, AIY_ERR_ARG, "null pointer");
  AIY_HIP(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(hook_poststates_kernel, dim3(hook_blocks(n)), dim3(kHookBlock), 0, as_stream(stream),
                     (long long)n, m, c, a_out);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_sum(aiy_handle* h, const double* x, int64_t n, double* out, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n < 0 || !out || (n > 0 && !x)) return fail(h, AIY_ERR_ARG, "bad arguments");
  AIY_HIP(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(hook_sum_kernel, dim3(1), dim3(1024), 0, as_stream(stream), (long long)n, x, out);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}
