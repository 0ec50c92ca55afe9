// Block-persistent Monte Carlo panel for small populations (SURVEY.md §8a rows B1-B6,
// C2), batched over calibrations (Table II in the reference's Krusell-Smith mode).
//
// The reference simulates 350-700 agents for act_T = 11 000 periods per GE iteration
// (Aiyagari-HARK.py:217-249).  At that size one launch per period would be launch-bound,
// so here ONE workgroup owns ONE calibration's whole panel for a block of periods:
// agents live in registers (K per lane), every period is
//   labour draw (np.random.choice inverse CDF, AS:1253-1254; host uniforms or Philox)
//   -> m = R a + W l (AS:1283) -> c = cFunc[4 l + 2 Mrkv + emp](m, M) (AS:1326-1408)
//   -> a = m - c (AS:1415) -> workgroup reduction of a (fixed order) -> calc_R_and_W
//   (AS:1867-1894) by lane 0 -> barrier,
// with no grid-wide synchronisation (calibrations are independent) and no memory
// traffic for the agents themselves.  Policy lookups use the same merged tables as the
// large-panel kernels (aiy_panel_build, panel_common.h).
#include "common.h"
#include "internal.h"
#include "panel_common.h"

#include <algorithm>
#include <vector>

namespace aiy {

struct BatchDev {
  int n_cal, S, n_M, n_a, n_lab, act_T;
  bool unemployed;
  const char* tables;        // [n_cal][g.bytes] merged policy tables
  PanelTabGeom g;
  const double* M_grid;      // [n_cal][n_M]
  const double* lab_level;   // [n_cal][n_lab]
  const double* lab_cdf;     // [n_cal][n_lab][n_lab]
  const int* mrkv_hist;      // [n_cal][act_T]
};

struct BlockRun {
  long long n;                     // agents per calibration
  double* a;                       // [n_cal][n]
  uint8_t* lab;                    // [n_cal][n]
  const double* u;                 // [n_cal][n_periods][n] or nullptr (Philox)
  const uint8_t* emp;              // [n_cal][n_periods][n] or nullptr (all employed)
  const unsigned long long* seeds; // [n_cal]
  const aiy_market* mk;            // [n_cal]
  unsigned ge_iter;
  int t0, n_periods;
  double* sow;                     // [n_cal][AIY_SOW_DOUBLES]
  double* hist_A;                  // [n_cal][act_T]
  double* hist_M;                  // [n_cal][act_T]
};

constexpr int kBlkMaxThreads = 1024;
constexpr int kBlkMaxAgents = 12288;   // a (f64) + lab (u8) resident in LDS: 108 KiB

// A agents per lane per sweep, as A/2 Philox pairs (2q, 2q + 1); a lane sweeps pair
// groups g = tid, tid + blockDim, ... .  a/lab live in LDS for the whole launch.
template <int A>
__global__ __launch_bounds__(kBlkMaxThreads) void panel_block_kernel(BatchDev B, BlockRun r) {
  static_assert(A % 2 == 0, "agents are processed in pairs");
  extern __shared__ double s_a[];        // [n] then lab bytes
  const int cal = blockIdx.x;
  const int tid = threadIdx.x;
  const int nthr = blockDim.x;
  const int n = (int)r.n;
  uint8_t* s_lab = reinterpret_cast<uint8_t*>(s_a + n);
  const int n_M = B.n_M, n_lab = B.n_lab;
  const PanelTab T = panel_tab(B.tables + (size_t)cal * B.g.bytes, B.g);
  const int n_J = B.g.n_J;
  const double* Mg = B.M_grid + (size_t)cal * n_M;
  const int* hist = B.mrkv_hist + (size_t)cal * B.act_T;
  const aiy_market mk = r.mk[cal];
  const unsigned long long seed = r.seeds[cal];
  double* sow = r.sow + (size_t)cal * AIY_SOW_DOUBLES;
  double* ga = r.a + (size_t)cal * n;
  uint8_t* glab = r.lab + (size_t)cal * n;

  __shared__ double s_cdf[kLdsLab * kLdsLab];
  __shared__ double s_lvl[kLdsLab];
  __shared__ CellHdr s_hdr[2 * kLdsLab];
  __shared__ double s_red[kBlkMaxThreads / kWave];
  __shared__ double s_price[4];   // Mnow, Rnow, Wnow, Mrkv
  for (int q = tid; q < n_lab * n_lab; q += nthr) s_cdf[q] = B.lab_cdf[(size_t)cal * n_lab * n_lab + q];
  for (int q = tid; q < n_lab; q += nthr) s_lvl[q] = B.lab_level[(size_t)cal * n_lab + q];
  for (int q = tid; q < n; q += nthr) {
    s_a[q] = ga[q];
    s_lab[q] = glab[q];
  }
  if (tid == 0) {
    s_price[0] = load_f64_agent(&sow[0]);
    s_price[1] = load_f64_agent(&sow[3]);
    s_price[2] = load_f64_agent(&sow[4]);
    s_price[3] = load_f64_agent(&sow[2]);
  }
  __syncthreads();

  const int n_groups = (n + A - 1) / A;
  Prices last{};
  for (int p = 0; p < r.n_periods; ++p) {
    const int t = r.t0 + p;
    const double Mnow = s_price[0], Rnow = s_price[1], Wnow = s_price[2];
    const int Mrkv = (int)s_price[3];
    int jc;
    double alpha;
    m_bracket(Mg, n_M, Mnow, jc, alpha);
    for (int q = tid; q < n_lab; q += nthr) {
      s_hdr[q] = cell_header(T, panel_cell(q, 1, Mrkv, n_lab, n_J, jc));
      if (r.emp) s_hdr[n_lab + q] = cell_header(T, panel_cell(q, 0, Mrkv, n_lab, n_J, jc));
    }
    __syncthreads();
    const unsigned ctr0 = (r.ge_iter << 20) | (unsigned)t;
    const double* u = r.u ? r.u + ((size_t)cal * r.n_periods + p) * n : nullptr;
    const uint8_t* em = r.emp ? r.emp + ((size_t)cal * r.n_periods + p) * n : nullptr;
    double local = 0.0;
    for (int g = tid; g < n_groups; g += nthr) {
      const int i0 = g * A;
      double m[A];
      int ln[A], ev[A];
#pragma unroll
      for (int kk = 0; kk < A / 2; ++kk) {
        const int ia = i0 + 2 * kk;
        double uu[2];
        if (u) {
          uu[0] = ia < n ? u[ia] : 0.0;
          uu[1] = ia + 1 < n ? u[ia + 1] : 0.0;
        } else {
          philox_uniform2(ctr0, (uint64_t)(ia >> 1), seed, 0u, uu[0], uu[1]);
        }
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int k = 2 * kk + e;
          const int i = ia + e < n ? ia + e : n - 1;
          const int l0 = s_lab[i];
          int l = 0;
          for (int q = 0; q < n_lab; ++q) l += (s_cdf[l0 * n_lab + q] <= uu[e]) ? 1 : 0;  // searchsorted 'right'
          ln[k] = l;
          ev[k] = em ? (int)em[i] : 1;                                                    // EmpNow (AS:1222-1240)
          m[k] = Rnow * s_a[i] + Wnow * (s_lvl[l] * (double)ev[k]);                      // AS:1283
        }
      }
      int cell[A], hx[A];
#pragma unroll
      for (int k = 0; k < A; ++k) {
        cell[k] = panel_cell(ln[k], ev[k], Mrkv, n_lab, n_J, jc);                      // AS:1326-1356
        hx[k] = panel_hdr(ln[k], ev[k], n_lab);
      }
      double c[A];
      tab_policy<A>(T, cell, s_hdr, hx, m, alpha, n_M > 1, c);                                  // AS:1326-1408
#pragma unroll
      for (int k = 0; k < A; ++k) {
        const int i = i0 + k;
        if (i < n) {
          const double an = m[k] - c[k];                                                 // AS:1415
          s_a[i] = an;
          s_lab[i] = (uint8_t)ln[k];
          local += an;
        }
      }
    }
    // workgroup sum of a (fixed order), then calc_R_and_W by lane 0
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) local += __shfl_down(local, o, kWave);
    if ((tid & (kWave - 1)) == 0) s_red[tid / kWave] = local;
    __syncthreads();
    if (tid == 0) {
      double tot = 0.0;
      for (int w = 0; w < nthr / kWave; ++w) tot += s_red[w];
      last = calc_prices(mk, hist[t], tot / (double)n);     // np.mean(np.array(aNow))
      s_price[0] = last.Mnow;
      s_price[1] = last.Rnow;
      s_price[2] = last.Wnow;
      s_price[3] = (double)last.Mrkv;
      if (r.hist_A) r.hist_A[(size_t)cal * B.act_T + t] = last.Aprev;
      if (r.hist_M) r.hist_M[(size_t)cal * B.act_T + t] = last.Mnow;
    }
    __syncthreads();
  }
  // LDS -> agents, final market state
  for (int q = tid; q < n; q += nthr) {
    ga[q] = s_a[q];
    glab[q] = s_lab[q];
  }
  if (tid == 0) {
    store_f64_agent(&sow[0], last.Mnow);
    store_f64_agent(&sow[1], last.Aprev);
    store_f64_agent(&sow[2], (double)last.Mrkv);
    store_f64_agent(&sow[3], last.Rnow);
    store_f64_agent(&sow[4], last.Wnow);
    store_f64_agent(&sow[5], 0.0);
    store_f64_agent(&sow[7], (double)(r.t0 + r.n_periods));
  }
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_sim_block_max_agents(void) { return kBlkMaxAgents; }

extern "C" int32_t aiy_sim_block_periods(aiy_handle* h, const aiy_panel_batch* model, const aiy_market* markets,
                                         int64_t n_agents, double* a, uint8_t* lab, const double* u,
                                         const uint8_t* emp, const uint64_t* seeds, uint32_t ge_iter, int32_t t0, int32_t n_periods,
                                         int32_t act_T, double* sow, double* hist_A, double* hist_M,
                                         aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!model || !markets || !sow || !seeds) return fail(h, AIY_ERR_ARG, "null model/markets/seeds/sow");
  const aiy_panel_batch& M = *model;
  if (M.n_cal < 1 || M.S < 1 || M.n_M < 1 || M.n_a < 2 || M.n_lab < 1 || M.n_lab > kLdsLab || M.S < 4 * M.n_lab)
    return fail(h, AIY_ERR_ARG, "bad batch model sizes");
  if (M.S != 4 * M.n_lab || 2LL * M.n_a >= BrkIdx::kMaxNodes) return fail(h, AIY_ERR_ARG, "bad batch model sizes");
  if (!M.tables || !M.lab_level || !M.lab_cdf || !M.mrkv_hist || (M.n_M > 1 && !M.M_grid))
    return fail(h, AIY_ERR_ARG, "null batch model array (tables come from aiy_panel_build)");
  if (n_agents < 1 || n_agents > kBlkMaxAgents) return fail(h, AIY_ERR_UNSUPPORTED, "n_agents out of range");
  if (!a || !lab) return fail(h, AIY_ERR_ARG, "null agent arrays");
  if (emp && !M.unemployed) return fail(h, AIY_ERR_ARG, "employment states need tables with the unemployed cells");
  if (t0 < 0 || n_periods < 0 || (int64_t)t0 + n_periods > act_T || act_T > (1 << 20))
    return fail(h, AIY_ERR_ARG, "bad period range");
  if (ge_iter >= (1u << 12)) return fail(h, AIY_ERR_ARG, "ge_iter too large for the Philox counter");
  if (n_periods == 0) return AIY_OK;
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  // per-calibration constants -> device scratch (stream-ordered copy of a pinned staging buffer)
  const size_t need = (size_t)M.n_cal * (sizeof(aiy_market) + sizeof(unsigned long long));
  if (need > h->blk_cap) {
    if (h->d_blk) (void)hipFree(h->d_blk);
    if (h->h_blk) (void)hipHostFree(h->h_blk);
    h->d_blk = nullptr; h->h_blk = nullptr; h->blk_cap = 0;
    AIY_HIP(h, hipMalloc(&h->d_blk, need));
    AIY_HIP(h, hipHostMalloc(&h->h_blk, need, hipHostMallocDefault));
    h->blk_cap = need;
  }
  AIY_HIP(h, hipStreamSynchronize(st));   // the staging buffer may still feed a previous copy
  std::memcpy(h->h_blk, markets, sizeof(aiy_market) * M.n_cal);
  std::memcpy((char*)h->h_blk + sizeof(aiy_market) * M.n_cal, seeds, sizeof(unsigned long long) * M.n_cal);
  AIY_HIP(h, hipMemcpyAsync(h->d_blk, h->h_blk, need, hipMemcpyHostToDevice, st));
  BatchDev B;
  B.n_cal = M.n_cal; B.S = M.S; B.n_M = M.n_M; B.n_a = M.n_a; B.n_lab = M.n_lab; B.act_T = act_T;
  B.unemployed = M.unemployed != 0;
  B.tables = static_cast<const char*>(M.tables); B.g = panel_tab_geom(M.n_lab, M.n_M, M.n_a, B.unemployed);
  B.M_grid = M.M_grid;
  B.lab_level = M.lab_level; B.lab_cdf = M.lab_cdf; B.mrkv_hist = M.mrkv_hist;
  BlockRun r;
  r.n = n_agents; r.a = a; r.lab = lab; r.u = u; r.emp = emp;
  r.mk = reinterpret_cast<const aiy_market*>(h->d_blk);
  r.seeds = reinterpret_cast<const unsigned long long*>((char*)h->d_blk + sizeof(aiy_market) * M.n_cal);
  r.ge_iter = ge_iter; r.t0 = t0; r.n_periods = n_periods; r.sow = sow; r.hist_A = hist_A; r.hist_M = hist_M;
  // 2 agents per lane up to 2048 agents (more waves to hide the lookup latency), then 4
  const int A = n_agents <= 2048 ? 2 : 4;
  const long long groups = (n_agents + A - 1) / A;
  int thr = (int)std::min<long long>(kBlkMaxThreads, std::max<long long>(kWave, (groups + kWave - 1) / kWave * kWave));
  const size_t lds = (size_t)n_agents * (sizeof(double) + 1);
  static bool attr_set = false;   // LDS beyond the 64 KiB default (gfx950: 160 KiB per CU)
  if (!attr_set) {
    const int max_lds = kBlkMaxAgents * (int)(sizeof(double) + 1);
    AIY_HIP(h, hipFuncSetAttribute(reinterpret_cast<const void*>(panel_block_kernel<2>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
    AIY_HIP(h, hipFuncSetAttribute(reinterpret_cast<const void*>(panel_block_kernel<4>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
    attr_set = true;
  }
  dim3 grid(M.n_cal), block(thr);
  if (A == 2) hipLaunchKernelGGL(panel_block_kernel<2>, grid, block, lds, st, B, r);
  else hipLaunchKernelGGL(panel_block_kernel<4>, grid, block, lds, st, B, r);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}
