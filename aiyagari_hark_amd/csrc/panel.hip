// Monte Carlo panel for gfx950.
//
// One period of Market.make_history ([HARK] sow -> cultivate -> reap -> mill) is ONE
// kernel launch on a single GPU:
//   every agent (one per lane, grid-stride): labour draw (np.random.choice inverse CDF,
//   Aiyagari_Support.py:1253-1254), m = R a + W l (AS:1283),
//   c = cFunc[4 l + 2 Mrkv + emp](m, M) (AS:1326-1408), a = m - c (AS:1415);
//   per-block partial sum of a -> the LAST block to arrive (write-through partials +
//   agent-scope ticket, cdna_hip_programming.md Guideline 16) sums the partials in
//   fixed order and runs mill/calc_R_and_W (AS:1867-1894), writing the next sow_state
//   and the history.
// The period index lives on the device (sow[7]) so every launch of a history has
// identical arguments: aiy_sim_periods captures a block of periods into a hipGraph
// once and replays it, which takes the host out of the per-period loop.
// With agents sharded over ranks the last block only publishes the
// local sum; an ncclAllReduce and a 1-thread price kernel follow on the same stream.
// The grid depends only on the local agent count and the partial sums are combined in
// fixed order, so every bit of the history is reproducible run to run.
#include "common.h"
#include "internal.h"
#include "panel_common.h"

#include <algorithm>

namespace aiy {

constexpr int kSimBlock = 256;
constexpr int kSimMaxBlocks = 8192;
// Arrival tickets: blocks count in kTicketGroups sub-counters (b % kTicketGroups), each on
// its own cache line; the last arriver of a group bumps the top counter.  One counter
// for ~3900 blocks serialised ~12 ns per atomic (measured 60 us per period at 1M agents,
// independent of data locality); with 16 groups each counter sees ~250 arrivals.
constexpr int kTicketGroups = 16;
constexpr int kTicketStride = 32;   // uints: 128 B apart
constexpr int kGraphPeriods = 64;

struct PanelRun {
  long long n, offset, n_total;
  double* a;
  uint8_t* lab;
  const double* u;   // uniforms [.. ][u_ld] starting at period u_t0, or nullptr (Philox)
  long long u_ld;
  int u_t0;
  const uint8_t* emp;   // employment [..][emp_ld] from period u_t0, or nullptr (all employed)
  long long emp_ld;
  unsigned long long seed;
  unsigned ge_iter;
  double* sow;
  double* partials;
  unsigned* ticket;
  double* hist_A;
  double* hist_M;
  int finish;        // 1: last block computes prices (single rank); 0: publish local sum only
};

// calc_R_and_W (AS:1839-1894) given the sum of end-of-period assets over all agents.
__device__ __forceinline__ void mill(const aiy_market& mk, const int* mrkv_hist, long long n_total, double sum_a,
                                     double* sow, double* hist_A, double* hist_M) {
  const int t = (int)load_f64_agent(&sow[7]);
  const Prices p = calc_prices(mk, mrkv_hist[t], sum_a / (double)n_total);   // np.mean(np.array(aNow))
  store_f64_agent(&sow[0], p.Mnow);
  store_f64_agent(&sow[1], p.Aprev);
  store_f64_agent(&sow[2], (double)p.Mrkv);
  store_f64_agent(&sow[3], p.Rnow);
  store_f64_agent(&sow[4], p.Wnow);
  store_f64_agent(&sow[5], 0.0);  // Urate is recorded by the caller (it draws the employment)
  store_f64_agent(&sow[7], (double)(t + 1));
  if (hist_A) hist_A[t] = p.Aprev;
  if (hist_M) hist_M[t] = p.Mnow;
}

__global__ __launch_bounds__(kSimBlock) void sim_period_kernel(PanelDev P, PanelRun r, aiy_market mk) {
  const double Mnow = load_f64_agent(&r.sow[0]);
  const int Mrkv = (int)load_f64_agent(&r.sow[2]);
  const double Rnow = load_f64_agent(&r.sow[3]);
  const double Wnow = load_f64_agent(&r.sow[4]);
  const int t = (int)load_f64_agent(&r.sow[7]);
  const unsigned ctr0 = (r.ge_iter << 20) | (unsigned)t;
  const double* u = r.u ? r.u + (size_t)(t - r.u_t0) * r.u_ld : nullptr;
  const uint8_t* em = r.emp ? r.emp + (size_t)(t - r.u_t0) * r.emp_ld : nullptr;
  const int n_M = P.n_M, n_lab = P.n_lab, n_J = P.tab.g.n_J;
  // LinearInterpOnInterp1D bracket in M: the same for every agent of the period.
  int jc;
  double alpha;
  m_bracket(P.M_grid, n_M, Mnow, jc, alpha);
  // Stage the labour chain (inverse CDF rows, levels) and the period's cell headers in
  // LDS: the per-agent dependent chain then has no global hop before the policy lookup.
  __shared__ double s_cdf[kLdsLab * kLdsLab];
  __shared__ double s_lvl[kLdsLab];
  __shared__ CellHdr s_hdr[2 * kLdsLab];
  for (int q = threadIdx.x; q < n_lab * n_lab; q += blockDim.x) s_cdf[q] = P.lab_cdf[q];
  for (int q = threadIdx.x; q < n_lab; q += blockDim.x) {
    s_lvl[q] = P.lab_level[q];
    s_hdr[q] = cell_header(P.tab, panel_cell(q, 1, Mrkv, n_lab, n_J, jc));
    if (em) s_hdr[n_lab + q] = cell_header(P.tab, panel_cell(q, 0, Mrkv, n_lab, n_J, jc));
  }
  __syncthreads();
  double local = 0.0;
  // kPairs agent PAIRS per lane (one Philox call and one 16-byte asset load per pair),
  // their dependent chains interleaved: the panel is latency-bound, and this puts the
  // whole population in flight in one wave round.
  const long long npairs = (r.n + 1) >> 1;
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  const bool even_offset = (r.offset & 1) == 0;
  for (long long pb = (long long)blockIdx.x * blockDim.x + threadIdx.x; pb < npairs; pb += nthreads * kPairs) {
    long long idx[kAgents];
    bool ok[kAgents];
    int lp[kAgents], ln[kAgents], ev[kAgents];
    double ap[kAgents], m[kAgents], uu[kAgents];
#pragma unroll
    for (int k = 0; k < kPairs; ++k) {
      const long long q = pb + k * nthreads;
      const long long i0 = 2 * q;
      idx[2 * k] = i0;
      idx[2 * k + 1] = i0 + 1;
      ok[2 * k] = i0 < r.n;
      ok[2 * k + 1] = i0 + 1 < r.n;
      if (ok[2 * k + 1]) {
        const double2 av = *reinterpret_cast<const double2*>(r.a + i0);
        const unsigned short lv = *reinterpret_cast<const unsigned short*>(r.lab + i0);
        ap[2 * k] = av.x; ap[2 * k + 1] = av.y;
        lp[2 * k] = lv & 0xff; lp[2 * k + 1] = lv >> 8;
      } else {
        ap[2 * k] = ok[2 * k] ? r.a[i0] : 0.0; ap[2 * k + 1] = 0.0;
        lp[2 * k] = ok[2 * k] ? r.lab[i0] : 0; lp[2 * k + 1] = 0;
      }
      ev[2 * k] = (em && ok[2 * k]) ? (int)em[i0] : 1;
      ev[2 * k + 1] = (em && ok[2 * k + 1]) ? (int)em[i0 + 1] : 1;
      if (u) {
        uu[2 * k] = ok[2 * k] ? u[i0] : 0.0;
        uu[2 * k + 1] = ok[2 * k + 1] ? u[i0 + 1] : 0.0;
      } else if (even_offset) {
        philox_uniform2(ctr0, (uint64_t)((r.offset + i0) >> 1), r.seed, 0u, uu[2 * k], uu[2 * k + 1]);
      } else {
        uu[2 * k] = philox_uniform(ctr0, (uint64_t)(r.offset + i0), r.seed, 0u);
        uu[2 * k + 1] = philox_uniform(ctr0, (uint64_t)(r.offset + i0 + 1), r.seed, 0u);
      }
    }
#ifdef AIY_DIAG_NO_PHILOX
#pragma unroll
    for (int k = 0; k < kAgents; ++k) uu[k] = 0.37 + 1e-9 * (double)(idx[k] & 1023);
#endif
    int cell[kAgents], hx[kAgents];
#pragma unroll
    for (int k = 0; k < kAgents; ++k) {
      int l = 0;
      for (int q = 0; q < n_lab; ++q) l += (s_cdf[lp[k] * n_lab + q] <= uu[k]) ? 1 : 0;  // searchsorted(cdf, u, 'right')
      ln[k] = l;
      m[k] = Rnow * ap[k] + Wnow * (s_lvl[l] * (double)ev[k]);                          // AS:1283
      cell[k] = panel_cell(l, ev[k], Mrkv, n_lab, n_J, jc);                              // AS:1326-1356
      hx[k] = panel_hdr(l, ev[k], n_lab);
    }
    double c[kAgents];
    tab_policy<kAgents>(P.tab, cell, s_hdr, hx, m, alpha, n_M > 1, c);                          // AS:1326-1408
#pragma unroll
    for (int k = 0; k < kAgents; ++k) {
      const double an = m[k] - c[k];                                                    // AS:1415
      if (ok[k]) {
        r.a[idx[k]] = an;
        r.lab[idx[k]] = (uint8_t)ln[k];
        local += an;
      }
    }
  }
  // ---- block partial, then the last block finishes the period ----
  __shared__ double red[kSimBlock / kWave];
  __shared__ int is_last;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) local += __shfl_down(local, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    // Hand-off without fences (MI355X_MICROARCH.md, "Valid forms", row 1): the partial is
    // stored write-through (sc1), drained, then counted with an agent-scope atomic; the
    // last arriver reads every partial with sc1 loads.  A per-block release fence here
    // would write back the XCD's whole L2 (the dirty a/lab lines) once per block.
    const double s = (red[0] + red[1]) + (red[2] + red[3]);
    store_f64_agent(&r.partials[blockIdx.x], s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int nb = (int)gridDim.x;
    const int ng = nb < kTicketGroups ? nb : kTicketGroups;
    const int g = blockIdx.x % kTicketGroups;
    const int gsize = (nb - g + kTicketGroups - 1) / kTicketGroups;
    const unsigned prev = __hip_atomic_fetch_add(to_global(&r.ticket[g * kTicketStride]), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    is_last = 0;
    if (prev == (unsigned)gsize - 1) {
      const unsigned top = __hip_atomic_fetch_add(to_global(&r.ticket[kTicketGroups * kTicketStride]), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      is_last = (top == (unsigned)ng - 1) ? 1 : 0;
    }
  }
  __syncthreads();
  if (!is_last) return;
  double acc = 0.0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) acc += load_f64_agent(&r.partials[b]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, kWave);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double total = (red[0] + red[1]) + (red[2] + red[3]);
    for (int g = 0; g <= kTicketGroups; ++g)
      __hip_atomic_store(to_global(&r.ticket[g * kTicketStride]), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r.finish) mill(mk, P.mrkv_hist, r.n_total, total, r.sow, r.hist_A, r.hist_M);
    else store_f64_agent(&r.sow[6], total);
  }
}

// Sharded path: prices from the all-reduced sum in sow[6].
__global__ void period_price_kernel(aiy_market mk, const int* __restrict__ mrkv_hist, long long n_total, double* sow,
                                    double* hist_A, double* hist_M) {
  if (threadIdx.x != 0) return;
  mill(mk, mrkv_hist, n_total, load_f64_agent(&sow[6]), sow, hist_A, hist_M);
}

// No local agents on this rank (sharded path only): publish a zero sum.
__global__ void zero_sum_kernel(double* sow) {
  if (threadIdx.x == 0) store_f64_agent(&sow[6], 0.0);
}

__global__ void set_period_kernel(double* sow, int t) {
  if (threadIdx.x == 0) store_f64_agent(&sow[7], (double)t);
}

static int sim_blocks(long long n) {
  long long nb = (n + (long long)kSimBlock * kAgents - 1) / ((long long)kSimBlock * kAgents);
  return (int)std::max(1LL, std::min<long long>(nb, kSimMaxBlocks));
}

static int32_t ensure_panel_scratch(aiy_handle* h) {
  if (h->partials_cap >= (size_t)kSimMaxBlocks) return AIY_OK;
  AIY_HIP(h, hipMalloc((void**)&h->d_partials, sizeof(double) * kSimMaxBlocks));
  const size_t tk = sizeof(unsigned) * (kTicketGroups + 1) * kTicketStride;
  AIY_HIP(h, hipMalloc((void**)&h->d_ticket, tk));
  AIY_HIP(h, hipMemset(h->d_ticket, 0, tk));
  AIY_HIP(h, hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
  h->partials_cap = kSimMaxBlocks;
  return AIY_OK;
}

// Enqueue one period (1 launch single-rank; 3 launches + 1 collective when sharded).
static int32_t enqueue_period(aiy_handle* h, const PanelDev& P, const PanelRun& r, const aiy_market& mk, int nb,
                              hipStream_t st) {
  if (r.n > 0) {
    hipLaunchKernelGGL(sim_period_kernel, dim3(nb), dim3(kSimBlock), 0, st, P, r, mk);
  } else {
    hipLaunchKernelGGL(zero_sum_kernel, dim3(1), dim3(64), 0, st, r.sow);
  }
  if (!r.finish) {
    ncclResult_t e = ncclAllReduce(r.sow + 6, r.sow + 6, 1, ncclDouble, ncclSum, h->comm, st);
    if (e != ncclSuccess) return fail(h, AIY_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(e));
    hipLaunchKernelGGL(period_price_kernel, dim3(1), dim3(64), 0, st, mk, P.mrkv_hist, r.n_total, r.sow, r.hist_A,
                       r.hist_M);
  }
  return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_sim_periods(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                                   int64_t n_local, int64_t agent_offset, int64_t n_total, double* a, uint8_t* lab,
                                   const double* u, int64_t u_ld, const uint8_t* emp, int64_t emp_ld, uint64_t seed,
                                   uint32_t ge_iter, int32_t t0, int32_t n_periods, double* sow, double* hist_A,
                                   double* hist_M, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!model || !mkt || !sow) return fail(h, AIY_ERR_ARG, "null model/market/sow");
  PanelDev P;
  int32_t rc = panel_dev(h, model, P);
  if (rc) return rc;
  if (n_local < 0 || n_total < 1 || agent_offset < 0) return fail(h, AIY_ERR_ARG, "bad agent counts");
  if (n_local > 0 && (!a || !lab)) return fail(h, AIY_ERR_ARG, "null agent arrays");
  if (u && u_ld < n_local) return fail(h, AIY_ERR_ARG, "u_ld < n_local");
  if (emp && emp_ld < n_local) return fail(h, AIY_ERR_ARG, "emp_ld < n_local");
  if (emp && !P.unemployed) return fail(h, AIY_ERR_ARG, "employment states need tables with the unemployed cells");
  if (t0 < 0 || n_periods < 0 || t0 + (int64_t)n_periods > P.act_T)
    return fail(h, AIY_ERR_ARG, "bad period range [%d, %lld) for act_T=%d", t0, (long long)t0 + n_periods, P.act_T);
  if (ge_iter >= (1u << 12)) return fail(h, AIY_ERR_ARG, "ge_iter too large for the Philox counter");
  if (!h->comm && n_local != n_total) return fail(h, AIY_ERR_ARG, "n_local != n_total without a communicator");
  if (n_periods == 0) return AIY_OK;
  AIY_HIP(h, hipSetDevice(h->device));
  rc = ensure_panel_scratch(h);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  rc = use_stream(h, st);
  if (rc) return rc;
  const int nb = sim_blocks(n_local);
  PanelRun r;
  r.n = n_local; r.offset = agent_offset; r.n_total = n_total; r.a = a; r.lab = lab; r.u = u; r.u_ld = u_ld;
  r.u_t0 = t0; r.emp = emp; r.emp_ld = emp_ld; r.seed = seed; r.ge_iter = ge_iter; r.sow = sow;
  r.partials = h->d_partials; r.ticket = h->d_ticket;
  r.hist_A = hist_A; r.hist_M = hist_M; r.finish = h->comm ? 0 : 1;
  const aiy_market mk = *mkt;

  // the persistent kernel simulates the employed sub-states only (Krusell-Smith mode runs
  // the per-period kernel)
  const bool res_ok = h->use_resident && !emp && n_local >= kResMinAgents && resident_supported(P) &&
                      resident_aligned(a, lab);
  // (its Philox pairs (2k, 2k + 1) must not straddle shards: an even agent_offset)
  if (h->comm && res_ok && (agent_offset & 1) == 0) {
    // sharded: per period ONE launch of the tuned resident kernel (its streaming form for shards
    // beyond LDS, e.g. 12.5M agents per rank at configs[3] on 8 GPUs) leaving the shard's sum in
    // sow[6], the RCCL all-reduce of that double, and the price kernel (mill, AS:1867-1894);
    // the next period's labour draws ride at the end of each launch
    // (period t's launch forms period t - 1's prices from the all-reduced sum itself; the price
    // kernel runs once, after the last all-reduce)
    hipLaunchKernelGGL(set_period_kernel, dim3(1), dim3(64), 0, st, sow, (int)t0);
    for (int p = 0; p < n_periods; ++p) {
      const int fl = kResSharded | (p == 0 ? kResDraw0 : kResPrices | kResKeepTmo) |
                     (p + 1 < n_periods ? kResDrawNext : 0);
      rc = launch_resident(h, P, mk, n_local, a, lab, u ? u + (size_t)p * u_ld : nullptr, u_ld, seed, ge_iter, t0 + p,
                           1, sow, hist_A, hist_M, st, agent_offset, fl, n_total);
      if (rc) return rc;
      const ncclResult_t e = ncclAllReduce(sow + 6, sow + 6, 1, ncclDouble, ncclSum, h->comm, st);
      if (e != ncclSuccess) return fail(h, AIY_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(e));
    }
    hipLaunchKernelGGL(period_price_kernel, dim3(1), dim3(64), 0, st, mk, P.mrkv_hist, (long long)n_total, sow,
                       hist_A, hist_M);
    AIY_CHECK_LAUNCH(h);
    return resident_status(h, st, false);
  }
  if (!h->comm && res_ok) {
    // one persistent launch for the whole block of periods (panel_resident.hip)
    hipLaunchKernelGGL(set_period_kernel, dim3(1), dim3(64), 0, st, sow, (int)t0);
    rc = launch_resident(h, P, mk, n_local, a, lab, u, u_ld, seed, ge_iter, t0, n_periods, sow, hist_A, hist_M, st);
    if (rc) return rc;
    AIY_CHECK_LAUNCH(h);
    return resident_status(h, st);
  }
  hipLaunchKernelGGL(set_period_kernel, dim3(1), dim3(64), 0, st, sow, (int)t0);
  int done = 0;
  if (h->use_graphs && !h->comm && n_periods >= 2 * kGraphPeriods) {
    // Capture kGraphPeriods identical periods on the handle's capture stream, replay.
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    AIY_HIP(h, hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
    for (int p = 0; p < kGraphPeriods; ++p) {
      rc = enqueue_period(h, P, r, mk, nb, h->cap_stream);
      if (rc) {
        hipGraph_t junk;
        (void)hipStreamEndCapture(h->cap_stream, &junk);
        return rc;
      }
    }
    AIY_HIP(h, hipStreamEndCapture(h->cap_stream, &g));
    AIY_HIP(h, hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const int reps = n_periods / kGraphPeriods;
    for (int k = 0; k < reps; ++k) AIY_HIP(h, hipGraphLaunch(ge, st));
    done = reps * kGraphPeriods;
    // the executable graph is released only after its replays ran: this call blocks
    AIY_HIP(h, hipStreamSynchronize(st));
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  for (int p = done; p < n_periods; ++p) {
    rc = enqueue_period(h, P, r, mk, nb, st);
    if (rc) return rc;
  }
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

// Two-step sharded period (caller-side all-reduce between the steps).
extern "C" int32_t aiy_sim_period_local(aiy_handle* h, const aiy_panel_model* model, int64_t n_local,
                                        int64_t agent_offset, double* a, uint8_t* lab, const double* u,
                                        const uint8_t* emp, uint64_t seed, uint32_t ge_iter, int32_t t, double* sow,
                                        aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!sow) return fail(h, AIY_ERR_ARG, "null sow");
  PanelDev P;
  int32_t rc = panel_dev(h, model, P);
  if (rc) return rc;
  if (n_local < 0 || agent_offset < 0) return fail(h, AIY_ERR_ARG, "bad agent counts");
  if (n_local > 0 && (!a || !lab)) return fail(h, AIY_ERR_ARG, "null agent arrays");
  if (t < 0 || t >= P.act_T) return fail(h, AIY_ERR_ARG, "period t=%d outside [0, act_T=%d)", t, P.act_T);
  if (ge_iter >= (1u << 12)) return fail(h, AIY_ERR_ARG, "ge_iter too large for the Philox counter");
  if (emp && !P.unemployed) return fail(h, AIY_ERR_ARG, "employment states need tables with the unemployed cells");
  AIY_HIP(h, hipSetDevice(h->device));
  rc = ensure_panel_scratch(h);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  rc = use_stream(h, st);
  if (rc) return rc;
  PanelRun r;
  r.n = n_local; r.offset = agent_offset; r.n_total = n_local; r.a = a; r.lab = lab; r.u = u; r.u_ld = n_local;
  r.u_t0 = t; r.emp = emp; r.emp_ld = n_local; r.seed = seed; r.ge_iter = ge_iter; r.sow = sow; r.partials = h->d_partials; r.ticket = h->d_ticket;
  r.hist_A = nullptr; r.hist_M = nullptr; r.finish = 0;
  hipLaunchKernelGGL(set_period_kernel, dim3(1), dim3(64), 0, st, sow, (int)t);
  if (h->use_resident && !emp && n_local >= kResMinAgents && resident_supported(P) && resident_aligned(a, lab) &&
      (agent_offset & 1) == 0) {
    // the tuned resident kernel, one period (its labour draws first), the shard's sum in sow[6]
    const aiy_market unused{};
    rc = launch_resident(h, P, unused, n_local, a, lab, u, n_local, seed, ge_iter, t, 1, sow, nullptr, nullptr, st,
                         agent_offset, kResSharded | kResDraw0);
    if (rc) return rc;
    AIY_CHECK_LAUNCH(h);
    return resident_status(h, st, false);
  }
  if (n_local > 0) {
    const aiy_market unused{};
    hipLaunchKernelGGL(sim_period_kernel, dim3(sim_blocks(n_local)), dim3(kSimBlock), 0, st, P, r, unused);
  } else {
    hipLaunchKernelGGL(zero_sum_kernel, dim3(1), dim3(64), 0, st, sow);
  }
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_sim_period_prices(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                                         int64_t n_total, int32_t t, double* sow, double* hist_A, double* hist_M,
                                         aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!mkt || !sow) return fail(h, AIY_ERR_ARG, "null market/sow");
  PanelDev P;
  int32_t rc = panel_dev(h, model, P);
  if (rc) return rc;
  if (n_total < 1) return fail(h, AIY_ERR_ARG, "n_total < 1");
  if (t < 0 || t >= P.act_T) return fail(h, AIY_ERR_ARG, "period t=%d outside [0, act_T=%d)", t, P.act_T);
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  rc = use_stream(h, st);
  if (rc) return rc;
  hipLaunchKernelGGL(period_price_kernel, dim3(1), dim3(64), 0, st, *mkt, P.mrkv_hist, (long long)n_total, sow, hist_A,
                     hist_M);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

// Timing hook for bench.py: n_launch back-to-back launches of the per-period kernel
// alone (agent update + block partials + last-block mill) between two HIP events on
// `stream`; returns the elapsed milliseconds.  Advances the panel state like
// n_launch periods of a history.
extern "C" int32_t aiy_sim_kernel_time(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                                       int64_t n_local, double* a, uint8_t* lab, uint64_t seed, uint32_t ge_iter,
                                       double* sow, int32_t n_launch, float* ms_out, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!model || !mkt || !sow || !a || !lab || !ms_out || n_local < 1 || n_launch < 1)
    return fail(h, AIY_ERR_ARG, "bad arguments");
  PanelDev P;
  int32_t rc = panel_dev(h, model, P);
  if (rc) return rc;
  if (n_launch > P.act_T) return fail(h, AIY_ERR_ARG, "n_launch=%d > act_T=%d", n_launch, P.act_T);
  AIY_HIP(h, hipSetDevice(h->device));
  rc = ensure_panel_scratch(h);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  rc = use_stream(h, st);
  if (rc) return rc;
  PanelRun r;
  r.n = n_local; r.offset = 0; r.n_total = n_local; r.a = a; r.lab = lab; r.u = nullptr; r.u_ld = 0; r.u_t0 = 0;
  r.emp = nullptr; r.emp_ld = 0; r.seed = seed; r.ge_iter = ge_iter; r.sow = sow; r.partials = h->d_partials; r.ticket = h->d_ticket;
  r.hist_A = nullptr; r.hist_M = nullptr; r.finish = 1;
  const int nb = sim_blocks(n_local);
  hipLaunchKernelGGL(set_period_kernel, dim3(1), dim3(64), 0, st, sow, 0);
  AIY_CHECK_LAUNCH(h);
  if (h->use_resident && n_local >= kResMinAgents && resident_supported(P) &&
      resident_aligned(a, lab)) {
    // one persistent launch of n_launch periods
    rc = time_launches(h, st, 1,
                       [&] {
                         (void)launch_resident(h, P, *mkt, n_local, a, lab, nullptr, 0, seed, ge_iter, 0, n_launch, sow,
                                               nullptr, nullptr, st);
                       },
                       ms_out);
    if (rc) return rc;
    return resident_status(h, st);
  }
  return time_launches(h, st, n_launch,
                       [&] { hipLaunchKernelGGL(sim_period_kernel, dim3(nb), dim3(kSimBlock), 0, st, P, r, *mkt); },
                       ms_out);
}

extern "C" int32_t aiy_set_option(aiy_handle* h, int32_t option, int64_t value) {
  if (!h) return AIY_ERR_ARG;
  switch (option) {
    case AIY_OPT_USE_GRAPHS: h->use_graphs = value != 0; return AIY_OK;
    case AIY_OPT_RESIDENT:
      h->use_resident = value != 0;
      return AIY_OK;
    case AIY_OPT_RESIDENT_SHAPE:
      if (value < 0 || value > 2) return fail(h, AIY_ERR_ARG, "AIY_OPT_RESIDENT_SHAPE must be 0, 1 or 2");
      h->res_shape = (int)value;
      return AIY_OK;
    case AIY_OPT_HIST_FUSED: h->hist_fused = value != 0; return AIY_OK;
    case AIY_OPT_RESIDENT_STREAM: h->res_stream = value != 0; return AIY_OK;
    case AIY_OPT_HIST_RESIDENT: h->hist_resident = value != 0; return AIY_OK;
    case AIY_OPT_HIST_ACCEL:
      if (value < 0 || value > (1 << 20)) return fail(h, AIY_ERR_ARG, "AIY_OPT_HIST_ACCEL must be >= 0");
      h->hist_accel = (int)value;
      return AIY_OK;
    case AIY_OPT_HIST_KRYLOV: h->hist_krylov = value != 0; return AIY_OK;
    case AIY_OPT_HIST_PULL: h->hist_pull = value != 0; return AIY_OK;
    case AIY_OPT_RESIDENT_SHAPE_STREAM:
      if (value < -1 || value > 2) return fail(h, AIY_ERR_ARG, "AIY_OPT_RESIDENT_SHAPE_STREAM must be -1, 0, 1 or 2");
      h->res_shape_stream = (int)value;
      return AIY_OK;
    case AIY_OPT_GE_LOOSE_HIST:
      if (value < 6 || value > 14) return fail(h, AIY_ERR_ARG, "AIY_OPT_GE_LOOSE_HIST must be in [6, 14]");
      h->ge_loose_hist = (int)value;
      return AIY_OK;
    case AIY_OPT_GE_RESIDENT: h->ge_resident = value != 0; return AIY_OK;
    case AIY_OPT_GE_LOGSEC:
      if (value < 0 || value > 2) return fail(h, AIY_ERR_ARG, "AIY_OPT_GE_LOGSEC must be 0, 1 or 2");
      h->ge_logsec = (int)value;
      return AIY_OK;
    case AIY_OPT_GE_EXTRAP_PERIOD:
      if (value < 4 || value > 1024) return fail(h, AIY_ERR_ARG, "AIY_OPT_GE_EXTRAP_PERIOD must be in [4, 1024]");
      h->ge_extrap_period = (int)value;
      return AIY_OK;
    case AIY_OPT_GE_ANDERSON:
      if (value != 0 && (value < 5 || value > 1024))
        return fail(h, AIY_ERR_ARG, "AIY_OPT_GE_ANDERSON must be 0 or in [5, 1024]");
      h->ge_anderson = (int)value;
      return AIY_OK;
    case AIY_OPT_GE_REBALANCE:
      if (value < 0 || value > 100) return fail(h, AIY_ERR_ARG, "AIY_OPT_GE_REBALANCE must be in [0, 100]");
      h->ge_rebalance = (int)value;
      return AIY_OK;
    case AIY_OPT_CU_LIMIT:
      if (value < 0 || value > 65536) return fail(h, AIY_ERR_ARG, "AIY_OPT_CU_LIMIT must be in [0, 65536]");
      h->cu_limit = (int)value;
      return AIY_OK;
    case AIY_OPT_HIST_CLUSTER:
      if (value < 0 || value > 128) return fail(h, AIY_ERR_ARG, "AIY_OPT_HIST_CLUSTER must be in [0, 128]");
      h->hist_cluster_cap = (int)value;
      return AIY_OK;
    default: return fail(h, AIY_ERR_ARG, "unknown option %d", option);
  }
}

// Current value of a handle option (the values aiy_set_option takes), so callers can save
// and restore what they change.
extern "C" int32_t aiy_get_option(aiy_handle* h, int32_t option, int64_t* value) {
  if (!h || !value) return AIY_ERR_ARG;
  switch (option) {
    case AIY_OPT_USE_GRAPHS: *value = h->use_graphs; return AIY_OK;
    case AIY_OPT_RESIDENT: *value = h->use_resident; return AIY_OK;
    case AIY_OPT_RESIDENT_SHAPE: *value = h->res_shape; return AIY_OK;
    case AIY_OPT_HIST_FUSED: *value = h->hist_fused; return AIY_OK;
    case AIY_OPT_RESIDENT_STREAM: *value = h->res_stream; return AIY_OK;
    case AIY_OPT_HIST_RESIDENT: *value = h->hist_resident; return AIY_OK;
    case AIY_OPT_HIST_ACCEL: *value = h->hist_accel; return AIY_OK;
    case AIY_OPT_HIST_KRYLOV: *value = h->hist_krylov; return AIY_OK;
    case AIY_OPT_HIST_PULL: *value = h->hist_pull; return AIY_OK;
    case AIY_OPT_RESIDENT_SHAPE_STREAM: *value = h->res_shape_stream; return AIY_OK;
    case AIY_OPT_GE_LOOSE_HIST: *value = h->ge_loose_hist; return AIY_OK;
    case AIY_OPT_GE_RESIDENT: *value = h->ge_resident; return AIY_OK;
    case AIY_OPT_GE_LOGSEC: *value = h->ge_logsec; return AIY_OK;
    case AIY_OPT_GE_EXTRAP_PERIOD: *value = h->ge_extrap_period; return AIY_OK;
    case AIY_OPT_GE_ANDERSON: *value = h->ge_anderson; return AIY_OK;
    case AIY_OPT_GE_REBALANCE: *value = h->ge_rebalance; return AIY_OK;
    case AIY_OPT_CU_LIMIT: *value = h->cu_limit; return AIY_OK;
    case AIY_OPT_HIST_CLUSTER: *value = h->hist_cluster_cap; return AIY_OK;
    default: return fail(h, AIY_ERR_ARG, "unknown option %d", option);
  }
}
