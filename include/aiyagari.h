/*
 * libaiyagari -- C ABI of the MI355X (gfx950) Aiyagari household block.
 *
 * Drop-in boundary for the hot path of Dostenlinus/Aiyagari-HARK:
 *   EGM backward step -> cross-sectional step (panel / histogram) -> GE loop.
 * Every entry point cites the reference interface it replaces
 * (AS = /root/reference/Aiyagari_Support.py, AH = /root/reference/Aiyagari-HARK.py,
 * [HARK] = econ-ark 0.12 library routine called from there).
 *
 * Conventions
 *  - All array arguments are DEVICE pointers owned by the caller (the Python host
 *    allocates them as PyTorch-ROCm tensors); the library allocates only inside a
 *    handle (small scratch).  Layouts are C-contiguous, float64 unless stated.
 *  - Every call returns 0 (AIY_OK) or a negative error code; aiy_last_error() gives
 *    the message.  Argument errors are detected on the host before any launch.
 *  - `stream` is a hipStream_t (NULL = the default stream).  Calls that only enqueue
 *    work are asynchronous; calls documented as BLOCKING synchronise `stream`.
 *  - One handle per (process, device); a handle is not re-entrant across threads.
 *  - Streams: calls that use the handle's scratch (EGM convergence slots and search
 *    index, panel partial sums, histogram slots, statistics scratch) may be given any
 *    stream; when a call arrives on a different stream than the previous one, the
 *    library makes the new stream wait for the old one (event hand-off), so work on two
 *    streams through one handle is serialised, never interleaved on the scratch.
 *
 * Table layout for consumption policies (the (x_list, y_list) of the reference's
 * 28 x 15 LinearInterp objects, AS:1509-1516):
 *    m[c][s][k][j], c[c][s][k][j]   c < n_cal, s < S, k < n_M, j <= n_a
 * where node j = 0 is the prepended (1e-7, 1e-7) point (AS:1503-1504).
 */
#ifndef AIYAGARI_H
#define AIYAGARI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIY_OK 0
#define AIY_ERR_ARG (-1)
#define AIY_ERR_HIP (-2)
#define AIY_ERR_STATE (-3)
#define AIY_ERR_UNSUPPORTED (-4)
#define AIY_ERR_COMM (-5)

#define AIY_MAX_STATES 64   /* S (discrete states) supported by the EGM kernel */

typedef struct aiy_handle aiy_handle;
typedef void* aiy_stream; /* hipStream_t */

/* Shapes of one batched EGM problem. */
typedef struct {
  int32_t n_cal; /* calibrations solved together (Table II batching)                 */
  int32_t S;     /* discrete states: 4 * LaborStatesNo (KS form) or N_l (stationary)  */
  int32_t n_M;   /* aggregate-M nodes (15 in the reference, AS:753-754); 1 = stationary */
  int32_t n_a;   /* exogenous end-of-period asset nodes (aGrid, AS:880)               */
} aiy_egm_dims;

/* Per-calibration inputs of solve_Aiyagari (AS:1423-1434) after precompute_arrays
 * (AS:906-1037) with the 28x-redundant current-state axis removed:
 *   mNextArray[a,k,s,s'] = R_next[k,s'] * a_grid[a] + W_next[k,s'] * lab[s']
 *   MnextArray[a,k,s,s'] = M_next[k,s'],  RnextArray[a,k,s,s'] = R_next[k,s'],
 *   ProbArray[a,k,s,s']  = P[s,s'].                                                  */
typedef struct {
  const double* a_grid; /* [n_cal][n_a]                                           */
  const double* M_grid; /* [n_cal][n_M]   Mgrid = MSS * MgridBase (AS:837-839)     */
  const double* P;      /* [n_cal][S][S]  MrkvIndArray (AS:1780)                    */
  const double* R_next; /* [n_cal][n_M][S]                                          */
  const double* W_next; /* [n_cal][n_M][S]                                          */
  const double* M_next; /* [n_cal][n_M][S] (ignored when n_M == 1)                  */
  const double* lab;    /* [n_cal][S]     LSStates[s' / 4] (AS:985, 990-1018)       */
  const double* beta;   /* [n_cal]        DiscFac                                  */
  const double* crra;   /* [n_cal]        CRRA                                     */
} aiy_egm_inputs;

/* Library version (major * 10000 + minor * 100 + patch). */
int32_t aiy_version(void);

/* Create / destroy a handle bound to HIP device `device`. */
int32_t aiy_create(int32_t device, aiy_handle** out);
int32_t aiy_destroy(aiy_handle* h);
const char* aiy_last_error(const aiy_handle* h);

/* One backward EGM step == one call of solve_Aiyagari (AS:1423-1520) for every
 * calibration of the batch.  m_next/c_next == NULL means the terminal guess
 * IdentityFunction (AS:892-904).  Asynchronous. */
int32_t aiy_egm_step(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in,
                     const double* m_next, const double* c_next, double* m_out, double* c_out,
                     aiy_stream stream);

/* Infinite-horizon solve == [HARK] solve_agent with cycles = 0 (AH:237): cold start
 * from the terminal guess (pre_solve, AS:806-808), iterate solve_Aiyagari until the
 * [HARK] MetricObject distance (max |dm|, |dc| over all tables) is <= tol, or
 * max_cycles + 1 cycles ran (HARK's 5000-cycle escape clause).  Each calibration
 * stops on its own cycle; converged calibrations are skipped on device.
 *   work_m/work_c: [2][n_cal][S][n_M][n_a+1] ping-pong scratch (caller-owned)
 *   m_out/c_out:   [n_cal][S][n_M][n_a+1] converged tables
 *   cycles_out/dist_out: HOST arrays [n_cal] (completed cycles, final distance)
 * BLOCKING (polls convergence every `chunk` cycles; chunk <= 0 selects 32). */
int32_t aiy_egm_solve(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in, double tol,
                      int32_t max_cycles, int32_t chunk, double* work_m, double* work_c,
                      double* m_out, double* c_out, int32_t* cycles_out, double* dist_out,
                      aiy_stream stream);

/* The same loop warm-started from caller tables m_init/c_init [n_cal][S][n_M][n_a+1]
 * instead of the terminal guess (build-defined: the stationary GE search E1 re-solves the
 * household at a nearby r every step; the KS-form GE keeps HARK's cold start, Q12).
 * Cycle 1 steps from the given tables.  BLOCKING. */
int32_t aiy_egm_solve_from(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in, double tol,
                           int32_t max_cycles, int32_t chunk, const double* m_init, const double* c_init,
                           double* work_m, double* work_c, double* m_out, double* c_out, int32_t* cycles_out,
                           double* dist_out, aiy_stream stream);

/* Measurement hook (bench.py): n_launch launches of the EGM cycle kernel alone from
 * (m_next, c_next) (search index built once, outside the timed region), each bracketed
 * by its own pair of HIP events on `stream`; *ms_out = sum of the per-launch elapsed
 * milliseconds (gaps between launches excluded).  BLOCKING. */
int32_t aiy_egm_kernel_time(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in,
                            const double* m_next, const double* c_next, double* m_out, double* c_out,
                            int32_t n_launch, float* ms_out, aiy_stream stream);

/* cFunc[state](m, M) for a batch of queries (interop for .solution[0].cFunc and the
 * notebook's plots, AH:271-275): HARK LinearInterpOnInterp1D semantics.
 *   tables [S][n_M][n_a+1]; state/m/M [n]; c_out [n].  Asynchronous. */
int32_t aiy_policy_eval(aiy_handle* h, int32_t S, int32_t n_M, int32_t n_a, const double* m_tab,
                        const double* c_tab, const double* M_grid, const int32_t* state,
                        const double* m, const double* M, int64_t n, double* c_out, aiy_stream stream);

/* Search index of policy rows (accelerates every HARK LinearInterp bracket search
 * without changing its result): for each of n_rows rows x[0..n1) (the m nodes of one
 * LinearInterp, x[0] > 0, sorted) build a log-bucket table of
 * aiy_index_ints_per_row() int32 so that lower_bound(x[:-1], q) is found by a search
 * over a few nodes.  Asynchronous. */
int32_t aiy_index_ints_per_row(void);
int32_t aiy_build_index(aiy_handle* h, int64_t n_rows, int32_t n1, const double* x, int32_t* index,
                        aiy_stream stream);

/* ----------------------------- panel (rows B1-B6, C2) ----------------------------- */

/* Market constants used by calc_R_and_W (AS:1839-1894). */
typedef struct {
  double cap_share;  /* CapShare */
  double depr_fac;   /* DeprFac */
  double prod[2];    /* ProdB, ProdG */
  double agg_L[2];   /* (1 - UrateB) LbrInd, (1 - UrateG) LbrInd */
} aiy_market;

/* Household panel model for one calibration (policy fixed during a history). */
typedef struct {
  int32_t S, n_M, n_a, n_lab; /* S = 4 n_lab (KS form)                                       */
  const void* tables;       /* merged policy tables of the converged policy
                               (AiyagariType.solution[0]), from aiy_panel_build              */
  const double* M_grid;     /* [n_M]                                                       */
  const double* lab_level;  /* [n_lab] LSStates (AS:1265)                                  */
  const double* lab_cdf;    /* [n_lab][n_lab] cumsum(P[l]) / last (np.random.choice)        */
  const int32_t* mrkv_hist; /* [act_T] MrkvNow_hist (AS:1793-1805)                          */
  int32_t act_T;            /* length of mrkv_hist and of the hist_A / hist_M buffers: every
                               call is checked to simulate periods t0 + n_periods <= act_T   */
  int32_t unemployed;       /* != 0: tables built with the unemployed sub-states too
                               (Krusell-Smith mode, UrateB/UrateG > 0)                       */
} aiy_panel_model;

/* Panel policy tables (get_controls, AS:1326-1408).  Each period an agent of labour
 * state l and employment e evaluates LinearInterpOnInterp1D = (1 - alpha) f_{j-1}(m) +
 * alpha f_j(m) of its sub-state s = 4 l + 2 Mrkv + e (e = 1 only unless `unemployed`).
 * For every (l, Mrkv, e, M interval j) the
 * two rows' nodes are merged into one sorted list; on each merged segment both rows'
 * brackets are fixed, so one 64-byte record holds both, and a bracket index over the
 * merged nodes (log buckets, one 64-bit entry each) finds the record with no search
 * in the common case.  HARK's arithmetic is unchanged (results bit-identical to
 * searching the two rows).
 *   aiy_panel_table_bytes: bytes of ONE calibration's tables (-1: unsupported sizes)
 *   aiy_panel_build: m_pol, c_pol [n_cal][S][n_M][n_a+1] (device) -> tables
 *                    [n_cal][aiy_panel_table_bytes] (device).  Asynchronous. */
int64_t aiy_panel_table_bytes(int32_t n_lab, int32_t n_M, int32_t n_a, int32_t unemployed);
int32_t aiy_panel_build(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_M, int32_t n_a, int32_t n_lab,
                        int32_t unemployed, const double* m_pol, const double* c_pol, void* tables,
                        aiy_stream stream);

/* Device-resident market state ("sow_state", AS:1585), 8 doubles:
 *   [0] Mnow [1] Aprev [2] Mrkv [3] Rnow [4] Wnow [5] Urate [6] sum(a) [7] period index t */
#define AIY_SOW_DOUBLES 8

/* Simulate periods t0 .. t0 + n_periods - 1 of Market.make_history (AH:249 ->
 * [HARK] Market.make_history): for each period one [HARK] sim_one_period of every
 * local agent (get_shocks AS:1217-1256, get_states AS:1259-1283, get_controls
 * AS:1286-1409, get_poststates AS:1411-1415), then mill/calc_R_and_W (AS:1839-1894)
 * on the mean of `a` over all n_total agents of all ranks, writing sow and
 * hist_A[t] = Aprev, hist_M[t] = Mnow (the track_vars of AS:1587).  sow[7] holds the
 * period index on device.
 *   a [n_local] (in: a_prev, out: a_now), lab [n_local] uint8 labour state
 *   u: NULL -> on-device Philox4x32-10 (counter (ge_iter<<20 | t, idx, 0), key seed),
 *      else host-supplied uniforms [n_periods][u_ld] starting at period t0 (parity
 *      with np.random.choice)
 *   emp: NULL -> everyone employed (UrateB = UrateG = 0), else the employment states
 *      (uint8 0/1, device) [n_periods][emp_ld] from period t0 -- this period's EmpNow of
 *      get_shocks (AS:1222-1240; exact-count permutations drawn with the agent RNG by the
 *      caller).  Needs tables with the unemployed cells (model->unemployed).
 *   agent_offset: global index of local agent 0 (Philox counter, sharding)
 * With a communicator bound (aiy_comm_init) the per-period sum of a is all-reduced
 * over RCCL before the prices are formed; otherwise n_local must equal n_total (or use
 * the two-step form below with a caller-side all-reduce).
 * Asynchronous, except that the persistent path (AIY_OPT_RESIDENT) and hipGraph replay
 * (single rank, n_periods >= 128) return after the periods completed. */
int32_t aiy_sim_periods(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                        int64_t n_local, int64_t agent_offset, int64_t n_total, double* a,
                        uint8_t* lab, const double* u, int64_t u_ld, const uint8_t* emp, int64_t emp_ld,
                        uint64_t seed, uint32_t ge_iter, int32_t t0, int32_t n_periods, double* sow,
                        double* hist_A, double* hist_M, aiy_stream stream);

/* One sharded period in two steps with the all-reduce left to the caller (any backend:
 * torch.distributed over RCCL or gloo, MPI, ...): the agent-sharded form of
 * np.mean(np.array(aNow)) (AS:1868).
 *   aiy_sim_period_local:  period t of the n_local agents (get_shocks .. get_poststates,
 *                          AS:1217-1415); leaves their sum of a in sow[6] (device).
 *                          u: NULL (Philox by global index) or n_local host uniforms of
 *                          period t; emp: NULL or the n_local employment states of t.
 *   -- caller: sow[6] <- sum over ranks of sow[6] --
 *   aiy_sim_period_prices: mill / calc_R_and_W (AS:1839-1894) on sow[6] / n_total; writes
 *                          sow, hist_A[t], hist_M[t] and advances sow[7] to t + 1.
 * Both asynchronous on `stream`, except that aiy_sim_period_local returns after the period
 * completed when it runs the resident kernel (>= 65536 local agents, even agent_offset, no
 * employment states).
 * Sharded aiy_sim_periods (a communicator bound) runs per period the same resident launch
 * (even agent_offset; parallel.shard_range splits on agent pairs), ncclAllReduce of sow[6]
 * and the price kernel, and returns after the periods completed. */
int32_t aiy_sim_period_local(aiy_handle* h, const aiy_panel_model* model, int64_t n_local,
                             int64_t agent_offset, double* a, uint8_t* lab, const double* u,
                             const uint8_t* emp, uint64_t seed, uint32_t ge_iter, int32_t t, double* sow,
                             aiy_stream stream);
int32_t aiy_sim_period_prices(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                              int64_t n_total, int32_t t, double* sow, double* hist_A, double* hist_M,
                              aiy_stream stream);

/* The reference's per-period simulation hooks one at a time, for a driver that steps
 * [HARK] Market.make_history period by period (sow -> cultivate -> reap -> mill -> store)
 * through AgentType.sim_one_period's get_shocks / get_states / get_controls /
 * get_poststates (AiyagariType, Aiyagari_Support.py:1217-1415).  One small launch each,
 * all asynchronous on `stream`; the fused aiy_sim_periods computes the same thing per
 * period in one pass.  All arrays are DEVICE arrays of the n agents unless noted.
 *   aiy_get_shocks:     lab <- inverse-CDF draw from lab_cdf[lab] (AS:1244-1256):
 *                       u = n uniforms (device) or NULL -> Philox counter
 *                       ((ge_iter << 20) | t, (agent_offset + i) / 2) as aiy_sim_periods
 *   aiy_get_states:     m = Rnow * a_prev + Wnow * lab_level[lab] * emp (AS:1276-1283);
 *                       emp NULL means everyone employed
 *   aiy_get_controls:   c = cFunc[4 lab + 2 Mrkv + emp](m, Mnow) on the RAW policy tables
 *                       m_tab / c_tab [S][n_M][n_a + 1] of aiy_egm_solve (HARK
 *                       LinearInterpOnInterp1D, AS:1295-1408); M_grid_host: HOST [n_M]
 *   aiy_get_poststates: a = m - c (AS:1415)
 *   aiy_sum:            out[0] (device) = sum of x in a fixed order (the mill's
 *                       np.mean(aNow) numerator, AS:1868) */
int32_t aiy_get_shocks(aiy_handle* h, int32_t n_lab, const double* lab_cdf, int64_t n, int64_t agent_offset,
                       uint8_t* lab, const double* u, uint64_t seed, uint32_t ge_iter, int32_t t,
                       aiy_stream stream);
int32_t aiy_get_states(aiy_handle* h, const double* lab_level, int64_t n, double Rnow, double Wnow,
                       const double* a_prev, const uint8_t* lab, const uint8_t* emp, double* m_out,
                       aiy_stream stream);
int32_t aiy_get_controls(aiy_handle* h, int32_t S, int32_t n_M, int32_t n_a, const double* m_tab,
                         const double* c_tab, const double* M_grid_host, int32_t Mrkv, double Mnow, int64_t n,
                         const double* m, const uint8_t* lab, const uint8_t* emp, double* c_out,
                         aiy_stream stream);
int32_t aiy_get_poststates(aiy_handle* h, int64_t n, const double* m, const double* c, double* a_out,
                           aiy_stream stream);
int32_t aiy_sum(aiy_handle* h, const double* x, int64_t n, double* out, aiy_stream stream);

/* Measurement hook (bench.py): n_launch periods of the panel kernel (single rank,
 * Philox shocks) -- n_launch per-period launches, each bracketed by its own pair of HIP
 * events on `stream`, or with AIY_OPT_RESIDENT one persistent launch of n_launch periods
 * between two events; *ms_out = kernel milliseconds for the n_launch periods.  Simulates
 * periods 0 .. n_launch - 1 (mrkv_hist must hold n_launch entries) and advances a/lab/sow.
 * BLOCKING. */
int32_t aiy_sim_kernel_time(aiy_handle* h, const aiy_panel_model* model, const aiy_market* mkt,
                            int64_t n_local, double* a, uint8_t* lab, uint64_t seed, uint32_t ge_iter,
                            double* sow, int32_t n_launch, float* ms_out, aiy_stream stream);

/* Persistent-panel launch statistics (measurement hook): kernel milliseconds summed over
 * the single-rank resident launches since the last reset (each bracketed by HIP events
 * on its stream), the number of launches and the periods they simulated.  reset != 0
 * zeroes the counters after reading them.  Host-only. */
int32_t aiy_panel_launch_stats(aiy_handle* h, double* ms_sum, int64_t* launches, int64_t* periods,
                               int32_t reset);

/* Batched small-population panel (Table II in the reference's Krusell-Smith mode: 350-700
 * agents per calibration, act_T = 11 000; AH:217-249).  One workgroup owns one
 * calibration: agents stay in registers for all n_periods, the per-period mean of `a`
 * is a workgroup reduction and calc_R_and_W runs on lane 0 (no grid synchronisation),
 * so a whole history is ONE launch.  Same per-period semantics as aiy_sim_periods.
 * All calibrations share (S, n_M, n_a, n_lab); arrays are stacked over calibrations. */
typedef struct {
  int32_t n_cal, S, n_M, n_a, n_lab;
  const void* tables;       /* [n_cal][aiy_panel_table_bytes], aiy_panel_build */
  const double* M_grid;     /* [n_cal][n_M] */
  const double* lab_level;  /* [n_cal][n_lab] */
  const double* lab_cdf;    /* [n_cal][n_lab][n_lab] */
  const int32_t* mrkv_hist; /* [n_cal][act_T] */
  int32_t unemployed;       /* != 0: tables with the unemployed sub-states (aiy_panel_build) */
} aiy_panel_batch;

/* Largest per-calibration population aiy_sim_block_periods accepts. */
int32_t aiy_sim_block_max_agents(void);

/* Periods t0 .. t0 + n_periods - 1 of every calibration's history.
 *   markets, seeds: HOST arrays [n_cal]
 *   a [n_cal][n_agents], lab [n_cal][n_agents] uint8 (device, in/out)
 *   u: NULL -> Philox (counter (ge_iter<<20 | t, idx/2, 0), key seeds[c]), else host
 *      uniforms [n_cal][n_periods][n_agents]
 *   emp: NULL (everyone employed) or employment states [n_cal][n_periods][n_agents]
 *      (uint8, device; as aiy_sim_periods)
 *   sow [n_cal][AIY_SOW_DOUBLES] (device, in/out); hist_A/hist_M [n_cal][act_T] or NULL.
 * Asynchronous (the call waits for earlier work on `stream` before it refills its
 * pinned staging buffer). */
int32_t aiy_sim_block_periods(aiy_handle* h, const aiy_panel_batch* model, const aiy_market* markets,
                              int64_t n_agents, double* a, uint8_t* lab, const double* u,
                              const uint8_t* emp, const uint64_t* seeds, uint32_t ge_iter, int32_t t0, int32_t n_periods,
                              int32_t act_T, double* sow, double* hist_A, double* hist_M,
                              aiy_stream stream);

/* Handle options. */
#define AIY_OPT_USE_GRAPHS 1 /* value != 0: replay panel periods from a captured hipGraph */
#define AIY_OPT_RESIDENT 2   /* value != 0 (default): single-rank panels of >= 65536 agents run
                                 a block of periods as ONE persistent launch (agents resident in
                                 LDS, in-kernel exchange of partial sums per period); 0: one launch
                                 per period */
#define AIY_OPT_HIST_FUSED 4 /* value != 0: aiy_hist_solve runs one fused push+mix launch per iteration
                              when every lottery row is monotone; 0 (default): the push/mix pair.  The
                              fused step moves 28 B per point but its borrowing-constraint tile pulls
                              thousands of sources serially: measured slower at Table II sizes */
#define AIY_OPT_RESIDENT_SHAPE 3 /* persistent panel workgroup: 0 (default) 512 threads x 8 agents
                                    per lane per pass, quad-cooperative record loads; 1: 1024
                                    threads x 4, quad-cooperative; 2: 512 x 8, per-lane record
                                    loads (results identical) */
#define AIY_OPT_RESIDENT_STREAM 5 /* value != 0: the persistent panel streams agents from HBM even
                                     when the workgroup slice would fit in LDS (the path panels of
                                     more than ~4M agents take; for tests and measurement) */
#define AIY_OPT_HIST_RESIDENT 6  /* value != 0 (default): aiy_hist_solve runs the whole distribution
                                    iteration in ONE device-resident launch (a cluster of workgroups
                                    per calibration, in-kernel barriers); 0: the push/mix launch pair */
#define AIY_OPT_HIST_CLUSTER 7   /* maximum workgroups per calibration cluster of the resident
                                    histogram (0: default 32; the minimum the grid size needs wins) */
#define AIY_OPT_HIST_ACCEL 8     /* value E > 0: the resident histogram extrapolates every E iterations
                                    along the last change when two consecutive estimates of its
                                    contraction ratio agree (Aitken; same fixed point, fewer
                                    iterations, counts differ from the plain iteration); 0 (default):
                                    the plain iteration of oracle/stationary.py */
#define AIY_OPT_HIST_KRYLOV 9     /* value != 0: the resident histogram solves (I - T) mass = 0 by
                                    BiCGSTAB from the given mass (hist_krylov.hip; stops at a mass
                                    T x with max|T x - x| < tol, the plain iteration's rule; counts
                                    are matvecs); takes precedence over AIY_OPT_HIST_ACCEL */
#define AIY_OPT_GE_RESIDENT 10    /* value != 0: aiy_ge_stationary runs the whole search of
                                    every calibration in ONE device-resident launch (each
                                    calibration's cluster: EGM cycles, lottery, BiCGSTAB, K_s and the
                                    root search on device, ge_resident.hip) when accel < 0, S <= 8
                                    and every cluster fits the device at once; else the host loop.
                                    A new handle starts at 0 (the host loop); the Python wrapper
                                    (stationary.solve_table2) sets it by default */
#define AIY_OPT_CU_LIMIT 11       /* compute units the resident launches of this handle may fill
                                    (0: the device's; several processes sharing one GPU: a share) */
#define AIY_OPT_GE_REBALANCE 12   /* value q in [1, 100] (default 55): the device-resident GE search
                                    stops every cluster at an evaluation boundary once q % of a
                                    launch's calibrations have finished and relaunches the rest on
                                    the freed compute units (larger clusters); 0: one launch */
#define AIY_OPT_GE_EXTRAP_PERIOD 13 /* device-resident GE search: EGM cycles between the geometric
                                    extrapolation checks (4 .. 1024; default 32) when
                                    AIY_OPT_GE_ANDERSON is 0 */
#define AIY_OPT_GE_ANDERSON 23     /* device-resident GE search with egm_extrapolate: every p-th EGM cycle
                                    (p in [5, 1024], default 12) the household iterate moves to the
                                    type-II Anderson combination of the last 4 plain cycles (m = 3),
                                    instead of the geometric extrapolation; the same fixed point and
                                    HARK stopping rule (sup-norm change <= tol); 0: off */
#define AIY_OPT_GE_LOGSEC 14      /* 1: with loose bracketing, while only K_s < K_d has been seen
                                    the next point is a secant of log(K_s / K_d) against
                                    log(1/beta - 1 - r) through the last two points (aimed 20 %
                                    past the predicted root, the distance to 1/beta - 1 cut by
                                    2 .. 16) instead of a bisection step, and Brent runs in those
                                    coordinates; 2 (default): also a unit-slope step from a single
                                    point; 0: bisection bracketing, Brent in r */
#define AIY_OPT_HIST_PULL 15       /* value != 0: the BiCGSTAB distribution solves of S <= 8 states
                                    (the resident GE search and aiy_hist_solve) form every matvec by
                                    PULLING each destination's lottery sources in ascending order
                                    (hist_pull.h's inverse lottery) instead of LDS-atomic pushes:
                                    deterministic run to run; 0: the push form.  S > 8 always pulls */
#define AIY_OPT_GE_LOOSE_HIST 17   /* value v in [6, 14] (default 8): the loose-bracketing evaluations'
                                    distribution tolerance is 10^-v (their sign needs |K_s - K_d| >= 5 %
                                    of K_d).  Brent's evaluations run at an adaptive tolerance
                                    between hist_tol and this one (ge_search.h ge_adapt_htol; an
                                    evaluation whose |K_s - K_d| is not well above its error is
                                    redone at hist_tol), and the evaluation the search ends on is
                                    always re-solved at hist_tol before Ks_out is reported */
#define AIY_OPT_RESIDENT_SHAPE_STREAM 18 /* workgroup shape (AIY_OPT_RESIDENT_SHAPE's values) of the resident
                                    panel's HBM-streaming form (agents beyond LDS, e.g. configs[3]);
                                    default 1 (1024 threads x 4 agents); -1: AIY_OPT_RESIDENT_SHAPE */
/* (options 16, 19, 20, 21 and 22 -- fused panel draws, the 25-state resident search, the
   loader-ring panel, loose Brent evaluations, the on-chip S > 8 solve -- were measured slower
   than the defaults and removed in round 5; setting them returns AIY_ERR_ARG) */
int32_t aiy_set_option(aiy_handle* h, int32_t option, int64_t value);
/* The current value of an option (so a caller can save and restore what it changes). */
int32_t aiy_get_option(aiy_handle* h, int32_t option, int64_t* value);

/* -------------------------- RCCL binding (multi-GPU, §8e) -------------------------- */
/* 128-byte ncclUniqueId created by rank 0 and broadcast by the host. */
int32_t aiy_comm_unique_id(void* out128);
int32_t aiy_comm_init(aiy_handle* h, const void* unique_id128, int32_t nranks, int32_t rank);
/* Bind a communicator the caller owns (an ncclComm_t, e.g. torch.distributed's RCCL group:
 * ProcessGroupNCCL._comm_ptr()) instead of creating one: one communicator per device in the
 * process.  It must be on the handle's device; aiy_comm_destroy then only unbinds it. */
int32_t aiy_comm_bind(aiy_handle* h, void* comm);
/* Unbind the communicator (destroying it when aiy_comm_init created it). */
int32_t aiy_comm_destroy(aiy_handle* h);
/* Sum-all-reduce of n doubles in place over the bound communicator (asynchronous). */
int32_t aiy_allreduce_sum(aiy_handle* h, double* buf, int64_t n, aiy_stream stream);

/* --------------------- stationary extensions (E1 / E2, no reference) --------------------- */

/* Young-lottery transition of each calibration's stationary household (build-defined
 * row E2): for state s and grid node j, m = R a_j + w lab[s], a' = m - c_s(m) (HARK
 * LinearInterp on the [S][n_a+1] tables), lottery onto a_grid:
 * lo[c][s][j] (int32) and wlo (weight on lo).  Asynchronous. */
int32_t aiy_hist_lottery(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_a, const double* m_tab,
                         const double* c_tab, const double* a_grid, const double* R, const double* w,
                         const double* lab, int32_t* lo, double* wlo, aiy_stream stream);

/* Iterate mass'[s', .] = sum_s P[s, s'] * lottery_push(mass[s, .]) until the sup-norm
 * change is < tol (per calibration) or max_iter.  mass [n_cal][S][n_a] in/out,
 * work [2][n_cal][S][n_a] scratch.  K_out (HOST [n_cal]) = sum mass * a_grid;
 * iters_out (HOST [n_cal]).  BLOCKING. */
int32_t aiy_hist_solve(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_a, const int32_t* lo,
                       const double* wlo, const double* P, const double* a_grid, double tol,
                       int32_t max_iter, int32_t chunk, double* mass, double* work, double* K_out,
                       int32_t* iters_out, aiy_stream stream);

/* ------------- stationary general equilibrium (E1 over E2, SURVEY §8b aiy_ge_bisect) ------------- */

/* A batch of stationary Aiyagari households: the EGM inputs of aiy_egm_solve with one
 * aggregate node (device arrays) and the firm of calc_R_and_W (AS:1886-1890, L = 1). */
typedef struct {
  int32_t n_cal, S, n_a;
  const double* a_grid;  /* [n_cal][n_a]  device                                  */
  const double* P;       /* [n_cal][S][S] device: income Markov chain               */
  const double* lab;     /* [n_cal][S]    device: labour levels (simple-mean norm.) */
  const double* beta;    /* [n_cal]       device: DiscFac                           */
  const double* crra;    /* [n_cal]       device: CRRA                              */
  const double* alpha;   /* [n_cal]       HOST: CapShare                            */
  const double* delta;   /* [n_cal]       HOST: DeprFac                             */
  const double* disc;    /* [n_cal]       HOST: DiscFac (bracket end 1 / beta - 1)  */
} aiy_stationary_model;

typedef struct {
  int32_t method;        /* 0: bisection on K_s(r) - K_d(r) (oracle ge_bisect); 1: bisection to a
                            sign change, then Brent's method (scipy brentq) per calibration     */
  double r_tol;          /* bracket width (bisection) / xtol (Brent)                          */
  double egm_tol;        /* household solve tolerance (sup-norm of the tables)                */
  double hist_tol;       /* distribution iteration tolerance (sup-norm of the mass)           */
  int32_t max_steps, max_egm_cycles, max_hist_iter;
  int32_t warm_hist;     /* != 0: each step's distribution starts from the previous step's     */
  int32_t warm_egm;      /* != 0: each step's household solve starts from the previous policy */
  int32_t accel;         /* Aitken period of the distribution iteration (0: plain; < 0: BiCGSTAB) */
  const double* r_lo;    /* HOST [n_cal] or NULL: -delta / 2                                   */
  const double* r_hi;    /* HOST [n_cal] or NULL: 1 / beta - 1 - 1e-9                          */
  int32_t secant_start;  /* != 0 (with warm_hist and warm_egm): from the third step on, each
                            evaluation starts its household and distribution solves at
                            cur + theta (cur - prev), theta = (r - r_cur) / (r_cur - r_prev)
                            clamped to [-1, 1] (the fixed points and stopping rules are
                            unchanged; iterates differ from the Python-driven loop)          */
  int32_t loose_bracket; /* != 0 (method 1): while a calibration's search is still bracketing
                            (bisection before the first sign change) its evaluations run to
                            the looser tolerances egm 1e-6 / hist 10^-AIY_OPT_GE_LOOSE_HIST
                            (default 1e-8); the sign of
                            K_s - K_d is taken only where |K_s - K_d| >= 5 % of K_d, else
                            the same r is evaluated again at the full tolerances          */
  int32_t egm_extrapolate; /* != 0: the household solves move a calibration's tables along
                            their last change by lambda / (1 - lambda) at chunk boundaries
                            where the cycle distances fall at a steady rate lambda (egm.hip;
                            the stopping rule is unchanged)                                   */
  int32_t* status_out;   /* HOST [n_cal] or NULL: per calibration, bit 1 = some evaluation's
                            household solve stopped at max_egm_cycles above its tolerance,
                            bit 2 = some distribution solve stopped at max_hist_iter, bit 4 =
                            the search stopped at max_steps before r_tol (0: converged)      */
} aiy_ge_options;

/* Device scratch the call needs (caller-owned `work`), -1 for bad sizes. */
int64_t aiy_ge_stationary_work_bytes(int32_t n_cal, int32_t S, int32_t n_a);

/* General equilibrium in r of every calibration (build-defined E1; no reference code):
 * per step, K_s(r) = sum(mass * a) of the stationary distribution (aiy_egm_solve ->
 * aiy_hist_lottery -> aiy_hist_solve) against K_d(r) = (alpha / (r + delta))^(1/(1-alpha)),
 * w(r) = (1 - alpha) K_d^alpha, R = 1 + r; the brackets move on the host.
 *   r_out, K_out (= K_d(r)), Ks_out (the last evaluation's K_s, may be NULL): HOST [n_cal];
 *   Ks_out always comes from a distribution solved to hist_tol: when the search ends on an
 *   evaluation at the adaptive Brent tolerance (loose bracketing), that evaluation's
 *   distribution is solved again at hist_tol from its mass before K_s is reported;
 *   steps_out: K_s evaluations; egm_cycles_out / hist_iters_out: their sums over steps and
 *   calibrations (may be NULL).  The converged tables, lottery and mass stay in `work`.
 * BLOCKING. */
int32_t aiy_ge_stationary(aiy_handle* h, const aiy_stationary_model* model, const aiy_ge_options* opt,
                          void* work, double* r_out, double* K_out, double* Ks_out, int32_t* steps_out,
                          int32_t* egm_cycles_out, int32_t* hist_iters_out, aiy_stream stream);

/* Plan of the device-resident GE search for (n_cal, S, n_a): returns 1 and out4 =
 * {workgroups per calibration cluster, asset columns per workgroup, columns per thread,
 * blocks of the launch} when aiy_ge_stationary would run it, else 0.  Host-only. */
int32_t aiy_ge_resident_plan(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_a, int32_t* out4);

/* Device-resident GE launch statistics (measurement hook): kernel milliseconds (HIP events
 * around each launch on its stream), launches, (state, node) point-matvecs of the
 * distribution solves and EGM cycles inside them, since the last reset.  Host-only. */
int32_t aiy_ge_launch_stats(aiy_handle* h, double* ms_sum, int64_t* launches, double* point_matvecs,
                            double* egm_cycles, int32_t reset);

/* Per-calibration profile of the last device-resident GE launch (measurement hook):
 * out[c * 8 + k], k = EGM, lottery, distribution solve, K reduction + search, whole search
 * (microseconds, workgroup 0's clock), EGM cycles, matvecs, evaluations.  Returns the
 * calibrations written (<= n_cal).  Host-only. */
int32_t aiy_ge_last_profile(aiy_handle* h, double* out, int32_t n_cal);
/* Per-evaluation log of the last device-resident search: out[(c * 32 + e) * 6 + k], k = r,
   (K_s - K_d) / K_d, EGM cycles, matvecs, loose flag, microseconds (measurement hook). */
int32_t aiy_ge_last_eval_log(aiy_handle* h, double* out, int32_t n_cal);

/* Launches of the last device-resident search (1 + its rebalancing relaunches) and how many
 * cluster stops happened inside a distribution solve (that solve resumes from its iterate in
 * the next launch).  Host-only. */
int32_t aiy_ge_last_rounds(aiy_handle* h, int32_t* launches, int32_t* mid_solve_stops);

/* Resident-histogram launch statistics (measurement hook): kernel milliseconds summed over
 * the device-resident distribution-iteration launches since the last reset (HIP events on
 * their stream) and their number.  reset != 0 zeroes the counters.  Host-only. */
int32_t aiy_hist_launch_stats(aiy_handle* h, double* ms_sum, int64_t* launches, int32_t reset);

/* ------------------- wealth-distribution statistics ------------------- */

/* HARK 0.12 get_lorenz_shares(data, weights, percentiles) and get_percentiles(...) of a
 * DEVICE array (the notebook's sim_wealth, Aiyagari-HARK.py:311-316): n doubles `data`,
 * optional device `weights` (NULL: unit weights), n_p <= 256 HOST percentiles in (0, 1).
 * lorenz_out / pctl_out: HOST [n_p] (either may be NULL).  Scratch is handle-owned.
 * BLOCKING (synchronises `stream`). */
int32_t aiy_wealth_stats(aiy_handle* h, const double* data, const double* weights, int64_t n,
                         const double* pctiles, int32_t n_p, double* lorenz_out, double* pctl_out,
                         aiy_stream stream);

#ifdef __cplusplus
}
#endif

#endif /* AIYAGARI_H */
