// Device-resident general equilibrium of the stationary Aiyagari household (build-defined
// row E1): the WHOLE root search of every calibration in ONE launch.
//
// aiy_ge_stationary's host loop (ge.hip) steps all calibrations of a batch together: each
// K_s(r) evaluation is an EGM solve (host checks every 32 cycles), a lottery launch and one
// distribution-solve launch, and every launch lasts as long as its slowest calibration.
// Here each calibration owns a CLUSTER of G workgroups (512 threads, one per CU; the same
// clusters as the resident histogram, hist_resident.hip) that runs, with no host round
// trip and no waiting for other calibrations:
//
//   loop over K_s(r) evaluations (the RootSearch of ge_search.h, every workgroup of the
//   cluster on bit-identical inputs):
//     prices      R = 1 + r, w = (1 - alpha) (alpha / (r + delta))^(alpha / (1 - alpha))
//     start       secant start of the household tables and the mass from the last two
//                 evaluations (x0 = cur + theta (cur - prev)), as ge.hip
//     EGM         cycles of solve_Aiyagari (Aiyagari_Support.py:1478-1504) over the
//                 workgroup's own asset nodes: V[s'][i] = R c_{s'}(R a_i + w l_{s'})^-rho by
//                 the wavefront-cooperative window interpolation of egm.hip (rows another
//                 workgroup wrote: `sc1` loads), E = beta sum_s' V P in NumPy's pairwise
//                 order, c = E^(-1/rho), m = a + c written write-through (`sc1`); the HARK
//                 stopping rule (sup-norm of the tables <= tol, NaN stops) rides on the
//                 cycle's cluster barrier; the geometric extrapolation of ge.hip every 32
//                 cycles
//     lottery     (s, j) -> a' = m - c_s(m), m = R a_j + w l_s, bracket in the asset grid
//     histogram   BiCGSTAB on (I - T) mass = 0 (hist_bicg.h, the kernel of hist_krylov.hip)
//     K_s         sum mass a (cluster reduction); f = K_s - K_d; loose-bracketing sign test
//   until the search is done; workgroup 0 writes r, K, K_s, the counts and the status.
//
// The launch ends when the slowest calibration's whole search ends (the host loop's launches
// each waited for the slowest calibration of that step).  Workgroup placement: block b runs
// on XCD b % 8 (observed dispatch, speed only), so the blocks are dealt XCD-contiguous and a
// cluster's exchanges mostly stay inside one XCD's L2; correctness never depends on it
// (every cross-workgroup value is written and read at agent scope).
#include "common.h"
#include "egm_common.h"
#include "ge_search.h"
#include "hist_bicg.h"
#include "hist_cluster.h"
#include "internal.h"

#include <algorithm>
#include <cmath>

namespace aiy {

// Workgroup size (template TH; the plan launches 512).  A cycle / matvec costs about the same
// per column of a workgroup whatever the thread organisation: 26.8 / 23.7 us at G = 10
// (1 000 columns, 512 threads x 2 columns), 23.0 / 25.5 us with 1 024 threads x 1 column
// (spills at 128 VGPRs), 15.5 / 12.4 us at G = 21 (477 columns, 512 threads x 1 column)
// (profiles/r03i_*, r03j_*): a cluster's time scales with its columns per CU.
constexpr int kGeTHMax = 1024;
constexpr int kGeWavesMax = kGeTHMax / kWave;   // 16
constexpr int kGeMaxTiles = 16;           // 64-node tiles of one workgroup's own columns (<= 1024)
constexpr int kGeBufs = 5;                // table buffers per calibration: ping, pong, cur, prev, init
// Periodic Anderson mixing of the EGM cycles (AIY_OPT_GE_ANDERSON): every p-th cycle the
// household iterate moves to the type-II Anderson combination of the last kGeAaM + 1 plain
// cycles (their outputs kept in a ring of kGeAaHist slots), plain cycles in between.  A CPU
// study on the oracle's EGM (scratch prototype; N_a = 3 000, the Table II cells near their
// roots, warm and cold starts) put it at 1.5-2.5x fewer cycles to the same HARK stopping rule
// than the period-32 geometric extrapolation it replaces (m = 3, p = 12: 97-128 against
// 196-248 cycles from a start 2e-2 away in r, 49-97 against 112-178 from 2e-5).
constexpr int kGeAaM = 3;
constexpr int kGeAaHist = kGeAaM + 2;
// One asset column per thread (G >= 20 at N_a = 10 000: every relaunch and the 8-GPU shape):
// the BiCGSTAB solve's alpha reduction rides on its first matvec's barrier (hist_bicg.h
// FUSEA), one cluster reduction per iteration instead of two.  A diagnostic build with
// -DAIY_DIAG_NO_FUSEA runs the plain recurrence everywhere (A/B timing).
#ifdef AIY_DIAG_NO_FUSEA
constexpr bool kGeFuseA = false;
#else
constexpr bool kGeFuseA = true;
#endif
// With two columns per thread (the first, 24-cell launch of a Table II sweep) the default keeps the
// two-reduction form: FUSEA there (-DAIY_FUSEA_KC2=2: u's own points read back from HBM beside the
// new p; =1: prefetched across the second reduction) measured SLOWER, 411-427 against 481-491 GE
// solves/s for the Table II sweep (gpurun_out/r08e_abaa_*: the last wave, which sweeps the riding
// reduction, owns columns at two per thread and delays its gather; the x loads move behind the
// matvec)
#ifndef AIY_FUSEA_KC2
#define AIY_FUSEA_KC2 0
#endif
constexpr bool kGeFuseAKc2 = AIY_FUSEA_KC2 != 0;
template <int NW>
constexpr size_t ge_egm_lds() { return (size_t)NW * (8 * kTile + 4 * kWin) * sizeof(double); }   // V tiles + windows

struct GeCalDev {
  double alpha, delta, disc, r_lo, r_hi;
};

struct GeState;
struct GeRun {
  int n_cal, S, n_a, G, nj, cap, n_work;   // n_work = G x (calibrations of this launch)
  const double* a_grid;   // [n_cal][n_a]
  const double* P;        // [n_cal][S][S]
  const double* lab;      // [n_cal][S]
  const double* beta;     // [n_cal]
  const double* crra;     // [n_cal]
  const GeCalDev* cal;    // [n_cal]
  int method;
  double r_tol, egm_tol, hist_tol;
  int max_steps, max_cyc, max_hist;
  int warm_hist, warm_egm, secant, loose, extrap;
  int extrap_period;      // EGM cycles between extrapolation checks (>= 4)
  int aa_period;          // EGM Anderson mixing every aa_period cycles (0: off; AIY_OPT_GE_ANDERSON)
  double* aah;            // [n_cal][kGeAaHist][S][n_a] the last kGeAaHist EGM outputs (c, own nodes)
  int logsec;             // log-secant bracketing (AIY_OPT_GE_LOGSEC, with loose bracketing)
  int pull;               // distribution solves by the lottery pull (AIY_OPT_HIST_PULL): deterministic
  double loose_hist;      // loose-bracketing histogram tolerance (AIY_OPT_GE_LOOSE_HIST)
  double* qb;             // [n_cal][S][n_a] pull form: the matvec input rows
  int* ainv;              // [n_cal][S][n_a + 1] pull form: inverse lottery
  double* tab;            // [n_cal][kGeBufs][2][S][n_a + 1]
  double* mass;           // [n_cal][S][n_a]
  double* pmass;          // [n_cal][S][n_a] previous evaluation's mass
  double* pg;             // [n_cal][S][n_a] BiCGSTAB p rows
  int* lo;                // [n_cal][S][n_a]
  double* wlo;            // [n_cal][S][n_a]
  double* slab;           // [launch cals][G][2][cap]
  int* span;              // [launch cals][G][SMAX][4]
  unsigned* ctr;          // [launch cals][kHcCtrStride]
  unsigned long long* gran;   // [launch cals][2][G][kHcRedRec]
  // rebalancing: a launch covers some calibrations (cal_ids) and stops at the next evaluation
  // boundary of every cluster once stop_at of them have finished; stopped ones save their
  // search state and the host relaunches them with larger clusters
  const int* cal_ids;     // [launch cals] cluster -> calibration
  GeState* saved;         // [n_cal] search state of a stopped calibration
  const int* resume;      // [n_cal] 1: start from saved[cal]
  unsigned* done_ctr;     // calibrations of this launch whose search has ended
  int stop_at;            // 0: never stop
  int* out_done;          // [n_cal] 1: search ended (outputs written), 0: stopped
  unsigned* err;
  double* out_r;
  double* out_K;
  double* out_Ks;
  int* out_steps;
  int* out_cyc;
  int* out_its;
  int* out_status;
  double* out_prof;       // [n_cal][kGeProf] workgroup 0's phase times (us) and counts
  double* out_evlog;      // [n_cal][kGeEvLog][kGeEvRec] per-evaluation record (measurement)
};
// per-calibration profile of the launch (workgroup 0, s_memrealtime at 100 MHz): EGM, lottery,
// distribution solve, K reduction + search, whole search (us); EGM cycles, matvecs, evaluations
constexpr int kGeProf = 8;
// per-evaluation log: r, (K_s - K_d) / K_d, EGM cycles, matvecs, loose, EGM + histogram us
constexpr int kGeEvLog = 32;
constexpr int kGeEvRec = 6;

// Search state of one calibration, one copy per workgroup (thread 0 writes, all read).
struct GeState {
  RootSearch rs;
  double R, wage, Kd, etol, htol, theta, r_cur, r_prev, Ks, dist, lam_prev, fext;
  double fmin;             // smallest |K_s - K_d| / K_d accepted so far (adaptive tolerance)
  int adapt;               // this evaluation runs at an adaptive histogram tolerance
  int steps, loose, refine, warm_egm, secant, fresh_mass, status, n, stop, nan_stop, moved, extrap;
  int in_hist;             // stopped (rebalancing) inside this evaluation's distribution solve
  int final_ks;            // the search ended on a loose or adaptive-tolerance evaluation: that r is
                           // evaluated once more at the full tolerances before K_s is reported
  int buf[kGeBufs];        // roles: 0 ping, 1 pong, 2 cur, 3 prev, 4 init -> buffer index
  long long cyc_sum, its_sum;
  unsigned long long t_egm, t_lot, t_hist, t_k, t0, t_ev0;
  unsigned nc_prev[2];
  unsigned nbc;            // counting barriers passed
};

// Cluster-wide reduction of nv per-thread values (bit v of kmax: NaN-propagating max, else
// sum) in a fixed order at every level, through tagged 8-byte granules (hist_bicg.h's
// protocol; every workgroup computes the same s_res).  It is also a barrier: every
// workgroup has published after all its waves drained their stores.
template <int TH>
__device__ __forceinline__ bool ge_reduce(unsigned long long* gran, int G, int w, unsigned& ne, const double* vals,
                                          int nv, unsigned kmax, double (*s_part)[kGeWavesMax], double* s_res,
                                          int* s_flag, unsigned* err) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int v = 0; v < nv; ++v) {
    const double x = (kmax >> v) & 1u ? wave_nan_max(vals[v]) : wave_sum_lane63(vals[v]);
    if (lane == kWave - 1) s_part[v][wid] = x;
  }
  __syncthreads();
  ++ne;
  const unsigned long long tag = (unsigned long long)ne << 32;
  unsigned long long* slot = gran + (size_t)(ne & 1) * G * kHcRedRec;
  if (tid < nv) {
    const int v = tid;
    double x = s_part[v][0];
    for (int q = 1; q < TH / kWave; ++q) x = (kmax >> v) & 1u ? nan_max(x, s_part[v][q]) : x + s_part[v][q];
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    unsigned long long* g = slot + (size_t)w * kHcRedRec + 2 * v;
    __hip_atomic_store(to_global(g), tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(to_global(g + 1), tag | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (wid == 0) {
    double xa[kHkRed], xb[kHkRed];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok;
    do {
      ok = true;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int w2 = lane + u * kWave;
#pragma unroll
        for (int v = 0; v < kHkRed; ++v) {
          double x = 0.0;
          if (v < nv && w2 < G) {
            const unsigned long long* g = slot + (size_t)w2 * kHcRedRec + 2 * v;
            const unsigned long long hi = __hip_atomic_load(to_global(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long lo = __hip_atomic_load(to_global(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = ok && (hi & 0xffffffff00000000ull) == tag && (lo & 0xffffffff00000000ull) == tag;
            x = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
          }
          if (u == 0) xa[v] = x;
          else xb[v] = x;
        }
      }
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kHcTimeoutTicks) {
        if (lane == 0) __hip_atomic_store(to_global(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    } while (true);
    if (lane == 0) *s_flag = ok ? 1 : 0;
#pragma unroll
    for (int v = 0; v < kHkRed; ++v) {
      if (v < nv) {
        const bool mx = (kmax >> v) & 1u;
        const double y = mx ? wave_nan_max(nan_max(xa[v], xb[v])) : wave_sum_lane63(xa[v] + xb[v]);
        if (lane == kWave - 1) s_res[v] = y;
      }
    }
  }
  __syncthreads();
  return *s_flag != 0;
}

// Interpolation pass over the workgroup's own asset columns, one 64-column tile per wave at
// a time (wave wv: tiles wv, wv + 8; column j = j0 + 64 tile + lane = j0 + tid + 512 k, the
// hist_bicg.h column of the same thread): for every row s of `src` (S rows of n_a + 1
// nodes) the HARK LinearInterp at q = R a_j + Wl[s], by the window search of egm.hip over
// agent-scope loads; sink(tile, lane column, s, q, value) takes the result.
template <int SMAX, int NW, typename Sink, typename Begin, typename End>
__device__ __forceinline__ void ge_rows_pass(int S, int n_a, int j0, int j1, const double* __restrict__ a_grid,
                                             const double* __restrict__ src_m, const double* __restrict__ src_c,
                                             double R, const double* s_Wl, int* s_hint, double* lds_win,
                                             Sink&& sink, Begin&& begin, End&& end) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int n = n_a, n1 = n_a + 1;
  const int ntile = (j1 - j0 + kTile - 1) / kTile;
  double* X = lds_win + (size_t)wv * 4 * kWin;
  double* Y = X + kWin;
  double* XB = X + 2 * kWin;
  double* YB = X + 3 * kWin;
#pragma unroll 1
  for (int tile = wv; tile < ntile; tile += NW) {
    const int jr = j0 + tile * kTile + lane;
    const int j = jr < j1 ? jr : j1 - 1;   // lanes past the range repeat the last column
    const double a = a_grid[j];
    int* hint = s_hint + tile * SMAX;
    begin(tile, j);
    auto fetch = [&](int r, RowWin& wn) {
      const int rr = r < S ? r : S - 1;
      load_win<true>(src_m + (size_t)rr * n1, src_c + (size_t)rr * n1, n, win_base(hint[rr], n1), lane, wn);
    };
    unsigned redo = 0u;
    auto step_unit = [&](int u, const RowWin& wa, const RowWin& wb) {
      const int ra = 2 * u, rb = 2 * u + 1;
      if (ra >= S) return;   // wave-uniform
      const bool has_b = rb < S;
      const int rbb = has_b ? rb : ra;
      const bool na = __any(stage_win(wa, n, X, Y, lane));
      const bool nb = __any(stage_win(wb, n, XB, YB, lane));
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const double qa = R * a + s_Wl[ra];   // mNextArray (AS:1024)
      const double qb = R * a + s_Wl[rbb];
      int lba, lbb;
      bool oka, okb;
      const double fa = search_win(wa.base, na, n, qa, X, Y, lba, oka);
      const double fb = search_win(wb.base, nb, n, qb, XB, YB, lbb, okb);
      hint[ra] = __builtin_amdgcn_readfirstlane(lba);
      if (has_b) hint[rb] = __builtin_amdgcn_readfirstlane(lbb);
      if (__any(!oka)) redo |= 1u << ra;
      else sink(tile, jr, j, ra, qa, fa);
      if (has_b) {
        if (__any(!okb)) redo |= 1u << rb;
        else sink(tile, jr, j, rb, qb, fb);
      }
    };
    RowWin a0, b0, a1, b1;
    fetch(0, a0);
    fetch(1, b0);
#pragma unroll 1
    for (int u = 0; 2 * u < S; u += 2) {
      fetch(2 * u + 2, a1);
      fetch(2 * u + 3, b1);
      step_unit(u, a0, b0);
      fetch(2 * u + 4, a0);
      fetch(2 * u + 5, b0);
      step_unit(u + 1, a1, b1);
    }
#pragma unroll 1
    while (redo != 0u) {   // wave-uniform
      const int s = __builtin_ctz(redo);
      redo &= redo - 1u;
      const double q = R * a + s_Wl[s];
      int lb;
      const double f = interp_row_global_agent(src_m + (size_t)s * n1, src_c + (size_t)s * n1, n, q, lb);
      hint[s] = __builtin_amdgcn_readfirstlane(lb);
      sink(tile, jr, j, s, q, f);
    }
    end(tile, j, a);
  }
}

// One EGM cycle of the workgroup's own nodes: src (cycle n - 1; nullptr: the terminal
// c = m) -> dst (cycle n).  Returns the workgroup's part of the HARK distance (track).
template <int SMAX, int SC, int PK, int NW>
__device__ __forceinline__ double ge_egm_cycle(int S, int n_a, int j0, int j1, const double* __restrict__ a_grid,
                                               const double* src_m, const double* src_c, double* dst_m,
                                               double* dst_c, bool track, double R, double beta, double gam,
                                               const double* s_Wl, const double* s_Pe, int* s_hint,
                                               double* lds_v, double* lds_win, double* ring) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int n1 = n_a + 1;
  double* Vw = lds_v + (size_t)wv * SMAX * kTile;   // this wave's V[s'][lane]
  const int ntile = (j1 - j0 + kTile - 1) / kTile;
  double dmax = 0.0;
  if (src_m == nullptr) {   // terminal guess: IdentityFunction (AS:898) of mNextArray
#pragma unroll 1
    for (int tile = wv; tile < ntile; tile += NW) {
      const int jr = j0 + tile * kTile + lane;
      const int j = jr < j1 ? jr : j1 - 1;
      const double a = a_grid[j];
      for (int sp = 0; sp < S; ++sp) {
        const double c = (R * a + s_Wl[sp]) * 1.0;
        Vw[sp * kTile + lane] = R * marg_u<PK>(c, gam);   // read back by the same lane only
      }
      for (int s = 0; s < S; ++s) {
        double sum;
        if constexpr (SC > 0) sum = pairwise_dot<SC>(Vw + lane, s_Pe + s * SC);
        else sum = np_pairwise_sum<SMAX>(S, [&](int t) { return Vw[t * kTile + lane] * uniform_f64(s_Pe[s * S + t]); });
        const double c = inv_marg<PK>(beta * sum, gam);
        store_f64_agent(&dst_m[(size_t)s * n1 + j + 1], a + c);
        store_f64_agent(&dst_c[(size_t)s * n1 + j + 1], c);
        if (ring) store_f64_agent(&ring[(size_t)s * n_a + j], c);
        if (j == 0) {
          store_f64_agent(&dst_m[(size_t)s * n1], kBorrowNode);
          store_f64_agent(&dst_c[(size_t)s * n1], kBorrowNode);
        }
      }
    }
    return 0.0;
  }
  // tiles one after another per wave: the previous tables' values at the lane's node
  // (distance) in flight from the tile's start, V of the tile's rows (phase 1), then its
  // outputs (phase 2)
  constexpr int NP = SC > 0 ? SC : SMAX;
  double pmv[NP], pcv[NP];
  auto begin = [&](int, int j) {
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      pmv[s] = 0.0;
      pcv[s] = 0.0;
      if (track && s < S) {
        pmv[s] = load_f64_agent(&src_m[(size_t)s * n1 + j + 1]);
        pcv[s] = load_f64_agent(&src_c[(size_t)s * n1 + j + 1]);
      }
    }
  };
  auto end = [&](int, int j, double a) {   // phase 2 (each lane reads its own V)
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      if (s < S) {
        __builtin_amdgcn_sched_barrier(0);   // one state's P reads at a time (no hoisting of all S x S)
        double sum;
        if constexpr (SC > 0) sum = pairwise_dot<SC>(Vw + lane, s_Pe + s * SC);
        else sum = np_pairwise_sum<SMAX>(S, [&](int t) { return Vw[t * kTile + lane] * uniform_f64(s_Pe[s * S + t]); });
        const double E = beta * sum;                     // EndOfPrdvP (AS:1485)
        const double c = inv_marg<PK>(E, gam);           // AS:1490
        const double m = a + c;                          // AS:1499
        store_f64_agent(&dst_m[(size_t)s * n1 + j + 1], m);
        store_f64_agent(&dst_c[(size_t)s * n1 + j + 1], c);
        if (ring) store_f64_agent(&ring[(size_t)s * n_a + j], c);   // Anderson history (own nodes)
        if (track) dmax = nan_max(dmax, nan_max(fabs(m - pmv[s]), fabs(c - pcv[s])));
        if (j == 0) {   // the (1e-7, 1e-7) node (AS:1503-1504)
          store_f64_agent(&dst_m[(size_t)s * n1], kBorrowNode);
          store_f64_agent(&dst_c[(size_t)s * n1], kBorrowNode);
        }
      }
    }
  };
  ge_rows_pass<SMAX, NW>(S, n_a, j0, j1, a_grid, src_m, src_c, R, s_Wl, s_hint, lds_win,
                     [&](int, int, int, int sp, double, double f) {
                       Vw[sp * kTile + lane] = R * marg_u<PK>(f, gam);   // RnextArray * MargValueFuncCRRA
                     },
                     begin, end);
  return dmax;
}

// The kernel's LDS at file scope, so the search loop, the EGM cycle and the lottery (their
// own non-inlined functions, each with its own register allocation) address it directly.
constexpr int kGeSmax = 8;    // the largest resident state count (Table II: 7)
extern __shared__ double ge_dyn[];                 // histogram: span buffer + v; EGM: V tiles + windows
__shared__ double ge_s_part[kHkRed][kGeWavesMax];
__shared__ double ge_s_res[kHkRed];
__shared__ int ge_s_flag;
__shared__ double ge_s_Pe[kGeSmax * kGeSmax];     // P[s][s'] unpadded (egm_phase2's layout)
__shared__ double ge_s_Wl[kGeSmax];               // w l(s')
__shared__ int ge_s_hint[kGeMaxTiles * kGeSmax];  // window hints per (tile, row)
__shared__ unsigned ge_s_nc;
__shared__ GeState ge_st;

template <int SMAX, int SC, int PK, int NW>
__device__ __forceinline__ double ge_egm_cycle_fn(int S, int n_a, int j0, int j1, const double* a_grid,
                                               const double* src_m, const double* src_c, double* dst_m,
                                               double* dst_c, bool track, double R, double beta, double gam,
                                               double* ring) {
  return ge_egm_cycle<SMAX, SC, PK, NW>(S, n_a, j0, j1, a_grid, src_m, src_c, dst_m, dst_c, track, R, beta, gam,
                                        ge_s_Wl, ge_s_Pe, ge_s_hint, ge_dyn, ge_dyn + (size_t)NW * SMAX * kTile, ring);
}

// lottery of the own columns on the final tables (hist.hip hist_lottery_kernel's arithmetic)
template <int SMAX, int NW>
__device__ __forceinline__ void ge_lottery_fn(int S, int n_a, int j0, int j1, const double* a_grid, const double* fm,
                                           const double* fc, double R, bool have_prev, int* LO, double* WL,
                                           bool write_through) {
  ge_rows_pass<SMAX, NW>(S, n_a, j0, j1, a_grid, fm, fc, R, ge_s_Wl, ge_s_hint, ge_dyn + (size_t)NW * SMAX * kTile,
                     [&](int, int jr, int, int s, double q, double c) {
                       if (jr >= j1) return;
                       const double ap = q - c;
                       const size_t o = (size_t)s * n_a + jr;
                       int d = -1;
                       if (have_prev) {   // last evaluation's bracket as the first guess
                         const int h = LO[o];
                         if (h >= 0 && h < n_a - 1 && a_grid[h] <= ap && ap < a_grid[h + 1]) d = h;
                       }
                       if (d < 0) {       // searchsorted(a_grid, a', 'right') - 1
                         int lo = 0, hi = n_a;
                         while (lo < hi) {
                           const int mid = lo + ((hi - lo) >> 1);
                           if (a_grid[mid] <= ap) lo = mid + 1; else hi = mid;
                         }
                         d = lo - 1;
                       }
                       d = d < 0 ? 0 : (d > n_a - 2 ? n_a - 2 : d);
                       double wl = (a_grid[d + 1] - ap) / (a_grid[d + 1] - a_grid[d]);
                       wl = wl < 0.0 ? 0.0 : (wl > 1.0 ? 1.0 : wl);
                       if (write_through) {   // the pull form reads foreign lottery entries
                         __hip_atomic_store(to_global(&LO[o]), d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                         store_f64_agent(&WL[o], wl);
                       } else {
                         LO[o] = d;
                         WL[o] = wl;
                       }
                     },
                     [](int, int) {}, [](int, int, double) {});
}

template <int SMAX, int SC, int KC, int TH>
__global__ __launch_bounds__(TH) void ge_cluster_kernel(GeRun g) {
  constexpr int NW = TH / kWave;
  static_assert(SMAX <= kGeSmax, "file-scope LDS sized for kGeSmax states");
  GeState& st = ge_st;
  double (*s_part)[kGeWavesMax] = ge_s_part;
  double* s_res = ge_s_res;
  int& s_flag = ge_s_flag;
  double* s_Pe = ge_s_Pe;
  double* s_Wl = ge_s_Wl;
  int* s_hint = ge_s_hint;
  unsigned& s_nc = ge_s_nc;

  const int per = gridDim.x >> 3;
  const int u = (blockIdx.x & 7) * per + (blockIdx.x >> 3);   // XCD-contiguous work order
  if (u >= g.n_work) return;
  const int G = g.G, S = g.S, n_a = g.n_a, n1 = n_a + 1;
  const int lc = u / G, w = u - lc * G;   // launch-local cluster, workgroup in it
  const int cal = g.cal_ids[lc];
  const int tid = threadIdx.x;
  const int j0 = w * g.nj, j1 = min(j0 + g.nj, n_a);
  const double* a_grid = g.a_grid + (size_t)cal * n_a;
  const double beta = g.beta[cal], gam = g.crra[cal];
  const GeCalDev cd = g.cal[cal];
  const size_t tab_sz = (size_t)S * n1;
  double* tab = g.tab + (size_t)cal * kGeBufs * 2 * tab_sz;
  auto tabm = [&](int b) { return tab + (size_t)b * 2 * tab_sz; };
  auto tabc = [&](int b) { return tab + (size_t)b * 2 * tab_sz + tab_sz; };
  const size_t row0 = (size_t)cal * S * n_a;
  double* X = g.mass + row0;
  double* PX = g.pmass + row0;
  int* LO = g.lo + row0;
  double* WL = g.wlo + row0;
  unsigned* ctr = g.ctr + (size_t)lc * kHcCtrStride;
  unsigned long long* cw = reinterpret_cast<unsigned long long*>(ctr + 2);   // counting-barrier words
  unsigned long long* gran = g.gran + (size_t)lc * 2 * G * kHcRedRec;
  unsigned nb = 0, ne = 0;   // plain barriers / reductions passed (hk_solve counts on)
  const int pk = gam == 1.0 ? 1 : (gam == 3.0 ? 3 : (gam == 5.0 ? 5 : 0));


  for (int q = tid; q < S * S; q += TH) s_Pe[q] = g.P[(size_t)cal * S * S + q];
  for (int q = tid; q < kGeMaxTiles * SMAX; q += TH) s_hint[q] = -1;
  if (tid == 0) {
    if (g.resume[cal]) {   // a calibration stopped by an earlier launch: its search goes on
      st = g.saved[cal];
      st.t0 = __builtin_amdgcn_s_memrealtime() - st.t0;   // saved: the time spent so far
    } else {
      st.rs.init(cd.r_lo, cd.r_hi, g.r_tol, g.method, g.loose ? g.logsec : 0);
      st.r_cur = st.r_prev = 0.0;
      st.Ks = 0.0;
      st.fmin = __builtin_inf();
      st.adapt = 0;
      st.steps = 0;
      st.refine = 0;
      st.in_hist = 0;
      st.final_ks = 0;
      st.status = 0;
      st.cyc_sum = st.its_sum = 0;
      for (int b = 0; b < kGeBufs; ++b) st.buf[b] = b;
      st.t_egm = st.t_lot = st.t_hist = st.t_k = 0ull;
      st.t0 = __builtin_amdgcn_s_memrealtime();
    }
    st.nc_prev[0] = st.nc_prev[1] = 0u;   // this launch's counting-barrier words start at 0
    st.nbc = 0u;
  }
  __syncthreads();
  auto plain_barrier = [&]() -> bool {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ++nb;
    return hc_barrier(g.err, ctr, (unsigned)G * nb, &s_flag);
  };

  bool stopped = false;
  while ((!st.rs.done && st.steps < g.max_steps) || st.final_ks) {
    // ---- rebalancing stop: once stop_at calibrations of the launch have finished, the
    //      cluster leaves at this evaluation boundary (the decision: any workgroup saw it,
    //      counted on the cluster's barrier, so every workgroup takes it) ----
    if (g.stop_at > 0 && st.steps > 0 && !st.in_hist) {
      unsigned flag = 0u;
      if (tid == 0) {
        flag = __hip_atomic_load(to_global(g.done_ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                       (unsigned)g.stop_at ? 1u : 0u;
        ++st.nbc;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const unsigned k = st.nbc, par = k & 1u;
      if (!hc_barrier_count(g.err, &cw[par], (unsigned)G * ((k + par) / 2), flag, &s_nc, &s_flag)) return;
      if (tid == 0) {
        const unsigned dlt = s_nc - st.nc_prev[par];
        st.nc_prev[par] = s_nc;
        st.stop = dlt != 0u;
      }
      __syncthreads();
      if (st.stop) {
        stopped = true;
        break;
      }
    }
    // a calibration stopped inside its distribution solve resumes there (prices, tables,
    // lottery and the iterate are in the saved state and HBM)
    unsigned long long tp = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && !st.in_hist) st.t_ev0 = tp;
    if (!st.in_hist) {
      // ---- this evaluation's prices, tolerances and starts (thread 0; identical everywhere) ----
      if (tid == 0) {
        // (the final pass re-evaluates the LAST evaluated r at the full tolerances)
        const double r = st.final_ks ? st.r_cur : st.rs.x, a = cd.alpha, d = cd.delta;
        const double KtoL = pow(a / (r + d), 1.0 / (1.0 - a));
        st.R = 1.0 + r;
        st.wage = (1.0 - a) * pow(KtoL, a);
        st.Kd = KtoL;
        st.loose = g.loose && g.method == 1 && !st.rs.brent && !st.rs.done && !st.refine;
        st.etol = st.loose ? fmax(g.egm_tol, AIY_GE_LOOSE_EGM) : g.egm_tol;
        st.htol = st.loose ? fmax(g.hist_tol, g.loose_hist) : g.hist_tol;
        // Brent's evaluations: the adaptive tolerance (ge_search.h), refined ones at the full one
        st.adapt = 0;
        if (kGeAdapt && g.loose && g.method == 1 && st.rs.brent && !st.rs.done && !st.refine) {
          st.htol = ge_adapt_htol(st.fmin, g.hist_tol, fmax(g.hist_tol, g.loose_hist));
          st.adapt = st.htol > g.hist_tol;
        }
        st.warm_egm = g.warm_egm && st.steps > 0;
        st.secant = g.secant && g.warm_egm && g.warm_hist && st.steps >= 2 && !st.final_ks;
        st.fresh_mass = !(g.warm_hist && st.steps > 0);
        double th = 0.0;
        if (st.secant) {
          const double den = st.r_cur - st.r_prev;
          th = den != 0.0 ? (r - st.r_cur) / den : 0.0;
          th = isfinite(th) ? fmax(-1.0, fmin(1.0, th)) : 0.0;
        }
        st.theta = th;
        st.extrap = g.extrap;
        st.moved = 0;
      }
      __syncthreads();
      if (tid < S) s_Wl[tid] = st.wage * g.lab[(size_t)cal * S + tid];   // W l(s') (mNextArray, AS:1024)
      const double R = st.R, theta = st.theta;
      // ---- starting tables: the secant start into `init` (own nodes), else cur ----
      const bool secant = st.secant != 0, warm = st.warm_egm != 0;
      const int b_cur = st.buf[2], b_prev = st.buf[3], b_init = st.buf[4];
      if (secant) {
        for (int s = 0; s < S; ++s) {
          for (int k = j0 + tid; k < j1; k += TH) {
            const size_t o = (size_t)s * n1 + k + 1;
            const double cm = load_f64_agent(&tabm(b_cur)[o]), pm = load_f64_agent(&tabm(b_prev)[o]);
            const double cc = load_f64_agent(&tabc(b_cur)[o]), pc = load_f64_agent(&tabc(b_prev)[o]);
            store_f64_agent(&tabm(b_init)[o], theta == 0.0 ? cm : cm + theta * (cm - pm));
            store_f64_agent(&tabc(b_init)[o], theta == 0.0 ? cc : cc + theta * (cc - pc));
          }
          if (j0 == 0 && tid == 0) {
            store_f64_agent(&tabm(b_init)[(size_t)s * n1], kBorrowNode);
            store_f64_agent(&tabc(b_init)[(size_t)s * n1], kBorrowNode);
          }
        }
      }
      // ---- the household solve ([HARK] solve_agent: cycles until the sup-norm change of the
      //      tables is <= tol, NaN stops; cold: cycle 1 from the terminal guess) ----
      tp = __builtin_amdgcn_s_memrealtime();
      const double* init_m = secant ? tabm(b_init) : (warm ? tabm(b_cur) : nullptr);
      const double* init_c = secant ? tabc(b_init) : (warm ? tabc(b_cur) : nullptr);
      int final_buf = -1;
      for (int attempt = 0; attempt < 2; ++attempt) {
        if (!plain_barrier()) return;   // every workgroup's start tables visible
        // Anderson mixing (the first attempt; a NaN after a mix reruns the solve plain) replaces
        // the geometric extrapolation
        const bool aa = g.aa_period > 0 && attempt == 0;
        const bool ext = st.extrap != 0 && attempt == 0 && !aa;
        auto ring_at = [&](int c) -> double* {
          return aa ? g.aah + ((size_t)cal * kGeAaHist + (size_t)(c % kGeAaHist)) * S * n_a : nullptr;
        };
        if (tid == 0) {
          st.lam_prev = -1.0;
          st.moved = 0;
          st.nan_stop = 0;
        }
        int n = 1;
        const int last_allowed = g.max_cyc + 1;
        bool converged = false;
        while (true) {
          const int b_dst = st.buf[n & 1], b_src = st.buf[(n - 1) & 1];
          const double* sm = n == 1 ? init_m : tabm(b_src);
          const double* sc = n == 1 ? init_c : tabc(b_src);
          const bool track = n >= 2;
          double dl;
          if (pk == 1)
            dl = ge_egm_cycle_fn<SMAX, SC, 1, NW>(S, n_a, j0, j1, a_grid, sm, sc, tabm(b_dst), tabc(b_dst), track, R, beta,
                                              gam, ring_at(n));
          else if (pk == 3)
            dl = ge_egm_cycle_fn<SMAX, SC, 3, NW>(S, n_a, j0, j1, a_grid, sm, sc, tabm(b_dst), tabc(b_dst), track, R, beta,
                                              gam, ring_at(n));
          else if (pk == 5)
            dl = ge_egm_cycle_fn<SMAX, SC, 5, NW>(S, n_a, j0, j1, a_grid, sm, sc, tabm(b_dst), tabc(b_dst), track, R, beta,
                                              gam, ring_at(n));
          else
            dl = ge_egm_cycle_fn<SMAX, SC, 0, NW>(S, n_a, j0, j1, a_grid, sm, sc, tabm(b_dst), tabc(b_dst), track, R, beta,
                                              gam, ring_at(n));
          // cluster distance: the value itself at the extrapolation checks (cycles 32k - 1,
          // 32k), else only its two facts (some part > tol; some part NaN) on a counting barrier
          const int xp = g.extrap_period;
          const bool want_value = ext && n >= xp - 1 && ((n % xp) == xp - 1 || (n % xp) == 0);
          double dclu = 0.0;
          bool go;
          if (want_value) {
            double v[1] = {dl};
            if (!ge_reduce<TH>(gran, G, w, ne, v, 1, 1u, s_part, s_res, &s_flag, g.err)) return;
            dclu = s_res[0];
            go = dclu > st.etol;   // NaN: stop (HARK: go = distance > tolerance)
            if (tid == 0) st.nan_stop = dclu != dclu;
          } else {
            const double dw = wave_nan_max(dl);
            if ((tid & (kWave - 1)) == 0) s_part[0][tid / kWave] = dw;
            __syncthreads();
            unsigned flag = 0u;
            if (tid == 0) {
              double d = s_part[0][0];
              for (int q = 1; q < TH / kWave; ++q) d = nan_max(d, s_part[0][q]);
              flag = (d > st.etol ? 1u : 0u) | (d != d ? (1u << 16) : 0u);
              ++st.nbc;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const unsigned k = st.nbc, par = k & 1u;
            if (!hc_barrier_count(g.err, &cw[par], (unsigned)G * ((k + par) / 2), flag, &s_nc, &s_flag)) return;
            if (tid == 0) {
              const unsigned dlt = s_nc - st.nc_prev[par];
              st.nc_prev[par] = s_nc;
              st.stop = (dlt & 0xffffu) == 0u || (dlt >> 16) != 0u;
              st.nan_stop = (dlt >> 16) != 0u;
            }
            __syncthreads();
            go = !st.stop;
          }
          if (track && !go) {
            converged = true;
            break;
          }
          if (n >= last_allowed) break;
          // geometric extrapolation at the checks (ge.hip / egm.hip egm_extrap_kernel)
          if (want_value && (n % xp) == 0) {
            if (tid == 0) {
              const double d1 = dclu, d0 = st.dist, lam = d1 / d0;
              st.fext = 0.0;
              if (n >= 4 && d1 > 100.0 * st.etol && lam > 0.5 && lam < 0.999 && st.lam_prev > 0.0 &&
                  fabs(lam - st.lam_prev) < 0.2 * (1.0 - lam)) {
                st.fext = lam / (1.0 - lam);
                st.moved = 1;
              }
              st.lam_prev = lam;
            }
            __syncthreads();
            const double f = st.fext;
            if (f != 0.0) {
              double* cm = tabm(b_dst);
              double* cc = tabc(b_dst);
              const double* pm = tabm(b_src);
              const double* pc = tabc(b_src);
              for (int s = 0; s < S; ++s)
                for (int k = j0 + tid; k < j1; k += TH) {
                  const size_t o = (size_t)s * n1 + k + 1;
                  const double x = load_f64_agent(&cm[o]), y = load_f64_agent(&cc[o]);
                  store_f64_agent(&cm[o], x + f * (x - load_f64_agent(&pm[o])));
                  store_f64_agent(&cc[o], y + f * (y - load_f64_agent(&pc[o])));
                }
              if (!plain_barrier()) return;
            }
          } else if (want_value) {
            if (tid == 0) st.dist = dclu;
          }
          if (aa && n >= g.aa_period && n >= kGeAaHist + 1 && (n % g.aa_period) == 0) {
            // type-II Anderson over the plain chain w0 .. w4 = the outputs of cycles n - 4 .. n
            // (p >= kGeAaHist: no mix inside the window): g_i = w_{i+1} - w_i, dG_i = g_{i+1} - g_i,
            // dF_i = w_{i+2} - w_{i+1}; gamma = argmin |g_3 - dG gamma| (Gram + 1e-12 trace
            // regularisation, two cluster reductions in fixed order: every workgroup solves the
            // same 3 x 3 system to the same bits); x_{n+1} = w4 - dF gamma replaces the cycle's
            // output (own nodes, m = a + c), visible to every workgroup after a barrier
            static_assert(kGeAaM == 3 && kGeAaHist == 5, "the mixing below is written for m = 3");
            const double* W0 = ring_at(n - 4);
            const double* W1 = ring_at(n - 3);
            const double* W2 = ring_at(n - 2);
            const double* W3 = ring_at(n - 1);
            const double* W4 = ring_at(n);
            double gp[9];
            for (int q = 0; q < 9; ++q) gp[q] = 0.0;
            for (int s = 0; s < S; ++s)
              for (int k = j0 + tid; k < j1; k += TH) {
                const size_t o = (size_t)s * n_a + k;
                const double w0 = load_f64_agent(W0 + o), w1 = load_f64_agent(W1 + o), w2 = load_f64_agent(W2 + o);
                const double w3 = load_f64_agent(W3 + o), w4 = load_f64_agent(W4 + o);
                const double g0 = w1 - w0, g1 = w2 - w1, g2 = w3 - w2, g3 = w4 - w3;
                const double d0 = g1 - g0, d1 = g2 - g1, d2 = g3 - g2;
                gp[0] += d0 * d0; gp[1] += d0 * d1; gp[2] += d0 * d2;
                gp[3] += d1 * d1; gp[4] += d1 * d2; gp[5] += d2 * d2;
                gp[6] += d0 * g3; gp[7] += d1 * g3; gp[8] += d2 * g3;
              }
            if (!ge_reduce<TH>(gran, G, w, ne, gp, 6, 0u, s_part, s_res, &s_flag, g.err)) return;
            double a00 = s_res[0], a01 = s_res[1], a02 = s_res[2], a11 = s_res[3], a12 = s_res[4], a22 = s_res[5];
            if (!ge_reduce<TH>(gran, G, w, ne, gp + 6, 3, 0u, s_part, s_res, &s_flag, g.err)) return;
            const double b0 = s_res[0], b1 = s_res[1], b2 = s_res[2];
            // Cholesky of the regularised Gram matrix (symmetric positive definite)
            const double reg = 1e-12 * (a00 + a11 + a22);
            a00 += reg; a11 += reg; a22 += reg;
            const double l00 = sqrt(a00), l10 = a01 / l00, l20 = a02 / l00;
            const double l11 = sqrt(a11 - l10 * l10), l21 = (a12 - l20 * l10) / l11;
            const double l22 = sqrt(a22 - l20 * l20 - l21 * l21);
            const double y0 = b0 / l00, y1 = (b1 - l10 * y0) / l11, y2 = (b2 - l20 * y0 - l21 * y1) / l22;
            const double c2 = y2 / l22, c1 = (y1 - l21 * c2) / l11, c0 = (y0 - l10 * c1 - l20 * c2) / l00;
            // (a degenerate or non-finite system -- a converging chain whose differences vanish,
            // NaN nodes -- skips the mix: the cycle's output stands)
            if (isfinite(c0) && isfinite(c1) && isfinite(c2) && reg > 0.0) {
              double* dm = tabm(b_dst);
              double* dc = tabc(b_dst);
              for (int s = 0; s < S; ++s)
                for (int k = j0 + tid; k < j1; k += TH) {
                  const size_t o = (size_t)s * n_a + k;
                  const double w1 = load_f64_agent(W1 + o), w2 = load_f64_agent(W2 + o);
                  const double w3 = load_f64_agent(W3 + o), w4 = load_f64_agent(W4 + o);
                  const double cn = w4 - ((c0 * (w2 - w1) + c1 * (w3 - w2)) + c2 * (w4 - w3));
                  store_f64_agent(&dm[(size_t)s * n1 + k + 1], a_grid[k] + cn);   // AS:1499
                  store_f64_agent(&dc[(size_t)s * n1 + k + 1], cn);
                }
              if (tid == 0) st.moved = 1;
              if (!plain_barrier()) return;
            }
          }
          ++n;
        }
        if (tid == 0) {
          st.n = n;
          if (!converged) st.status |= 1;
        }
        __syncthreads();
        final_buf = st.buf[n & 1];
        // an extrapolated solve that ended in NaN: the whole solve again, plain (ge.hip)
        if (!(st.moved && st.nan_stop)) break;
        if (tid == 0) {
          st.extrap = 0;
          st.status &= ~1;
        }
        __syncthreads();
      }
      if (tid == 0) {
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
        st.t_egm += tn - tp;
        st.cyc_sum += st.n;
        // buffer roles: prev <- cur, cur <- the solve's final tables, the freed ones ping-pong
        const int fb = final_buf;
        const int other = st.buf[0] == fb ? st.buf[1] : st.buf[0];
        const int old_prev = st.buf[3];
        st.buf[3] = st.buf[2];
        st.buf[2] = fb;
        st.buf[0] = other;
        st.buf[1] = old_prev;
      }
      __syncthreads();
      // ---- lottery of the own columns on the final tables (hist.hip hist_lottery_kernel) ----
      tp = __builtin_amdgcn_s_memrealtime();
      ge_lottery_fn<SMAX, NW>(S, n_a, j0, j1, a_grid, tabm(st.buf[2]), tabc(st.buf[2]), R, st.steps > 0, LO, WL,
                              g.pull != 0);
      // ---- the distribution's start (own columns) ----
      if (st.fresh_mass) {
        const double u0 = 1.0 / ((double)S * n_a);
        for (int s = 0; s < S; ++s)
          for (int k = j0 + tid; k < j1; k += TH) X[(size_t)s * n_a + k] = u0;
      } else if (warm) {
        for (int s = 0; s < S; ++s)
          for (int k = j0 + tid; k < j1; k += TH) {
            const size_t o = (size_t)s * n_a + k;
            const double x = X[o];
            if (secant) X[o] = theta == 0.0 ? x : x + theta * (x - PX[o]);
            PX[o] = x;
          }
      }
      __syncthreads();
      if (tid == 0) {
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
        st.t_lot += tn - tp;
        tp = tn;
      }
    }
    // ---- the stationary distribution: BiCGSTAB on (I - T) mass = 0 ----
    int mv;
    {
      HkArgs hk;
      hk.G = G; hk.S = S; hk.n_a = n_a; hk.cap = g.cap; hk.w = w; hk.j0 = j0; hk.j1 = j1;
      hk.LO = to_global((const int*)LO); hk.WL = to_global((const double*)WL); hk.X = to_global(X);
      hk.Pg = to_global(g.pg + row0); hk.Vg = to_global((double*)nullptr);
      hk.slab_cl = to_global(g.slab + (size_t)lc * G * 2 * g.cap);
      hk.span_cl = to_global(g.span + (size_t)lc * G * SMAX * 4);
      hk.ctr = to_global(ctr); hk.gran = to_global(gran); hk.Pc = to_global(g.P + (size_t)cal * S * S);
      hk.max_iter = g.max_hist; hk.err = to_global(g.err);
      hk.tol = st.htol;
      hk.stop_ctr = to_global((const unsigned*)(g.stop_at > 0 ? g.done_ctr : nullptr));
      hk.stop_at = (unsigned)g.stop_at;
      hk.Qg = to_global(g.qb + row0);
      hk.Ainv = to_global(g.ainv + (size_t)cal * S * (n_a + 1));
      hk.lottery_fresh = true;
      mv = g.pull ? hk_solve_inlined<SMAX, KC, TH, true>(hk, &nb, &ne)
                  : hk_solve_isolated<SMAX, KC, TH, false, (KC == 1 || kGeFuseAKc2) && kGeFuseA>(hk, &nb, &ne);
    }
    if (mv == -1) return;
    if (tid == 0) {
      const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
      st.t_hist += tn - tp;
      tp = tn;
    }
    if (mv <= -2) {   // rebalancing stop inside the solve: resume it in the next launch
      if (tid == 0) {
        st.its_sum += -mv - 2;
        st.in_hist = 1;
        if (w == 0) __hip_atomic_fetch_add(to_global(g.done_ctr + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      stopped = true;
      break;
    }
    if (tid == 0) st.in_hist = 0;
    // ---- K_s = sum mass a over the cluster ----
    double part = 0.0;
    for (int k = j0 + tid; k < j1; k += TH) {
      double ms = 0.0;
      for (int s = 0; s < S; ++s) ms += X[(size_t)s * n_a + k];
      part += ms * a_grid[k];
    }
    {
      double v[1] = {part};
      if (!ge_reduce<TH>(gran, G, w, ne, v, 1, 0u, s_part, s_res, &s_flag, g.err)) return;
    }
    const bool fin = st.final_ks != 0;   // (set in an earlier pass; never cleared: the loop ends here)
    if (tid == 0) {
      const double Ks = s_res[0];
      if (w == 0 && st.steps < kGeEvLog && !fin) {
        double* ev = g.out_evlog + ((size_t)cal * kGeEvLog + st.steps) * kGeEvRec;
        ev[0] = st.rs.x;
        ev[1] = (Ks - st.Kd) / st.Kd;
        ev[2] = (double)st.n;
        ev[3] = (double)mv;
        ev[4] = (double)st.loose;
        ev[5] = (double)(__builtin_amdgcn_s_memrealtime() - st.t_ev0) * 0.01;
      }
      st.its_sum += mv;
      if (mv >= g.max_hist) st.status |= 2;
    }
    if (fin) {   // the full-tolerance re-solve of the last evaluation: K_s only
      if (tid == 0) st.Ks = s_res[0];
      __syncthreads();
      break;
    }
    if (tid == 0) {
      const double Ks = s_res[0];
      st.r_prev = st.r_cur;
      st.r_cur = st.rs.x;
      const double f = Ks - st.Kd;
      st.refine = (st.loose && !(fabs(f) >= kGeSignMargin * st.Kd)) ||   // NaN: refine
                  (st.adapt && !(fabs(f) >= kGeAdaptMargin * st.htol * st.Kd));
      if (!st.refine) {
        st.rs.update(f, st.Kd);
        st.fmin = fmin(st.fmin, fabs(f) / st.Kd);
      }
      st.Ks = Ks;
      ++st.steps;
      // a search that ends on an evaluation at looser tolerances (a loose bracketing
      // one, or Brent's at the adaptive distribution tolerance) reports K_s only after that r is
      // evaluated again at egm_tol / hist_tol (one more pass, warm from its tables and mass: a few
      // cycles and matvecs; searches normally end on full-tolerance evaluations near the root)
      if (st.rs.done && (st.adapt || st.loose)) st.final_ks = 1;
      st.t_k += __builtin_amdgcn_s_memrealtime() - tp;
    }
    __syncthreads();
  }
  if (stopped) {
    if (w == 0 && tid == 0) {
      st.t0 = __builtin_amdgcn_s_memrealtime() - st.t0;
      g.saved[cal] = st;
      g.out_done[cal] = 0;
    }
    return;
  }
  if (w == 0 && tid == 0) {
    __hip_atomic_fetch_add(to_global(g.done_ctr), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g.out_done[cal] = 1;
    const double r = st.rs.x, a = cd.alpha, d = cd.delta;
    g.out_r[cal] = r;
    g.out_K[cal] = pow(a / (r + d), 1.0 / (1.0 - a));
    g.out_Ks[cal] = st.Ks;
    g.out_steps[cal] = st.steps;
    g.out_cyc[cal] = (int)min(st.cyc_sum, 0x7fffffffll);
    g.out_its[cal] = (int)min(st.its_sum, 0x7fffffffll);
    g.out_status[cal] = st.status | (st.rs.done ? 0 : 4);
    double* pf = g.out_prof + (size_t)cal * kGeProf;
    pf[0] = st.t_egm * 0.01;
    pf[1] = st.t_lot * 0.01;
    pf[2] = st.t_hist * 0.01;
    pf[3] = st.t_k * 0.01;
    pf[4] = (__builtin_amdgcn_s_memrealtime() - st.t0) * 0.01;
    pf[5] = (double)st.cyc_sum;
    pf[6] = (double)st.its_sum;
    pf[7] = (double)st.steps;
  }
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
struct GePlan {
  int G = 0, nj = 0, kc = 0, smax = 0, sc = 0, cap = 0, blocks = 0, th = 0;
  size_t lds = 0;
  const void* fn = nullptr;
};

template <int SMAX, int SC, int KC, int TH>
static const void* ge_fn() {
  return reinterpret_cast<const void*>(ge_cluster_kernel<SMAX, SC, KC, TH>);
}

// Launch shape of the device-resident search for (n_cal, S, n_a): every calibration's
// cluster resident at once (n_cal G workgroups, one per CU, within the handle's CU limit).
static bool ge_make_plan(aiy_handle* h, int n_cal, int S, int n_a, GePlan& p) {
  if (S < 1 || S > kGeSmax || n_a < 2 || n_cal < 1) return false;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus < 1) return false;
  if (h->cu_limit > 0) cus = std::min(cus, h->cu_limit);
  const int g_min = (n_a + 2 * 512 - 1) / (2 * 512);
  // the cluster reductions (ge_reduce, hist_bicg.h) read at most kHcMaxG workgroups
  if (g_min > kHcMaxG || g_min > cus) return false;
  const int g_cap = h->hist_cluster_cap > 0 ? h->hist_cluster_cap : 32;
  int G = std::max(g_min, std::min(std::min(g_cap, kHcMaxG), cus / n_cal));
  G = std::min(G, n_a);
  p.nj = (n_a + G - 1) / G;
  p.G = (n_a + p.nj - 1) / p.nj;
  if (p.G > kHcMaxG) return false;
  if (p.nj > kGeMaxTiles * kTile) return false;
  if ((long long)p.G * n_cal > cus) return false;
  p.th = 512;
  const int th = p.th;
  p.kc = p.nj <= th ? 1 : 2;
  p.smax = S == 7 ? 7 : 8;   // the Table II shape: exact state count (fewer registers in the solve)
  p.sc = S == 7 ? 7 : 0;
  if (p.sc == 7) p.fn = p.kc == 1 ? ge_fn<7, 7, 1, 512>() : ge_fn<7, 7, 2, 512>();
  else p.fn = p.kc == 1 ? ge_fn<8, 0, 1, 512>() : ge_fn<8, 0, 2, 512>();
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, p.fn) != hipSuccess) return false;
  int lds_dev = 0;
  if (hipDeviceGetAttribute(&lds_dev, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device) != hipSuccess)
    return false;
  const size_t lds_total = std::min<size_t>(kHcLdsTotal, (size_t)lds_dev);
  const size_t stat = fa.sharedSizeBytes;
  if (stat + 4096 >= lds_total) return false;
  p.lds = (lds_total - stat - 1024) / 256 * 256;
  const size_t vbytes = (size_t)p.kc * p.smax * th * sizeof(double);   // BiCGSTAB v behind the spans
  const size_t egm_lds = ge_egm_lds<8>();
  if (p.lds < egm_lds || p.lds <= vbytes + 4096) return false;
  p.cap = (int)((p.lds - vbytes) / sizeof(double));
  p.blocks = (p.G * n_cal + 7) / 8 * 8;
  return true;
}

struct GeScratch {
  size_t tab, mass, pmass, pg, qb, ainv, lo, wlo, slab, span, ctr, gran, ids, saved, resume, done, err, cal, outd, outi, prof,
      evlog, aah, bytes;
};
// Per-calibration arrays (kept across the rebalancing launches) first, then the per-launch
// cluster arrays sized for the most workgroups any launch can hold (cus) and the largest span
// capacity (cap_max doubles).
static GeScratch ge_scratch_layout(int n_cal, int S, int n_a, int cus, int cap_max) {
  GeScratch L;
  size_t o = 0;
  auto take = [&](size_t bytes) { const size_t at = o; o += (bytes + 255) / 256 * 256; return at; };
  const size_t pts = (size_t)n_cal * S * n_a;
  L.tab = take((size_t)n_cal * kGeBufs * 2 * S * (n_a + 1) * sizeof(double));
  L.mass = take(pts * 8); L.pmass = take(pts * 8); L.pg = take(pts * 8); L.qb = take(pts * 8);
  L.ainv = take((size_t)n_cal * S * (n_a + 1) * sizeof(int));
  L.lo = take(pts * 4); L.wlo = take(pts * 8);
  L.slab = take((size_t)cus * 2 * cap_max * sizeof(double));
  L.span = take((size_t)cus * 8 * 4 * sizeof(int));
  L.ctr = take((size_t)n_cal * kHcCtrStride * sizeof(unsigned));
  L.gran = take((size_t)cus * 2 * kHcRedRec * sizeof(unsigned long long));
  L.ids = take((size_t)n_cal * sizeof(int));
  L.saved = take((size_t)n_cal * sizeof(GeState));
  L.resume = take((size_t)n_cal * sizeof(int));
  L.done = take((size_t)n_cal * sizeof(int));
  L.err = take(256);
  L.cal = take((size_t)n_cal * sizeof(GeCalDev));
  L.outd = take((size_t)n_cal * 3 * sizeof(double));
  L.outi = take((size_t)n_cal * 4 * sizeof(int));
  L.prof = take((size_t)n_cal * kGeProf * sizeof(double));
  L.evlog = take((size_t)n_cal * kGeEvLog * kGeEvRec * sizeof(double));
  L.aah = take((size_t)n_cal * kGeAaHist * S * n_a * sizeof(double));
  L.bytes = o;
  return L;
}

// The whole search on device when the shape allows it (1: done; 0: not applicable, the caller
// runs the host-driven loop; < 0: error).  With rebalancing (AIY_OPT_GE_REBALANCE = q > 0,
// default 55) a launch whose calibrations are more than 4 stops every cluster at its next
// evaluation boundary once q % of them have finished, and the unfinished ones are launched
// again with the freed compute units (a cluster's time scales with its columns per CU): with
// q = 50 the 24 Table II cells run as 24 x 10, then ~12 x 21, ~6 x 32, ~3 x 32 workgroups.
int32_t ge_stationary_resident(aiy_handle* h, const aiy_stationary_model* M, const aiy_ge_options* o, double* r_out,
                               double* K_out, double* Ks_out, int32_t* steps_out, int32_t* cyc_out,
                               int32_t* its_out, int32_t* status_out, hipStream_t st) {
  if (!h->ge_resident || o->accel >= 0) return 0;   // BiCGSTAB distribution solves only
  const int n_cal = M->n_cal, S = M->S, n_a = M->n_a;
  GePlan p0;
  if (!ge_make_plan(h, n_cal, S, n_a, p0)) return 0;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) return 0;
  if (h->cu_limit > 0) cus = std::min(cus, h->cu_limit);
  const int cap_max = (int)(kHcLdsTotal / sizeof(double));
  const GeScratch L = ge_scratch_layout(n_cal, S, n_a, cus, cap_max);
  if (L.bytes > h->ge_cap) {
    if (h->d_ge) (void)hipFree(h->d_ge);
    h->d_ge = nullptr;
    h->ge_cap = 0;
    AIY_HIP(h, hipMalloc(&h->d_ge, L.bytes));
    h->ge_cap = L.bytes;
  }
  char* base = static_cast<char*>(h->d_ge);
  std::vector<GeCalDev> cals(n_cal);
  for (int c = 0; c < n_cal; ++c) {
    cals[c].alpha = M->alpha[c];
    cals[c].delta = M->delta[c];
    cals[c].disc = M->disc[c];
    cals[c].r_lo = o->r_lo ? o->r_lo[c] : -0.5 * M->delta[c];
    cals[c].r_hi = o->r_hi ? o->r_hi[c] : 1.0 / M->disc[c] - 1.0 - 1e-9;
  }
  GeRun g;
  g.n_cal = n_cal; g.S = S; g.n_a = n_a;
  g.a_grid = M->a_grid; g.P = M->P; g.lab = M->lab; g.beta = M->beta; g.crra = M->crra;
  g.cal = reinterpret_cast<const GeCalDev*>(base + L.cal);
  g.method = o->method; g.r_tol = o->r_tol; g.egm_tol = o->egm_tol; g.hist_tol = o->hist_tol;
  g.max_steps = o->max_steps;
  g.max_cyc = o->max_egm_cycles > 0 ? o->max_egm_cycles : 5000;
  g.max_hist = o->max_hist_iter > 0 ? o->max_hist_iter : 200000;
  g.warm_hist = o->warm_hist != 0; g.warm_egm = o->warm_egm != 0;
  g.secant = o->secant_start != 0; g.loose = o->loose_bracket != 0; g.extrap = o->egm_extrapolate != 0;
  g.extrap_period = h->ge_extrap_period;
  g.aa_period = o->egm_extrapolate != 0 ? h->ge_anderson : 0;   // (with the EGM acceleration on)
  g.aah = reinterpret_cast<double*>(base + L.aah);
  g.logsec = h->ge_logsec;
  g.tab = reinterpret_cast<double*>(base + L.tab);
  g.mass = reinterpret_cast<double*>(base + L.mass);
  g.pmass = reinterpret_cast<double*>(base + L.pmass);
  g.pg = reinterpret_cast<double*>(base + L.pg);
  g.qb = reinterpret_cast<double*>(base + L.qb);
  g.ainv = reinterpret_cast<int*>(base + L.ainv);
  g.pull = h->hist_pull;
  g.loose_hist = std::pow(10.0, -(double)h->ge_loose_hist);
  g.lo = reinterpret_cast<int*>(base + L.lo);
  g.wlo = reinterpret_cast<double*>(base + L.wlo);
  g.slab = reinterpret_cast<double*>(base + L.slab);
  g.span = reinterpret_cast<int*>(base + L.span);
  g.ctr = reinterpret_cast<unsigned*>(base + L.ctr);
  g.gran = reinterpret_cast<unsigned long long*>(base + L.gran);
  int* d_ids = reinterpret_cast<int*>(base + L.ids);
  int* d_resume = reinterpret_cast<int*>(base + L.resume);
  g.cal_ids = d_ids;
  g.saved = reinterpret_cast<GeState*>(base + L.saved);
  g.resume = d_resume;
  g.out_done = reinterpret_cast<int*>(base + L.done);
  g.err = reinterpret_cast<unsigned*>(base + L.err);
  g.done_ctr = g.err + 1;
  double* outd = reinterpret_cast<double*>(base + L.outd);
  int* outi = reinterpret_cast<int*>(base + L.outi);
  g.out_r = outd; g.out_K = outd + n_cal; g.out_Ks = outd + 2 * n_cal;
  g.out_steps = outi; g.out_cyc = outi + n_cal; g.out_its = outi + 2 * n_cal; g.out_status = outi + 3 * n_cal;
  g.out_prof = reinterpret_cast<double*>(base + L.prof);
  g.out_evlog = reinterpret_cast<double*>(base + L.evlog);
  AIY_HIP(h, hipMemsetAsync(g.out_evlog, 0, (size_t)n_cal * kGeEvLog * kGeEvRec * sizeof(double), st));
  AIY_HIP(h, hipMemcpyAsync(base + L.cal, cals.data(), sizeof(GeCalDev) * n_cal, hipMemcpyHostToDevice, st));
  AIY_HIP(h, hipMemsetAsync(d_resume, 0, (size_t)n_cal * sizeof(int), st));
  AIY_HIP(h, hipMemsetAsync(g.out_done, 0, (size_t)n_cal * sizeof(int), st));
  for (hipEvent_t& e : h->ge_ev)
    if (!e) AIY_HIP(h, hipEventCreate(&e));
  std::vector<int> active(n_cal), done(n_cal, 0), resume(n_cal, 0);
  for (int c = 0; c < n_cal; ++c) active[c] = c;
  h->ge_rounds = 0;
  h->ge_mid_stops = 0;
  while (!active.empty()) {
    const int n = (int)active.size();
    GePlan p;
    if (!ge_make_plan(h, n, S, n_a, p)) return fail(h, AIY_ERR_STATE, "device-resident GE: no plan for %d calibrations", n);
    if (hipFuncSetAttribute(p.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess) {
      (void)hipGetLastError();
      if (h->ge_rounds == 0) return 0;
      return fail(h, AIY_ERR_STATE, "device-resident GE: dynamic LDS attribute");
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, p.fn, p.th, p.lds) != hipSuccess || per_cu < 1) {
      (void)hipGetLastError();
      if (h->ge_rounds == 0) return 0;
      return fail(h, AIY_ERR_STATE, "device-resident GE: occupancy query");
    }
    g.G = p.G; g.nj = p.nj; g.cap = p.cap; g.n_work = n * p.G;
    g.stop_at = (h->ge_rebalance > 0 && n > 4) ? std::max(1, (n * h->ge_rebalance + 99) / 100) : 0;
    std::vector<int> res_h(n_cal);
    for (int c = 0; c < n_cal; ++c) res_h[c] = resume[c];
    AIY_HIP(h, hipMemcpyAsync(d_ids, active.data(), sizeof(int) * n, hipMemcpyHostToDevice, st));
    AIY_HIP(h, hipMemcpyAsync(d_resume, res_h.data(), sizeof(int) * n_cal, hipMemcpyHostToDevice, st));
    AIY_HIP(h, hipMemsetAsync(g.ctr, 0, (size_t)n * kHcCtrStride * sizeof(unsigned), st));
    AIY_HIP(h, hipMemsetAsync(g.gran, 0, (size_t)n * 2 * p.G * kHcRedRec * sizeof(unsigned long long), st));
    AIY_HIP(h, hipMemsetAsync(g.err, 0, 256, st));
    void* args[] = {&g};
    AIY_HIP(h, hipEventRecord(h->ge_ev[0], st));
    AIY_HIP(h, hipLaunchKernel(p.fn, dim3(p.blocks), dim3(p.th), args, p.lds, st));
    AIY_HIP(h, hipEventRecord(h->ge_ev[1], st));
    unsigned errw[3] = {0, 0, 0};   // error, finished clusters, clusters stopped inside a solve
    AIY_HIP(h, hipMemcpyAsync(errw, g.err, sizeof(errw), hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipMemcpyAsync(done.data(), g.out_done, sizeof(int) * n_cal, hipMemcpyDeviceToHost, st));
    AIY_HIP(h, hipStreamSynchronize(st));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->ge_ev[0], h->ge_ev[1]) == hipSuccess) {
      h->ge_ms_sum += ms;
      h->ge_launches += 1;
    }
    ++h->ge_rounds;
    h->ge_mid_stops += errw[2];
    const unsigned err = errw[0];
    if (err == 1u)
      return fail(h, AIY_ERR_STATE, "device-resident GE: cluster barrier timed out (workgroups not co-resident?)");
    if (err) return fail(h, AIY_ERR_STATE, "device-resident GE: histogram shape does not fit (error %u)", err);
    std::vector<int> next;
    for (int c : active) {
      if (!done[c]) {
        next.push_back(c);
        resume[c] = 1;
      }
    }
    if ((int)next.size() == n && g.stop_at > 0)
      return fail(h, AIY_ERR_STATE, "device-resident GE: a rebalancing launch finished no calibration");
    active.swap(next);
  }
  std::vector<double> hd(3 * (size_t)n_cal);
  std::vector<int> hi(4 * (size_t)n_cal);
  AIY_HIP(h, hipMemcpyAsync(hd.data(), outd, sizeof(double) * 3 * n_cal, hipMemcpyDeviceToHost, st));
  AIY_HIP(h, hipMemcpyAsync(hi.data(), outi, sizeof(int) * 4 * n_cal, hipMemcpyDeviceToHost, st));
  h->ge_prof.assign((size_t)n_cal * kGeProf, 0.0);
  h->ge_evlog.assign((size_t)n_cal * kGeEvLog * kGeEvRec, 0.0);
  AIY_HIP(h, hipMemcpyAsync(h->ge_evlog.data(), g.out_evlog, sizeof(double) * kGeEvLog * kGeEvRec * n_cal,
                            hipMemcpyDeviceToHost, st));
  AIY_HIP(h, hipMemcpyAsync(h->ge_prof.data(), g.out_prof, sizeof(double) * kGeProf * n_cal, hipMemcpyDeviceToHost,
                            st));
  AIY_HIP(h, hipStreamSynchronize(st));
  long long cyc = 0, its = 0;
  int steps = 0;
  for (int c = 0; c < n_cal; ++c) {
    r_out[c] = hd[c];
    K_out[c] = hd[n_cal + c];
    if (Ks_out) Ks_out[c] = hd[2 * n_cal + c];
    steps = std::max(steps, hi[c]);
    cyc += hi[n_cal + c];
    its += hi[2 * n_cal + c];
    if (status_out) status_out[c] = hi[3 * n_cal + c];
    h->ge_points += (double)hi[2 * n_cal + c] * S * n_a;
    h->ge_egm_cycles += hi[n_cal + c];
  }
  if (steps_out) *steps_out = steps;
  if (cyc_out) *cyc_out = (int32_t)std::min<long long>(cyc, 0x7fffffff);
  if (its_out) *its_out = (int32_t)std::min<long long>(its, 0x7fffffff);
  return 1;
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_ge_resident_plan(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_a, int32_t* out4) {
  if (!h || !out4) return AIY_ERR_ARG;
  GePlan p;
  if (!h->ge_resident || !ge_make_plan(h, n_cal, S, n_a, p)) {
    out4[0] = out4[1] = out4[2] = out4[3] = 0;
    return 0;
  }
  out4[0] = p.G;
  out4[1] = p.nj;
  out4[2] = p.kc;
  out4[3] = p.blocks;
  return 1;
}

// Launches of the last device-resident search (1 + rebalancing relaunches) and how many of
// its cluster stops happened inside a distribution solve (resumed from the iterate).
extern "C" int32_t aiy_ge_last_rounds(aiy_handle* h, int32_t* launches, int32_t* mid_solve_stops) {
  if (!h) return AIY_ERR_ARG;
  if (launches) *launches = h->ge_rounds;
  if (mid_solve_stops) *mid_solve_stops = h->ge_mid_stops;
  return AIY_OK;
}

extern "C" int32_t aiy_ge_launch_stats(aiy_handle* h, double* ms_sum, int64_t* launches, double* point_matvecs,
                                       double* egm_cycles, int32_t reset) {
  if (!h) return AIY_ERR_ARG;
  if (ms_sum) *ms_sum = h->ge_ms_sum;
  if (launches) *launches = h->ge_launches;
  if (point_matvecs) *point_matvecs = h->ge_points;
  if (egm_cycles) *egm_cycles = h->ge_egm_cycles;
  if (reset) {
    h->ge_ms_sum = 0.0;
    h->ge_launches = 0;
    h->ge_points = 0.0;
    h->ge_egm_cycles = 0.0;
  }
  return AIY_OK;
}

// Per-evaluation log of the last device-resident search (measurement hook): out[(c * 32 + e)
// * 6 + k] for evaluation e of calibration c, k = r, (K_s - K_d) / K_d, EGM cycles, matvecs,
// loose (1: a bracketing evaluation at the loose tolerances), microseconds from the
// evaluation's start (workgroup 0's clock; a solve split by a rebalancing stop includes the
// relaunch gap, its matvecs count the resumed part only); rows past
// a calibration's evaluations are zero.  Returns the calibrations written.  Host-only.
extern "C" int32_t aiy_ge_last_eval_log(aiy_handle* h, double* out, int32_t n_cal) {
  if (!h || !out || n_cal < 0) return AIY_ERR_ARG;
  const int have = (int)(h->ge_evlog.size() / (kGeEvLog * kGeEvRec));
  const int n = std::min(have, (int)n_cal);
  std::copy(h->ge_evlog.begin(), h->ge_evlog.begin() + (size_t)n * kGeEvLog * kGeEvRec, out);
  return n;
}

// Per-calibration profile of the last device-resident GE launch (measurement hook):
// out[c * 8 + k] for k = EGM, lottery, distribution solve, K reduction + search, whole
// search (microseconds, workgroup 0's clock), EGM cycles, matvecs, evaluations.  Returns
// the calibrations written (<= n_cal).  Host-only.
extern "C" int32_t aiy_ge_last_profile(aiy_handle* h, double* out, int32_t n_cal) {
  if (!h || !out || n_cal < 0) return AIY_ERR_ARG;
  const int have = (int)(h->ge_prof.size() / kGeProf);
  const int n = std::min(have, (int)n_cal);
  std::copy(h->ge_prof.begin(), h->ge_prof.begin() + (size_t)n * kGeProf, out);
  return n;
}
