// Host-side internals shared by the libaiyagari translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/aiyagari.h"

struct aiy_handle {
  int device = 0;
  std::string err;
  // EGM convergence bookkeeping: [n_cal][3] distance slots (bit patterns of
  // non-negative doubles, atomicMax) and [n_cal] last completed cycle.
  unsigned long long* d_dist = nullptr;
  int* d_last = nullptr;
  size_t egm_cap = 0;
  int* d_egm_hint = nullptr;         // EGM row hints [work item][rows x S] (egm.hip)
  double* d_egm_aa = nullptr;        // Anderson mixing of the host-driven EGM solve (egm.hip): the c
  size_t egm_aa_cap = 0;             //   tables of the last 5 cycles + Gram partials + gamma (doubles)
  size_t egm_hint_cap = 0;           // ints
  unsigned long long egm_hint_sig = ~0ull;   // shape the hints belong to
  // host pinned mirrors
  unsigned long long* h_dist = nullptr;
  int* h_last = nullptr;
  // panel: per-block partial sums
  double* d_partials = nullptr;
  unsigned* d_ticket = nullptr;      // last-block-done counter of the period kernel
  size_t partials_cap = 0;
  hipStream_t cap_stream = nullptr;  // hipGraph capture stream
  bool use_graphs = true;
  // histogram: per-calibration sup-norm slots [n_cal][3] + sums of K
  unsigned long long* d_hdist = nullptr;
  double* d_K = nullptr;
  int* d_hlast = nullptr;
  size_t hist_cap = 0;
  bool hist_fused = false;           // AIY_OPT_HIST_FUSED
  bool hist_resident = true;         // AIY_OPT_HIST_RESIDENT (hist_resident.hip)
  int hist_cluster_cap = 0;          // AIY_OPT_HIST_CLUSTER: max workgroups per calibration (0: 32)
  int hist_accel = 0;                // AIY_OPT_HIST_ACCEL: Aitken period of the resident histogram (0: off)
  int hist_krylov = 0;               // AIY_OPT_HIST_KRYLOV: resident histogram solves by BiCGSTAB
  int res_shape_stream = 1;          // AIY_OPT_RESIDENT_SHAPE_STREAM: shape of the HBM-streaming form (-1: res_shape)
  int hist_pull = 0;                 // AIY_OPT_HIST_PULL: BiCGSTAB matvecs of S <= 8 by the lottery pull
  int ge_loose_hist = 8;             // AIY_OPT_GE_LOOSE_HIST: loose-bracketing histogram tolerance 10^-value
  // per-calibration tolerances for one call (aiy_ge_stationary's loose bracketing); null: the
  // scalar tolerance of the call.  Device arrays [n_cal]; egm_tolh: the host copy.
  const double* egm_tolv = nullptr;
  const double* egm_tolh = nullptr;
  const double* hist_tolv = nullptr;
  int egm_extrap = 0;                // aiy_ge_stationary: extrapolate the EGM iterates (egm.hip)
  void* d_hcd = nullptr;             // resident histogram: stored differences (Aitken)
  size_t hc_dcap = 0;
  void* d_hc = nullptr;              // resident histogram: slabs, spans, counters, distances
  size_t hc_cap = 0;
  hipEvent_t hc_ev[2] = {nullptr, nullptr};
  double hc_ms_sum = 0.0;
  long long hc_launches = 0;
  // device-resident GE search (ge_resident.hip)
  bool ge_resident = false;          // AIY_OPT_GE_RESIDENT
  int cu_limit = 0;                  // AIY_OPT_CU_LIMIT: compute units resident launches may fill (0: all)
  int ge_rebalance = 55;             // AIY_OPT_GE_REBALANCE: % finished that stops a launch (0: one launch)
  int ge_rounds = 0;                 // launches of the last device-resident search
  int ge_mid_stops = 0;              // of its clusters, those stopped inside a distribution solve
  int ge_extrap_period = 32;         // AIY_OPT_GE_EXTRAP_PERIOD: EGM cycles between extrapolation checks
  int ge_anderson = 12;              // AIY_OPT_GE_ANDERSON: EGM cycles between Anderson mixes (0: off)
  int ge_logsec = 2;                 // AIY_OPT_GE_LOGSEC: 0 off, 1 two-point log-secant bracketing, 2 also from one point (with loose bracketing)
  void* d_ge = nullptr;              // tables, masses, lottery, cluster sync of the launch
  size_t ge_cap = 0;
  hipEvent_t ge_ev[2] = {nullptr, nullptr};
  double ge_ms_sum = 0.0, ge_points = 0.0, ge_egm_cycles = 0.0;
  long long ge_launches = 0;
  std::vector<double> ge_prof;       // [n_cal][8] per-calibration profile of the last launch
  std::vector<double> ge_evlog;      // [n_cal][32][6] per-evaluation log of the last search
  // wealth statistics (stats.hip): sort / scan scratch
  void* d_stats = nullptr;
  size_t stats_cap = 0;
  unsigned long long* h_hdist = nullptr;
  double* h_K = nullptr;
  int* h_hlast = nullptr;
  // resident panel: tagged partial-sum granules + timeout word; option
  void* d_res_sync = nullptr;
  bool use_resident = true;
  int res_shape = 0;                 // resident workgroup shape (AIY_OPT_RESIDENT_SHAPE)
  hipEvent_t res_ev[2] = {nullptr, nullptr};   // bracket every resident launch (aiy_panel_launch_stats)
  double res_ms_sum = 0.0;
  long long res_launches = 0, res_periods = 0;
  unsigned res_epoch = 0;            // granule tag base of the next resident launch
  const void* res_occ_fn = nullptr;  // resident shape whose occupancy was last checked
  size_t res_occ_lds = 0;
  // block panel: per-calibration markets + seeds (device + pinned staging)
  void* d_blk = nullptr;
  void* h_blk = nullptr;
  size_t blk_cap = 0;
  bool res_stream = false;           // AIY_OPT_RESIDENT_STREAM
  // RCCL
  ncclComm_t comm = nullptr;
  bool comm_owned = false;           // created by aiy_comm_init (destroyed with the handle)
  int nranks = 1, rank = 0;
  // stream hand-off between calls that share the scratch above (aiy::use_stream)
  hipStream_t last_stream = nullptr;
  bool has_last_stream = false;
  hipEvent_t hand_ev = nullptr;
};

// EGM solve loop, cold (m_init == NULL) or warm-started (egm.hip).
int32_t aiy_egm_solve_impl(aiy_handle* h, const aiy_egm_dims* dims, const aiy_egm_inputs* in, double tol,
                           int32_t max_cycles, int32_t chunk, const double* m_init, const double* c_init,
                           double* work_m, double* work_c, double* m_out, double* c_out, int32_t* cycles_out,
                           double* dist_out, aiy_stream stream);

namespace aiy {

int32_t launch_build_index(aiy_handle* h, const double* x, long long n_rows, int n1, int* H, hipStream_t st);
int32_t hist_solve_resident(aiy_handle* h, int n_cal, int S, int n_a, const int* lo, const double* wlo,
                            const double* P, double tol, int max_iter, double* mass, int* d_iters, hipStream_t st);
int32_t hist_resident_plan(aiy_handle* h, int n_cal, int S, int n_a, int* out4);
int32_t ge_stationary_resident(aiy_handle* h, const aiy_stationary_model* M, const aiy_ge_options* o, double* r_out,
                               double* K_out, double* Ks_out, int32_t* steps_out, int32_t* cyc_out,
                               int32_t* its_out, int32_t* status_out, hipStream_t st);

inline int32_t fail(aiy_handle* h, int32_t code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  return code;
}

#define AIY_HIP(h, expr)                                                                 \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return aiy::fail((h), AIY_ERR_HIP, "%s failed: %s (%s:%d)", #expr,                \
                       hipGetErrorString(_e), __FILE__, __LINE__);                        \
  } while (0)

#define AIY_CHECK_LAUNCH(h) AIY_HIP(h, hipGetLastError())

inline hipStream_t as_stream(aiy_stream s) { return reinterpret_cast<hipStream_t>(s); }

// Calls that use handle scratch go through here with their stream: when the stream
// differs from the previous call's, the new stream waits (device-side) for everything
// already enqueued on the old one, so two streams never interleave on the scratch.
inline int32_t use_stream(aiy_handle* h, hipStream_t st) {
  if (h->has_last_stream && h->last_stream != st) {
    if (!h->hand_ev) AIY_HIP(h, hipEventCreateWithFlags(&h->hand_ev, hipEventDisableTiming));
    if (hipEventRecord(h->hand_ev, h->last_stream) == hipSuccess) {
      AIY_HIP(h, hipStreamWaitEvent(st, h->hand_ev, 0));
    } else {
      (void)hipGetLastError();   // the old stream is gone: nothing left to order against
    }
  }
  h->last_stream = st;
  h->has_last_stream = true;
  return AIY_OK;
}
#define AIY_USE_STREAM(h, st)                        \
  do {                                               \
    int32_t _r = aiy::use_stream((h), (st));         \
    if (_r) return _r;                               \
  } while (0)

// Measurement hooks: n launches, each bracketed by its own pair of HIP events on `st`,
// *ms = sum of the per-launch elapsed times (so inter-launch gaps are not charged to
// the kernel; comparable with rocprofv3 --kernel-trace durations).
template <class Launch>
int32_t time_launches(aiy_handle* h, hipStream_t st, int n, Launch launch, float* ms) {
  std::vector<hipEvent_t> ev(2 * (size_t)n, nullptr);
  int32_t rc = AIY_OK;
  for (auto& e : ev)
    if (hipEventCreate(&e) != hipSuccess) { rc = fail(h, AIY_ERR_HIP, "hipEventCreate failed"); break; }
  for (int k = 0; rc == AIY_OK && k < n; ++k) {
    if (hipEventRecord(ev[2 * k], st) != hipSuccess) rc = fail(h, AIY_ERR_HIP, "hipEventRecord failed");
    launch();
    if (hipGetLastError() != hipSuccess) rc = fail(h, AIY_ERR_HIP, "kernel launch failed");
    if (hipEventRecord(ev[2 * k + 1], st) != hipSuccess) rc = fail(h, AIY_ERR_HIP, "hipEventRecord failed");
  }
  if (rc == AIY_OK && hipStreamSynchronize(st) != hipSuccess) rc = fail(h, AIY_ERR_HIP, "hipStreamSynchronize failed");
  float tot = 0.f;
  for (int k = 0; rc == AIY_OK && k < n; ++k) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, ev[2 * k], ev[2 * k + 1]) != hipSuccess) rc = fail(h, AIY_ERR_HIP, "hipEventElapsedTime failed");
    tot += t;
  }
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  if (rc == AIY_OK) *ms = tot;
  return rc;
}

}  // namespace aiy
