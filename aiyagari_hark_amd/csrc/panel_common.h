// Device helpers shared by the panel kernels (panel.hip, panel_block.hip,
// panel_resident.hip) and the merged policy tables they read (panel_tab.hip).
#pragma once

#include "common.h"
#include "internal.h"

namespace aiy {

// ---------------------------------------------------------------------------------
// Merged policy tables ("cells", built once per history by aiy_panel_build).
//
// get_controls (AS:1326-1408) evaluates, for an agent of labour state l in aggregate
// state g, HARK's LinearInterpOnInterp1D of the employed sub-state s = 4 l + 2 g + 1:
//   c = (1 - alpha) f_{j-1}(m) + alpha f_j(m),
// two LinearInterp rows at the M nodes bracketing the period's Mnow.  Cell (l, g, j)
// merges the two rows' searched nodes x0[0..n), x1[0..n) (n = n_a: HARK searches
// x[:-1]) into one sorted list z[0..Z), Z = 2 n.  For q in (z[k-1], z[k]] both rows'
// lower_bounds are constant, so record k (k = 0..Z) holds both rows' brackets
//   {x0[i0-1], x0[i0]}, {c0[i0-1], c0[i0]}, {x1[i1-1], x1[i1]}, {c1[i1-1], c1[i1]}
// with i = max(lower_bound, 1).  A panel lookup is then ONE bracket-index load (BrkIdx
// encoding, common.h, over z) plus ONE 64-byte record -- instead of two index loads,
// two bracket searches and four pair loads -- with the reference's arithmetic unchanged.
// n_M == 1 (no aggregate dimension): row 1 = row 0.
//
// Per-calibration layout (bytes; sections 256-aligned):
//   rec [cells][Z + 1][4] double2 | z [cells][Z] double | idx [cells][buckets + 2] u64
// cells = 2 n_lab n_J (employed sub-states only) or 4 n_lab n_J (with the unemployed
// ones, Krusell-Smith mode), n_J = max(n_M - 1, 1); employed cell(l, g, j) =
// (2 l + g) n_J + (j - 1), unemployed cell(l, g, j) = (2 n_lab + 2 l + g) n_J + (j - 1).
// The index starts at z[2]: z[0] = z[1] is both rows' (1e-7, 1e-7) borrowing node
// (AS:1503-1504), far below the first real node.
// ---------------------------------------------------------------------------------
struct PanelTabGeom {
  int n, Z, n_J, n_cells;
  int shift, buckets;       // index over z: 2^(52 - shift) buckets per octave, kTabOctaves octaves
  long long rec_stride;     // double2 per cell
  long long z_stride;       // doubles per cell
  long long idx_stride;     // u64 per cell
  long long rec_off, z_off, idx_off, bytes;
};

constexpr int kTabOctaves = 12;
constexpr int kTabFirst = 2;   // first indexed node of z

__host__ __device__ inline long long tab_align(long long b) { return (b + 255) / 256 * 256; }

__host__ __device__ inline PanelTabGeom panel_tab_geom(int n_lab, int n_M, int n_a, bool unemployed = false) {
  PanelTabGeom g;
  g.n = n_a;
  g.Z = 2 * n_a;
  g.n_J = n_M > 1 ? n_M - 1 : 1;
  g.n_cells = (unemployed ? 4 : 2) * n_lab * g.n_J;
#ifndef AIY_TAB_LG_MAX
#define AIY_TAB_LG_MAX 13
#endif
  int lg = 4;                                  // ~n_a buckets per octave (~Z / 2), 16 .. 8192
  while (lg < AIY_TAB_LG_MAX && (1 << lg) < n_a) ++lg;
  g.shift = 52 - lg;
  g.buckets = kTabOctaves << lg;
  g.rec_stride = 4LL * (g.Z + 1);
  g.z_stride = g.Z;
  g.idx_stride = (long long)g.buckets + 2;
  g.rec_off = 0;
  g.z_off = tab_align((long long)g.n_cells * g.rec_stride * 16);
  g.idx_off = tab_align(g.z_off + (long long)g.n_cells * g.z_stride * 8);
  g.bytes = tab_align(g.idx_off + (long long)g.n_cells * g.idx_stride * 8);
  return g;
}

struct PanelTab {
  const double2* rec;
  const double* z;
  const unsigned long long* idx;
  PanelTabGeom g;
};
__host__ __device__ inline PanelTab panel_tab(const void* base, const PanelTabGeom& g) {
  const char* b = static_cast<const char*>(base);
  PanelTab t;
  t.rec = reinterpret_cast<const double2*>(b + g.rec_off);
  t.z = reinterpret_cast<const double*>(b + g.z_off);
  t.idx = reinterpret_cast<const unsigned long long*>(b + g.idx_off);
  t.g = g;
  return t;
}

// Per-cell header, staged in LDS: index base and last bucket, both rows' first node
// (the NaN guard of HARK's LinearInterp below the grid).
struct CellHdr {
  int base, last;
  double first0, first1;
};
__device__ __forceinline__ CellHdr cell_header(const PanelTab& T, int cell) {
  const unsigned long long* E = T.idx + (size_t)cell * T.g.idx_stride;
  const double2* r = T.rec + (size_t)cell * T.g.rec_stride;   // record 0 brackets nodes (0, 1) of both rows
  CellHdr h;
  h.last = (int)(long long)E[T.g.buckets];
  h.base = (int)(long long)E[T.g.buckets + 1];
  h.first0 = r[0].x;
  h.first1 = r[2].x;
  return h;
}

// Raw buffer resource over a table section (32-bit byte offsets: one address VGPR per
// lookup, the four record loads share it through immediate offsets).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tab_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(unsigned)bytes, 0x00020000);
}
__device__ __forceinline__ unsigned long long buf_u64(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(unsigned long long, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ double2 buf_f64x2(__amdgpu_buffer_rsrc_t r, unsigned off, int imm) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, imm, 0));
}

#ifdef AIY_DIAG_PHASES
__device__ unsigned diag_search_iters;   // diagnostic build only: wave search-loop trips
#endif

// c = cFunc(m, Mnow) for the NA agents of one lane, in lock step so the index loads,
// the rare searches and the record loads of all NA agents overlap.  Agent k uses cell
// cell[k] whose header is hdr[hidx[k]] (LDS; read where needed, not held in registers).
// BLEND = false: one row (n_M == 1).  Every load is unconditional and BLEND is a
// compile-time choice: a data-dependent branch between the loads makes the compiler
// wait for each agent's record before issuing the next (measured: 8 serial round trips).
// Quad-cooperative record loads (QUAD = true; the four lanes of every quad must be
// active).  The per-lane pattern -- four 16-byte loads of the lane's own record --
// touches 64 cache lines per load instruction; here the quad loads one agent's record
// per instruction (lane q the q-th 16-byte chunk: 16 lines per instruction, the same
// instruction count) and a 4 x 4 transpose across the quad (two DPP exchange stages)
// hands every lane its own record.  Measured at configs[1]: 23.3 -> 21.2 us per period.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
  return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = dpp_u32<CTRL>((unsigned)b), hi = dpp_u32<CTRL>((unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int CTRL>
__device__ __forceinline__ double2 dpp_f64x2(double2 v) {
  return make_double2(dpp_f64<CTRL>(v.x), dpp_f64<CTRL>(v.y));
}
__device__ __forceinline__ double2 sel2(bool p, double2 a, double2 b) {
  return make_double2(p ? a.x : b.x, p ? a.y : b.y);
}
constexpr int kDppXor1 = 0xB1;   // quad_perm [1, 0, 3, 2]
constexpr int kDppXor2 = 0x4E;   // quad_perm [2, 3, 0, 1]
// t[r] = chunk q of agent r (lane q of the quad)  ->  t[c] = chunk c of agent q.
__device__ __forceinline__ void quad_transpose(double2 (&t)[4], int q) {
  const bool b0 = q & 1, b1 = q & 2;
  const double2 x0 = dpp_f64x2<kDppXor1>(t[0]), x1 = dpp_f64x2<kDppXor1>(t[1]);
  const double2 x2 = dpp_f64x2<kDppXor1>(t[2]), x3 = dpp_f64x2<kDppXor1>(t[3]);
  const double2 a0 = sel2(b0, x1, t[0]), a1 = sel2(b0, t[1], x0);
  const double2 a2 = sel2(b0, x3, t[2]), a3 = sel2(b0, t[3], x2);
  const double2 y0 = dpp_f64x2<kDppXor2>(a0), y1 = dpp_f64x2<kDppXor2>(a1);
  const double2 y2 = dpp_f64x2<kDppXor2>(a2), y3 = dpp_f64x2<kDppXor2>(a3);
  t[0] = sel2(b1, y2, a0);
  t[2] = sel2(b1, a2, y0);
  t[1] = sel2(b1, y3, a1);
  t[3] = sel2(b1, a3, y1);
}

template <int NA, bool BLEND, bool QUAD = false>
__device__ __forceinline__ void tab_policy_t(const PanelTab& T, const int (&cell)[NA], const CellHdr* hdr,
                                             const int (&hidx)[NA], const double (&m)[NA], double alpha,
                                             double (&c)[NA]) {
  const PanelTabGeom& g = T.g;
  const __amdgpu_buffer_rsrc_t ridx = tab_rsrc(T.idx, (long long)g.n_cells * g.idx_stride * 8);
  const __amdgpu_buffer_rsrc_t rrec = tab_rsrc(T.rec, (long long)g.n_cells * g.rec_stride * 16);
  int slot[NA], lo[NA], hi[NA];
  long long raw[NA];
  bool nx[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) slot[k] = brk_slot(g.shift, g.buckets, hdr[hidx[k]].base, m[k], raw[k]);
#ifdef AIY_DIAG_NO_INDEX
#pragma unroll
  for (int k = 0; k < NA; ++k) {   // diagnostic build only: record position from the bucket, no index load
    lo[k] = hi[k] = (int)((long long)slot[k] * g.Z / g.buckets);
    nx[k] = false;
  }
#else
  unsigned long long e[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) e[k] = buf_u64(ridx, (unsigned)(((long long)cell[k] * g.idx_stride + slot[k]) * 8));
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    const CellHdr& H = hdr[hidx[k]];
    const double z0 = H.first0 < H.first1 ? H.first0 : H.first1;
    const double z1 = H.first0 < H.first1 ? H.first1 : H.first0;
    brk_resolve(g.shift, g.buckets, H.base, H.last, g.Z, raw[k], e[k], m[k], z0, z1, lo[k], hi[k], nx[k]);
  }
#endif
#ifdef AIY_DIAG_NO_RECORD
#pragma unroll
  for (int k = 0; k < NA; ++k) c[k] = 0.9 * m[k] + 1e-30 * lo[k];   // diagnostic build only: no record load
  return;
#endif
  // Rare: buckets of >= 7 nodes (window to the end of z), truncated-field ties,
  // degenerate tables -- binary search over z.  The common case falls through with no
  // branch between the index trip and the record trip.
  bool more = false;
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    if (nx[k]) hi[k] = g.Z;
    more = more || (lo[k] < hi[k]);
  }
  while (more) {
    more = false;
#ifdef AIY_DIAG_PHASES
    if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(&diag_search_iters, 1u);
#endif
    double v[NA];
    int mid[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      mid[k] = lo[k] + ((hi[k] - lo[k]) >> 1);
      v[k] = lo[k] < hi[k] ? T.z[(size_t)cell[k] * g.z_stride + mid[k]] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      if (lo[k] < hi[k]) {
        if (v[k] < m[k]) lo[k] = mid[k] + 1; else hi[k] = mid[k];
        more = more || (lo[k] < hi[k]);
      }
    }
  }
  double2 p0[NA], p1[NA], p2[NA], p3[NA];
  if constexpr (QUAD && BLEND) {
    const int q = (int)(threadIdx.x & 3);
    const unsigned qo = 16u * (unsigned)q;
    double2 t[NA][4];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const unsigned off = (unsigned)(((long long)cell[k] * g.rec_stride + 4LL * lo[k]) * 16);
      t[k][0] = buf_f64x2(rrec, dpp_u32<0x00>(off) + qo, 0);   // agent of quad lane 0
      t[k][1] = buf_f64x2(rrec, dpp_u32<0x55>(off) + qo, 0);
      t[k][2] = buf_f64x2(rrec, dpp_u32<0xAA>(off) + qo, 0);
      t[k][3] = buf_f64x2(rrec, dpp_u32<0xFF>(off) + qo, 0);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      quad_transpose(t[k], q);
      p0[k] = t[k][0];
      p1[k] = t[k][1];
      p2[k] = t[k][2];
      p3[k] = t[k][3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const unsigned off = (unsigned)(((long long)cell[k] * g.rec_stride + 4LL * lo[k]) * 16);
      p0[k] = buf_f64x2(rrec, off, 0);
      p1[k] = buf_f64x2(rrec, off, 16);
      if constexpr (BLEND) {
        p2[k] = buf_f64x2(rrec, off, 32);
        p3[k] = buf_f64x2(rrec, off, 48);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    // HARK LinearInterp (AS:1512): alpha = (q - x_lo) / (x_hi - x_lo),
    // y = (1 - alpha) y_lo + alpha y_hi, NaN below the row's first node
    const double a0 = (m[k] - p0[k].x) / (p0[k].y - p0[k].x);
    const double v0 = (1.0 - a0) * p1[k].x + a0 * p1[k].y;
    const double f0 = (m[k] < hdr[hidx[k]].first0) ? __builtin_nan("") : v0;
    if constexpr (BLEND) {
      const double a1 = (m[k] - p2[k].x) / (p2[k].y - p2[k].x);
      const double v1 = (1.0 - a1) * p3[k].x + a1 * p3[k].y;
      const double f1 = (m[k] < hdr[hidx[k]].first1) ? __builtin_nan("") : v1;
      c[k] = (1 - alpha) * f0 + alpha * f1;                                     // LinearInterpOnInterp1D
    } else {
      c[k] = f0;
    }
  }
}

template <int NA, bool QUAD = false>
__device__ __forceinline__ void tab_policy(const PanelTab& T, const int (&cell)[NA], const CellHdr* hdr,
                                           const int (&hidx)[NA], const double (&m)[NA], double alpha, bool blend,
                                           double (&c)[NA]) {
  if (blend) tab_policy_t<NA, true, QUAD>(T, cell, hdr, hidx, m, alpha, c);
  else tab_policy_t<NA, false, QUAD>(T, cell, hdr, hidx, m, alpha, c);
}

// The period's M bracket (LinearInterpOnInterp1D: clip(searchsorted(Mgrid, M), 1,
// n_M - 1)) as the cell's j - 1 and the blend weight.
__device__ __forceinline__ void m_bracket(const double* __restrict__ Mg, int n_M, double Mnow, int& jc, double& alpha) {
  jc = 0;
  alpha = 0.0;
  if (n_M > 1) {
    int j = lower_bound(Mg, 0, n_M, Mnow);
    j = j > n_M - 1 ? n_M - 1 : j;
    j = j < 1 ? 1 : j;
    alpha = (Mnow - Mg[j - 1]) / (Mg[j] - Mg[j - 1]);
    jc = j - 1;
  }
}

// Cell of an agent with labour state l and employment e in aggregate state Mrkv, and the
// index of its header among the period's staged headers (employed: l, unemployed:
// n_lab + l).
__device__ __forceinline__ int panel_cell(int l, int e, int Mrkv, int n_lab, int n_J, int jc) {
  return (2 * l + Mrkv + (e ? 0 : 2 * n_lab)) * n_J + jc;
}
__device__ __forceinline__ int panel_hdr(int l, int e, int n_lab) { return e ? l : n_lab + l; }

// One calibration's panel model on device (aiy_panel_model).
struct PanelDev {
  int S, n_M, n_a, n_lab, act_T;
  bool unemployed;   // tables hold the unemployed cells too
  const double* M_grid;
  const double* lab_level;
  const double* lab_cdf;
  const int* mrkv_hist;
  PanelTab tab;
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

constexpr int kLdsLab = 16;   // labour states (the KS form has S = 4 n_lab <= 64)
constexpr int kPairs = 2;     // agent pairs per lane per pass
constexpr int kAgents = 2 * kPairs;

// Host: check the model of one calibration and fill its device view.
int32_t panel_dev(aiy_handle* h, const aiy_panel_model* model, PanelDev& P);

// Persistent panel (panel_resident.hip), used by aiy_sim_periods.  Single rank: a block of
// periods in one launch.  Sharded (kResSharded): ONE period per launch whose workgroup 0 leaves
// the shard's sum of a in sow[6] for the caller's all-reduce and the price kernel (kResDraw0: the
// launch draws its period's labour states first; kResDrawNext: it draws the next period's after
// the lookups, as the multi-period launch does while the partial sums travel).
// kResPrices: the launch first forms period t0 - 1's prices from the all-reduced sum in sow[6]
// (the mill of the price kernel, by every workgroup; workgroup 0 writes sow and the history)
// instead of reading them from sow -- one kernel fewer per period.  kResKeepTmo: the timeout
// word is not re-zeroed (an earlier launch of the same call zeroed it; the host reads it once
// at the end).
constexpr int kResSharded = 1, kResDraw0 = 2, kResDrawNext = 4, kResPrices = 8, kResKeepTmo = 16;
int32_t launch_resident(aiy_handle* h, const PanelDev& P, const aiy_market& mk, long long n, double* a, uint8_t* lab,
                        const double* u, long long u_ld, unsigned long long seed, unsigned ge_iter, int t0,
                        int n_periods, double* sow, double* hist_A, double* hist_M, hipStream_t st,
                        long long offset = 0, int flags = kResDraw0, long long n_total = 0);
int32_t resident_status(aiy_handle* h, hipStream_t st, bool timed = true);
bool resident_supported(const PanelDev& P);
// the persistent kernel moves agent pairs as 16-byte asset / 2-byte labour accesses
inline bool resident_aligned(const double* a, const uint8_t* lab) {
  return (reinterpret_cast<uintptr_t>(a) & 15) == 0 && (reinterpret_cast<uintptr_t>(lab) & 1) == 0;
}
constexpr long long kResMinAgents = 65536;

}  // namespace aiy
