// Merged policy tables of the panel (layout and lookup: panel_common.h), built once
// per history from the converged policy (AiyagariType.solution[0], AS:1509-1519).
//
//   tab_merge_kernel  one lane per node of the two rows of a cell: its position in the
//                     merged list z is its own index plus its rank in the other row
//                     (row 0 first on ties: a stable merge, no sort); the lane writes z
//                     and the record of the segment that starts at its node.
//   tab_index_kernel  one lane per merged node: the bracket index of z (common.h),
//                     streaming, no searches.
#include "common.h"
#include "internal.h"
#include "panel_common.h"

namespace aiy {

// #{x[0..n) <= v}
__device__ __forceinline__ int count_le(const double* __restrict__ x, int n, double v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = lo + ((hi - lo) >> 1);
    if (x[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void tab_merge_kernel(const double* __restrict__ m_pol,
                                                        const double* __restrict__ c_pol, int S, int n_M,
                                                        PanelTabGeom g, char* __restrict__ tabs) {
  const int cell = blockIdx.y, cal = blockIdx.z;
  const int n = g.n, n1 = n + 1;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e > 2 * n) return;
  const int lgc = cell / g.n_J, jc = cell - lgc * g.n_J;
  const int n_lg = 2 * (S / 4);                       // employed cells first, then the unemployed
  const int emp = lgc < n_lg ? 1 : 0;
  const int lg = emp ? lgc : lgc - n_lg;
  const int s = 4 * (lg >> 1) + 2 * (lg & 1) + emp;   // sub-state 4 l + 2 g + emp (AS:1326-1356)
  const int j0 = n_M > 1 ? jc : 0, j1 = n_M > 1 ? jc + 1 : 0;
  const size_t r0 = (((size_t)cal * S + s) * n_M + j0) * n1;
  const size_t r1 = (((size_t)cal * S + s) * n_M + j1) * n1;
  const double* x0 = m_pol + r0;
  const double* y0 = c_pol + r0;
  const double* x1 = m_pol + r1;
  const double* y1 = c_pol + r1;
  char* base = tabs + (size_t)cal * g.bytes;
  double2* rec = reinterpret_cast<double2*>(base + g.rec_off) + (size_t)cell * g.rec_stride;
  double* z = reinterpret_cast<double*>(base + g.z_off) + (size_t)cell * g.z_stride;
  int p, c0, c1;   // merged position of this lane's node; nodes of each row at positions <= p
  if (e < n) {
    const double v = x0[e];
    const int cb = lower_bound(x1, 0, n, v);           // row-1 nodes < v
    p = e + cb;
    c0 = e + 1;
    c1 = cb;
    z[p] = v;
  } else if (e < 2 * n) {
    const int b = e - n;
    const double v = x1[b];
    const int ca = count_le(x0, n, v);                 // row-0 nodes <= v (row 0 first on ties)
    p = b + ca;
    c0 = ca;
    c1 = b + 1;
    z[p] = v;
  } else {
    p = -1;                                            // record 0: queries at or below z[0]
    c0 = 0;
    c1 = 0;
  }
  const int i0 = c0 < 1 ? 1 : c0, i1 = c1 < 1 ? 1 : c1;   // HARK: max(searchsorted, 1)
  double2* r = rec + 4 * (size_t)(p + 1);
  r[0] = make_double2(x0[i0 - 1], x0[i0]);
  r[1] = make_double2(y0[i0 - 1], y0[i0]);
  r[2] = make_double2(x1[i1 - 1], x1[i1]);
  r[3] = make_double2(y1[i1 - 1], y1[i1]);
}

// Bracket index of z (BrkIdx, common.h), bucketed from z[kTabFirst]: lane i writes the
// empty buckets strictly between its predecessor's bucket and its own (lo = i) and, as
// the first node of its bucket, that bucket's entry; lane Z writes the bucket past the
// last node and the header.  Every bucket up to last + 1 is written exactly once.
__global__ __launch_bounds__(256) void tab_index_kernel(PanelTabGeom g, char* __restrict__ tabs) {
  const int cell = blockIdx.y, cal = blockIdx.z;
  char* base = tabs + (size_t)cal * g.bytes;
  const double* z = reinterpret_cast<const double*>(base + g.z_off) + (size_t)cell * g.z_stride;
  unsigned long long* E = reinterpret_cast<unsigned long long*>(base + g.idx_off) + (size_t)cell * g.idx_stride;
  const int n = g.Z;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const double xf = n > kTabFirst ? z[kTabFirst] : 0.0;
  if (!(xf > 0.0)) {
    if (i == 0) {
      E[g.buckets] = 0ull;
      E[g.buckets + 1] = (unsigned long long)(long long)kIdxNoBase;
    }
    return;
  }
  const long long bk = (long long)((unsigned long long)__double_as_longlong(xf) >> g.shift);
  auto c = [&](int k) -> long long {
    const double v = z[k];
    if (!(v > 0.0)) return -1;
    const long long b = (long long)((unsigned long long)__double_as_longlong(v) >> g.shift) - bk;
    return b > g.buckets - 1 ? g.buckets - 1 : (b < -1 ? -1 : b);
  };
  if (i < n) {
    const long long hi = c(i);
    const long long lo = (i == 0) ? -1 : c(i - 1);
    for (long long b = lo + 1; b < hi; ++b) E[b] = brk_encode(i, 0, 0);
    if (hi > lo && hi >= 0) {
      int cnt = 1;
      while (cnt < BrkIdx::kCntSat && i + cnt < n && c(i + cnt) == hi) ++cnt;
      unsigned long long fields = 0;
      if (cnt <= 3) {   // top w within-bucket bits of each node (brk_decode)
        const int w = brk_field_bits(cnt, g.shift);
        const unsigned long long mask = (1ull << w) - 1;
        for (int j = 0; j < cnt; ++j)
          fields |= ((((unsigned long long)__double_as_longlong(z[i + j])) >> (g.shift - w)) & mask) << (j * w);
      }
      E[hi] = brk_encode(i, cnt, fields);
    }
  } else {
    const long long last = c(n - 1);
    if (last + 1 <= g.buckets - 1) E[last + 1] = brk_encode(n, 0, 0);
    E[g.buckets] = (unsigned long long)last;
  }
  if (i == 0) E[g.buckets + 1] = (unsigned long long)bk;
}

int32_t panel_dev(aiy_handle* h, const aiy_panel_model* model, PanelDev& P) {
  if (!model) return fail(h, AIY_ERR_ARG, "null model");
  if (model->S < 1 || model->n_M < 1 || model->n_a < 2 || model->n_lab < 1 || model->n_lab > 255)
    return fail(h, AIY_ERR_ARG, "bad model sizes");
  if (model->S != 4 * model->n_lab) return fail(h, AIY_ERR_ARG, "S must be 4 * n_lab (KS form)");
  if (model->n_lab > kLdsLab) return fail(h, AIY_ERR_UNSUPPORTED, "n_lab=%d > %d", model->n_lab, kLdsLab);
  if (2LL * model->n_a >= BrkIdx::kMaxNodes) return fail(h, AIY_ERR_UNSUPPORTED, "n_a too large");
  if (!model->tables || !model->lab_level || !model->lab_cdf || !model->mrkv_hist)
    return fail(h, AIY_ERR_ARG, "null model array (tables come from aiy_panel_build)");
  if (model->n_M > 1 && !model->M_grid) return fail(h, AIY_ERR_ARG, "null M_grid");
  if (model->act_T < 1 || model->act_T > (1 << 20)) return fail(h, AIY_ERR_ARG, "bad act_T=%d", model->act_T);
  P.S = model->S; P.n_M = model->n_M; P.n_a = model->n_a; P.n_lab = model->n_lab; P.act_T = model->act_T;
  P.M_grid = model->M_grid; P.lab_level = model->lab_level; P.lab_cdf = model->lab_cdf;
  P.mrkv_hist = model->mrkv_hist;
  P.unemployed = model->unemployed != 0;
  P.tab = panel_tab(model->tables, panel_tab_geom(model->n_lab, model->n_M, model->n_a, P.unemployed));
  return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" int64_t aiy_panel_table_bytes(int32_t n_lab, int32_t n_M, int32_t n_a, int32_t unemployed) {
  if (n_lab < 1 || n_lab > kLdsLab || n_M < 1 || n_a < 2 || 2LL * n_a >= BrkIdx::kMaxNodes) return -1;
  return panel_tab_geom(n_lab, n_M, n_a, unemployed != 0).bytes;
}

extern "C" int32_t aiy_panel_build(aiy_handle* h, int32_t n_cal, int32_t S, int32_t n_M, int32_t n_a, int32_t n_lab,
                                   int32_t unemployed, const double* m_pol, const double* c_pol, void* tables,
                                   aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_cal < 1 || n_cal > 65535 || n_M < 1 || n_a < 2 || n_lab < 1 || n_lab > kLdsLab || S != 4 * n_lab)
    return fail(h, AIY_ERR_ARG, "bad panel table sizes (n_cal=%d S=%d n_M=%d n_a=%d n_lab=%d)", n_cal, S, n_M, n_a,
                n_lab);
  if (2LL * n_a >= BrkIdx::kMaxNodes) return fail(h, AIY_ERR_UNSUPPORTED, "n_a=%d too large", n_a);
  if (!m_pol || !c_pol || !tables) return fail(h, AIY_ERR_ARG, "null pointer");
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  const PanelTabGeom g = panel_tab_geom(n_lab, n_M, n_a, unemployed != 0);
  char* tabs = static_cast<char*>(tables);
  dim3 gm((2 * n_a + 1 + 255) / 256, g.n_cells, n_cal);
  hipLaunchKernelGGL(tab_merge_kernel, gm, dim3(256), 0, st, m_pol, c_pol, S, n_M, g, tabs);
  dim3 gi((g.Z + 1 + 255) / 256, g.n_cells, n_cal);
  hipLaunchKernelGGL(tab_index_kernel, gi, dim3(256), 0, st, g, tabs);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}
