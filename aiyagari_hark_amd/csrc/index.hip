// Build the log-bucket search index (common.h) of many policy rows at once.
//
// One lane per node i of a row (i = 0..n-1, n = n_a: the HARK search runs over
// x[:-1]): with c(i) = clamp(key(x_i) - base, -1, K - 1), lane i writes H[b] = i for
// every bucket b in (c(i-1), c(i)]; lane n writes H[last + 1] = n and the header
// last = c(n-1).  Every bucket up to last + 1 is written exactly once and
// H[b] = first i with x_i >= edge_b -- a streaming pass, no searches.  Buckets above
// last + 1 are never read (their queries exceed every node: lower_bound = n).  Starting the buckets at x[1] keeps the per-lane ranges short: the huge gap
// between the 1e-7 borrowing node and the first real node is not bucketed.
#include "common.h"
#include "internal.h"

namespace aiy {

template <class I>
__global__ __launch_bounds__(256) void build_index_kernel(const double* __restrict__ x, long long stride, long long n_rows,
                                                          int n1, int* __restrict__ H) {
  const long long row = blockIdx.y + (long long)blockIdx.z * gridDim.y;
  if (row >= n_rows) return;
  const int n = n1 - 1;
  const double* xr0 = x + row * n1 * stride;
  auto xr = [&](int k) { return xr0[(size_t)k * stride]; };
  int* Hr = H + row * I::kRow;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const double x1 = n >= 2 ? xr(1) : 0.0;
  if (!(x1 > 0.0)) {
    if (i == 0) Hr[I::kBuckets + 1] = kIdxNoBase;
    return;
  }
  const long long base = idx_key<I>(x1);
  // c(k): bucket of node k relative to base, -1 below bucket 0, capped at K - 1.
  auto c = [&](int k) -> long long {
    const double v = xr(k);
    if (!(v > 0.0)) return -1;
    const long long b = idx_key<I>(v) - base;
    return b > I::kBuckets - 1 ? I::kBuckets - 1 : (b < -1 ? -1 : b);
  };
  if (i < n) {
    const long long hi = c(i);
    const long long lo = (i == 0) ? -1 : c(i - 1);
    for (long long b = lo + 1; b <= hi; ++b) Hr[b] = i;
  } else {
    // one bucket past the last node's (its lower_bound is n), and the header
    const long long last = c(n - 1);
    if (last + 1 <= I::kBuckets - 1) Hr[last + 1] = n;
    Hr[I::kBuckets] = (int)last;
  }
  if (i == 0) Hr[I::kBuckets + 1] = (int)base;
}

int32_t launch_build_index(aiy_handle* h, const double* x, long long n_rows, int n1, int* H, hipStream_t st) {
  if (n_rows <= 0) return AIY_OK;
  const long long gy = n_rows < 65535 ? n_rows : 65535;
  const long long gz = (n_rows + gy - 1) / gy;
  dim3 grid((n1 + 255) / 256, (unsigned)gy, (unsigned)gz);
  hipLaunchKernelGGL(build_index_kernel<EgmIdx>, grid, dim3(256), 0, st, x, 1LL, n_rows, n1, H);
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

// Bracket index (BrkIdx, common.h) of pair rows (x at stride 2): one lane per node i.
// Lane i writes the empty buckets strictly between its predecessor's bucket and its
// own as (lo = i, cnt = 0) and, when it is the first node of its bucket, that bucket's
// entry (lo = i, cnt = nodes in the bucket (<= 7), low bits of x_i); lane n writes the
// bucket past the last node (lo = n) and the header.  Every bucket up to last + 1 is
// written exactly once.
__global__ __launch_bounds__(256) void build_brk_kernel(const double* __restrict__ x, long long n_rows, int n1,
                                                        unsigned long long* __restrict__ E) {
  const long long row = blockIdx.y + (long long)blockIdx.z * gridDim.y;
  if (row >= n_rows) return;
  const int n = n1 - 1;
  const double* xr0 = x + row * n1 * 2;
  auto xr = [&](int k) { return xr0[(size_t)k * 2]; };
  unsigned long long* Er = E + row * BrkIdx::kRowU64;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const double x1 = n >= 2 ? xr(1) : 0.0;
  if (!(x1 > 0.0)) {
    if (i == 0) Er[BrkIdx::kBuckets + 1] = (unsigned long long)(long long)kIdxNoBase;
    return;
  }
  const long long base = idx_key<BrkIdx>(x1);
  auto c = [&](int k) -> long long {
    const double v = xr(k);
    if (!(v > 0.0)) return -1;
    const long long b = idx_key<BrkIdx>(v) - base;
    return b > BrkIdx::kBuckets - 1 ? BrkIdx::kBuckets - 1 : (b < -1 ? -1 : b);
  };
  if (i < n) {
    const long long hi = c(i);
    const long long lo = (i == 0) ? -1 : c(i - 1);
    for (long long b = lo + 1; b < hi; ++b) Er[b] = brk_encode(i, 0, 0);
    if (hi > lo && hi >= 0) {
      int cnt = 1;
      while (cnt < BrkIdx::kCntSat && i + cnt < n && c(i + cnt) == hi) ++cnt;
      Er[hi] = brk_encode(i, cnt, (unsigned long long)__double_as_longlong(xr(i)));
    }
  } else {
    const long long last = c(n - 1);
    if (last + 1 <= BrkIdx::kBuckets - 1) Er[last + 1] = brk_encode(n, 0, 0);
    Er[BrkIdx::kBuckets] = (unsigned long long)last;
  }
  if (i == 0) Er[BrkIdx::kBuckets + 1] = (unsigned long long)base;
}

// Interleave a policy table into (m, c) pairs and build its panel bracket index.
__global__ __launch_bounds__(256) void interleave_kernel(const double* __restrict__ m, const double* __restrict__ c,
                                                         long long n, double* __restrict__ pairs) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  reinterpret_cast<double2*>(pairs)[t] = make_double2(m[t], c[t]);
}

}  // namespace aiy

extern "C" int32_t aiy_panel_index_ints_per_row(void) { return aiy::PanelIdx::kRow; }

extern "C" int32_t aiy_panel_prepare(aiy_handle* h, int64_t n_rows, int32_t n1, const double* m_pol,
                                     const double* c_pol, double* pairs, int32_t* index, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_rows < 1 || n1 < 2 || !m_pol || !c_pol || !pairs || !index) return aiy::fail(h, AIY_ERR_ARG, "bad prepare args");
  if (n1 > aiy::BrkIdx::kMaxNodes) return aiy::fail(h, AIY_ERR_UNSUPPORTED, "n_a + 1 = %d > %d", n1, aiy::BrkIdx::kMaxNodes);
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = aiy::as_stream(stream);
  const long long n = n_rows * (long long)n1;
  hipLaunchKernelGGL(aiy::interleave_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, m_pol, c_pol, n, pairs);
  const long long gy = n_rows < 65535 ? n_rows : 65535;
  const long long gz = (n_rows + gy - 1) / gy;
  dim3 grid((n1 + 255) / 256, (unsigned)gy, (unsigned)gz);
  hipLaunchKernelGGL(aiy::build_brk_kernel, grid, dim3(256), 0, st, pairs, (long long)n_rows, n1,
                     reinterpret_cast<unsigned long long*>(index));
  AIY_CHECK_LAUNCH(h);
  return AIY_OK;
}

extern "C" int32_t aiy_index_ints_per_row(void) { return aiy::kIdxRow; }

extern "C" int32_t aiy_build_index(aiy_handle* h, int64_t n_rows, int32_t n1, const double* x, int32_t* index,
                                   aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_rows < 0 || n1 < 2 || (n_rows > 0 && (!x || !index))) return aiy::fail(h, AIY_ERR_ARG, "bad index args");
  AIY_HIP(h, hipSetDevice(h->device));
  return aiy::launch_build_index(h, x, n_rows, n1, index, aiy::as_stream(stream));
}
