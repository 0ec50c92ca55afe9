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

}  // namespace aiy

extern "C" int32_t aiy_index_ints_per_row(void) { return aiy::kIdxRow; }

extern "C" int32_t aiy_build_index(aiy_handle* h, int64_t n_rows, int32_t n1, const double* x, int32_t* index,
                                   aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (n_rows < 0 || n1 < 2 || (n_rows > 0 && (!x || !index))) return aiy::fail(h, AIY_ERR_ARG, "bad index args");
  AIY_HIP(h, hipSetDevice(h->device));
  return aiy::launch_build_index(h, x, n_rows, n1, index, aiy::as_stream(stream));
}
