// Wealth-distribution statistics of a simulated panel: HARK's
// get_lorenz_shares and get_percentiles as the reference notebook calls them on the
// simulated wealth (Aiyagari-HARK.py:298-316), over a device-resident panel of up to
// 1e8 agents, so the assets never leave HBM.
//
//   sort      rocPRIM radix sort of the wealth (pairs with the weights when given);
//   scan      inclusive sums of w (cum_dist numerator) and a w (cum_data numerator);
//   interp    one thread per requested percentile: np.interp(p, cum_dist, cum_data)
//             (Lorenz) and scipy interp1d(cum_dist, sorted, bounds_error=False)(p)
//             (percentiles), each reading only the two bracketing entries.
// Unit weights (weights == nullptr, the notebook's sim_wealth call) skip the weight
// sort and scan: cum_dist[k] = (k + 1) / n exactly as cumsum(ones) / sum(ones).
// The sums are tree-ordered (rocPRIM scan) where NumPy's cumsum is sequential, so the
// results agree with HARK to rounding (~1e-15 relative), not bit for bit.
#include "common.h"
#include "internal.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstring>

namespace aiy {

constexpr int kMaxPct = 256;

__global__ void stats_product_kernel(const double* __restrict__ x, const double* __restrict__ w, long long n,
                                     double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = x[i] * w[i];   // temp2 = temp * weights
}

// cum_dist[k]: (k + 1) / n for unit weights, else cw[k] / cw[n - 1].
__device__ __forceinline__ double cum_dist_at(const double* cw, long long n, long long k) {
  return cw ? cw[k] / cw[n - 1] : (double)(k + 1) / (double)n;
}

// First k in [0, n) with cum_dist[k] > p (searchsorted side='right'), or with
// cum_dist[k] >= p (side='left').
__device__ __forceinline__ long long cd_search(const double* cw, long long n, double p, bool right) {
  long long lo = 0, hi = n;
  while (lo < hi) {
    const long long mid = lo + ((hi - lo) >> 1);
    const double v = cum_dist_at(cw, n, mid);
    if (right ? (v <= p) : (v < p)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void stats_interp_kernel(const double* __restrict__ sorted, const double* __restrict__ cw,
                                    const double* __restrict__ cd, long long n, const double* __restrict__ pct,
                                    int n_p, double* __restrict__ lorenz, double* __restrict__ pctl) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_p) return;
  const double p = pct[t];
  const double total = cd[n - 1];
  // np.interp(p, xp = cum_dist, fp = cum_data), cum_data = cumsum(temp2) / sum(temp2)
  {
    const double x0 = cum_dist_at(cw, n, 0), xl = cum_dist_at(cw, n, n - 1);
    double r;
    if (p < x0) {
      r = cd[0] / total;
    } else if (p >= xl) {
      r = cd[n - 1] / total;
    } else {
      const long long j = cd_search(cw, n, p, true) - 1;   // xp[j] <= p < xp[j + 1]
      const double xj = cum_dist_at(cw, n, j), xj1 = cum_dist_at(cw, n, j + 1);
      const double yj = cd[j] / total, yj1 = cd[j + 1] / total;
      if (p == xj) {
        r = yj;
      } else {
        const double slope = (yj1 - yj) / (xj1 - xj);
        r = slope * (p - xj) + yj;
        if (r != r) {                                        // numpy's NaN retry
          r = slope * (p - xj1) + yj1;
          if (r != r && yj == yj1) r = yj;
        }
      }
    }
    lorenz[t] = r;
  }
  // scipy interp1d(cum_dist, sorted, bounds_error=False): NaN outside [x[0], x[-1]]
  {
    const double x0 = cum_dist_at(cw, n, 0), xl = cum_dist_at(cw, n, n - 1);
    double r = __builtin_nan("");
    if (!(p < x0) && !(p > xl) && n >= 2) {
      long long hi = cd_search(cw, n, p, false);             // searchsorted(x, p) (left)
      hi = hi < 1 ? 1 : (hi > n - 1 ? n - 1 : hi);
      const long long lo = hi - 1;
      const double xa = cum_dist_at(cw, n, lo), xb = cum_dist_at(cw, n, hi);
      const double slope = (sorted[hi] - sorted[lo]) / (xb - xa);
      r = slope * (p - xa) + sorted[lo];
    }
    pctl[t] = r;
  }
}

static int32_t grow(aiy_handle* h, void** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return AIY_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  AIY_HIP(h, hipMalloc(p, bytes));
  *cap = bytes;
  return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" int32_t aiy_wealth_stats(aiy_handle* h, const double* data, const double* weights, int64_t n,
                                    const double* pctiles, int32_t n_p, double* lorenz_out, double* pctl_out,
                                    aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!data || !pctiles || n_p < 1) return fail(h, AIY_ERR_ARG, "null data/pctiles or n_p < 1");
  if (n < 1) return fail(h, AIY_ERR_ARG, "n must be >= 1");
  if (n_p > kMaxPct) return fail(h, AIY_ERR_UNSUPPORTED, "n_p=%d exceeds %d", n_p, kMaxPct);
  for (int i = 0; i < n_p; ++i)
    if (!(pctiles[i] > 0.0 && pctiles[i] < 1.0)) return fail(h, AIY_ERR_ARG, "percentiles must lie in (0, 1)");
  AIY_HIP(h, hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  AIY_USE_STREAM(h, st);
  const size_t nb = (size_t)n * sizeof(double);
  int32_t rc;
  // scratch: [sorted][cd] (+ [w_sorted][cw][w sorted x a] with weights) + percentiles/results + rocPRIM temp
  const int nbuf = weights ? 5 : 2;
  const size_t small = 3 * kMaxPct * sizeof(double);
  size_t tmp_sort = 0, tmp_scan = 0;
  if (weights) {
    AIY_HIP(h, rocprim::radix_sort_pairs(nullptr, tmp_sort, data, (double*)nullptr, weights, (double*)nullptr,
                                         (size_t)n, 0, 64, st));
  } else {
    AIY_HIP(h, rocprim::radix_sort_keys(nullptr, tmp_sort, data, (double*)nullptr, (size_t)n, 0, 64, st));
  }
  AIY_HIP(h, rocprim::inclusive_scan(nullptr, tmp_scan, (const double*)nullptr, (double*)nullptr, (size_t)n,
                                     rocprim::plus<double>(), st));
  const size_t head = (nbuf * nb + small + 255) / 256 * 256;   // rocPRIM temp 256-aligned
  const size_t tmp = (tmp_sort > tmp_scan ? tmp_sort : tmp_scan) + 256;
  rc = grow(h, &h->d_stats, &h->stats_cap, head + tmp);
  if (rc) return rc;
  char* base = reinterpret_cast<char*>(h->d_stats);
  double* sorted = reinterpret_cast<double*>(base);
  double* cd = reinterpret_cast<double*>(base + nb);
  double* ws = weights ? reinterpret_cast<double*>(base + 2 * nb) : nullptr;
  double* cw = weights ? reinterpret_cast<double*>(base + 3 * nb) : nullptr;
  double* prod = weights ? reinterpret_cast<double*>(base + 4 * nb) : nullptr;
  double* d_pct = reinterpret_cast<double*>(base + nbuf * nb);
  double* d_lor = d_pct + kMaxPct;
  double* d_pcl = d_lor + kMaxPct;
  void* d_tmp = reinterpret_cast<void*>(base + head);
  size_t ts = tmp_sort;
  if (weights) {
    AIY_HIP(h, rocprim::radix_sort_pairs(d_tmp, ts, data, sorted, weights, ws, (size_t)n, 0, 64, st));
    size_t tc = tmp_scan;
    AIY_HIP(h, rocprim::inclusive_scan(d_tmp, tc, ws, cw, (size_t)n, rocprim::plus<double>(), st));
    hipLaunchKernelGGL(stats_product_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sorted, ws,
                       (long long)n, prod);
    AIY_CHECK_LAUNCH(h);
    tc = tmp_scan;
    AIY_HIP(h, rocprim::inclusive_scan(d_tmp, tc, prod, cd, (size_t)n, rocprim::plus<double>(), st));
  } else {
    AIY_HIP(h, rocprim::radix_sort_keys(d_tmp, ts, data, sorted, (size_t)n, 0, 64, st));
    size_t tc = tmp_scan;
    AIY_HIP(h, rocprim::inclusive_scan(d_tmp, tc, sorted, cd, (size_t)n, rocprim::plus<double>(), st));
  }
  AIY_HIP(h, hipMemcpyAsync(d_pct, pctiles, n_p * sizeof(double), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(stats_interp_kernel, dim3((n_p + 63) / 64), dim3(64), 0, st, sorted, cw, cd, (long long)n,
                     d_pct, n_p, d_lor, d_pcl);
  AIY_CHECK_LAUNCH(h);
  double res[2 * kMaxPct];
  AIY_HIP(h, hipMemcpyAsync(res, d_lor, 2 * kMaxPct * sizeof(double), hipMemcpyDeviceToHost, st));
  AIY_HIP(h, hipStreamSynchronize(st));
  if (lorenz_out) std::memcpy(lorenz_out, res, n_p * sizeof(double));
  if (pctl_out) std::memcpy(pctl_out, res + kMaxPct, n_p * sizeof(double));
  return AIY_OK;
}
