// Shared device helpers for libaiyagari (gfx950 / CDNA4, wave64).
//
// Numerics policy: the library is compiled with -ffp-contract=off so every product and
// sum rounds exactly as the NumPy expressions of the reference do
// (Aiyagari_Support.py:1024, 1485, 1490, 1499; HARK LinearInterp /
// LinearInterpOnInterp1D).  Sums over next-period states replicate NumPy's pairwise
// summation order (8 running partials, numpy/_core/src/umath/loops_utils.h) so the
// CRRA = 1 path is bit-identical to the oracle; other CRRA values differ only by the
// device pow's last-ulp rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aiy {

constexpr int kWave = 64;
constexpr double kBorrowNode = 0.0000001;  // Aiyagari_Support.py:1503-1504

// ---------------------------------------------------------------------------------
// Cross-kernel control words (convergence slots, the device market state) are read
// with agent-scope atomic loads.  A plain load of a block-uniform address compiles to
// s_load through the scalar cache, which is not kept coherent with the vector-memory
// atomics and stores of the previous kernels: measured on MI355X, a solve whose
// convergence slot was read with s_load kept iterating ~20 cycles past convergence.
// ---------------------------------------------------------------------------------
// Every control word and hand-off buffer lives in global memory (hipMalloc): the accesses
// are typed global so they compile to global_load/store ... sc1 even where the compiler
// cannot prove the address space of a generic pointer (a flat_ access is slower and is not
// a valid stand-in for the agent-scope acquire, MI355X_MICROARCH.md hand-off rules).
template <class T>
using gptr = __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr<T> to_global(T* p) {
  return (gptr<T>)p;
}
__device__ __forceinline__ unsigned long long load_u64_agent(const unsigned long long* p) {
  return __hip_atomic_load(to_global(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_f64_agent(const double* p) {
  return __longlong_as_double((long long)load_u64_agent(reinterpret_cast<const unsigned long long*>(p)));
}
__device__ __forceinline__ void store_u64_agent(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(to_global(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_f64_agent(double* p, double v) {
  store_u64_agent(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v));
}

// ---------------------------------------------------------------------------------
// Wave-level helpers
// ---------------------------------------------------------------------------------
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
  return v;
}
// Sum over the wave by xor butterflies (a fixed order per lane: lane 0's value is
// reproducible run to run).
__device__ __forceinline__ double wave_sum_fixed(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
// NaN-propagating max (np.max semantics): a NaN anywhere makes the result NaN.
__device__ __forceinline__ double nan_max(double a, double b) {
  return (a != a || a > b) ? a : b;
}
__device__ __forceinline__ double wave_nan_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nan_max(v, __shfl_xor(v, o, kWave));
  return v;
}

// ---------------------------------------------------------------------------------
// Lower bound (numpy searchsorted side='left') over x[lo, hi): first index with
// x[idx] >= q, or hi.  For a sorted row every correct lower bound returns the index
// numpy's npy_binsearch<left> returns.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ int lower_bound(const double* __restrict__ x, int lo, int hi, double q) {
  while (lo < hi) {
    int mid = lo + ((hi - lo) >> 1);
    if (x[mid] < q) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// HARK 0.12 LinearInterp._evaluate for one query given the bracket index
// i = max(searchsorted(x[:-1], q), 1):
//   alpha = (q - x[i-1]) / (x[i] - x[i-1]); y = (1 - alpha) y[i-1] + alpha y[i];
//   NaN when q < x[0] (lower_extrap = False).
__device__ __forceinline__ double lerp_at(const double* __restrict__ x, const double* __restrict__ y,
                                          int i, double q, double x0) {
  double xl = x[i - 1], xh = x[i];
  double alpha = (q - xl) / (xh - xl);
  double v = (1.0 - alpha) * y[i - 1] + alpha * y[i];
  return (q < x0) ? __builtin_nan("") : v;
}

// Wave-cooperative monotone interpolation on one row (x, y) of length n + 1.
// All 64 lanes of the wave must call it together (inactive lanes pass active=false).
// The bracket search is narrowed to [lb(qmin), lb(qmax)] found by two wave-uniform
// searches, so each lane's private search runs over a few dozen nodes instead of n.
__device__ __forceinline__ double interp_row_wave(const double* __restrict__ x, const double* __restrict__ y,
                                                  int n, double q, bool active) {
  double qmin = wave_min(active ? q : __builtin_inf());
  double qmax = wave_max(active ? q : -__builtin_inf());
  int lo = 0, hi = n;
  if (qmin == qmin && qmax == qmax && qmin <= qmax) {   // all-NaN / no active lanes: full search
    lo = lower_bound(x, 0, n, qmin);
    hi = lower_bound(x, lo, n, qmax);   // lb(q) lies in [lb(qmin), lb(qmax)] for q in range
  }
  int i = lower_bound(x, lo, hi, q);    // NaN lanes get some index; their value is NaN anyway
  i = i < 1 ? 1 : i;
  return lerp_at(x, y, i, q, x[0]);
}

// Plain per-lane search version (no wave cooperation); used where lanes are independent.
__device__ __forceinline__ double interp_row(const double* __restrict__ x, const double* __restrict__ y,
                                             int n, double q) {
  int i = lower_bound(x, 0, n, q);
  i = i < 1 ? 1 : i;
  return lerp_at(x, y, i, q, x[0]);
}

// ---------------------------------------------------------------------------------
// Log-bucket search index of a sorted, positive row x[0..n) (the m nodes of one
// LinearInterp, searched over x[:-1]).  Bucket b covers the doubles whose bit
// pattern >> SHIFT equals base + b, base = key(x[1]) (x[0] is the 1e-7 borrowing node,
// far below the rest of the row): 2^(52 - SHIFT) buckets per binary octave.
// H[b] = first i with x[i] >= edge_b = lower_bound(x, edge_b).  A query in bucket b has
// its lower_bound in [H[b], H[b+1]] (queries below edge_0: [0, H[0]]; above the last
// node's bucket: n), found exactly -- bucket edges are bit-level, no floating-point
// rounding -- by a search over a handful of nodes.
//   layout per row: H[0 .. BUCKETS - 1] (entries up to last + 1 valid),
//   last = bucket of the last node at [BUCKETS], base at [BUCKETS + 1]
// EgmIdx (256 / octave) is rebuilt every EGM cycle; the panel uses the finer bracket
// index below (BrkIdx), built once per history.
// ---------------------------------------------------------------------------------
template <int SHIFT, int BUCKETS>
struct IdxSpec {
  static constexpr int kShift = SHIFT;
  static constexpr int kBuckets = BUCKETS;
  static constexpr int kRow = BUCKETS + 2;   // ints per row
};
using EgmIdx = IdxSpec<44, 16 * 256>;
constexpr int kIdxShift = EgmIdx::kShift;
constexpr int kIdxBuckets = EgmIdx::kBuckets;
constexpr int kIdxRow = EgmIdx::kRow;
constexpr int kIdxNoBase = -2147483647 - 1;     // x[1] <= 0 or n < 2: index unusable -> full search

template <class I = EgmIdx>
__device__ __forceinline__ long long idx_key(double q) {
  return (long long)(__double_as_longlong(q) >> I::kShift);
}

// ---------------------------------------------------------------------------------
// BRACKET index (the panel's merged policy tables, panel_common.h): log buckets of a
// sorted positive node list -- 2^(52 - shift) per binary octave, `buckets` in all,
// starting at a base node -- with one 64-bit entry per bucket:
//   bits 43..63  lo  = first i with key(x_i) >= bucket (= lower_bound of the edge)
//   bits 40..42  cnt = nodes inside the bucket (saturated at 7)
//   bits  0..39  for cnt <= 3: the top w = min(40 / cnt, shift) of the `shift`
//                within-bucket bits of each of those nodes, node j at bits [j w, j w + w)
// All doubles of one bucket share their bits above `shift`, so comparing q's top w
// within-bucket bits with the stored fields counts the bucket's nodes below q: the
// lower bound comes from the entry alone -- ONE index load, no dependent search step --
// unless a field ties with q's when w < shift (then a one-node search) or cnt >= 4.
// Layout (uint64): E[0 .. buckets - 1], E[buckets] = last bucket, E[buckets + 1] = base
// key (int64).
// ---------------------------------------------------------------------------------
struct BrkIdx {
  static constexpr unsigned long long kLow = (1ull << 40) - 1;
  static constexpr int kCntSat = 7;
  static constexpr int kMaxNodes = 1 << 21;
};

__host__ __device__ __forceinline__ unsigned long long brk_encode(int lo, int cnt, unsigned long long low) {
  return ((unsigned long long)lo << 43) | ((unsigned long long)cnt << 40) | (low & BrkIdx::kLow);
}
// Width of one node's field in an entry holding cnt (1..3) nodes.
__host__ __device__ __forceinline__ int brk_field_bits(int cnt, int shift) {
  const int w = 40 / cnt;
  return w < shift ? w : shift;
}
__device__ __forceinline__ int brk_lo(unsigned long long e) { return (int)(e >> 43); }

// Bracket-index lookup in two branch-free steps, so callers issue the entry load
// themselves (a buffer load) and keep many lookups in flight:
//   brk_slot:    the entry to load -- always in [0, buckets): q below the first bucket
//                (or q <= 0, NaN) loads E[0], q at or beyond the capped top bucket
//                E[buckets - 1] -- and the raw bucket key for brk_resolve;
//   brk_resolve: [lo, hi) from that entry; lo == hi means the lower bound is known,
//                need_next that hi is brk_lo(E[slot + 1]) (a bucket of >= 7 nodes).
// Every case is a select, so a wave decodes each lookup as soon as its entry arrives
// (no branch, no wait for the other lookups in flight).  Below the first bucket the
// window [0, E[0].lo) holds at most the two borrowing nodes z[0], z[1] (E[0].lo <= 2:
// the base bucket is z[2]'s), so the lower bound is counted from them directly (z01 =
// {z[0], z[1]}, held by the caller) -- the borrowing-constrained agents resolve without
// a search step.
__device__ __forceinline__ int brk_slot(int shift, int buckets, int base, double q, long long& raw) {
  const long long k = (long long)((unsigned long long)__double_as_longlong(q) >> shift) - (long long)base;
  raw = (q > 0.0) ? k : -1;
  const long long c = raw < 0 ? 0 : (raw > buckets - 1 ? buckets - 1 : raw);
  return (int)c;
}
__device__ __forceinline__ void brk_resolve(int shift, int buckets, int base, int last, int n, long long raw,
                                            unsigned long long e, double q, double z0, double z1, int& lo, int& hi,
                                            bool& need_next) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(q);
  const int l = brk_lo(e);
  const int c = (int)((e >> 40) & 7u);
  const int w0 = c <= 1 ? 40 : (c == 2 ? 20 : 13);   // brk_field_bits for c = 1..3
  const int w = w0 < shift ? w0 : shift;
  const unsigned long long mask = (1ull << w) - 1;
  const unsigned long long qf = (bits >> (shift - w)) & mask;
  const unsigned long long f0 = e & mask, f1 = (e >> w) & mask, f2 = (e >> (2 * w)) & mask;
  const int below = (f0 < qf ? 1 : 0) + (c >= 2 && f1 < qf ? 1 : 0) + (c >= 3 && f2 < qf ? 1 : 0);
  const int upto = (f0 <= qf ? 1 : 0) + (c >= 2 && f1 <= qf ? 1 : 0) + (c >= 3 && f2 <= qf ? 1 : 0);
  const bool fields = c >= 1 && c <= 3;
  int nlo = fields ? l + below : l;
  int nhi = fields ? (w == shift ? nlo : l + upto) : (c < BrkIdx::kCntSat ? l + c : l);
  bool nx = c == BrkIdx::kCntSat;
  if (raw < 0) {                                       // below the first bucket (E[0] loaded)
    const int b = (l > 0 && z0 < q ? 1 : 0) + (l > 1 && z1 < q ? 1 : 0);
    nlo = b; nhi = b; nx = false;
    if (l > 2) { nlo = 0; nhi = l; }                   // not a table of ours: search the window
  } else if (raw >= buckets - 1) {                     // capped top bucket (E[buckets - 1] loaded)
    const bool capped = last == buckets - 1;
    nlo = capped ? l : n; nhi = n; nx = false;
  } else if (raw > last) {                             // above every node
    nlo = n; nhi = n; nx = false;
  }
  if (base == kIdxNoBase) { nlo = 0; nhi = n; nx = false; }   // no positive node: full search
  if (!nx && (nlo < 0 || nhi > n || nlo > nhi)) { nlo = 0; nhi = n; }   // defensive: unsorted rows
  lo = nlo; hi = nhi; need_next = nx;
}

// Search window [lo, hi) of lower_bound(x[0..n), q) from the row index H (base given).
template <class I>
__device__ __forceinline__ void index_window(const int* __restrict__ H, int base, int n, double q, int& lo, int& hi) {
  lo = 0;
  hi = n;
  if (H == nullptr || base == kIdxNoBase) return;
  const long long key = idx_key<I>(q) - (long long)base;
  const int last = H[I::kBuckets];
  if (!(q > 0.0) || key < 0) { lo = 0; hi = H[0]; }
  else if (key >= I::kBuckets - 1) {                    // capped top bucket / beyond the span
    if (last == I::kBuckets - 1) { lo = H[I::kBuckets - 1]; hi = n; } else { lo = n; hi = n; }
  }
  else if (key > last) { lo = n; hi = n; }              // above every node
  else { lo = H[key]; hi = H[key + 1]; }
  if (lo < 0 || hi > n || lo > hi) { lo = 0; hi = n; }  // defensive: unsorted rows
}

// lower_bound(x[0..n), q) using the row index H (nullptr -> plain binary search).
template <class I = EgmIdx>
__device__ __forceinline__ int locate(const double* __restrict__ x, int n, const int* __restrict__ H, double q) {
  int lo = 0, hi = n;
  if (H != nullptr) index_window<I>(H, H[I::kBuckets + 1], n, q, lo, hi);
  return lower_bound(x, lo, hi, q);
}

// HARK LinearInterp of one row through the index.
__device__ __forceinline__ double interp_row_idx(const double* __restrict__ x, const double* __restrict__ y, int n,
                                                 const int* __restrict__ H, double q) {
  int i = locate(x, n, H, q);
  i = i < 1 ? 1 : i;
  return lerp_at(x, y, i, q, x[0]);
}

// ---------------------------------------------------------------------------------
// x ** -gam and x ** (-1/gam) with NumPy's fast scalar-power path for gam == 1
// (ndarray ** -1.0 is np.reciprocal).  kind: 1 -> gam == 1; 0 -> generic pow.
// ---------------------------------------------------------------------------------
template <int KIND>
__device__ __forceinline__ double crra_marg(double c, double gam) {
  if constexpr (KIND == 1) return 1.0 / c;
  else return pow(c, -gam);
}
template <int KIND>
__device__ __forceinline__ double crra_inv(double e, double gam) {
  if constexpr (KIND == 1) return 1.0 / e;
  else return pow(e, -1.0 / gam);
}

// ---------------------------------------------------------------------------------
// NumPy pairwise sum of f(0..n) for n <= NMAX <= 128 (numpy's pairwise_sum for
// n <= PW_BLOCKSIZE): n < 8 -> sequential from 0.0; else 8 running partials r[t % 8]
// over t < n - n % 8, combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail added
// in order.  Every f(t) index is a compile-time constant so register arrays behind f
// stay in registers.
// ---------------------------------------------------------------------------------
template <int NMAX, typename F>
__device__ __forceinline__ double np_pairwise_sum(int n, F f) {
  if (n < 8) {
    double res = 0.0;
#pragma unroll
    for (int t = 0; t < (NMAX < 8 ? NMAX : 8); ++t)
      if (t < n) res += f(t);
    return res;
  }
  if constexpr (NMAX >= 8) {
    const int nfull = n - (n % 8);
    double r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) r[t] = f(t);
#pragma unroll
    for (int t = 8; t < NMAX; ++t)
      if (t < nfull) r[t % 8] += f(t);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int t = 8; t < NMAX; ++t)
      if (t >= nfull && t < n) res += f(t);
    return res;
  } else {
    return 0.0;
  }
}

// ---------------------------------------------------------------------------------
// Philox4x32-10 (Random123 constants) and the 53-bit uniform used by the panel.
// counter = (c0, idx_lo, idx_hi, stream), key = (seed_lo, seed_hi).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
// One Philox call per agent PAIR (2j, 2j + 1): counter = (ctr0, j, 0, stream); words
// (0, 1) give agent 2j's 53-bit uniform, words (2, 3) agent 2j+1's.
__device__ __forceinline__ void philox_uniform2(uint32_t ctr0, uint64_t pair, uint64_t seed, uint32_t stream,
                                                double& u_even, double& u_odd) {
  uint32_t c[4] = {ctr0, (uint32_t)pair, (uint32_t)(pair >> 32), stream};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  u_even = ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) / 9007199254740992.0;
  u_odd = ((double)(c[2] >> 5) * 67108864.0 + (double)(c[3] >> 6)) / 9007199254740992.0;
}
__device__ __forceinline__ double philox_uniform(uint32_t ctr0, uint64_t idx, uint64_t seed, uint32_t stream) {
  double e, o;
  philox_uniform2(ctr0, idx >> 1, seed, stream, e, o);
  return (idx & 1) ? o : e;
}

}  // namespace aiy
