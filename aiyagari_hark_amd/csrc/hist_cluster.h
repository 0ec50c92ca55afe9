// Shared pieces of the device-resident distribution-iteration kernels (hist_resident.hip:
// plain / Aitken iteration; hist_krylov.hip: BiCGSTAB): the per-calibration cluster run
// description, the covering-span record, the cluster barrier and wave sums.
#pragma once

#include "common.h"

namespace aiy {

constexpr int kHcMaxG = 128;                       // workgroups per calibration cluster
constexpr int kHcCand = 32;                        // covering workgroups per (row, workgroup)
constexpr int kHcRows = 8;                         // rows whose push loads are in flight together
// rows whose gather loads are in flight together: all (S <= 8) for one column per thread
template <int SMAX, int KC, int TH>
struct HcGather {
  static constexpr int kRows = SMAX == 8 ? 8 : 4;
};
constexpr size_t kHcLdsTotal = 160 * 1024;         // per CU
constexpr unsigned long long kHcTimeoutTicks = 200000000ull;   // 2 s of the 100 MHz clock
constexpr int kHcCtrStride = 32;
constexpr int kHcRedRec = 16;                     // 8-byte words per (parity, workgroup) record of `dist`                   // uints between cluster counters (128 B)

struct HcRun {
  int n_cal, cal0, S, n_a, G, nj, cap;   // cap: doubles of the span buffer / one slab
  int cw;                 // pull form: columns of one matvec chunk (hist_pull_plan)
  const int* lo;          // [n_cal][S][n_a]
  const double* wlo;      // [n_cal][S][n_a]
  const double* P;        // [n_cal][S][S]
  double* mass;           // [n_cal][S][n_a] in: start, out: final
  double* slab;           // [launch cals][G][2][cap]
  int* span;              // [launch cals][G][SMAX][4] (first, len, left base, right base)
  unsigned* ctr;          // [launch cals][kHcCtrStride]
  double* dist;           // [launch cals][2][G][4]: sup-norm change, Aitken dot products, valid
  double* dbuf;           // [n_cal][S][n_a] stored differences for the Aitken step (accel > 0);
                          // pull form (hist_pull.h): [n_cal][4][S][n_a] BiCGSTAB vectors r, p, v, t
  int* ainv;              // pull form: [n_cal][S][n_a + 1] inverse lottery
  int accel;              // Aitken extrapolation period E (0: plain iteration = the oracle's)
  int* iters_out;         // [n_cal]
  unsigned* err;          // 0 ok, 1 timeout, 2 span overflow / not monotone, 3 candidate overflow
  double tol;
  const double* tolv;     // [n_cal] per-calibration tolerance (device) or null: tol
  int max_iter;
};

struct HcCand {
  int w, first, len, base;   // destination d of the covering span sits at slab/LDS index base + d
};

// Cluster barrier: lane 0 adds one to the cluster counter (after the caller's drained sc1
// stores) and waits until it reaches `target`.  False on timeout (error word set).
__device__ __forceinline__ bool hc_barrier(unsigned* err, unsigned* ctr, unsigned target, int* s_flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(to_global(ctr), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while (__hip_atomic_load(to_global(ctr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kHcTimeoutTicks) {
        __hip_atomic_store(to_global(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *s_flag = ok;
  }
  __syncthreads();
  return *s_flag != 0;
}
__device__ __forceinline__ bool hc_barrier(const HcRun& r, unsigned* ctr, unsigned target, int* s_flag) {
  return hc_barrier(r.err, ctr, target, s_flag);
}

// Cluster barrier that also counts the workgroups whose `flag` is set: lane 0 adds
// (1 | flag << 32) to the 64-bit word of the barrier's parity (low half: arrivals, high
// half: cumulative flags of that parity; a workgroup can run at most one barrier ahead, so
// the other parity's word takes its early add) and waits for `target` arrivals (G times
// the barriers of this parity so far).  *nc_out: the flag count of this parity after every
// workgroup's add.  False on timeout (error word set).
__device__ __forceinline__ bool hc_barrier_count(unsigned* err, unsigned long long* cw, unsigned target,
                                                 unsigned flag, unsigned* nc_out, int* s_flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long v = __hip_atomic_fetch_add(to_global(cw), 1ull | ((unsigned long long)flag << 32), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) +
                           (1ull | ((unsigned long long)flag << 32));
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while ((unsigned)v < target) {
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(to_global(cw), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kHcTimeoutTicks) {
        __hip_atomic_store(to_global(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *nc_out = (unsigned)(v >> 32);
    *s_flag = ok;
  }
  __syncthreads();
  return *s_flag != 0;
}

// One covering span's value at destination d: the own span from LDS (read once by the
// column's owner, then re-zeroed for the next push), a foreign one from its published slab.
__device__ __forceinline__ double hc_take(const HcCand& c, int w, int d, int par, int cap, const double* slab_cl,
                                          double* Tacc) {
  const int q = c.base + d;
  // two destinations (added at the use): one shared register would make the LDS read
  // wait for every earlier slab load in flight (write-after-write on the register)
  double vg = 0.0, vl = 0.0;
  if (c.w == w) {
    vl = Tacc[q];
    Tacc[q] = 0.0;
  } else {
    vg = load_f64_agent(&slab_cl[((size_t)c.w * 2 + par) * cap + q]);
  }
  return vg + vl;
}

// Sum over the 64 lanes (DPP: row shifts, then row broadcasts), valid in lane 63.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_add_src(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROWS, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_sum_lane63(double v) {
  v += dpp_add_src<0x111, 0xF>(v);   // row_shr:1
  v += dpp_add_src<0x112, 0xF>(v);   // row_shr:2
  v += dpp_add_src<0x114, 0xF>(v);   // row_shr:4
  v += dpp_add_src<0x118, 0xF>(v);   // row_shr:8   (lane 15 of every row: the row's sum)
  v += dpp_add_src<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
  v += dpp_add_src<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3
  return v;
}

// BiCGSTAB form of the cluster kernel (hist_krylov.hip) for (S, padded S, columns per
// thread) and its state count (*smax_k); nullptr when there is no instantiation
const void* hist_bicg_pick(int S, int smax, int kc, int* smax_k, bool pull = false);
// pull form (hist_pull.h) for S > 8: the kernel, and its dynamic LDS for n_own columns
const void* hist_pull_pick(int S);
// pull form: the column chunk of a matvec (fewest item rounds + mix passes whose LDS fits
// `budget`) and its dynamic LDS bytes; false when even one-column chunks do not fit
bool hist_pull_plan(int S, int n_own, size_t budget, int* cw, size_t* lds);
#ifdef AIY_HP_TH
constexpr int kHpTH = AIY_HP_TH;   // tuning builds only
#else
constexpr int kHpTH = 512;
#endif

}  // namespace aiy
