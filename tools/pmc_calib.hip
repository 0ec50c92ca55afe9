// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths this repository's
// kernels use (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the bytes of a 16-B-per-lane
// streaming read on gfx950; other widths are uncalibrated).  Streams a 1 GiB buffer (beyond
// the 256 MiB Infinity Cache) once per kernel with a known byte count:
//   read8   8 B per lane  (a double per lane: the EGM window loads, the histogram vectors)
//   read16  16 B per lane (a double2 per lane)
//   write8  8 B per lane stores
//   write16 16 B per lane stores
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/bin/pmc_calib
// Run:   rocprofv3 --pmc FETCH_SIZE -d <dir> -o run --output-format csv -- tools/bin/pmc_calib
//        (and a separate pass with WRITE_SIZE); python tools/pmc_calib_summary.py <dir> <dir>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__global__ void read8(const double* __restrict__ a, size_t n, double* __restrict__ out) {
  double acc = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += a[i];
  if (acc == 12345.678) out[0] = acc;   // keeps the loads; never true for the zero-filled buffer
}

__global__ void read16(const double2* __restrict__ a, size_t n2, double* __restrict__ out) {
  double acc = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;
}

__global__ void write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = 1.0;
}

__global__ void write16(double2* __restrict__ a, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_double2(1.0, 2.0);
}

int main() {
  const size_t bytes = (size_t)1 << 30;   // 1 GiB
  const size_t n = bytes / sizeof(double);
  double* a = nullptr;
  double* out = nullptr;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&out, sizeof(double)));
  CHECK(hipMemset(a, 0, bytes));
  CHECK(hipDeviceSynchronize());
  const dim3 grid(256 * 8), block(256);
  for (int rep = 0; rep < 2; ++rep) {
    read8<<<grid, block>>>(a, n, out);
    read16<<<grid, block>>>(reinterpret_cast<const double2*>(a), n / 2, out);
    write8<<<grid, block>>>(a, n);
    write16<<<grid, block>>>(reinterpret_cast<double2*>(a), n / 2);
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::printf("pmc_calib: %zu bytes per kernel\n", bytes);
  CHECK(hipFree(a));
  CHECK(hipFree(out));
  return 0;
}
