#include "common.h"
#include "internal.h"
#include "hist_cluster.h"
#include "hist_bicg.h"
namespace aiy {
template <int SMAX, int KC, int TH, bool PIPE>
__global__ __launch_bounds__(TH) void probe_kernel(HkArgs a, unsigned* o) {
  unsigned nb = 0, ne = 0;
  o[blockIdx.x] = hk_solve_inlined<SMAX, KC, TH, false, PIPE>(a, &nb, &ne);
}
template __global__ void probe_kernel<7, 1, 512, true>(HkArgs, unsigned*);
}
