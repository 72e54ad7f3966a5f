// Diagnostic (not product): cost of the wave-level top-K primitives.
// One wave per block; each wave runs REPS iterations of a primitive on
// register data; the kernel trace gives the time per iteration.
#include "../../hhfm_amd/csrc/topk_common.h"
#include <cstdio>
using namespace hhfm;

template <int MODE>
__global__ __launch_bounds__(64) void bench(float* out, int reps) {
  const int l = lane_id();
  float s = __int_as_float(0x3f000000 + l * 977 % 64 * 1000);
  int32_t i = l;
  for (int r = 0; r < reps; ++r) {
    if constexpr (MODE == 0) bitonic_sort_desc<64>(s, i);
    if constexpr (MODE == 1) bitonic_merge_desc<32>(s, i);
    if constexpr (MODE == 2) { s = xor_lane(s, 16); }
    if constexpr (MODE == 3) { s = xor_lane(s, 32); }
    if constexpr (MODE == 4) { s = xor_lane(s, 1); }
    if constexpr (MODE == 5) { s = xor_lane(s, 4); }
    if constexpr (MODE == 6) { s = __shfl_xor(s, 16, 64); }
    if constexpr (MODE == 7) { cx(s, i, 1, (l & 1) == 0); }
    if constexpr (MODE == 8) { s = s * 1.0001f + 0.5f; }
    s += 1e-7f;
  }
  out[blockIdx.x * 64 + l] = s + i;
}

int main() {
  float* d;
  hipMalloc(&d, 1 << 20);
  const int reps = 10000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"sort64", "merge32", "xor16", "xor32", "xor1", "xor4", "shfl_xor16", "cx1", "fma"};
  for (int m = 0; m < 9; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      switch (m) {
        case 0: hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 1: hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 2: hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 3: hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 4: hipLaunchKernelGGL(bench<4>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 5: hipLaunchKernelGGL(bench<5>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 6: hipLaunchKernelGGL(bench<6>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 7: hipLaunchKernelGGL(bench<7>, dim3(1), dim3(64), 0, 0, d, reps); break;
        case 8: hipLaunchKernelGGL(bench<8>, dim3(1), dim3(64), 0, 0, d, reps); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("%-10s %8.1f ns/iter  (%.0f cycles at 2.4 GHz)\n", names[m], ms * 1e6 / reps, ms * 1e6 / reps * 2.4);
    }
  }
  return 0;
}
