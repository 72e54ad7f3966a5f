// Diagnostic probe (round 6): is a once-per-dispatch straight-line code path
// instruction-fetch bound on gfx950?  One 512-thread workgroup per CU runs
// (a) 2,048 VALU instructions straight-line (~16 KB of code), (b) the same
// 2,048 as a loop of 8 x 256 (~2 KB fetched once), (c) 256 straight-line
// once; s_memtime around each, wave 0's cycles written per workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define V8(x) x x x x x x x x
#define V64(x) V8(V8(x))
#define V256(x) V64(x) V64(x) V64(x) V64(x)
#define STEP asm volatile("v_add_f32 %0, %0, %1\n v_mul_f32 %1, %1, %0" : "+v"(a), "+v"(b));

__global__ __launch_bounds__(512) void probe(unsigned long long* out, float* sink, int reps) {
  float a = threadIdx.x, b = 1.0001f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  V256(STEP) V256(STEP) V256(STEP) V256(STEP)   // 2 x 1,024 instructions straight-line
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) { V64(STEP) }   // reps x 128 instructions, one body
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  V64(STEP)                                      // 128 straight-line, code not yet fetched
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = t1 - t0;
    out[blockIdx.x * 4 + 1] = t2 - t1;
    out[blockIdx.x * 4 + 2] = t3 - t2;
  }
  if (a == 12345.f) sink[0] = b;
}

int main() {
  const int nwg = 40;
  unsigned long long* d;
  float* s;
  hipMalloc(&d, nwg * 4 * 8);
  hipMalloc(&s, 4);
  std::vector<unsigned long long> h(nwg * 4);
  for (int it = 0; it < 5; ++it) {
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(512), 0, 0, d, s, 16);
    hipDeviceSynchronize();
  }
  hipMemcpy(h.data(), d, nwg * 4 * 8, hipMemcpyDeviceToHost);
  double a = 0, b = 0, c = 0;
  for (int i = 0; i < nwg; ++i) { a += h[i * 4]; b += h[i * 4 + 1]; c += h[i * 4 + 2]; }
  printf("{\"straight_2048_instr_cycles\": %.0f, \"loop_16x128_instr_cycles\": %.0f, \"straight_128_cold_cycles\": %.0f}\n",
         a / nwg, b / nwg, c / nwg);
  return 0;
}
