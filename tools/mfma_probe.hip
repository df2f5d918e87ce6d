// Micro-probe (tools only, not part of the product): issue rate of
// v_mfma_f32_32x32x2_f32 as a single dependent accumulation chain vs
// round-robin over K independent accumulators, at 1 or 2 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mfma_probe.hip -o build/mfma_probe.so
// probe_run(kacc, iters, waves_per_block, blocks, out_ms) -> 0
#include <hip/hip_runtime.h>

typedef float f16v __attribute__((ext_vector_type(16)));

template <int K>
__global__ __launch_bounds__(512) void probe_kernel(float* out, int iters, float a0, float b0) {
  f16v acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[k][i] = 0.f;
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
    // 16 MFMAs per iteration, accumulator (m mod K): K = 1 is one dependent chain
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m % K] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m % K], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[k][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

extern "C" int probe_run(int kacc, int iters, int waves, int blocks, float* out_ms) {
  float* out;
  if (hipMalloc(&out, (size_t)blocks * waves * 64 * 4) != hipSuccess) return 1;
  auto launch = [&]() {
    dim3 g(blocks), b(64 * waves);
    switch (kacc) {
      case 1: hipLaunchKernelGGL(probe_kernel<1>, g, b, 0, 0, out, iters, 1.f, 1.f); break;
      case 2: hipLaunchKernelGGL(probe_kernel<2>, g, b, 0, 0, out, iters, 1.f, 1.f); break;
      case 4: hipLaunchKernelGGL(probe_kernel<4>, g, b, 0, 0, out, iters, 1.f, 1.f); break;
      default: hipLaunchKernelGGL(probe_kernel<8>, g, b, 0, 0, out, iters, 1.f, 1.f); break;
    }
  };
  launch();
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int r = 0; r < 5; ++r) launch();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  *out_ms = ms / 5;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(out);
  return 0;
}
