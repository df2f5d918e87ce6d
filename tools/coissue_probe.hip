// Micro-probe (tools only, not part of the product): does a v_mfma_f32_32x32x2_f32
// stream on a SIMD leave room for another wave's VALU / LDS-read / LDS-DMA issue,
// or for the same wave's VALU between its MFMAs?  
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/coissue_probe.hip -o tools/coissue_probe.so
//
// pair_run(other, roles, iters_m, iters_o, out_ms): one 512-thread block per CU (256
// blocks); waves 0-3 (one per SIMD) run iters_m x 16 MFMAs on 4 accumulators when
// roles & 1, waves 4-7 (the SIMD partners) run iters_o x 16 "other" instructions when
// roles & 2: other 1 = v_fma_f32 (8 independent chains), 2 = ds_read_b128 (8 per
// lgkmcnt(0) wait), 3 = global_load_lds_dwordx4 LDS-DMA from an L2-resident 64 KB
// buffer (4 per vmcnt(0) wait), 4 = the Winograd chunk mix (8 ds_read_b128 + 32 VALU
// + 2 DMA per 16).  T(both) ~ max(T(m), T(o)) means the pipes overlap; ~ sum, they
// serialise.
// self_run(k, iters, out_ms): waves 0-3 alone, each MFMA followed by k v_fma_f32 of its
// own (sched_group_barrier pins the pattern): cycles per MFMA vs k.
#include <hip/hip_runtime.h>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ inline void dma16(const uint4* src, uint4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <int OTHER>
__global__ __launch_bounds__(512, 1) void pair_kernel(float* out, const uint4* buf, int roles, int iters_m,
                                                      int iters_o, float a0) {
  extern __shared__ __attribute__((aligned(16))) uint4 sm[];
  const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  float res = 0.f;
  if (wv < 4) {
    if (roles & 1) {
      f16v acc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = f16v{};
      const float a = a0 + tid * 1e-7f, b = a0 - tid * 1e-7f;
      for (int it = 0; it < iters_m; ++it) {
#pragma unroll
        for (int m = 0; m < 16; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 3], 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) res += acc[k][i];
    }
  } else if (roles & 2) {
    if constexpr (OTHER == 1) {
      float r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = a0 + k + tid;
      const float m = 1.0000001f, c = 1e-9f;
      for (int it = 0; it < iters_o; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[k & 7]) : "v"(m), "v"(c));
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) res += r[k];
    } else if constexpr (OTHER == 2) {
      f4v s = f4v{};
      const f4v* p = reinterpret_cast<const f4v*>(sm) + (tid - 256);
      for (int it = 0; it < iters_o; ++it) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f4v v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = p[k * 256];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(v[k]));
          s += v[it & 7];
        }
      }
      res = s[0] + s[1] + s[2] + s[3];
    } else if constexpr (OTHER == 3) {
      uint4* dst = sm + ((tid - 256) & ~63);
      const uint4* src = buf + (tid - 256);
      for (int it = 0; it < iters_o; ++it) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
#pragma unroll
          for (int k = 0; k < 4; ++k) dma16(src + ((h * 4 + k) & 15) * 256, dst + k * 256);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      res = reinterpret_cast<const float*>(sm)[tid];
    } else if constexpr (OTHER == 4) {
      f4v s = f4v{};
      const f4v* p = reinterpret_cast<const f4v*>(sm) + (tid - 256);
      uint4* dst = sm + 4096 + ((tid - 256) & ~63);
      const uint4* src = buf + (tid - 256);
      for (int it = 0; it < iters_o; ++it) {
        dma16(src + (it & 7) * 256, dst);
        dma16(src + ((it + 1) & 7) * 256, dst + 256);
        f4v v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[k * 256];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        f4v t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) t[k][e] = fmaf(-1.f, v[2 * k + 1][e], v[2 * k][e]);
        f4v w0 = t[0] - t[2], w1 = t[1] + t[2], w2 = t[2] - t[1], w3 = t[1] - t[3];
        asm volatile("" ::"v"(w0), "v"(w1), "v"(w2), "v"(w3));
        s += w0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      res = s[0] + s[1] + s[2] + s[3];
    }
  }
  out[blockIdx.x * 512 + tid] = res;
}

template <int K>
__global__ __launch_bounds__(256, 1) void self_kernel(float* out, int iters, float a0) {
  f16v acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = f16v{};
  const int tid = threadIdx.x;
  const float a = a0 + tid * 1e-7f, b = a0 - tid * 1e-7f;
  float r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = a0 + k + tid;
  const float m = 1.0000001f, c = 1e-9f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc[q & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[q & 3], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < K; ++k) r[k & 7] = fmaf(r[k & 7], m, c + (float)k);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (K) __builtin_amdgcn_sched_group_barrier(0x002, K, 0);
    }
  }
  float res = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) res += acc[k][i];
#pragma unroll
  for (int k = 0; k < 8; ++k) res += r[k];
  out[blockIdx.x * 256 + tid] = res;
}

template <class L>
static int timed(L launch, float* out_ms) {
  launch();
  if (hipDeviceSynchronize() != hipSuccess) return 2;
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
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

extern "C" int pair_run(int other, int roles, int iters_m, int iters_o, float* out_ms) {
  float* out;
  uint4* buf;
  if (hipMalloc(&out, 256 * 512 * 4) != hipSuccess) return 1;
  if (hipMalloc(&buf, 64 * 1024) != hipSuccess) return 1;
  hipMemset(buf, 0, 64 * 1024);
  const size_t lds = 128 * 1024;  // one block per CU
  int rc = 0;
  auto go = [&](auto k) {
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    rc = timed([&]() { hipLaunchKernelGGL(k, dim3(256), dim3(512), lds, 0, out, buf, roles, iters_m, iters_o, 1.f); },
               out_ms);
  };
  switch (other) {
    case 1: go(pair_kernel<1>); break;
    case 2: go(pair_kernel<2>); break;
    case 3: go(pair_kernel<3>); break;
    default: go(pair_kernel<4>); break;
  }
  hipFree(out);
  hipFree(buf);
  return rc;
}

extern "C" int self_run(int k, int iters, float* out_ms) {
  float* out;
  if (hipMalloc(&out, 256 * 256 * 4) != hipSuccess) return 1;
  int rc = 0;
  auto go = [&](auto kern) {
    rc = timed([&]() { hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, out, iters, 1.f); }, out_ms);
  };
  switch (k) {
    case 0: go(self_kernel<0>); break;
    case 2: go(self_kernel<2>); break;
    case 4: go(self_kernel<4>); break;
    case 8: go(self_kernel<8>); break;
    case 12: go(self_kernel<12>); break;
    case 16: go(self_kernel<16>); break;
    default: go(self_kernel<24>); break;
  }
  hipFree(out);
  return rc;
}
