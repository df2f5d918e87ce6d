// Micro-probe 2 (tools only): the SIMD-time price of each instruction kind issued
// beside a v_mfma_f32_32x32x2_f32 stream, and whether the MFMA's
// accumulator file (AGPR vs VGPR) changes it.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/coissue_probe2.hip -o tools/coissue_probe2.so
// run(kind, acc_vgpr, roles, iters_m, iters_o, out_ms): one 512-thread block per CU;
// waves 0-3 run iters_m x 16 MFMAs (accumulators in AGPRs, or VGPRs when acc_vgpr)
// when roles & 1; waves 4-7 run iters_o x 16 instructions of `kind` when roles & 2:
//   1 v_fma_f32   2 v_mov_b32   3 ds_read_b32   4 ds_read_b64   5 ds_read_b128
//   6 ds_write_b128   7 global_load_dwordx4 (L2-resident 64 KB)   8 LDS-DMA 16 B
//   9 s_add_u32 (SALU)   10 s_nop 0
// (reads/loads: one s_waitcnt per 16; 1-6: lgkmcnt, 7-8: vmcnt).  self(kind, k, iters,
// out_ms): waves 0-3 alone, each MFMA followed by k instructions of `kind` of its own.
#include <hip/hip_runtime.h>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

template <bool V>
__device__ inline void mfma(f16v& acc, float a, float b) {
  if constexpr (V)
    asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int K>
__device__ inline void other16(float* r, const uint4* buf, uint4* sm, int lid, float& sink) {
  if constexpr (K == 1) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[k & 7]) : "v"(r[8]), "v"(r[9]));
  } else if constexpr (K == 2) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("v_mov_b32 %0, %1" : "=v"(r[k & 7]) : "v"(r[8 + (k & 1)]));
  } else if constexpr (K == 3 || K == 4 || K == 5) {
    const char* base = reinterpret_cast<const char*>(sm);
    constexpr int B = K == 3 ? 4 : (K == 4 ? 8 : 16);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const char* p = base + (k * 64 + lid) * B;
      if constexpr (K == 3) {
        float v = *reinterpret_cast<const float*>(p);
        asm volatile("" ::"v"(v));
      } else if constexpr (K == 4) {
        f2v v = *reinterpret_cast<const f2v*>(p);
        asm volatile("" ::"v"(v));
      } else {
        f4v v = *reinterpret_cast<const f4v*>(p);
        asm volatile("" ::"v"(v));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sink += acc;
  } else if constexpr (K == 6) {
    f4v v = {r[0], r[1], r[2], r[3]};
#pragma unroll
    for (int k = 0; k < 16; ++k) *reinterpret_cast<f4v*>(sm + 2048 + k * 64 + lid) = v;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else if constexpr (K == 7) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(buf) + k * 64 + lid);
      asm volatile("" ::"v"(v));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if constexpr (K == 8) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(buf + k * 64 + lid),
                                       (__attribute__((address_space(3))) void*)(sm + 4096 + (k & 7) * 64), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if constexpr (K == 9) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("s_add_u32 s0, s0, 1" ::: "s0", "scc");
  } else if constexpr (K == 10) {
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("s_nop 0");
  }
}

template <int K, bool V>
__global__ __launch_bounds__(512, 1) void pair_kernel(float* out, const uint4* buf, int roles, int iters_m, int iters_o) {
  extern __shared__ __attribute__((aligned(16))) uint4 sm[];
  const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  float res = 0.f;
  if (wv < 4) {
    if (roles & 1) {
      f16v acc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = f16v{};
      const float a = 1.f + tid * 1e-7f, b = 1.f - tid * 1e-7f;
      for (int it = 0; it < iters_m; ++it) {
#pragma unroll
        for (int m = 0; m < 16; ++m) mfma<V>(acc[m & 3], a, b);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) res += acc[k][i];
    }
  } else if (roles & 2) {
    float r[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) r[k] = 1.f + k * 1e-3f + tid * 1e-7f;
    float sink = 0.f;
    for (int it = 0; it < iters_o; ++it) other16<K>(r, buf, sm, lane, sink);
#pragma unroll
    for (int k = 0; k < 10; ++k) res += r[k];
    res += sink;
  }
  out[blockIdx.x * 512 + tid] = res;
}

// waves 0-3 alone: each MFMA followed by k of its own `kind` instructions (kind 1, 5, 8)
template <int K, int N>
__global__ __launch_bounds__(256, 1) void self_kernel(float* out, const uint4* buf, int iters) {
  extern __shared__ __attribute__((aligned(16))) uint4 sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  f16v acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = f16v{};
  const float a = 1.f + tid * 1e-7f, b = 1.f - tid * 1e-7f;
  float r[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) r[k] = 1.f + k * 1e-3f;
  f4v s = f4v{};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      mfma<false>(acc[q & 3], a, b);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        if constexpr (K == 1) {
          asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[k & 7]) : "v"(r[8]), "v"(r[9]));
        } else if constexpr (K == 5) {
          f4v v = *reinterpret_cast<const f4v*>(sm + ((q * N + k) & 31) * 64 + lane);
          asm volatile("" ::"v"(v));
          s += v;
        } else {
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(buf + ((q * N + k) & 15) * 64 + lane),
                                           (__attribute__((address_space(3))) void*)(sm + 4096 + ((q + k) & 7) * 64), 16, 0, 0);
        }
      }
    }
    if constexpr (K == 5) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (K == 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float res = s[0] + s[1];
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
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < 5; ++r) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  *out_ms = ms / 5;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

static float* g_out = nullptr;
static uint4* g_buf = nullptr;
static int setup() {
  if (g_out) return 0;
  if (hipMalloc(&g_out, 256 * 512 * 4) != hipSuccess) return 1;
  if (hipMalloc(&g_buf, 1 << 20) != hipSuccess) return 1;
  return hipMemset(g_buf, 0, 1 << 20) == hipSuccess ? 0 : 1;
}

template <int K, bool V>
static int run_k(int roles, int im, int io, float* ms) {
  auto k = pair_kernel<K, V>;
  const size_t lds = 128 * 1024;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return timed([&]() { hipLaunchKernelGGL(k, dim3(256), dim3(512), lds, 0, g_out, g_buf, roles, im, io); }, ms);
}

extern "C" int run(int kind, int accv, int roles, int im, int io, float* ms) {
  if (setup()) return 1;
#define CASE(K)                                                                       \
  case K:                                                                             \
    return accv ? run_k<K, true>(roles, im, io, ms) : run_k<K, false>(roles, im, io, ms);
  switch (kind) {
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10)
  }
#undef CASE
  return 9;
}

template <int K, int N>
static int self_k(int iters, float* ms) {
  auto k = self_kernel<K, N>;
  const size_t lds = 128 * 1024;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return timed([&]() { hipLaunchKernelGGL(k, dim3(256), dim3(256), lds, 0, g_out, g_buf, iters); }, ms);
}

extern "C" int self_run(int kind, int n, int iters, float* ms) {
  if (setup()) return 1;
#define S(K, N) \
  if (kind == K && n == N) return self_k<K, N>(iters, ms);
  S(1, 0) S(1, 1) S(1, 2) S(1, 4)
  S(5, 1) S(5, 2) S(5, 4)
  S(8, 1) S(8, 2)
#undef S
  return 9;
}
