// Does fp32 MFMA (v_mfma_f32_16x16x4_f32) co-execute with fp32 VALU work on
// the same SIMD?  One workgroup of 4 waves per CU (one wave per SIMD), every
// CU busy; each wave runs N iterations of {M MFMAs on independent
// accumulators, V independent v_pk_fma_f32}.  Times: MFMA only, VALU only,
// both interleaved.  hipcc --offload-arch=gfx950 -O3 mfma_valu_overlap.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int M, int V>
__global__ __launch_bounds__(256, 1) void k(float* out, int iters, float s) {
  f32x4 acc[8];
  for (int u = 0; u < 8; ++u) acc[u] = (f32x4){s, s + 1, s + 2, s + 3};
  f32x2 v[8];
  for (int u = 0; u < 8; ++u) v[u] = (f32x2){s * u, s + u};
  const float a = s * 0.5f + threadIdx.x, b = s * 0.25f - threadIdx.x;
  const f32x2 w = {1.0001f, 0.9999f}, c = {1e-7f, -1e-7f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int u = 0; u < M; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[u], 0, 0, 0);
#pragma unroll
      for (int u = 0; u < V; ++u) v[u & 7] = __builtin_elementwise_fma(v[u & 7], w, c);
    }
  }
  float t = 0.f;
  for (int u = 0; u < 8; ++u) t += acc[u][0] + acc[u][3] + v[u][0] + v[u][1];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

// two waves per SIMD: waves 0-3 run M MFMAs per step only, waves 4-7 V
// pk_fma per step only (separate waves sharing each SIMD)
template <int M, int V>
__global__ __launch_bounds__(512, 1) void k2(float* out, int iters, float s) {
  f32x4 acc[8];
  for (int u = 0; u < 8; ++u) acc[u] = (f32x4){s, s + 1, s + 2, s + 3};
  f32x2 v[8];
  for (int u = 0; u < 8; ++u) v[u] = (f32x2){s * u, s + u};
  const float a = s * 0.5f + threadIdx.x, b = s * 0.25f - threadIdx.x;
  const f32x2 w = {1.0001f, 0.9999f}, c = {1e-7f, -1e-7f};
  const bool mf = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < 4;
  if (mf) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int u = 0; u < M; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[u], 0, 0, 0);
  } else {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int u = 0; u < V; ++u) v[u & 7] = __builtin_elementwise_fma(v[u & 7], w, c);
  }
  float t = 0.f;
  for (int u = 0; u < 8; ++u) t += acc[u][0] + acc[u][3] + v[u][0] + v[u][1];
  out[blockIdx.x * 512 + threadIdx.x] = t;
}

template <int M, int V>
float run2(float* out, int iters, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k2<M, V><<<ncu, 512>>>(out, 2, 1.f);
  hipEventRecord(e0);
  k2<M, V><<<ncu, 512>>>(out, iters, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

template <int M, int V>
float run(float* out, int iters, int ncu) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<M, V><<<ncu, 256>>>(out, 2, 1.f);
  hipEventRecord(e0);
  k<M, V><<<ncu, 256>>>(out, iters, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  int ncu;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, ncu * 512 * 4);
  const int iters = 2000;
  // per iteration: 8 * M MFMAs (32 cyc each) and 8 * V pk_fma
  float m = run<4, 0>(out, iters, ncu);
  float v8 = run<0, 8>(out, iters, ncu);
  float v16 = run<0, 16>(out, iters, ncu);
  float mv8 = run<4, 8>(out, iters, ncu);
  float mv16 = run<4, 16>(out, iters, ncu);
  float v4 = run<0, 4>(out, iters, ncu);
  float mv4 = run<4, 4>(out, iters, ncu);
  const double mf = 8.0 * 4 * iters;  // MFMAs per wave
  printf("MFMA only (4/step):          %8.3f ms  %.1f cyc/MFMA at 2.4 GHz\n", m, m * 2.4e6 / mf);
  printf("VALU only 4 pk_fma/step:      %8.3f ms\n", v4);
  printf("VALU only 8 pk_fma/step:      %8.3f ms\n", v8);
  printf("VALU only 16 pk_fma/step:     %8.3f ms\n", v16);
  printf("4 MFMA + 4 pk_fma per step:   %8.3f ms  (sum %.3f, max %.3f)\n", mv4, m + v4, m > v4 ? m : v4);
  printf("4 MFMA + 8 pk_fma per step:   %8.3f ms  (sum %.3f, max %.3f)\n", mv8, m + v8, m > v8 ? m : v8);
  printf("4 MFMA + 16 pk_fma per step:  %8.3f ms  (sum %.3f, max %.3f)\n", mv16, m + v16, m > v16 ? m : v16);
  float x_m = run2<4, 0>(out, iters, ncu);
  float x_v = run2<0, 16>(out, iters, ncu);
  float x_mv = run2<4, 16>(out, iters, ncu);
  float x_mv8 = run2<4, 8>(out, iters, ncu);
  printf("two waves/SIMD: MFMA wave only %.3f, VALU(16) wave only %.3f, both %.3f, both with VALU(8) %.3f ms\n",
         x_m, x_v, x_mv, x_mv8);
  return 0;
}
