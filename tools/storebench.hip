// Store-pattern microbenchmark for GEMM epilogues: writes an [M][N] fp32
// matrix (N = 256) in different per-instruction shapes and reports the write
// rate.  hipcc --offload-arch=gfx950 -O3 tools/storebench.hip -o /tmp/storebench
#include <hip/hip_runtime.h>
#include <stdio.h>

// mode 0: a wave owns 32 rows x 128 columns (one N half, the half chosen by
//         blockIdx parity); an instruction = 8 rows x 128 B (the 32x32
//         kernel's epilogue shape)
// mode 1: a wave owns 32 rows x 256 columns; an instruction = 8 rows x 128 B
// mode 2: a wave owns 32 rows x 256 columns; an instruction = 4 rows x 256 B
// mode 3: a wave owns 32 rows x 256 columns; an instruction = 1 row x 1 KB
// mode 4: flat: an instruction = 1 KB contiguous, consecutive waves consecutive KB
__global__ __launch_bounds__(256) void store_kernel(float* __restrict__ y, long M, int mode,
                                                   int reps_per_wave) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long gw = (long)blockIdx.x * 4 + wave;
  const long nw = (long)gridDim.x * 4;
  const float4 v = make_float4(1.f, 2.f, 3.f, (float)lane);
  const long ntile = M / 32;
  for (int it = 0; it < reps_per_wave; ++it) {
    if (mode == 4) {
      const long t = gw + it * nw;  // 32 rows x 1 KB per wave step, flat
      if (t >= ntile) return;
      float* base = y + t * 32 * 256;
#pragma unroll 4
      for (int i = 0; i < 32; ++i) *reinterpret_cast<float4*>(base + i * 256 + lane * 4) = v;
      continue;
    }
    if (mode == 0) {
      const long t2 = gw + it * nw;  // (tile, half) pairs
      const long t = t2 >> 1;
      const int half = (int)(t2 & 1);
      if (t >= ntile) return;
      float* base = y + t * 32 * 256 + half * 128;
      const int rp = lane >> 3, q = lane & 7;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<float4*>(base + (rp + 8 * r) * 256 + u * 32 + 4 * q) = v;
      continue;
    }
    const long t = gw + it * nw;
    if (t >= ntile) return;
    float* base = y + t * 32 * 256;
    if (mode == 1) {
      const int rp = lane >> 3, q = lane & 7;
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<float4*>(base + (rp + 8 * r) * 256 + u * 32 + 4 * q) = v;
    } else if (mode == 2) {
      const int rp = lane >> 4, q = lane & 15;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int r = 0; r < 8; ++r)
          *reinterpret_cast<float4*>(base + (rp + 4 * r) * 256 + u * 64 + 4 * q) = v;
    } else {
#pragma unroll 4
      for (int r = 0; r < 32; ++r) *reinterpret_cast<float4*>(base + r * 256 + 4 * lane) = v;
    }
  }
}

int main() {
  const long M = 4194304, N = 256;
  float* y = nullptr;
  if (hipMalloc(&y, M * N * sizeof(float)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"32x128 per wave, 8 rows x 128 B", "32x256 per wave, 8 rows x 128 B",
                         "32x256 per wave, 4 rows x 256 B", "32x256 per wave, 1 row x 1 KB",
                         "flat 1 KB"};
  for (int grid : {768, 2048, 8192}) {
    for (int mode = 0; mode < 5; ++mode) {
      const long units = mode == 0 ? 2 * (M / 32) : M / 32;
      const int reps = (int)((units + (long)grid * 4 - 1) / ((long)grid * 4));
      for (int w = 0; w < 2; ++w) store_kernel<<<grid, 256>>>(y, M, mode, reps);
      hipEventRecord(e0);
      for (int i = 0; i < 5; ++i) store_kernel<<<grid, 256>>>(y, M, mode, reps);
      hipEventRecord(e1);
      if (hipEventSynchronize(e1) != hipSuccess) return 2;
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1000.0 / 5;
      printf("grid %5d  mode %d  %-34s %8.1f us  %6.2f TB/s\n", grid, mode, names[mode], us,
             M * N * 4.0 / us / 1e6);
    }
  }
  hipFree(y);
  return 0;
}
