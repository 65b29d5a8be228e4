// the optimizer step after backward — torch.optim.Adam
// (train_mobilenetV3_ecagai.py:564: Adam(lr, weight_decay=5e-4), amsgrad off)
// over every parameter tensor in ONE launch.
//
// The tensors are described by a device table of {param, grad, exp_avg,
// exp_avg_sq, numel} rows; a second table maps each 1024-element chunk to its
// (tensor, offset), so a workgroup of 256 threads updates one chunk as
// float4s (scalar tail for a tensor whose numel % 4 != 0).  Per element, in
// torch's order (single-tensor / foreach Adam):
//   g  = grad + weight_decay * p
//   m  = lerp(m, g, 1 - beta1)            (torch lerp: w < 0.5 ? m + w (g - m)
//                                                   : g - (g - m)(1 - w))
//   v  = v * beta2 + (1 - beta2) * g * g
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// with bc1 = 1 - beta1^step, bc2 = 1 - beta2^step computed on the host.
#include "common.h"

namespace jabd {

struct AdamRow {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
};

constexpr int kAdamChunk = 1024;

__device__ __forceinline__ float adam_lerp(float a, float b, float w) {
  return w < 0.5f ? a + w * (b - a) : b - (b - a) * (1.f - w);
}

// The scalars arrive as torch computes them: Python doubles (1 - beta2,
// lr / bc1, sqrt(bc2)) rounded once to fp32.
struct AdamScalars {
  float step_size, w1, b2, omb2, bc2s, eps, wd;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v,
                                          const AdamScalars& s) {
  if (s.wd != 0.f) g = g + s.wd * p;
  m = adam_lerp(m, g, s.w1);
  v = v * s.b2 + (s.omb2 * g) * g;
  const float denom = sqrtf(v) / s.bc2s + s.eps;
  p = p - s.step_size * (m / denom);
}

__global__ __launch_bounds__(256) void adam_kernel(const AdamRow* __restrict__ rows,
                                                   const int64_t* __restrict__ chunks,
                                                   AdamScalars s) {
  const int64_t ck = chunks[blockIdx.x];
  const int ti = (int)(ck >> 40);                 // tensor index
  const int64_t off = ck & ((1ll << 40) - 1);     // first element of the chunk
  const AdamRow r = rows[ti];
  const int64_t end = min(off + kAdamChunk, r.n);
  const bool vec = ((reinterpret_cast<uintptr_t>(r.p) | reinterpret_cast<uintptr_t>(r.g) |
                     reinterpret_cast<uintptr_t>(r.m) | reinterpret_cast<uintptr_t>(r.v)) &
                    15) == 0;
  if (vec) {
    const int64_t i = off + 4 * (int64_t)threadIdx.x;
    if (i + 3 < end) {
      float4 p = *reinterpret_cast<const float4*>(r.p + i);
      const float4 g = *reinterpret_cast<const float4*>(r.g + i);
      float4 m = *reinterpret_cast<const float4*>(r.m + i);
      float4 v = *reinterpret_cast<const float4*>(r.v + i);
      adam_elem(p.x, g.x, m.x, v.x, s);
      adam_elem(p.y, g.y, m.y, v.y, s);
      adam_elem(p.z, g.z, m.z, v.z, s);
      adam_elem(p.w, g.w, m.w, v.w, s);
      *reinterpret_cast<float4*>(r.p + i) = p;
      *reinterpret_cast<float4*>(r.m + i) = m;
      *reinterpret_cast<float4*>(r.v + i) = v;
    } else {
      for (int64_t e = i; e < end; ++e)
        adam_elem(r.p[e], r.g[e], r.m[e], r.v[e], s);
    }
    return;
  }
  for (int64_t e = off + threadIdx.x; e < end; e += blockDim.x)
    adam_elem(r.p[e], r.g[e], r.m[e], r.v[e], s);
}

}  // namespace jabd

using namespace jabd;

extern "C" int64_t jabd_adam_num_chunks(const int64_t* numel, int64_t ntensors) {
  if (!numel || ntensors < 0) return -1;
  int64_t c = 0;
  for (int64_t i = 0; i < ntensors; ++i) c += cdiv(numel[i], kAdamChunk);
  return c;
}

extern "C" int jabd_adam_fill_chunks(const int64_t* numel, int64_t ntensors, int64_t* chunks) {
  JABD_REQUIRE(numel && chunks && ntensors >= 0 && ntensors < (1 << 23), "adam: bad table");
  int64_t c = 0;
  for (int64_t i = 0; i < ntensors; ++i) {
    JABD_REQUIRE(numel[i] >= 0 && numel[i] < (1ll << 40), "adam: tensor too large");
    for (int64_t off = 0; off < numel[i]; off += kAdamChunk) chunks[c++] = (i << 40) | off;
  }
  return JABD_OK;
}

extern "C" int jabd_adam_step_f32(const void* rows, const int64_t* chunks, int64_t nchunks,
                                  double lr, double beta1, double beta2, double eps,
                                  double weight_decay, double bias_correction1,
                                  double bias_correction2, jabd_stream_t stream) {
  JABD_REQUIRE(rows && chunks && nchunks >= 0 && nchunks < ((int64_t)1 << 31),
               "adam: bad arguments");
  JABD_REQUIRE(bias_correction1 > 0 && bias_correction2 > 0, "adam: bias corrections must be > 0");
  if (nchunks == 0) return JABD_OK;
  AdamScalars sc;
  sc.step_size = (float)(lr / bias_correction1);
  sc.w1 = (float)(1.0 - beta1);
  sc.b2 = (float)beta2;
  sc.omb2 = (float)(1.0 - beta2);
  sc.bc2s = (float)sqrt(bias_correction2);
  sc.eps = (float)eps;
  sc.wd = (float)weight_decay;
  adam_kernel<<<(unsigned)nchunks, 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const AdamRow*>(rows), chunks, sc);
  return check_launch("adam");
}
