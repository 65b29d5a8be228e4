// BECA gate — the contrast-ECA block of the bicubic variant
// (train_mobilenetV3_ecagai.py:286-316: y = stdv_channels(x) (population std
// over H*W, two-pass: mean then mean squared deviation, sqrt), conv1d over
// channels (k taps, zero pad (k-1)/2, no bias), Hardsigmoid, x * y), §8f rank 4.
// NHWC fp32.  Forward: stats (64-channel x 4-pixel-group workgroups, LDS
// combine), gate (one thread per (b, c)), apply (elementwise).  Backward:
//   dgate[b,c] = Σ_p g*x,  dv = dgate * [−3 < v < 3] / 6,
//   dstd[b,j] = Σ_k w[k] dv[b, j−k+pad],  dw[k] = Σ_{b,c} dv[b,c] std[b,c+k−pad],
//   dx = g*gate + dstd * (x − mean) / (HW * std)   (the mean term sums to zero).
#include <math.h>

#include "common.h"

namespace jabd {

// x NHWC [B, P, C]; out0[b*C+c] = Σ_p f(p), two modes: 0 -> mean/std of x,
// 1 -> Σ g*x (dgate).
__global__ __launch_bounds__(256) void beca_stats_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ g, int64_t P,
                                                         int C, int mode,
                                                         float* __restrict__ mean,
                                                         float* __restrict__ stdv) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int64_t b = blockIdx.y;
  const bool ok = c < C;
  const float* xb = x + b * P * C + c;
  const float* gb = g ? g + b * P * C + c : nullptr;
  float s = 0.f;
  if (ok) {
    if (mode == 0)
      for (int64_t p = grp; p < P; p += 4) s += xb[p * C];
    else
      for (int64_t p = grp; p < P; p += 4) s += gb[p * C] * xb[p * C];
  }
  red[grp][cl] = s;
  __syncthreads();
  const float tot = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
  if (mode == 1) {
    if (grp == 0 && ok) mean[b * C + c] = tot;
    return;
  }
  const float mu = tot / (float)P;
  __syncthreads();
  float q = 0.f;
  if (ok)
    for (int64_t p = grp; p < P; p += 4) {
      const float d = xb[p * C] - mu;
      q += d * d;
    }
  red[grp][cl] = q;
  __syncthreads();
  if (grp == 0 && ok) {
    mean[b * C + c] = mu;
    stdv[b * C + c] = sqrtf((red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]) / (float)P);
  }
}

__global__ void beca_gate_kernel(const float* __restrict__ stdv, const float* __restrict__ w,
                                 int k, int C, int64_t BC, float* __restrict__ v,
                                 float* __restrict__ gate) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= BC) return;
  const int c = (int)(i % C);
  const int64_t base = i - c;
  const int pad = (k - 1) / 2;
  float a = 0.f;
  for (int t = 0; t < k; ++t) {
    const int j = c + t - pad;
    if (j >= 0 && j < C) a += w[t] * stdv[base + j];
  }
  v[i] = a;
  gate[i] = fminf(fmaxf(a + 3.f, 0.f), 6.f) / 6.f;  // Hardsigmoid = relu6(x + 3) / 6
}

__global__ void beca_apply_kernel(const float* __restrict__ x, const float* __restrict__ gate,
                                  int C, int64_t P, int64_t total, float* __restrict__ y) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const int64_t b = i / (P * C);
  y[i] = x[i] * gate[b * C + c];
}

// dv from dgate (in place), then dstd per (b, j) and dw per tap.
__global__ void beca_dv_kernel(float* __restrict__ dgate_dv, const float* __restrict__ v,
                               int64_t BC) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= BC) return;
  const float a = v[i];
  dgate_dv[i] = (a > -3.f && a < 3.f) ? dgate_dv[i] / 6.f : 0.f;
}

__global__ void beca_dstd_kernel(const float* __restrict__ dv, const float* __restrict__ w, int k,
                                 int C, int64_t BC, float* __restrict__ dstd) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= BC) return;
  const int j = (int)(i % C);
  const int64_t base = i - j;
  const int pad = (k - 1) / 2;
  float a = 0.f;
  for (int t = 0; t < k; ++t) {
    const int c = j - t + pad;
    if (c >= 0 && c < C) a += w[t] * dv[base + c];
  }
  dstd[i] = a;
}

__global__ __launch_bounds__(256) void beca_dw_kernel(const float* __restrict__ dv,
                                                      const float* __restrict__ stdv, int k,
                                                      int C, int64_t BC, float* __restrict__ dw) {
  const int t = blockIdx.x;  // one workgroup per tap, fixed-order reduction
  const int pad = (k - 1) / 2;
  float a = 0.f;
  for (int64_t i = threadIdx.x; i < BC; i += blockDim.x) {
    const int c = (int)(i % C);
    const int j = c + t - pad;
    if (j >= 0 && j < C) a += dv[i] * stdv[i - c + j];
  }
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
  __shared__ float s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) dw[t] = s[0] + s[1] + s[2] + s[3];
}

__global__ void beca_dx_kernel(const float* __restrict__ x, const float* __restrict__ g,
                               const float* __restrict__ gate, const float* __restrict__ mean,
                               const float* __restrict__ stdv, const float* __restrict__ dstd,
                               int C, int64_t P, int64_t total, float* __restrict__ dx) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const int64_t bc = (i / (P * C)) * C + c;
  dx[i] = g[i] * gate[bc] + dstd[bc] * (x[i] - mean[bc]) / ((float)P * stdv[bc]);
}

}  // namespace jabd

using namespace jabd;

// stats: float [4, B*C] = mean, std, v, gate (kept for the backward).
extern "C" int jabd_beca_fwd_f32(const float* x, int64_t batch, int64_t pixels, int C,
                                 const float* w, int k, float* y, float* stats,
                                 jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && pixels > 0 && C > 0 && k > 0 && (k & 1), "beca: bad size");
  if (batch == 0) return JABD_OK;
  JABD_REQUIRE(x && w && stats, "beca: null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t BC = batch * C, total = BC * pixels;
  float *mean = stats, *sd = stats + BC, *v = stats + 2 * BC, *gate = stats + 3 * BC;
  beca_stats_kernel<<<dim3((unsigned)cdiv(C, 64), (unsigned)batch), 256, 0, st>>>(
      x, nullptr, pixels, C, 0, mean, sd);
  if (int e = check_launch("beca_stats")) return e;
  beca_gate_kernel<<<(unsigned)cdiv(BC, 256), 256, 0, st>>>(sd, w, k, C, BC, v, gate);
  if (int e = check_launch("beca_gate")) return e;
  if (!y) return JABD_OK;  // gate only: stats[3] = the [B][C] gate
  beca_apply_kernel<<<(unsigned)cdiv(total, 256), 256, 0, st>>>(x, gate, C, pixels, total, y);
  return check_launch("beca_apply");
}

// ws: float [2, B*C].  Writes dx [B, P, C] and dw [k].
extern "C" int jabd_beca_bwd_f32(const float* x, const float* grad_y, int64_t batch,
                                 int64_t pixels, int C, const float* w, int k,
                                 const float* stats, float* grad_x, float* grad_w, float* ws,
                                 jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && pixels > 0 && C > 0 && k > 0 && (k & 1), "beca_bwd: bad size");
  if (batch == 0) return JABD_OK;
  JABD_REQUIRE(x && grad_y && w && stats && grad_x && grad_w && ws, "beca_bwd: null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t BC = batch * C, total = BC * pixels;
  const float *mean = stats, *sd = stats + BC, *v = stats + 2 * BC, *gate = stats + 3 * BC;
  float *dv = ws, *dstd = ws + BC;
  beca_stats_kernel<<<dim3((unsigned)cdiv(C, 64), (unsigned)batch), 256, 0, st>>>(
      x, grad_y, pixels, C, 1, dv, nullptr);
  if (int e = check_launch("beca_dgate")) return e;
  beca_dv_kernel<<<(unsigned)cdiv(BC, 256), 256, 0, st>>>(dv, v, BC);
  beca_dstd_kernel<<<(unsigned)cdiv(BC, 256), 256, 0, st>>>(dv, w, k, C, BC, dstd);
  beca_dw_kernel<<<(unsigned)k, 256, 0, st>>>(dv, sd, k, C, BC, grad_w);
  if (int e = check_launch("beca_dw")) return e;
  beca_dx_kernel<<<(unsigned)cdiv(total, 256), 256, 0, st>>>(x, grad_y, gate, mean, sd, dstd, C,
                                                              pixels, total, grad_x);
  return check_launch("beca_dx");
}
