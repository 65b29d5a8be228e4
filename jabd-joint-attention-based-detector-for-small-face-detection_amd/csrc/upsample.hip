// Bicubic align_corners upsampling — the CSAF fusion of the bicubic FPN variant
// (train_mobilenetV3_ecagai.py:270,279: F.interpolate(x, size, mode="bicubic",
// align_corners=True)), §8f rank 4.  NHWC fp32 (the engine's activation layout),
// one thread per output element with the channel fastest (coalesced).
// PyTorch's algorithm: scale = (in-1)/(out-1) (0 if out == 1), src = scale*o,
// i = floor(src), t = src - i, cubic-convolution weights with A = -0.75, taps
// i-1..i+2 clamped to [0, in-1], x first then y.  Backward gathers: each input
// element sums the weighted gradients of the outputs that read it, in a fixed
// order (deterministic; clamped taps that share an input are summed per axis).
#include <math.h>

#include "common.h"

namespace jabd {

__device__ __forceinline__ void cubic_w(float t, float w[4]) {
  const float A = -0.75f;
  float x = t + 1.f;
  w[0] = ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A;
  x = t;
  w[1] = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  x = 1.f - t;
  w[2] = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  x = 2.f - t;
  w[3] = ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A;
}

__device__ __forceinline__ void cubic_src(int o, float scale, int n, int idx[4], float w[4]) {
  const float real = scale * (float)o;
  const int i = (int)floorf(real);
  cubic_w(real - (float)i, w);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int j = i - 1 + k;
    idx[k] = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
  }
}

__global__ __launch_bounds__(256) void upsample_bicubic_fwd(const float* __restrict__ x, int H,
                                                            int W, int C, float* __restrict__ y,
                                                            int OH, int OW, float sh, float sw,
                                                            int64_t total) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  int64_t r = e / C;
  const int ox = (int)(r % OW);
  r /= OW;
  const int oy = (int)(r % OH);
  const int64_t b = r / OH;
  int xi[4], yi[4];
  float wx[4], wy[4];
  cubic_src(ox, sw, W, xi, wx);
  cubic_src(oy, sh, H, yi, wy);
  const float* xb = x + b * H * W * C + c;
  float acc = 0.f;
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    const float* row = xb + (int64_t)yi[ky] * W * C;
    float rv = row[(int64_t)xi[0] * C] * wx[0] + row[(int64_t)xi[1] * C] * wx[1] +
               row[(int64_t)xi[2] * C] * wx[2] + row[(int64_t)xi[3] * C] * wx[3];
    acc += rv * wy[ky];
  }
  y[e] = acc;
}

// Sum of the cubic weights with which output o's four (clamped) taps read
// input index i along one axis — the same index math as the forward.
__device__ __forceinline__ float tap_weight(int o, float scale, int n, int i) {
  int idx[4];
  float w[4];
  cubic_src(o, scale, n, idx, w);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) s += idx[k] == i ? w[k] : 0.f;
  return s;
}

// Outputs whose taps can reach input i: floor(scale*o) in [i-2, i+1] (one
// index of slack for rounding); the edge inputs also collect the clamped taps.
__device__ __forceinline__ void out_range(int i, int n, int on, float scale, int& lo, int& hi) {
  if (scale <= 0.f) {
    lo = 0;
    hi = on - 1;
    return;
  }
  lo = i == 0 ? 0 : max(0, (int)floorf((float)(i - 2) / scale) - 1);
  hi = i == n - 1 ? on - 1 : min(on - 1, (int)ceilf((float)(i + 2) / scale) + 1);
}

// Gather form: one thread per input element sums, in a fixed order, the
// weighted gradients of every output that reads it — deterministic (no
// atomics), and each grad_x element is written once.
__global__ __launch_bounds__(256) void upsample_bicubic_bwd(const float* __restrict__ gy, int H,
                                                            int W, int C, float* __restrict__ gx,
                                                            int OH, int OW, float sh, float sw,
                                                            int64_t total) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  int64_t r = e / C;
  const int ix = (int)(r % W);
  r /= W;
  const int iy = (int)(r % H);
  const int64_t b = r / H;
  int ylo, yhi, xlo, xhi;
  out_range(iy, H, OH, sh, ylo, yhi);
  out_range(ix, W, OW, sw, xlo, xhi);
  const float* gb = gy + b * OH * OW * C + c;
  float acc = 0.f;
  for (int oy = ylo; oy <= yhi; ++oy) {
    const float wy = tap_weight(oy, sh, H, iy);
    if (wy == 0.f) continue;
    const float* row = gb + (int64_t)oy * OW * C;
    float rs = 0.f;
    for (int ox = xlo; ox <= xhi; ++ox) {
      const float wx = tap_weight(ox, sw, W, ix);
      if (wx != 0.f) rs = fmaf(wx, row[(int64_t)ox * C], rs);
    }
    acc = fmaf(wy, rs, acc);
  }
  gx[e] = acc;
}

static float ac_scale(int in, int out) {
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_upsample_bicubic_ac_f32(const float* x, int64_t batch, int H, int W, int C,
                                            float* y, int OH, int OW, jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0,
               "upsample_bicubic: bad size");
  const int64_t total = batch * OH * OW * C;
  if (total == 0) return JABD_OK;
  JABD_REQUIRE(x && y, "upsample_bicubic: null pointer");
  upsample_bicubic_fwd<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      x, H, W, C, y, OH, OW, ac_scale(H, OH), ac_scale(W, OW), total);
  return check_launch("upsample_bicubic");
}

extern "C" int jabd_upsample_bicubic_ac_bwd_f32(const float* grad_y, int64_t batch, int H, int W,
                                                int C, float* grad_x, int OH, int OW,
                                                jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0,
               "upsample_bicubic_bwd: bad size");
  const int64_t total = batch * H * W * C;
  if (batch == 0) return JABD_OK;
  JABD_REQUIRE(grad_y && grad_x, "upsample_bicubic_bwd: null pointer");
  hipStream_t st = as_stream(stream);
  upsample_bicubic_bwd<<<(unsigned)cdiv(total, 256), 256, 0, st>>>(
      grad_y, H, W, C, grad_x, OH, OW, ac_scale(H, OH), ac_scale(W, OW), total);
  return check_launch("upsample_bicubic_bwd");
}
