// Module-level kernels on gfx950: what the reference's individual nn.Modules
// compute when a caller runs them one by one (nn.Sequential children, the
// body of a torchvision IntermediateLayerGetter, a standalone eca_block or
// PSPModule), rather than inside the fused RetinaFace plan:
//   activations    nn.ReLU / LeakyReLU / Hardswish / Hardsigmoid / Sigmoid,
//                  forward and backward, layout-agnostic over dense storage
//   bn_eval        eval-mode BatchNorm2d/1d (running statistics) + activation
//   channel_scale  x * s[b][c] (ECA / SE gate application), NHWC
//   adaptive_pool  nn.AdaptiveAvgPool2d at several output sizes concatenated
//                  (PSPModule, nets/retinaface_r.py:85-104) and its backward
// All memory-bound elementwise/gather work: float4 where the layout allows.
#include <math.h>

#include "common.h"
#include "conv_args.h"

namespace jabd {

__device__ __forceinline__ float mact(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return relu_f(v);
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: return hswish_f(v);
    case ACT_HSIGMOID: return hsigmoid_f(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// d act / d x at the input x (PyTorch's *_backward conventions).
__device__ __forceinline__ float mact_d(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? 1.f : 0.f;
    case ACT_LEAKY: return v > 0.f ? 1.f : slope;
    case ACT_HSWISH: return v < -3.f ? 0.f : (v <= 3.f ? v / 3.f + 0.5f : 1.f);
    case ACT_HSIGMOID: return (v > -3.f && v < 3.f) ? 1.f / 6.f : 0.f;
    case ACT_SIGMOID: {
      const float s = 1.f / (1.f + expf(-v));
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}

__global__ __launch_bounds__(256) void act_kernel(const float4* __restrict__ x, int64_t n4, int act,
                                                  float slope, float4* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    y[i] = make_float4(mact(v.x, act, slope), mact(v.y, act, slope), mact(v.z, act, slope),
                       mact(v.w, act, slope));
  }
}

// scalar grid-stride twin: the < 4 tail, or storage that is not 16-byte aligned
__global__ __launch_bounds__(256) void act_scalar_kernel(const float* __restrict__ x, int64_t lo,
                                                         int64_t n, int act, float slope,
                                                         float* __restrict__ y) {
  for (int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = mact(x[i], act, slope);
}

__global__ __launch_bounds__(256) void act_bwd_kernel(const float4* __restrict__ x,
                                                      const float4* __restrict__ dy, int64_t n4,
                                                      int act, float slope,
                                                      float4* __restrict__ dx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i], g = dy[i];
    dx[i] = make_float4(g.x * mact_d(v.x, act, slope), g.y * mact_d(v.y, act, slope),
                        g.z * mact_d(v.z, act, slope), g.w * mact_d(v.w, act, slope));
  }
}

__global__ __launch_bounds__(256) void act_bwd_scalar_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ dy,
                                                             int64_t lo, int64_t n, int act,
                                                             float slope,
                                                             float* __restrict__ dx) {
  for (int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = dy[i] * mact_d(x[i], act, slope);
}

static unsigned ew_grid(int64_t n4) {
  const int64_t g = cdiv(n4 > 0 ? n4 : 1, 256);
  return (unsigned)(g < 8192 ? g : 8192);  // grid-stride beyond 2M float4
}

// y[m][c] = act((x[m][c] - rm[c]) / sqrt(rv[c] + eps) * g[c] + b[c]), any C
// (the module path also meets the 10-channel SSH branches).
__global__ __launch_bounds__(256) void bn_eval_kernel(const float* __restrict__ x, int64_t M, int C,
                                                      const float* __restrict__ rm,
                                                      const float* __restrict__ rv, float eps,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ b, int act,
                                                      float slope, float* __restrict__ y) {
  const int64_t n = M * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    // (x - mean) * invstd * gamma + beta, the order of torch's batch_norm
    const float inv = 1.f / sqrtf(rv[c] + eps);
    y[i] = mact((x[i] - rm[c]) * inv * g[c] + b[c], act, slope);
  }
}

// y[b][p][c] = x[b][p][c] * s[b][c] (NHWC, C % 4 == 0)
__global__ __launch_bounds__(256) void channel_scale_kernel(const float4* __restrict__ x,
                                                            int64_t HW, int C4,
                                                            const float4* __restrict__ s,
                                                            float4* __restrict__ y,
                                                            int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    const int64_t b = i / ((int64_t)C4 * HW);
    const float4 v = x[i], g = s[b * C4 + c4];
    y[i] = make_float4(v.x * g.x, v.y * g.y, v.z * g.z, v.w * g.w);
  }
}

struct PoolSizes {
  int n;
  int v[8];
};

__device__ __forceinline__ void pool_bin(const PoolSizes& sz, int s, int H, int W, int& h0, int& h1,
                                         int& w0, int& w1) {
  int base = 0, lvl = 0;
  for (; lvl < sz.n - 1; ++lvl) {
    const int n = sz.v[lvl] * sz.v[lvl];
    if (s < base + n) break;
    base += n;
  }
  const int z = sz.v[lvl];
  const int bi = (s - base) / z, bj = (s - base) % z;
  // AdaptiveAvgPool2d bin [floor(i*H/z), ceil((i+1)*H/z))
  h0 = (bi * H) / z;
  h1 = ((bi + 1) * H + z - 1) / z;
  w0 = (bj * W) / z;
  w1 = ((bj + 1) * W + z - 1) / z;
}

// One workgroup per (bin, image); threads stride the channels, pixels summed
// in row-major order (fixed order: deterministic).
__global__ __launch_bounds__(256) void adaptive_pool_kernel(const float* __restrict__ x,
                                                            int64_t x_bs, int H, int W, int C,
                                                            const PoolSizes sz, int S,
                                                            float* __restrict__ out) {
  const int s = blockIdx.x, b = blockIdx.y;
  int h0, h1, w0, w1;
  pool_bin(sz, s, H, W, h0, h1, w0, w1);
  const float cnt = (float)((h1 - h0) * (w1 - w0));
  const float* xb = x + (int64_t)b * x_bs;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f;
    for (int i = h0; i < h1; ++i)
      for (int j = w0; j < w1; ++j) a += xb[((int64_t)i * W + j) * C + c];
    out[((int64_t)b * S + s) * C + c] = a / cnt;  // sum / count, as torch
  }
}

// Two-pass form (workspace): pass 1, one workgroup per (row, image), sums
// each column bin q (q enumerates (level, bj)) of the row for every channel
// into rowpart[b][y][q][c]; pass 2, one workgroup per (bin, image), sums the
// bin's rows of rowpart.  x is read from HBM once (the one-pass kernel above
// has the 1x1 bin's workgroup read the whole image alone).  Fixed order.
__device__ __forceinline__ void col_bin(const PoolSizes& sz, int q, int& lvl, int& bj) {
  lvl = 0;
  while (lvl < sz.n - 1 && q >= sz.v[lvl]) {
    q -= sz.v[lvl];
    ++lvl;
  }
  bj = q;
}

__global__ __launch_bounds__(256) void pool_rows_kernel(const float* __restrict__ x,
                                                        int64_t x_bs, int H, int W, int C,
                                                        const PoolSizes sz, int Q,
                                                        float* __restrict__ rowpart) {
  const int y = blockIdx.x, b = blockIdx.y;
  const float* xr = x + (int64_t)b * x_bs + (int64_t)y * W * C;
  float* rp = rowpart + (((int64_t)b * H + y) * Q) * C;
  for (int it = threadIdx.x; it < Q * C; it += blockDim.x) {
    const int q = it / C, c = it - q * C;
    int lvl, bj;
    col_bin(sz, q, lvl, bj);
    const int z = sz.v[lvl];
    const int w0 = (bj * W) / z, w1 = ((bj + 1) * W + z - 1) / z;
    float a = 0.f;
    for (int j = w0; j < w1; ++j) a += xr[(int64_t)j * C + c];
    rp[it] = a;
  }
}

__global__ __launch_bounds__(256) void pool_bins_kernel(const float* __restrict__ rowpart, int H,
                                                        int W, int C, const PoolSizes sz, int S,
                                                        int Q, float* __restrict__ out) {
  const int s = blockIdx.x, b = blockIdx.y;
  int h0, h1, w0, w1;
  pool_bin(sz, s, H, W, h0, h1, w0, w1);
  // column-bin index q of this bin: levels before it, then bj
  int base = 0, qb = 0, lvl = 0;
  for (; lvl < sz.n - 1; ++lvl) {
    const int n = sz.v[lvl] * sz.v[lvl];
    if (s < base + n) break;
    base += n;
    qb += sz.v[lvl];
  }
  const int q = qb + (s - base) % sz.v[lvl];
  const float cnt = (float)((h1 - h0) * (w1 - w0));
  const float* rp = rowpart + ((int64_t)b * H * Q + q) * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f;
    for (int i = h0; i < h1; ++i) a += rp[(int64_t)i * Q * C + c];
    out[((int64_t)b * S + s) * C + c] = a / cnt;
  }
}

// dx[b][p][c] = sum over the bins containing p of dy[b][s][c] / |bin s|
// (gather form: every pixel owns its sum, no atomics).  Per level only the
// bins around floor(i*z/H) can hold row i (likewise for columns).
__global__ __launch_bounds__(256) void adaptive_pool_bwd_kernel(const float* __restrict__ dy,
                                                                int H, int W, int C,
                                                                const PoolSizes sz, int S,
                                                                float* __restrict__ dx) {
  const int b = blockIdx.y;
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= (int64_t)H * W * C) return;
  const int c = (int)(idx % C);
  const int p = (int)(idx / C);
  const int i = p / W, j = p % W;
  float a = 0.f;
  int base = 0;
  for (int l = 0; l < sz.n; ++l) {
    const int z = sz.v[l];
    const int bi0 = max(0, (i * z) / H - 1), bi1 = min(z - 1, (i * z) / H + 1);
    const int bj0 = max(0, (j * z) / W - 1), bj1 = min(z - 1, (j * z) / W + 1);
    for (int bi = bi0; bi <= bi1; ++bi) {
      const int r0 = (bi * H) / z, r1 = ((bi + 1) * H + z - 1) / z;
      if (i < r0 || i >= r1) continue;
      for (int bj = bj0; bj <= bj1; ++bj) {
        const int c0 = (bj * W) / z, c1 = ((bj + 1) * W + z - 1) / z;
        if (j < c0 || j >= c1) continue;
        a += dy[((int64_t)b * S + base + bi * z + bj) * C + c] / (float)((r1 - r0) * (c1 - c0));
      }
    }
    base += z * z;
  }
  dx[(int64_t)b * H * W * C + idx] = a;
}

// F.interpolate(mode='nearest', size=...) source index (ATen nearest_idx).
__device__ __forceinline__ int near_src(int dst, int in, int out) {
  if (out == in) return dst;
  if (out == 2 * in) return dst >> 1;
  const int s = (int)floorf((float)dst * ((float)in / (float)out));
  return s < in - 1 ? s : in - 1;
}

// out = lateral + nearest(src -> h x w), NHWC, C % 4 == 0 (the plain FPN's
// up-sample and add, nets/layers.py:106-117)
__global__ __launch_bounds__(256) void up_add_kernel(const float* __restrict__ src, int hs, int ws,
                                                     int h, int w, int C,
                                                     const float* __restrict__ lat,
                                                     float* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int C4 = C >> 2;
  const int b = blockIdx.y;
  if (idx >= (int64_t)h * w * C4) return;
  const int c4 = (int)(idx % C4);
  const int p = (int)(idx / C4);
  const int i = p / w, j = p - (p / w) * w;
  const int64_t o = ((int64_t)b * h * w + p) * C4 + c4;
  const float4 a = reinterpret_cast<const float4*>(lat)[o];
  const float4 u = reinterpret_cast<const float4*>(
      src + (((int64_t)b * hs + near_src(i, hs, h)) * ws + near_src(j, ws, w)) * C)[c4];
  reinterpret_cast<float4*>(out)[o] = make_float4(a.x + u.x, a.y + u.y, a.z + u.z, a.w + u.w);
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_upsample_nearest_add_f32(const float* src, int32_t B, int32_t hs, int32_t ws,
                                             int32_t h, int32_t w, int32_t C,
                                             const float* lateral, float* out,
                                             jabd_stream_t stream) {
  JABD_REQUIRE(src && lateral && out && B > 0 && C % 4 == 0 && hs <= h && ws <= w,
               "upsample_add: bad args");
  dim3 g((unsigned)cdiv((int64_t)h * w * (C / 4), 256), (unsigned)B);
  up_add_kernel<<<g, 256, 0, as_stream(stream)>>>(src, hs, ws, h, w, C, lateral, out);
  return check_launch("upsample_add");
}

extern "C" int jabd_act_f32(const float* x, int64_t n, int32_t act, float slope, float* y,
                            jabd_stream_t stream) {
  JABD_REQUIRE(n >= 0 && (n == 0 || (x && y)), "act: bad args");
  JABD_REQUIRE(act >= ACT_NONE && act <= ACT_SIGMOID, "act: kind %d", act);
  if (n == 0) return JABD_OK;
  hipStream_t st = as_stream(stream);
  const bool al = ((uintptr_t)x % 16 == 0) && ((uintptr_t)y % 16 == 0);
  const int64_t n4 = al ? n / 4 : 0;
  if (n4) {
    act_kernel<<<ew_grid(n4), 256, 0, st>>>(reinterpret_cast<const float4*>(x), n4, act, slope,
                                           reinterpret_cast<float4*>(y));
    if (int e = check_launch("act")) return e;
  }
  if (4 * n4 < n)
    act_scalar_kernel<<<ew_grid(cdiv(n - 4 * n4, 4)), 256, 0, st>>>(x, 4 * n4, n, act, slope, y);
  return check_launch("act_scalar");
}

extern "C" int jabd_act_bwd_f32(const float* x, const float* dy, int64_t n, int32_t act,
                                float slope, float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(n >= 0 && (n == 0 || (x && dy && dx)), "act_bwd: bad args");
  JABD_REQUIRE(act >= ACT_NONE && act <= ACT_SIGMOID, "act_bwd: kind %d", act);
  if (n == 0) return JABD_OK;
  hipStream_t st = as_stream(stream);
  const bool al = ((uintptr_t)x % 16 == 0) && ((uintptr_t)dy % 16 == 0) &&
                  ((uintptr_t)dx % 16 == 0);
  const int64_t n4 = al ? n / 4 : 0;
  if (n4) {
    act_bwd_kernel<<<ew_grid(n4), 256, 0, st>>>(reinterpret_cast<const float4*>(x),
                                               reinterpret_cast<const float4*>(dy), n4, act,
                                               slope, reinterpret_cast<float4*>(dx));
    if (int e = check_launch("act_bwd")) return e;
  }
  if (4 * n4 < n)
    act_bwd_scalar_kernel<<<ew_grid(cdiv(n - 4 * n4, 4)), 256, 0, st>>>(x, dy, 4 * n4, n, act,
                                                                       slope, dx);
  return check_launch("act_bwd_scalar");
}

extern "C" int jabd_bn_eval_f32(const float* x, int64_t M, int32_t C, const float* running_mean,
                                const float* running_var, float eps, const float* gamma,
                                const float* beta, int32_t act, float slope, float* y,
                                jabd_stream_t stream) {
  JABD_REQUIRE(x && running_mean && running_var && gamma && beta && y && M >= 0 && C > 0,
               "bn_eval: bad args");
  JABD_REQUIRE(act >= ACT_NONE && act <= ACT_SIGMOID, "bn_eval: act %d", act);
  if (M == 0) return JABD_OK;
  const int64_t n = M * C;
  bn_eval_kernel<<<ew_grid(cdiv(n, 4)), 256, 0, as_stream(stream)>>>(
      x, M, C, running_mean, running_var, eps, gamma, beta, act, slope, y);
  return check_launch("bn_eval");
}

extern "C" int jabd_channel_scale_f32(const float* x, int64_t B, int64_t HW, int32_t C,
                                      const float* scale, float* y, jabd_stream_t stream) {
  JABD_REQUIRE(x && scale && y && B > 0 && HW > 0 && C > 0 && C % 4 == 0,
               "channel_scale: bad args (C %% 4 == 0 required)");
  const int64_t n4 = B * HW * C / 4;
  channel_scale_kernel<<<ew_grid(n4), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const float4*>(x), HW, C / 4, reinterpret_cast<const float4*>(scale),
      reinterpret_cast<float4*>(y), n4);
  return check_launch("channel_scale");
}

static int pool_sizes(const int32_t* sizes, int32_t nsizes, PoolSizes& sz, int& S) {
  JABD_REQUIRE(sizes && nsizes > 0 && nsizes <= 8, "adaptive_pool: 1..8 output sizes");
  sz.n = nsizes;
  S = 0;
  for (int i = 0; i < 8; ++i) {
    sz.v[i] = i < nsizes ? sizes[i] : 0;
    if (i < nsizes) {
      JABD_REQUIRE(sizes[i] > 0, "adaptive_pool: bad size");
      S += sizes[i] * sizes[i];
    }
  }
  return JABD_OK;
}

extern "C" int64_t jabd_adaptive_pool_ws_floats(int32_t B, int32_t H, int32_t C,
                                                const int32_t* sizes, int32_t nsizes) {
  if (!sizes || nsizes <= 0 || B <= 0 || H <= 0 || C <= 0) return -1;
  int64_t Q = 0;
  for (int i = 0; i < nsizes; ++i) Q += sizes[i];
  return (int64_t)B * H * Q * C;
}

extern "C" int jabd_adaptive_pool_f32(const float* x, int64_t x_bs, int32_t B, int32_t H,
                                      int32_t W, int32_t C, const int32_t* sizes, int32_t nsizes,
                                      float* out, float* ws, int64_t ws_floats,
                                      jabd_stream_t stream) {
  JABD_REQUIRE(x && out && B > 0 && H > 0 && W > 0 && C > 0, "adaptive_pool: bad args");
  PoolSizes sz;
  int S;
  if (int e = pool_sizes(sizes, nsizes, sz, S)) return e;
  hipStream_t st = as_stream(stream);
  if (ws && ws_floats >= jabd_adaptive_pool_ws_floats(B, H, C, sizes, nsizes)) {
    int Q = 0;
    for (int i = 0; i < nsizes; ++i) Q += sizes[i];
    pool_rows_kernel<<<dim3((unsigned)H, (unsigned)B), 256, 0, st>>>(x, x_bs, H, W, C, sz, Q, ws);
    if (int e = check_launch("adaptive_pool_rows")) return e;
    pool_bins_kernel<<<dim3((unsigned)S, (unsigned)B), 256, 0, st>>>(ws, H, W, C, sz, S, Q, out);
    return check_launch("adaptive_pool_bins");
  }
  adaptive_pool_kernel<<<dim3((unsigned)S, (unsigned)B), 256, 0, st>>>(x, x_bs, H, W, C, sz, S,
                                                                      out);
  return check_launch("adaptive_pool");
}

extern "C" int jabd_adaptive_pool_bwd_f32(const float* dy, int32_t B, int32_t H, int32_t W,
                                          int32_t C, const int32_t* sizes, int32_t nsizes,
                                          float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(dy && dx && B > 0 && H > 0 && W > 0 && C > 0, "adaptive_pool_bwd: bad args");
  PoolSizes sz;
  int S;
  if (int e = pool_sizes(sizes, nsizes, sz, S)) return e;
  dim3 g((unsigned)cdiv((int64_t)H * W * C, 256), (unsigned)B);
  adaptive_pool_bwd_kernel<<<g, 256, 0, as_stream(stream)>>>(dy, H, W, C, sz, S, dx);
  return check_launch("adaptive_pool_bwd");
}
