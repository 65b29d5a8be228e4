// BECA gate — the contrast-ECA block of the bicubic variant
// (train_mobilenetV3_ecagai.py:286-316: y = stdv_channels(x) (population std
// over H*W, two-pass: mean then mean squared deviation, sqrt), conv1d over
// channels (k taps, zero pad (k-1)/2, no bias), Hardsigmoid, x * y), §8f rank 4.
// NHWC fp32.  Forward: stats (C % 4 == 0: pixel-chunk x image workgroups
// writing per-chunk partials to the caller's workspace, summed in a fixed
// order — mean pass, then squared-deviation pass; otherwise 64-channel
// workgroups), gate (one thread per (b, c)), apply (elementwise).  Backward:
//   dgate[b,c] = Σ_p g*x,  dv = dgate * [−3 < v < 3] / 6,
//   dstd[b,j] = Σ_k w[k] dv[b, j−k+pad],  dw[k] = Σ_{b,c} dv[b,c] std[b,c+k−pad],
//   dx = g*gate + dstd * (x − mean) / (HW * std)   (the mean term sums to zero).
#include <math.h>

#include <algorithm>

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

// Parallel form of the same sums for C % 4 == 0 (every BECA width JABD
// uses): grid (nblk, B), each workgroup reduces `per` pixels of one image for
// all channels — thread t takes channel quad t % C4 and pixel row t / C4
// (TPX = 256 / C4 rows), the rows combine in LDS in a fixed order — and
// writes part[b][blk][C]; beca_final_kernel sums the nblk partials per
// (b, c) in order.  MODE 0: x;  1: (x - mean)^2;  2: g * x.
template <int MODE>
__global__ __launch_bounds__(256) void beca_part_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ mean,
                                                        int64_t P, int C, int64_t per,
                                                        float* __restrict__ part) {
  __shared__ float4 red[256];
  const int t = threadIdx.x, C4 = C >> 2;
  const int64_t b = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = min(P, p0 + per);
  const float4* xb = reinterpret_cast<const float4*>(x + b * P * C);
  const float4* gb = MODE == 2 ? reinterpret_cast<const float4*>(g + b * P * C) : nullptr;
  float4* pb = reinterpret_cast<float4*>(part + (b * gridDim.x + blockIdx.x) * C);
  if (C4 > 256) {  // one pixel row, channel quads strided over the threads
    for (int cq = t; cq < C4; cq += 256) {
      float4 mu = make_float4(0.f, 0.f, 0.f, 0.f);
      if (MODE == 1) mu = reinterpret_cast<const float4*>(mean + b * C)[cq];
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t p = p0; p < p1; ++p) {
        const float4 v = xb[p * C4 + cq];
        if (MODE == 0) { s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
        if (MODE == 1) {
          const float a = v.x - mu.x, bb = v.y - mu.y, c = v.z - mu.z, d = v.w - mu.w;
          s.x += a * a; s.y += bb * bb; s.z += c * c; s.w += d * d;
        }
        if (MODE == 2) {
          const float4 q = gb[p * C4 + cq];
          s.x += q.x * v.x; s.y += q.y * v.y; s.z += q.z * v.z; s.w += q.w * v.w;
        }
      }
      pb[cq] = s;
    }
    return;
  }
  const int TPX = 256 / C4;
  const int cq = t % C4, r = t / C4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (r < TPX) {
    float4 mu = make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE == 1) mu = reinterpret_cast<const float4*>(mean + b * C)[cq];
    for (int64_t p = p0 + r; p < p1; p += TPX) {
      const float4 v = xb[p * C4 + cq];
      if (MODE == 0) { s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
      if (MODE == 1) {
        const float a = v.x - mu.x, bb = v.y - mu.y, c = v.z - mu.z, d = v.w - mu.w;
        s.x += a * a; s.y += bb * bb; s.z += c * c; s.w += d * d;
      }
      if (MODE == 2) {
        const float4 q = gb[p * C4 + cq];
        s.x += q.x * v.x; s.y += q.y * v.y; s.z += q.z * v.z; s.w += q.w * v.w;
      }
    }
  }
  red[t] = s;
  __syncthreads();
  if (t < C4) {
    float4 a = red[t];
    for (int k = 1; k < TPX; ++k) {
      const float4 v = red[k * C4 + t];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    pb[t] = a;
  }
}

// out[b*C + c] = f(sum over blk of part[b][blk][c]): MODE 0 mean, 1 std, 2 raw sum.
template <int MODE>
__global__ void beca_final_kernel(const float* __restrict__ part, int nblk, int C, int64_t BC,
                                  int64_t P, float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= BC) return;
  const int c = (int)(i % C);
  const int64_t b = i / C;
  const float* pp = part + b * nblk * C + c;
  float s = 0.f;
  for (int k = 0; k < nblk; ++k) s += pp[(int64_t)k * C];
  out[i] = MODE == 0 ? s / (float)P : (MODE == 1 ? sqrtf(s / (float)P) : s);
}

static int beca_nblk(int64_t pixels) {
  return (int)std::min<int64_t>(64, std::max<int64_t>(1, pixels / 1024));
}

static bool beca_par_ok(const float* x, const float* g, int C) {
  return C % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)g % 16 == 0;
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
extern "C" int64_t jabd_beca_ws_floats(int64_t batch, int64_t pixels, int C) {
  if (batch < 0 || pixels <= 0 || C <= 0) return -1;
  return batch * beca_nblk(pixels) * (int64_t)C;
}

extern "C" int jabd_beca_fwd_f32(const float* x, int64_t batch, int64_t pixels, int C,
                                 const float* w, int k, float* y, float* stats, float* ws,
                                 int64_t ws_floats, jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && pixels > 0 && C > 0 && k > 0 && (k & 1), "beca: bad size");
  if (batch == 0) return JABD_OK;
  JABD_REQUIRE(x && w && stats, "beca: null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t BC = batch * C, total = BC * pixels;
  float *mean = stats, *sd = stats + BC, *v = stats + 2 * BC, *gate = stats + 3 * BC;
  if (ws && beca_par_ok(x, nullptr, C) && ws_floats >= jabd_beca_ws_floats(batch, pixels, C)) {
    const int nb = beca_nblk(pixels);
    const int64_t per = cdiv(pixels, nb);
    const dim3 g((unsigned)nb, (unsigned)batch);
    const unsigned gf = (unsigned)cdiv(BC, 256);
    beca_part_kernel<0><<<g, 256, 0, st>>>(x, nullptr, nullptr, pixels, C, per, ws);
    beca_final_kernel<0><<<gf, 256, 0, st>>>(ws, nb, C, BC, pixels, mean);
    beca_part_kernel<1><<<g, 256, 0, st>>>(x, nullptr, mean, pixels, C, per, ws);
    beca_final_kernel<1><<<gf, 256, 0, st>>>(ws, nb, C, BC, pixels, sd);
  } else {
    beca_stats_kernel<<<dim3((unsigned)cdiv(C, 64), (unsigned)batch), 256, 0, st>>>(
        x, nullptr, pixels, C, 0, mean, sd);
  }
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
                                 float* part, int64_t part_floats, jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && pixels > 0 && C > 0 && k > 0 && (k & 1), "beca_bwd: bad size");
  if (batch == 0) return JABD_OK;
  JABD_REQUIRE(x && grad_y && w && stats && grad_x && grad_w && ws, "beca_bwd: null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t BC = batch * C, total = BC * pixels;
  const float *mean = stats, *sd = stats + BC, *v = stats + 2 * BC, *gate = stats + 3 * BC;
  float *dv = ws, *dstd = ws + BC;
  if (part && beca_par_ok(x, grad_y, C) &&
      part_floats >= jabd_beca_ws_floats(batch, pixels, C)) {
    const int nb = beca_nblk(pixels);
    beca_part_kernel<2><<<dim3((unsigned)nb, (unsigned)batch), 256, 0, st>>>(
        x, grad_y, nullptr, pixels, C, cdiv(pixels, nb), part);
    beca_final_kernel<2><<<(unsigned)cdiv(BC, 256), 256, 0, st>>>(part, nb, C, BC, pixels, dv);
  } else {
    beca_stats_kernel<<<dim3((unsigned)cdiv(C, 64), (unsigned)batch), 256, 0, st>>>(
        x, grad_y, pixels, C, 1, dv, nullptr);
  }
  if (int e = check_launch("beca_dgate")) return e;
  beca_dv_kernel<<<(unsigned)cdiv(BC, 256), 256, 0, st>>>(dv, v, BC);
  beca_dstd_kernel<<<(unsigned)cdiv(BC, 256), 256, 0, st>>>(dv, w, k, C, BC, dstd);
  beca_dw_kernel<<<(unsigned)k, 256, 0, st>>>(dv, sd, k, C, BC, grad_w);
  if (int e = check_launch("beca_dw")) return e;
  beca_dx_kernel<<<(unsigned)cdiv(total, 256), 256, 0, st>>>(x, grad_y, gate, mean, sd, dstd, C,
                                                              pixels, total, grad_x);
  return check_launch("beca_dx");
}
