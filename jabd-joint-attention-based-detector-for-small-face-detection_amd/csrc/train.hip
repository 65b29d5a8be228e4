// A11 training kernels on gfx950 (fp32, NHWC): batch-statistics BatchNorm
// forward/backward fused with the activation (and the residual add of a
// MobileNetV3 block), convolution weight gradients on the fp32 MFMA,
// depthwise weight/data gradients, the ECA gate backward, the detection-head
// gradient gather and the max-pool backward.  Reductions over pixels are
// block partials summed in a fixed order (deterministic).
#include <math.h>

#include "common.h"
#include "conv_args.h"

namespace jabd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float act_f(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: {
      float r = fminf(fmaxf(v + 3.f, 0.f), 6.f);
      return v * r / 6.f;
    }
    default: return v;
  }
}

// d act / d z at pre-activation z (PyTorch's *_backward conventions).
__device__ __forceinline__ float act_d(float z, int act, float slope) {
  switch (act) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_LEAKY: return z > 0.f ? 1.f : slope;
    case ACT_HSWISH: return z < -3.f ? 0.f : (z <= 3.f ? z / 3.f + 0.5f : 1.f);
    default: return 1.f;
  }
}

constexpr int kRedThreads = 256;

// Rows per block of the BN reductions (>= 1 pass of the block).
static int64_t bn_rows_per_blk(int64_t M, int C) {
  const int C4 = C / 4;
  const int lanes = C4 < kRedThreads ? C4 : kRedThreads;
  const int rows_pass = kRedThreads / lanes;
  int64_t per = cdiv(M, 1024);  // ~1024 blocks
  per = cdiv(per, rows_pass) * rows_pass;
  if (per < rows_pass) per = rows_pass;
  return per;
}

// part[blk][0][c] = sum (x - shift[c]), part[blk][1][c] = sum (x - shift[c])^2
// over this block's rows; shift = row 0 of the tensor (limits cancellation).
__global__ __launch_bounds__(kRedThreads) void bn_stats_part_kernel(
    const float* __restrict__ x, int ldx, int64_t M, int C, int64_t rows_per_blk,
    float* __restrict__ part) {
  const int C4 = C >> 2;
  const int lanes = C4 < kRedThreads ? C4 : kRedThreads;
  const int rows_pass = kRedThreads / lanes;
  const int t = threadIdx.x;
  const int r0 = t / lanes;
  const int64_t m0 = blockIdx.x * rows_per_blk;
  const int64_t m1 = min(m0 + rows_per_blk, M);
  __shared__ float4 rs[kRedThreads], rq[kRedThreads];
  for (int cgb = 0; cgb < C4; cgb += lanes) {  // uniform trip count (barriers inside)
    const int cg = cgb + t % lanes;
    const bool cv = cg < C4;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
    if (r0 < rows_pass) {
      const float4 sh = cv ? reinterpret_cast<const float4*>(x)[cg] : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t m = m0 + r0; cv && m < m1; m += rows_pass) {
        float4 v = reinterpret_cast<const float4*>(x + m * ldx)[cg];
        v.x -= sh.x; v.y -= sh.y; v.z -= sh.z; v.w -= sh.w;
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        q.x = fmaf(v.x, v.x, q.x); q.y = fmaf(v.y, v.y, q.y);
        q.z = fmaf(v.z, v.z, q.z); q.w = fmaf(v.w, v.w, q.w);
      }
    }
    __syncthreads();
    rs[t] = s;
    rq[t] = q;
    __syncthreads();
    if (t < lanes && cv) {
      float4 S = make_float4(0.f, 0.f, 0.f, 0.f), Q = S;
      for (int r = 0; r < rows_pass; ++r) {
        const float4 a = rs[r * lanes + t], b = rq[r * lanes + t];
        S.x += a.x; S.y += a.y; S.z += a.z; S.w += a.w;
        Q.x += b.x; Q.y += b.y; Q.z += b.z; Q.w += b.w;
      }
      reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C)[cg] = S;
      reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C + C)[cg] = Q;
    }
  }
}

__global__ void bn_stats_final_kernel(const float* __restrict__ x, const float* __restrict__ part,
                                      int64_t nblk, int64_t M, int C, float momentum, float eps,
                                      float* __restrict__ mean, float* __restrict__ invstd,
                                      float* __restrict__ rmean, float* __restrict__ rvar) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double S = 0.0, Q = 0.0;  // 1024 partials: fp64 accumulation is free here
  for (int64_t b = 0; b < nblk; ++b) {
    S += part[b * 2 * C + c];
    Q += part[b * 2 * C + C + c];
  }
  const double ms = S / (double)M;
  double var = Q / (double)M - ms * ms;
  if (var < 0.0) var = 0.0;
  const float mu = (float)((double)x[c] + ms);
  mean[c] = mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
  if (rvar) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
  }
}

// y = act((x - mean) * invstd * gamma + beta [+ res])
__global__ void bn_act_fwd_kernel(const float* __restrict__ x, int ldx, int64_t M, int C,
                                  const float* __restrict__ mean, const float* __restrict__ invstd,
                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                  const float* __restrict__ res, int ldr, int act, float slope,
                                  float* __restrict__ y, int ldy, int yc0) {
  const int C4 = C >> 2;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= M * C4) return;
  const int64_t m = i / C4;
  const int c = (int)(i - m * C4) * 4;
  const float4 v = *reinterpret_cast<const float4*>(x + m * ldx + c);
  const float4 mu = *reinterpret_cast<const float4*>(mean + c);
  const float4 is = *reinterpret_cast<const float4*>(invstd + c);
  const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
  const float4 bt = *reinterpret_cast<const float4*>(beta + c);
  float4 o;
  o.x = (v.x - mu.x) * is.x * gm.x + bt.x;
  o.y = (v.y - mu.y) * is.y * gm.y + bt.y;
  o.z = (v.z - mu.z) * is.z * gm.z + bt.z;
  o.w = (v.w - mu.w) * is.w * gm.w + bt.w;
  if (res) {
    const float4 r = *reinterpret_cast<const float4*>(res + m * ldr + c);
    o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
  }
  o.x = act_f(o.x, act, slope);
  o.y = act_f(o.y, act, slope);
  o.z = act_f(o.z, act, slope);
  o.w = act_f(o.w, act, slope);
  *reinterpret_cast<float4*>(y + m * ldy + yc0 + c) = o;
}

// dz = dy * act'(z);  part[blk][0][c] = sum dz, part[blk][1][c] = sum dz * xhat
__global__ __launch_bounds__(kRedThreads) void bn_bwd_part_kernel(
    const float* __restrict__ dy, int lddy, int dyc0, const float* __restrict__ x, int ldx,
    const float* __restrict__ res, int ldr, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int act, float slope, int64_t rows_per_blk,
    float* __restrict__ part) {
  const int C4 = C >> 2;
  const int lanes = C4 < kRedThreads ? C4 : kRedThreads;
  const int rows_pass = kRedThreads / lanes;
  const int t = threadIdx.x;
  const int r0 = t / lanes;
  const int64_t m0 = blockIdx.x * rows_per_blk;
  const int64_t m1 = min(m0 + rows_per_blk, M);
  __shared__ float4 rs[kRedThreads], rq[kRedThreads];
  for (int cgb = 0; cgb < C4; cgb += lanes) {  // uniform trip count (barriers inside)
    const int cg = cgb + t % lanes;
    const bool cv = cg < C4;
    const int c = cv ? cg * 4 : 0;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
    if (r0 < rows_pass && cv) {
      const float4 mu = *reinterpret_cast<const float4*>(mean + c);
      const float4 is = *reinterpret_cast<const float4*>(invstd + c);
      const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
      const float4 bt = *reinterpret_cast<const float4*>(beta + c);
      for (int64_t m = m0 + r0; m < m1; m += rows_pass) {
        const float4 v = *reinterpret_cast<const float4*>(x + m * ldx + c);
        const float4 g = *reinterpret_cast<const float4*>(dy + m * lddy + dyc0 + c);
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        if (res) r = *reinterpret_cast<const float4*>(res + m * ldr + c);
        float xh[4] = {(v.x - mu.x) * is.x, (v.y - mu.y) * is.y, (v.z - mu.z) * is.z,
                       (v.w - mu.w) * is.w};
        float gg[4] = {g.x, g.y, g.z, g.w};
        float gmm[4] = {gm.x, gm.y, gm.z, gm.w};
        float btt[4] = {bt.x, bt.y, bt.z, bt.w};
        float rr[4] = {r.x, r.y, r.z, r.w};
        float dz[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) dz[e] = gg[e] * act_d(xh[e] * gmm[e] + btt[e] + rr[e], act, slope);
        s.x += dz[0]; s.y += dz[1]; s.z += dz[2]; s.w += dz[3];
        q.x = fmaf(dz[0], xh[0], q.x); q.y = fmaf(dz[1], xh[1], q.y);
        q.z = fmaf(dz[2], xh[2], q.z); q.w = fmaf(dz[3], xh[3], q.w);
      }
    }
    __syncthreads();
    rs[t] = s;
    rq[t] = q;
    __syncthreads();
    if (t < lanes && cv) {
      float4 S = make_float4(0.f, 0.f, 0.f, 0.f), Q = S;
      for (int r = 0; r < rows_pass; ++r) {
        const float4 a = rs[r * lanes + t], b = rq[r * lanes + t];
        S.x += a.x; S.y += a.y; S.z += a.z; S.w += a.w;
        Q.x += b.x; Q.y += b.y; Q.z += b.z; Q.w += b.w;
      }
      reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C)[cg] = S;
      reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C + C)[cg] = Q;
    }
  }
}

__global__ void bn_bwd_final_kernel(const float* __restrict__ part, int64_t nblk, int C,
                                    float* __restrict__ dbeta, float* __restrict__ dgamma) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double S = 0.0, Q = 0.0;
  for (int64_t b = 0; b < nblk; ++b) {
    S += part[b * 2 * C + c];
    Q += part[b * 2 * C + C + c];
  }
  dbeta[c] = (float)S;
  dgamma[c] = (float)Q;
}

// dx = gamma*invstd*(dz - sum(dz)/M - xhat*sum(dz*xhat)/M); dres = dz
__global__ void bn_bwd_apply_kernel(const float* __restrict__ dy, int lddy, int dyc0,
                                    const float* __restrict__ x, int ldx,
                                    const float* __restrict__ res, int ldr, int64_t M, int C,
                                    const float* __restrict__ mean,
                                    const float* __restrict__ invstd,
                                    const float* __restrict__ gamma,
                                    const float* __restrict__ beta, int act, float slope,
                                    const float* __restrict__ sdz, const float* __restrict__ sdzx,
                                    float* __restrict__ dx, float* __restrict__ dres) {
  const int C4 = C >> 2;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= M * C4) return;
  const int64_t m = i / C4;
  const int c = (int)(i - m * C4) * 4;
  const float invM = 1.f / (float)M;
  const float4 v = *reinterpret_cast<const float4*>(x + m * ldx + c);
  const float4 g = *reinterpret_cast<const float4*>(dy + m * lddy + dyc0 + c);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (res) r = *reinterpret_cast<const float4*>(res + m * ldr + c);
  float vv[4] = {v.x, v.y, v.z, v.w}, gg[4] = {g.x, g.y, g.z, g.w}, rr[4] = {r.x, r.y, r.z, r.w};
  float o[4], dzo[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float mu = mean[c + e], is = invstd[c + e], gm = gamma[c + e], bt = beta[c + e];
    const float xh = (vv[e] - mu) * is;
    const float dz = gg[e] * act_d(xh * gm + bt + rr[e], act, slope);
    dzo[e] = dz;
    o[e] = gm * is * (dz - sdz[c + e] * invM - xh * sdzx[c + e] * invM);
  }
  *reinterpret_cast<float4*>(dx + m * (int64_t)C + c) = make_float4(o[0], o[1], o[2], o[3]);
  if (dres) *reinterpret_cast<float4*>(dres + m * (int64_t)C + c) = make_float4(dzo[0], dzo[1], dzo[2], dzo[3]);
}

// ---------------------------------------------------------------------------
// Conv weight gradient: dW[k][n] = sum_m A[m][k] * dY[m][n]  (A = im2col of x,
// including the forward's ECA A-scale).  Workgroup = 64 k x 64 n tile over a
// chunk of pixels; X^T and dY^T tiles staged through LDS so both MFMA
// operands are float4 LDS reads (4 pixels per lane per k-step).
// ---------------------------------------------------------------------------
template <bool VEC4>
__device__ __forceinline__ float4 wg_load_a(const ConvArgs& p, int64_t m, int k4) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (m >= p.M) return r;
  const int OHW = p.OH * p.OW;
  const int b = (int)(m / OHW);
  const int rr = (int)(m - (int64_t)b * OHW);
  const int oh = rr / p.OW, ow = rr - (rr / p.OW) * p.OW;
  const int Ktot = p.KH * p.KW * p.Cin;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = 0.f;
    const int k = k4 + e;
    if (k >= Ktot) continue;
    const int tap = k / p.Cin, ci = k - tap * p.Cin;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
    const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
    if (ih < 0 || ih >= p.H || iw < 0 || iw >= p.W) continue;
    float xv;
    if (p.nchw_in)
      xv = p.x[(int64_t)b * p.x_bs + ((int64_t)ci * p.H + ih) * p.W + iw];
    else
      xv = p.x[(int64_t)b * p.x_bs + ((int64_t)ih * p.W + iw) * p.x_ps + p.x_c0 + ci];
    if (p.ascale) xv *= p.ascale[(int64_t)b * p.ascale_bs + ci];
    v[e] = xv;
  }
  if (VEC4) {
    (void)r;
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

constexpr int kWgT = 64;       // k and n tile
constexpr int kWgPx = 64;      // pixels per LDS stage
constexpr int kWgLd = kWgPx + 4;

__global__ __launch_bounds__(256) void conv_wgrad_kernel(const ConvArgs p, int64_t px_per_wg,
                                                         float* __restrict__ part) {
  __shared__ float XT[kWgT * kWgLd];
  __shared__ float DT[kWgT * kWgLd];
  const int K = p.KH * p.KW * p.Cin;
  const int k0 = blockIdx.x * kWgT, n0 = blockIdx.y * kWgT;
  const int chunk = blockIdx.z;
  const int64_t mbeg = (int64_t)chunk * px_per_wg;
  const int64_t mend = min(mbeg + px_per_wg, p.M);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i = lane & 15, g = lane >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const float* dy = p.y;  // dY, NHWC [M][y_ps] at channel offset y_c0
  const int OHW = p.OH * p.OW;
  for (int64_t px0 = mbeg; px0 < mend; px0 += kWgPx) {
    // stage X^T (64 k x 64 px) and dY^T (64 n x 64 px): 1024 float4 each
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = q * 256 + t;
      const int px = idx >> 4, c4 = (idx & 15) * 4;
      const int64_t m = px0 + px;
      const bool mv = m < mend;
      float4 a = mv ? wg_load_a<false>(p, m, k0 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      XT[(c4 + 0) * kWgLd + px] = a.x;
      XT[(c4 + 1) * kWgLd + px] = a.y;
      XT[(c4 + 2) * kWgLd + px] = a.z;
      XT[(c4 + 3) * kWgLd + px] = a.w;
      float dv[4] = {0.f, 0.f, 0.f, 0.f};
      if (mv) {
        const int b = (int)(m / OHW);
        const int64_t pix = m - (int64_t)b * OHW;
        const float* dr = dy + (int64_t)b * p.y_bs + pix * p.y_ps + p.y_c0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n0 + c4 + e < p.Cout) dv[e] = dr[n0 + c4 + e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) DT[(c4 + e) * kWgLd + px] = dv[e];
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kWgPx / 16; ++s) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(XT + (16 * wave + i) * kWgLd + 16 * s + 4 * g);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(DT + (16 * u + i) * kWgLd + 16 * s + 4 * g);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc[u], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // acc[u][r] = dW[k0 + 16*wave + 4g + r][n0 + 16u + i]
  float* pc = part + (int64_t)chunk * K * p.Cout;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int n = n0 + 16 * u + i;
    if (n >= p.Cout) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 16 * wave + 4 * g + r;
      if (k < K) pc[(int64_t)k * p.Cout + n] = acc[u][r];
    }
  }
}

// dW (torch layout [Cout][Cin][KH][KW]) = sum over chunks of part[chunk][k][n]
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int64_t nchunk, int K, int Cout,
                                    int Cin, int KHW, float* __restrict__ dw) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)K * Cout) return;
  const int k = (int)(i / Cout), n = (int)(i - (int64_t)k * Cout);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t c = 0;
  for (; c + 4 <= nchunk; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += part[(c + u) * K * Cout + i];
  }
  for (; c < nchunk; ++c) s[0] += part[c * K * Cout + i];
  const int tap = k / Cin, ci = k - tap * Cin;
  dw[((int64_t)n * Cin + ci) * KHW + tap] = (s[0] + s[1]) + (s[2] + s[3]);
}

static int64_t wgrad_chunks(const ConvArgs& a) {
  const int64_t K = (int64_t)a.KH * a.KW * a.Cin;
  const int64_t tiles = cdiv(K, kWgT) * cdiv(a.Cout, kWgT);
  int64_t nchunk = cdiv(2048, tiles);
  const int64_t maxchunk = cdiv(a.M, kWgPx);
  if (nchunk > maxchunk) nchunk = maxchunk;
  // keep the partial buffer <= 64M floats
  const int64_t cap = ((int64_t)64 << 20) / (K * a.Cout);
  if (nchunk > cap) nchunk = cap;
  return nchunk < 1 ? 1 : nchunk;
}

// ---------------------------------------------------------------------------
// Depthwise gradients.  dgrad: dx[i] = sum_{taps with (i+pad-kh) % s == 0}
// dy[(i+pad-kh)/s] * w[kh][kw]  (a gather, so no atomics).  wgrad: per tap
// and channel, sum over pixels of dy * x (block partials, fixed order).
// ---------------------------------------------------------------------------
__global__ void dw_dgrad_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                int H, int W, int C, int OH, int OW, int k, int s, int pad,
                                int64_t total4, float* __restrict__ dx) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int C4 = C >> 2;
  const int c4 = (int)(i % C4);
  int64_t r = i / C4;
  const int iw = (int)(r % W);
  r /= W;
  const int ih = (int)(r % H);
  const int b = (int)(r / H);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kh = 0; kh < k; ++kh) {
    const int nh = ih + pad - kh;
    if (nh < 0 || nh % s) continue;
    const int oh = nh / s;
    if (oh >= OH) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int nw = iw + pad - kw;
      if (nw < 0 || nw % s) continue;
      const int ow = nw / s;
      if (ow >= OW) continue;
      const float4 g = reinterpret_cast<const float4*>(dy + (((int64_t)b * OH + oh) * OW + ow) * C)[c4];
      const float4 wv = reinterpret_cast<const float4*>(w + (kh * k + kw) * C)[c4];
      acc.x = fmaf(g.x, wv.x, acc.x); acc.y = fmaf(g.y, wv.y, acc.y);
      acc.z = fmaf(g.z, wv.z, acc.z); acc.w = fmaf(g.w, wv.w, acc.w);
    }
  }
  reinterpret_cast<float4*>(dx)[i] = acc;
}

// part[blk][tap][c]; block = (rows of output pixels) x (channel groups)
template <int K>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ dy, int H, int W,
                                                       int C, int OH, int OW, int s, int pad,
                                                       int64_t M, int64_t px_per_blk,
                                                       float* __restrict__ part) {
  const int C4 = C >> 2;
  const int lanes = C4 < 256 ? C4 : 256;
  const int rows_pass = 256 / lanes;
  const int t = threadIdx.x;
  const int r0 = t / lanes;
  const int64_t m0 = blockIdx.x * px_per_blk, m1 = min(m0 + px_per_blk, M);
  __shared__ float4 red[256];
  const int OHW = OH * OW;
  for (int cgb = 0; cgb < C4; cgb += lanes) {  // uniform trip count (barriers inside)
    const int cg = cgb + t % lanes;
    const bool cv = cg < C4;
    float4 acc[K * K];
#pragma unroll
    for (int q = 0; q < K * K; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 < rows_pass && cv) {
      for (int64_t m = m0 + r0; m < m1; m += rows_pass) {
        const int b = (int)(m / OHW);
        const int rr = (int)(m - (int64_t)b * OHW);
        const int oh = rr / OW, ow = rr - (rr / OW) * OW;
        const float4 g = reinterpret_cast<const float4*>(dy + m * C)[cg];
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
          const int ih = oh * s - pad + kh;
          if (ih < 0 || ih >= H) continue;
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            const int iw = ow * s - pad + kw;
            if (iw < 0 || iw >= W) continue;
            const float4 v = reinterpret_cast<const float4*>(x + (((int64_t)b * H + ih) * W + iw) * C)[cg];
            float4& a = acc[kh * K + kw];
            a.x = fmaf(g.x, v.x, a.x); a.y = fmaf(g.y, v.y, a.y);
            a.z = fmaf(g.z, v.z, a.z); a.w = fmaf(g.w, v.w, a.w);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < K * K; ++q) {
      __syncthreads();
      red[t] = acc[q];
      __syncthreads();
      if (t < lanes && cv) {
        float4 S = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int r = 0; r < rows_pass; ++r) {
          const float4 a = red[r * lanes + t];
          S.x += a.x; S.y += a.y; S.z += a.z; S.w += a.w;
        }
        reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * K * K + q) * C)[cg] = S;
      }
    }
  }
}

// dw torch layout [C][1][k][k] = sum over blocks of part[blk][tap][c]
__global__ void dw_wgrad_reduce_kernel(const float* __restrict__ part, int64_t nblk, int KK, int C,
                                       float* __restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= KK * C) return;
  const int tap = i / C, c = i - tap * C;
  double s = 0.0;
  for (int64_t b = 0; b < nblk; ++b) s += part[b * KK * C + i];
  dw[c * KK + tap] = (float)s;
}

// ---------------------------------------------------------------------------
// ECA-scaled operand backward.  The consumer conv saw a = x * s[b][c]; given
// da: dx = da * s, and ds[b][c] = sum_hw da * x (block partials).
// ---------------------------------------------------------------------------
__global__ void scale_bwd_kernel(const float* __restrict__ da, const float* __restrict__ x,
                                 const float* __restrict__ s, int64_t HW, int C, int64_t per_blk,
                                 int nblk, float* __restrict__ dx, float* __restrict__ part) {
  const int b = blockIdx.y;
  const int C4 = C >> 2;
  const int lanes = C4 < 256 ? C4 : 256;
  const int rows_pass = 256 / lanes;
  const int t = threadIdx.x, r0 = t / lanes;
  const int64_t p0 = blockIdx.x * per_blk, p1 = min(p0 + per_blk, HW);
  __shared__ float4 red[256];
  for (int cgb = 0; cgb < C4; cgb += lanes) {  // uniform trip count (barriers inside)
    const int cg = cgb + t % lanes;
    const bool cv = cg < C4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 sc = cv ? reinterpret_cast<const float4*>(s + (int64_t)b * C)[cg]
                         : make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 < rows_pass && cv) {
      for (int64_t q = p0 + r0; q < p1; q += rows_pass) {
        const int64_t off = ((int64_t)b * HW + q) * C;
        const float4 g = reinterpret_cast<const float4*>(da + off)[cg];
        const float4 v = reinterpret_cast<const float4*>(x + off)[cg];
        reinterpret_cast<float4*>(dx + off)[cg] =
            make_float4(g.x * sc.x, g.y * sc.y, g.z * sc.z, g.w * sc.w);
        acc.x = fmaf(g.x, v.x, acc.x); acc.y = fmaf(g.y, v.y, acc.y);
        acc.z = fmaf(g.z, v.z, acc.z); acc.w = fmaf(g.w, v.w, acc.w);
      }
    }
    __syncthreads();
    red[t] = acc;
    __syncthreads();
    if (t < lanes && cv) {
      float4 S = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < rows_pass; ++r) {
        const float4 a = red[r * lanes + t];
        S.x += a.x; S.y += a.y; S.z += a.z; S.w += a.w;
      }
      reinterpret_cast<float4*>(part + ((int64_t)b * nblk + blockIdx.x) * C)[cg] = S;
    }
  }
}

// Per image: ds -> dz = ds * gate'(z) -> dmean (transposed Conv1d) -> the
// per-(b,c) term added to dx, and the Conv1d weight-gradient partial per image.
__global__ void eca_gate_bwd_kernel(const float* __restrict__ part, int nblk, int C,
                                    const float* __restrict__ mean, const float* __restrict__ s,
                                    const float* __restrict__ w1d, int k, int gate, float inv_hw,
                                    float* __restrict__ dmean_hw, float* __restrict__ dw1d_img) {
  extern __shared__ float sm[];  // dz [C], mean [C]
  float* dz = sm;
  float* mu = sm + C;
  const int b = blockIdx.x;
  const int h = (k - 1) / 2;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float ds = 0.f;
    for (int q = 0; q < nblk; ++q) ds += part[((int64_t)b * nblk + q) * C + c];
    const float sv = s[(int64_t)b * C + c];
    float gd;
    if (gate == ACT_SIGMOID) {
      gd = sv * (1.f - sv);
    } else {  // Hardsigmoid'(z) = 1/6 on (-3, 3): recompute z
      float z = 0.f;
      for (int t = 0; t < k; ++t) {
        const int cc = c + t - h;
        if (cc >= 0 && cc < C) z = fmaf(w1d[t], mean[(int64_t)b * C + cc], z);
      }
      gd = (z > -3.f && z < 3.f) ? 1.f / 6.f : 0.f;
    }
    dz[c] = ds * gd;
    mu[c] = mean[(int64_t)b * C + c];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float dm = 0.f;
    for (int t = 0; t < k; ++t) {  // z[c'] = sum_t w[t] mean[c' + t - h]  =>  c' = c - t + h
      const int cp = c - t + h;
      if (cp >= 0 && cp < C) dm = fmaf(w1d[t], dz[cp], dm);
    }
    dmean_hw[(int64_t)b * C + c] = dm * inv_hw;
  }
  if (threadIdx.x < k) {
    const int t = threadIdx.x;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) {
      const int cc = c + t - h;
      if (cc >= 0 && cc < C) acc = fmaf(dz[c], mu[cc], acc);
    }
    dw1d_img[(int64_t)b * k + t] = acc;
  }
}

__global__ void add_bc_kernel(float* __restrict__ dx, const float* __restrict__ v, int64_t HW, int C,
                              int64_t total4) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int C4 = C >> 2;
  const int64_t m = i / C4;
  const int c4 = (int)(i - m * C4);
  const int b = (int)(m / HW);
  const float4 a = reinterpret_cast<const float4*>(v + (int64_t)b * C)[c4];
  float4 d = reinterpret_cast<float4*>(dx)[i];
  d.x += a.x; d.y += a.y; d.z += a.z; d.w += a.w;
  reinterpret_cast<float4*>(dx)[i] = d;
}

__global__ void eca_w_reduce_kernel(const float* __restrict__ dw1d_img, int B, int k,
                                    float* __restrict__ dw1d) {
  const int t = threadIdx.x;
  if (t >= k) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += dw1d_img[(int64_t)b * k + t];
  dw1d[t] = s;
}

// ---------------------------------------------------------------------------
// Heads: gather d(loc|conf|landm) of one pyramid level into [B][HW][32].
// ---------------------------------------------------------------------------
__global__ void heads_gather_kernel(const float* __restrict__ gl, const float* __restrict__ gc,
                                    const float* __restrict__ glm, int64_t A, int64_t a_off,
                                    int HW, float* __restrict__ dout) {
  const int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (pix >= HW) return;
  const int64_t row = (int64_t)b * A + a_off + pix * 2;
  float* o = dout + ((int64_t)b * HW + pix) * 32;
  const float4* l4 = reinterpret_cast<const float4*>(gl + row * 4);
  reinterpret_cast<float4*>(o)[0] = l4[0];
  reinterpret_cast<float4*>(o)[1] = l4[1];
  reinterpret_cast<float4*>(o)[2] = reinterpret_cast<const float4*>(gc + row * 2)[0];
  for (int n = 0; n < 20; ++n) o[12 + n] = glm[row * 10 + n];
}

// ---------------------------------------------------------------------------
// Max-pool backward (gather form): each input pixel sums dy of the windows
// whose (first, NaN-propagating) argmax it is — F.max_pool2d semantics.
// ---------------------------------------------------------------------------
__global__ void maxpool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, int H,
                                   int W, int C, int OH, int OW, int k, int s, int pad,
                                   int64_t total, float* __restrict__ dx) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  int64_t r = i / C;
  const int iw = (int)(r % W);
  r /= W;
  const int ih = (int)(r % H);
  const int b = (int)(r / H);
  float acc = 0.f;
  for (int kh = 0; kh < k; ++kh) {
    const int nh = ih + pad - kh;
    if (nh < 0 || nh % s) continue;
    const int oh = nh / s;
    if (oh >= OH) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int nw = iw + pad - kw;
      if (nw < 0 || nw % s) continue;
      const int ow = nw / s;
      if (ow >= OW) continue;
      // recompute the argmax of window (oh, ow)
      float best = -INFINITY;
      int bh = -1, bw = -1;
      for (int a = 0; a < k; ++a) {
        const int yh = oh * s - pad + a;
        if (yh < 0 || yh >= H) continue;
        for (int q = 0; q < k; ++q) {
          const int yw = ow * s - pad + q;
          if (yw < 0 || yw >= W) continue;
          const float v = x[(((int64_t)b * H + yh) * W + yw) * C + c];
          if (bh < 0 || v > best || v != v) { best = v; bh = yh; bw = yw; }
        }
      }
      if (bh == ih && bw == iw) acc += dy[(((int64_t)b * OH + oh) * OW + ow) * C + c];
    }
  }
  dx[i] = acc;
}

}  // namespace jabd

using namespace jabd;

extern "C" int64_t jabd_bn_nblk(int64_t M, int32_t C) {
  if (M <= 0 || C <= 0 || C % 4) return -1;
  return cdiv(M, bn_rows_per_blk(M, C));
}

extern "C" int jabd_bn_stats_f32(const float* x, int32_t ldx, int64_t M, int32_t C, float* part,
                                 float* mean, float* invstd, float* running_mean,
                                 float* running_var, float momentum, float eps,
                                 jabd_stream_t stream) {
  JABD_REQUIRE(x && part && mean && invstd && M > 0 && C > 0 && C % 4 == 0 && ldx % 4 == 0,
               "bn_stats: bad args");
  hipStream_t st = as_stream(stream);
  const int64_t per = bn_rows_per_blk(M, C), nblk = cdiv(M, per);
  bn_stats_part_kernel<<<(unsigned)nblk, kRedThreads, 0, st>>>(x, ldx, M, C, per, part);
  if (int e = check_launch("bn_stats_part")) return e;
  bn_stats_final_kernel<<<(unsigned)cdiv(C, 256), 256, 0, st>>>(x, part, nblk, M, C, momentum, eps,
                                                                mean, invstd, running_mean,
                                                                running_var);
  return check_launch("bn_stats_final");
}

extern "C" int jabd_bn_act_fwd_f32(const float* x, int32_t ldx, int64_t M, int32_t C,
                                   const float* mean, const float* invstd, const float* gamma,
                                   const float* beta, const float* res, int32_t ldr, int32_t act,
                                   float slope, float* y, int32_t ldy, int32_t yc0,
                                   jabd_stream_t stream) {
  JABD_REQUIRE(x && mean && invstd && gamma && beta && y && C % 4 == 0 && ldx % 4 == 0 &&
                   ldy % 4 == 0 && yc0 % 4 == 0 && (!res || ldr % 4 == 0),
               "bn_act_fwd: bad args");
  const int64_t total = M * (C / 4);
  if (total == 0) return JABD_OK;
  bn_act_fwd_kernel<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      x, ldx, M, C, mean, invstd, gamma, beta, res, ldr, act, slope, y, ldy, yc0);
  return check_launch("bn_act_fwd");
}

extern "C" int jabd_bn_act_bwd_f32(const float* dy, int32_t lddy, int32_t dyc0, const float* x,
                                   int32_t ldx, const float* res, int32_t ldr, int64_t M,
                                   int32_t C, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, int32_t act,
                                   float slope, float* part, float* dgamma, float* dbeta,
                                   float* dx, float* dres, jabd_stream_t stream) {
  JABD_REQUIRE(dy && x && mean && invstd && gamma && beta && part && dgamma && dbeta && dx &&
                   C % 4 == 0 && lddy % 4 == 0 && dyc0 % 4 == 0 && ldx % 4 == 0,
               "bn_act_bwd: bad args");
  hipStream_t st = as_stream(stream);
  const int64_t per = bn_rows_per_blk(M, C), nblk = cdiv(M, per);
  bn_bwd_part_kernel<<<(unsigned)nblk, kRedThreads, 0, st>>>(dy, lddy, dyc0, x, ldx, res, ldr, M,
                                                            C, mean, invstd, gamma, beta, act,
                                                            slope, per, part);
  if (int e = check_launch("bn_bwd_part")) return e;
  bn_bwd_final_kernel<<<(unsigned)cdiv(C, 256), 256, 0, st>>>(part, nblk, C, dbeta, dgamma);
  if (int e = check_launch("bn_bwd_final")) return e;
  const int64_t total = M * (C / 4);
  bn_bwd_apply_kernel<<<(unsigned)cdiv(total, 256), 256, 0, st>>>(
      dy, lddy, dyc0, x, ldx, res, ldr, M, C, mean, invstd, gamma, beta, act, slope, dbeta, dgamma,
      dx, dres);
  return check_launch("bn_bwd_apply");
}

extern "C" int64_t jabd_conv_wgrad_part_floats(const jabd_conv_args* args) {
  if (!args) return -1;
  ConvArgs a = *args;
  a.M = (int64_t)a.B * a.OH * a.OW;
  return wgrad_chunks(a) * (int64_t)a.KH * a.KW * a.Cin * a.Cout;
}

extern "C" int jabd_conv_wgrad_f32(const jabd_conv_args* args, float* part, float* dw,
                                   jabd_stream_t stream) {
  JABD_REQUIRE(args && part && dw, "conv_wgrad: null");
  ConvArgs a = *args;
  JABD_REQUIRE(a.x && a.y && !a.x2 && !a.tconv, "conv_wgrad: bad args");
  a.M = (int64_t)a.B * a.OH * a.OW;
  JABD_REQUIRE(a.M < (int64_t)0x7fffffff, "conv_wgrad: M too large");
  const int K = a.KH * a.KW * a.Cin;
  const int64_t nchunk = wgrad_chunks(a);
  const int64_t per = cdiv(cdiv(a.M, nchunk), kWgPx) * kWgPx;
  const int64_t nch = cdiv(a.M, per);
  hipStream_t st = as_stream(stream);
  dim3 g((unsigned)cdiv(K, kWgT), (unsigned)cdiv(a.Cout, kWgT), (unsigned)nch);
  conv_wgrad_kernel<<<g, 256, 0, st>>>(a, per, part);
  if (int e = check_launch("conv_wgrad")) return e;
  const int64_t tot = (int64_t)K * a.Cout;
  wgrad_reduce_kernel<<<(unsigned)cdiv(tot, 256), 256, 0, st>>>(part, nch, K, a.Cout, a.Cin,
                                                                a.KH * a.KW, dw);
  return check_launch("wgrad_reduce");
}

extern "C" int jabd_dw_dgrad_f32(const float* dy, const float* w, int32_t B, int32_t H, int32_t W,
                                 int32_t C, int32_t OH, int32_t OW, int32_t k, int32_t stride,
                                 int32_t pad, float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(dy && w && dx && C % 4 == 0, "dw_dgrad: bad args");
  const int64_t total4 = (int64_t)B * H * W * (C / 4);
  dw_dgrad_kernel<<<(unsigned)cdiv(total4, 256), 256, 0, as_stream(stream)>>>(
      dy, w, H, W, C, OH, OW, k, stride, pad, total4, dx);
  return check_launch("dw_dgrad");
}

extern "C" int64_t jabd_dw_wgrad_part_floats(int64_t M, int32_t C, int32_t k) {
  return 1024 * (int64_t)k * k * C;
}

extern "C" int jabd_dw_wgrad_f32(const float* x, const float* dy, int32_t B, int32_t H, int32_t W,
                                 int32_t C, int32_t OH, int32_t OW, int32_t k, int32_t stride,
                                 int32_t pad, float* part, float* dw, jabd_stream_t stream) {
  JABD_REQUIRE(x && dy && part && dw && C % 4 == 0, "dw_wgrad: bad args");
  const int64_t M = (int64_t)B * OH * OW;
  int64_t per = cdiv(M, 1024);
  if (per < 1) per = 1;
  const int64_t nblk = cdiv(M, per);
  hipStream_t st = as_stream(stream);
  if (k == 3)
    dw_wgrad_kernel<3><<<(unsigned)nblk, 256, 0, st>>>(x, dy, H, W, C, OH, OW, stride, pad, M, per,
                                                       part);
  else if (k == 5)
    dw_wgrad_kernel<5><<<(unsigned)nblk, 256, 0, st>>>(x, dy, H, W, C, OH, OW, stride, pad, M, per,
                                                       part);
  else {
    set_error("dw_wgrad: k=%d unsupported", k);
    return JABD_EINVAL;
  }
  if (int e = check_launch("dw_wgrad")) return e;
  dw_wgrad_reduce_kernel<<<(unsigned)cdiv((int64_t)k * k * C, 256), 256, 0, st>>>(part, nblk, k * k,
                                                                                C, dw);
  return check_launch("dw_wgrad_reduce");
}

extern "C" int jabd_eca_bwd_f32(const float* da, const float* x, int64_t B, int64_t HW,
                                int32_t C, const float* scale, const float* mean,
                                const float* w1d, int32_t k, int32_t gate, float* part,
                                int32_t nblk, float* dmean_ws, float* dw1d_ws, float* dx,
                                float* dw1d, jabd_stream_t stream) {
  JABD_REQUIRE(da && x && scale && mean && w1d && part && dmean_ws && dw1d_ws && dx && dw1d &&
                   C % 4 == 0 && nblk > 0,
               "eca_bwd: bad args");
  hipStream_t st = as_stream(stream);
  const int64_t per = cdiv(HW, nblk);
  dim3 g((unsigned)nblk, (unsigned)B);
  scale_bwd_kernel<<<g, 256, 0, st>>>(da, x, scale, HW, C, per, nblk, dx, part);
  if (int e = check_launch("scale_bwd")) return e;
  eca_gate_bwd_kernel<<<(unsigned)B, 256, 2 * C * sizeof(float), st>>>(
      part, nblk, C, mean, scale, w1d, k, gate, 1.f / (float)HW, dmean_ws, dw1d_ws);
  if (int e = check_launch("eca_gate_bwd")) return e;
  const int64_t total4 = B * HW * (C / 4);
  add_bc_kernel<<<(unsigned)cdiv(total4, 256), 256, 0, st>>>(dx, dmean_ws, HW, C, total4);
  if (int e = check_launch("eca_add")) return e;
  eca_w_reduce_kernel<<<1, 64, 0, st>>>(dw1d_ws, (int)B, k, dw1d);
  return check_launch("eca_w_reduce");
}

extern "C" int jabd_scale_bwd_f32(const float* da, const float* x, int64_t B, int64_t HW,
                                  int32_t C, const float* scale, float* part, int32_t nblk,
                                  float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(da && x && scale && part && dx && C % 4 == 0 && nblk > 0, "scale_bwd: bad args");
  dim3 g((unsigned)nblk, (unsigned)B);
  scale_bwd_kernel<<<g, 256, 0, as_stream(stream)>>>(da, x, scale, HW, C, cdiv(HW, nblk), nblk, dx,
                                                     part);
  return check_launch("scale_bwd");
}

extern "C" int jabd_heads_gather_f32(const float* gloc, const float* gconf, const float* glandm,
                                     int32_t B, int64_t A, int64_t a_off, int32_t HW, float* dout,
                                     jabd_stream_t stream) {
  JABD_REQUIRE(gloc && gconf && glandm && dout, "heads_gather: null");
  dim3 g((unsigned)cdiv(HW, 256), (unsigned)B);
  heads_gather_kernel<<<g, 256, 0, as_stream(stream)>>>(gloc, gconf, glandm, A, a_off, HW, dout);
  return check_launch("heads_gather");
}

extern "C" int jabd_maxpool_bwd_f32(const float* x, const float* dy, int32_t B, int32_t H,
                                    int32_t W, int32_t C, int32_t k, int32_t stride, int32_t pad,
                                    float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(x && dy && dx, "maxpool_bwd: null");
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  const int64_t total = (int64_t)B * H * W * C;
  maxpool_bwd_kernel<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      x, dy, H, W, C, OH, OW, k, stride, pad, total, dx);
  return check_launch("maxpool_bwd");
}
