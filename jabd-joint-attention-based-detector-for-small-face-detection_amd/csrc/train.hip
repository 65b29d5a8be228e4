// A11 training kernels on gfx950 (fp32, NHWC): batch-statistics BatchNorm
// forward/backward fused with the activation (and the residual add of a
// MobileNetV3 block), convolution weight gradients on the fp32 MFMA,
// depthwise weight/data gradients, the ECA gate backward, the detection-head
// gradient gather and the max-pool backward.  Reductions over pixels are
// block partials summed in a fixed order (deterministic).
#include <math.h>

#include <algorithm>

#include "common.h"
#include "conv_args.h"

namespace jabd {
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float act_f(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return relu_f(v);
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: {
      float r = fminf(fmaxf(v + 3.f, 0.f), 6.f);
      return v * r * (1.f / 6.f);
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

// Rows whose loads a BN reduction thread issues before accumulating them.
constexpr int kBnBatch = 8;

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
    if (r0 < rows_pass && cv) {
      const float4 sh = reinterpret_cast<const float4*>(x)[cg];
      auto acc = [&](float4 v) {
        v.x -= sh.x; v.y -= sh.y; v.z -= sh.z; v.w -= sh.w;
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        q.x = fmaf(v.x, v.x, q.x); q.y = fmaf(v.y, v.y, q.y);
        q.z = fmaf(v.z, v.z, q.z); q.w = fmaf(v.w, v.w, q.w);
      };
      // kBnBatch rows' loads in flight before their (in-order) accumulation:
      // one load per iteration left each wave one HBM round trip per row
      int64_t m = m0 + r0;
      for (; m + (kBnBatch - 1) * rows_pass < m1; m += kBnBatch * rows_pass) {
        float4 v[kBnBatch];
#pragma unroll
        for (int u = 0; u < kBnBatch; ++u)
          v[u] = reinterpret_cast<const float4*>(x + (m + u * rows_pass) * ldx)[cg];
#pragma unroll
        for (int u = 0; u < kBnBatch; ++u) acc(v[u]);
      }
      for (; m < m1; m += rows_pass) acc(reinterpret_cast<const float4*>(x + m * ldx)[cg]);
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

// Deterministic fp64 sum over the nblk partial blocks of part[b][0|1][c] for
// the kFinLanes channels of this workgroup: kFinThreads / kFinLanes rows of
// threads stride the blocks (8 independent loads in flight per thread, so
// ~1024 partials take two L2 round trips instead of a 256-deep chain), then a
// fixed-shape LDS tree over the rows.  Valid in threads t < kFinLanes.
constexpr int kFinThreads = 1024, kFinLanes = 16, kFinRows = kFinThreads / kFinLanes;

template <typename T>
__device__ __forceinline__ void bn_final_sums(const T* __restrict__ part, int64_t nblk, int C,
                                              double& S, double& Q) {
  __shared__ double ls[kFinThreads], lq[kFinThreads];
  const int t = threadIdx.x;
  const int r = t / kFinLanes;
  const int c = blockIdx.x * kFinLanes + t % kFinLanes;
  double s = 0.0, q = 0.0;
  if (c < C) {
    int64_t b = r;
    for (; b + 7 * kFinRows < nblk; b += 8 * kFinRows) {
      T vs[8], vq[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        vs[u] = part[(b + u * kFinRows) * 2 * C + c];
        vq[u] = part[(b + u * kFinRows) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += vs[u];
        q += vq[u];
      }
    }
    for (; b < nblk; b += kFinRows) {
      s += part[b * 2 * C + c];
      q += part[b * 2 * C + C + c];
    }
  }
  ls[t] = s;
  lq[t] = q;
  __syncthreads();
#pragma unroll
  for (int h = kFinThreads / 2; h >= kFinLanes; h >>= 1) {
    if (t < h) {
      ls[t] += ls[t + h];
      lq[t] += lq[t + h];
    }
    __syncthreads();
  }
  S = ls[t % kFinLanes];
  Q = lq[t % kFinLanes];
}

template <typename T>
__global__ __launch_bounds__(kFinThreads) void bn_stats_final_kernel(
    const float* __restrict__ x, const T* __restrict__ part, int64_t nblk, int64_t M, int C,
    float momentum, float eps, float* __restrict__ mean, float* __restrict__ invstd,
    float* __restrict__ rmean, float* __restrict__ rvar) {
  double S, Q;
  bn_final_sums(part, nblk, C, S, Q);
  const int c = blockIdx.x * kFinLanes + threadIdx.x;
  if (threadIdx.x >= kFinLanes || c >= C) return;
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

// Statistics rows of a producer that takes them per 32-pixel tile (the 32x32
// GEMM's ST epilogue, conv32.hip): rows[r][0][c] = the tile's mean,
// rows[r][1][c] = its sum of squared deviations, r < nrow = ceil(M / 32),
// row pitch 2 * ldc.  First stage of the exact combination: per chunk of
// kRowChunk rows, in fp64 and row order, the sums around the shift
// sh = rows[0][0][c] (tile 0's mean):
//   S = sum n_r (mean_r - sh),  Q = sum M2_r + n_r (mean_r - sh)^2,
// to out[chunk][0|1][c] (bn_stats_part's layout in double); the second stage
// is bn_stats_final_kernel<double> with x = rows (shift = row 0's means).
constexpr int kRowChunk = 64;

__global__ __launch_bounds__(256) void bn_rows_chunk_kernel(const float* __restrict__ rows,
                                                            int ldc, int64_t nrow, int64_t M,
                                                            int C, double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t chunk = i / C;
  const int c = (int)(i - chunk * C);
  const int64_t r0 = chunk * kRowChunk;
  if (r0 >= nrow) return;
  const int64_t r1 = min(r0 + kRowChunk, nrow);
  const double sh = (double)rows[c];
  double S = 0.0, Q = 0.0;
  int64_t r = r0;
  auto acc = [&](int64_t rr, float mu, float m2) {
    const double n = (double)min<int64_t>(32, M - rr * 32);
    const double d = (double)mu - sh;
    S += n * d;
    Q += (double)m2 + n * d * d;
  };
  for (; r + 8 <= r1; r += 8) {
    float mu[8], m2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      mu[u] = rows[(r + u) * 2 * ldc + c];
      m2[u] = rows[(r + u) * 2 * ldc + ldc + c];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc(r + u, mu[u], m2[u]);
  }
  for (; r < r1; ++r) acc(r, rows[r * 2 * ldc + c], rows[r * 2 * ldc + ldc + c]);
  out[chunk * 2 * C + c] = S;
  out[chunk * 2 * C + C + c] = Q;
}

// Plain fp64 sums of kRowChunk-row chunks of rows[r][0|1][C] (the 32x32
// GEMM's BatchNorm-backward epilogue rows), in row order, to out[chunk][0|1][C].
__global__ __launch_bounds__(256) void bn_rows_sum_kernel(const float* __restrict__ rows,
                                                          int64_t nrow, int C,
                                                          double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t chunk = i / C;
  const int c = (int)(i - chunk * C);
  const int64_t r0 = chunk * kRowChunk;
  if (r0 >= nrow) return;
  const int64_t r1 = min(r0 + kRowChunk, nrow);
  double S = 0.0, Q = 0.0;
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
    float a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = rows[(r + u) * 2 * C + c];
      b[u] = rows[(r + u) * 2 * C + C + c];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      S += (double)a[u];
      Q += (double)b[u];
    }
  }
  for (; r < r1; ++r) {
    S += (double)rows[r * 2 * C + c];
    Q += (double)rows[r * 2 * C + C + c];
  }
  out[chunk * 2 * C + c] = S;
  out[chunk * 2 * C + C + c] = Q;
}

int64_t bn_rows_sum_doubles(int64_t M, int C) {
  return cdiv(cdiv(M, (int64_t)32), (int64_t)kRowChunk) * 2 * C;
}

int64_t bn_rows_chunk_doubles(int64_t M, int C) {
  return cdiv(cdiv(M, (int64_t)32), (int64_t)kRowChunk) * 2 * C;
}

int bn_rows_final_launch(const float* rows, int ldc, int64_t M, int C, double* chunks,
                         float* mean, float* invstd, float* rmean, float* rvar, float momentum,
                         float eps, hipStream_t st) {
  const int64_t nrow = cdiv(M, (int64_t)32), nch = cdiv(nrow, (int64_t)kRowChunk);
  bn_rows_chunk_kernel<<<(unsigned)cdiv(nch * C, (int64_t)256), 256, 0, st>>>(rows, ldc, nrow, M,
                                                                             C, chunks);
  if (int e = check_launch("bn_rows_chunk")) return e;
  bn_stats_final_kernel<double><<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, st>>>(
      rows, chunks, nch, M, C, momentum, eps, mean, invstd, rmean, rvar);
  return check_launch("bn_stats_final (rows)");
}

// Elementwise BN kernels: workgroup = `lanes` float4 channel groups x
// (256 / lanes) rows, `iters` row passes; per-channel parameters live in
// registers (no per-element index division).
constexpr int kEwIters = 8;

struct EwMap {
  int64_t m0;
  int rows_pass, cg;
  bool ok;
};

__device__ __forceinline__ EwMap ew_map(int lanes, int C4) {
  EwMap e;
  const int t = threadIdx.x;
  e.rows_pass = kRedThreads / lanes;
  const int r0 = t / lanes;
  e.cg = blockIdx.y * lanes + t % lanes;
  e.ok = r0 < e.rows_pass && e.cg < C4;
  e.m0 = (int64_t)blockIdx.x * e.rows_pass * kEwIters + r0;
  return e;
}

// y = act((x - mean) * invstd * gamma + beta [+ res])
// RES / TR: residual / dy-transform operand present (compile time: a runtime
// select of a float4 operand was lowered through scratch)
template <bool RES>
__global__ __launch_bounds__(kRedThreads) void bn_act_fwd_kernel(
    const float* __restrict__ x, int ldx, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ res, int ldr, int act, float slope,
    float* __restrict__ y, int ldy, int yc0, int lanes) {
  const EwMap e = ew_map(lanes, C >> 2);
  if (!e.ok) return;
  const int c = e.cg * 4;
  const float4 mu = *reinterpret_cast<const float4*>(mean + c);
  const float4 is = *reinterpret_cast<const float4*>(invstd + c);
  const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
  const float4 bt = *reinterpret_cast<const float4*>(beta + c);
  auto one = [&](int64_t m, float4 v, float4 r) {
    float4 o;
    o.x = (v.x - mu.x) * is.x * gm.x + bt.x;
    o.y = (v.y - mu.y) * is.y * gm.y + bt.y;
    o.z = (v.z - mu.z) * is.z * gm.z + bt.z;
    o.w = (v.w - mu.w) * is.w * gm.w + bt.w;
    if (RES) {
      o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
    }
    o.x = act_f(o.x, act, slope);
    o.y = act_f(o.y, act, slope);
    o.z = act_f(o.z, act, slope);
    o.w = act_f(o.w, act, slope);
    *reinterpret_cast<float4*>(y + m * ldy + yc0 + c) = o;
  };
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e.m0 + (int64_t)(kEwIters - 1) * e.rows_pass < M) {
    // full block: every row's loads in flight first
    float4 v[kEwIters], r[kEwIters];
#pragma unroll
    for (int k = 0; k < kEwIters; ++k) {
      const int64_t m = e.m0 + (int64_t)k * e.rows_pass;
      v[k] = *reinterpret_cast<const float4*>(x + m * ldx + c);
      r[k] = RES ? *reinterpret_cast<const float4*>(res + m * ldr + c) : z4;
    }
#pragma unroll
    for (int k = 0; k < kEwIters; ++k) one(e.m0 + (int64_t)k * e.rows_pass, v[k], r[k]);
    return;
  }
  for (int k = 0; k < kEwIters; ++k) {
    const int64_t m = e.m0 + (int64_t)k * e.rows_pass;
    if (m >= M) break;
    one(m, *reinterpret_cast<const float4*>(x + m * ldx + c),
        RES ? *reinterpret_cast<const float4*>(res + m * ldr + c) : z4);
  }
}

// y = act((x - mean) * invstd * gamma + beta) and, for the ECA gate that
// follows BN2 in a MobileNetV3 block (nets/mobilenetV3.py:141-148), the
// channel sums of y per block of RB = rp * kEwIters rows (rp a power of two
// dividing H*W / kEwIters, so no block straddles an image): part[blk][c],
// i.e. [B][HW / RB][C] — the pass over y that F.channel_sums would make.
__global__ __launch_bounds__(kRedThreads) void bn_act_fwd_sum_kernel(
    const float* __restrict__ x, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int act, float slope, float* __restrict__ y, int lanes,
    int rp, float* __restrict__ part) {
  __shared__ float4 red[kRedThreads];
  const int t = threadIdx.x, r0 = t / lanes, cl = t - r0 * lanes;
  const int C4 = C >> 2;
  const int cg = blockIdx.y * lanes + cl;
  const bool ok = r0 < rp && cg < C4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    const int c = cg * 4;
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
    const float4 bt = *reinterpret_cast<const float4*>(beta + c);
    const int64_t m0 = (int64_t)blockIdx.x * rp * kEwIters + r0;
    auto one = [&](int64_t m, float4 v) {
      float4 o;
      o.x = act_f((v.x - mu.x) * is.x * gm.x + bt.x, act, slope);
      o.y = act_f((v.y - mu.y) * is.y * gm.y + bt.y, act, slope);
      o.z = act_f((v.z - mu.z) * is.z * gm.z + bt.z, act, slope);
      o.w = act_f((v.w - mu.w) * is.w * gm.w + bt.w, act, slope);
      *reinterpret_cast<float4*>(y + m * C + c) = o;
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
    };
    if (m0 + (int64_t)(kEwIters - 1) * rp < M) {  // full block: loads first
      float4 v[kEwIters];
#pragma unroll
      for (int k = 0; k < kEwIters; ++k)
        v[k] = *reinterpret_cast<const float4*>(x + (m0 + (int64_t)k * rp) * C + c);
#pragma unroll
      for (int k = 0; k < kEwIters; ++k) one(m0 + (int64_t)k * rp, v[k]);
    } else {
      for (int k = 0; k < kEwIters; ++k) {
        const int64_t m = m0 + (int64_t)k * rp;
        if (m >= M) break;
        one(m, *reinterpret_cast<const float4*>(x + m * C + c));
      }
    }
  }
  red[t] = acc;
  __syncthreads();
  if (r0 == 0 && cg < C4) {
    float4 S = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < rp; ++r) {
      const float4 a = red[r * lanes + cl];
      S.x += a.x; S.y += a.y; S.z += a.z; S.w += a.w;
    }
    reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * C)[cg] = S;
  }
}

// dz = dy * act'(z);  part[blk][0][c] = sum dz, part[blk][1][c] = sum dz * xhat
// Optional per-(image, channel) affine map of the incoming gradient,
// dy' = dy * dys[b][c] + dya[b][c] (b = row / hw): the backward of an ECA
// gate applied after this BN (x * s[b][c], and the pooled-mean term of the
// gate's own gradient), fused here instead of a separate pass over dy.
// The image's (dys, dya) row is cached: a thread's rows only increase, so the
// 64-bit m / hw and the two loads happen once per image crossing instead of
// once per row.
struct DyImgCache {
  int64_t lo = 0, hi = -1;
  float4 sc, ad;
  __device__ __forceinline__ float4 apply(float4 g, const float* __restrict__ dys,
                                          const float* __restrict__ dya, int64_t m, int64_t hw,
                                          int C, int c) {
    if (m >= hi || m < lo) {
      const int64_t b = m / hw;
      lo = b * hw;
      hi = lo + hw;
      sc = *reinterpret_cast<const float4*>(dys + b * C + c);
      ad = *reinterpret_cast<const float4*>(dya + b * C + c);
    }
    return make_float4(fmaf(g.x, sc.x, ad.x), fmaf(g.y, sc.y, ad.y), fmaf(g.z, sc.z, ad.z),
                       fmaf(g.w, sc.w, ad.w));
  }
};

template <bool RES, bool TR>
__global__ __launch_bounds__(kRedThreads) void bn_bwd_part_kernel(
    const float* __restrict__ dy, int lddy, int dyc0, const float* __restrict__ x, int ldx,
    const float* __restrict__ res, int ldr, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int act, float slope, int64_t rows_per_blk,
    float* __restrict__ part, const float* __restrict__ dys, const float* __restrict__ dya,
    int64_t hw) {
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
      DyImgCache ic;
      auto acc = [&](int64_t m, float4 v, float4 g, float4 r) {
        if (TR) g = ic.apply(g, dys, dya, m, hw, C, c);
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
      };
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      int64_t m = m0 + r0;
      // kBnBatch / 2 rows (x, dy and the residual) in flight, accumulated in order
      constexpr int NB = kBnBatch / 2;
      for (; m + (NB - 1) * rows_pass < m1; m += NB * rows_pass) {
        float4 v[NB], g[NB], r[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int64_t mu_ = m + u * rows_pass;
          v[u] = *reinterpret_cast<const float4*>(x + mu_ * ldx + c);
          g[u] = *reinterpret_cast<const float4*>(dy + mu_ * lddy + dyc0 + c);
          r[u] = RES ? *reinterpret_cast<const float4*>(res + mu_ * ldr + c) : z4;
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) acc(m + u * rows_pass, v[u], g[u], r[u]);
      }
      for (; m < m1; m += rows_pass)
        acc(m, *reinterpret_cast<const float4*>(x + m * ldx + c),
            *reinterpret_cast<const float4*>(dy + m * lddy + dyc0 + c),
            RES ? *reinterpret_cast<const float4*>(res + m * ldr + c) : z4);
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

template <typename T>
__global__ __launch_bounds__(kFinThreads) void bn_bwd_final_kernel(
    const T* __restrict__ part, int64_t nblk, int C, float* __restrict__ dbeta,
    float* __restrict__ dgamma) {
  double S, Q;
  bn_final_sums(part, nblk, C, S, Q);
  const int c = blockIdx.x * kFinLanes + threadIdx.x;
  if (threadIdx.x >= kFinLanes || c >= C) return;
  dbeta[c] = (float)S;
  dgamma[c] = (float)Q;
}

// dx = gamma*invstd*(dz - sum(dz)/M - xhat*sum(dz*xhat)/M); dres = dz
template <bool RES, bool TR>
__global__ __launch_bounds__(kRedThreads) void bn_bwd_apply_kernel(
    const float* __restrict__ dy, int lddy, int dyc0, const float* __restrict__ x, int ldx,
    const float* __restrict__ res, int ldr, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int act, float slope, const float* __restrict__ sdz,
    const float* __restrict__ sdzx, float* __restrict__ dx, float* __restrict__ dres, int lanes,
    const float* __restrict__ dys, const float* __restrict__ dya, int64_t hw) {
  const EwMap e = ew_map(lanes, C >> 2);
  if (!e.ok) return;
  const int c = e.cg * 4;
  const float invM = 1.f / (float)M;
  float mu[4], is[4], gm[4], bt[4], a1[4], a2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mu[j] = mean[c + j];
    is[j] = invstd[c + j];
    gm[j] = gamma[c + j];
    bt[j] = beta[c + j];
    a1[j] = sdz[c + j] * invM;
    a2[j] = sdzx[c + j] * invM;
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  DyImgCache ic;
  auto one = [&](int64_t m, float4 v, float4 g, float4 r) {
    if (TR) g = ic.apply(g, dys, dya, m, hw, C, c);
    const float vv[4] = {v.x, v.y, v.z, v.w}, gg[4] = {g.x, g.y, g.z, g.w},
                rr[4] = {r.x, r.y, r.z, r.w};
    float o[4], dzo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (vv[j] - mu[j]) * is[j];
      const float dz = gg[j] * act_d(xh * gm[j] + bt[j] + rr[j], act, slope);
      dzo[j] = dz;
      o[j] = gm[j] * is[j] * (dz - a1[j] - xh * a2[j]);
    }
    *reinterpret_cast<float4*>(dx + m * (int64_t)C + c) = make_float4(o[0], o[1], o[2], o[3]);
    if (dres)
      *reinterpret_cast<float4*>(dres + m * (int64_t)C + c) =
          make_float4(dzo[0], dzo[1], dzo[2], dzo[3]);
  };
  // half-blocks of rows with every load in flight before the math
  constexpr int NH = kEwIters / 2;
  for (int h = 0; h < 2; ++h) {
    const int64_t mb = e.m0 + (int64_t)h * NH * e.rows_pass;
    if (mb + (int64_t)(NH - 1) * e.rows_pass < M) {
      float4 v[NH], g[NH], r[NH];
#pragma unroll
      for (int k = 0; k < NH; ++k) {
        const int64_t m = mb + (int64_t)k * e.rows_pass;
        v[k] = *reinterpret_cast<const float4*>(x + m * ldx + c);
        g[k] = *reinterpret_cast<const float4*>(dy + m * lddy + dyc0 + c);
        r[k] = RES ? *reinterpret_cast<const float4*>(res + m * ldr + c) : z4;
      }
#pragma unroll
      for (int k = 0; k < NH; ++k) one(mb + (int64_t)k * e.rows_pass, v[k], g[k], r[k]);
      continue;
    }
    for (int k = 0; k < NH; ++k) {
      const int64_t m = mb + (int64_t)k * e.rows_pass;
      if (m >= M) break;
      one(m, *reinterpret_cast<const float4*>(x + m * ldx + c),
          *reinterpret_cast<const float4*>(dy + m * lddy + dyc0 + c),
          RES ? *reinterpret_cast<const float4*>(res + m * ldr + c) : z4);
    }
  }
}

static dim3 ew_grid(int64_t M, int C, int& lanes) {
  const int C4 = C / 4;
  lanes = C4 < 64 ? C4 : 64;
  const int rows_pass = kRedThreads / lanes;
  return dim3((unsigned)cdiv(M, (int64_t)rows_pass * kEwIters), (unsigned)cdiv(C4, lanes), 1);
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

// Vector wgrad (NHWC x with Cin % 4 == 0, contiguous dY with Cout % 4 == 0):
// tile KT (im2col k) x NT (out channels) over a chunk of pixels.  X and dY
// stage through LDS in their natural [pixel][channel] layout with float4
// global loads and float4 LDS stores (no transposition); the MFMA reduction
// index runs over pixels, lane (i, g) feeding pixel 16S + g + 4e of step e, so
// the operand reads are conflict-free ds_read_b32 (row pitch = 16 mod 32
// dwords).  Tiles smaller than 4 MFMA blocks split the pixels across waves
// and combine in LDS in a fixed order.  Global loads of stage s+1 are issued
// before the MFMAs of stage s (register prefetch).
constexpr int kWvP = 64;  // pixels per stage

template <int KT>
struct WvPitch {
  static constexpr int v = (KT % 32 == 16) ? KT : KT + 16;
};

// host-built divisors of the im2col decode (OH*OW, OW, Cin, KW)
struct WgDivs {
  FastDiv ohw, ow, cin, kw;
};

template <int KT, int NT>
__global__ __launch_bounds__(256) void conv_wgrad_v_kernel(const ConvArgs p, int px_per_wg,
                                                           int fast1x1, float* __restrict__ part,
                                                           const WgDivs dv) {
  constexpr int LDA = WvPitch<KT>::v, LDN = WvPitch<NT>::v;
  constexpr int QA = KT / 16, QD = NT / 16;  // float4 loads per thread per stage
  constexpr int NBK = KT / 16, NBN = NT / 16, NB = NBK * NBN;
  constexpr int BPW = NB >= 4 ? NB / 4 : 1;  // MFMA blocks per wave
  constexpr int WPB = NB >= 4 ? 1 : 4 / NB;  // waves sharing a block (pixel split)
  __shared__ float Xs[kWvP * LDA];
  __shared__ float Ds[kWvP * LDN];
  const int K = p.KH * p.KW * p.Cin;
  const int k0 = blockIdx.x * KT, n0 = blockIdx.y * NT;
  const int chunk = blockIdx.z;
  const int mbeg = chunk * px_per_wg;
  const int mend = min(mbeg + px_per_wg, (int)p.M);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int OHW = p.OH * p.OW;

  float4 ra[QA], rd[QD];
  auto load_stage = [&](int px0) {
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int idx = q * 256 + t;
      const int px = idx / (KT / 4), c4 = (idx % (KT / 4)) * 4;
      const int m = px0 + px;
      const int k = k0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < mend && k < K) {
        if (fast1x1) {
          v = *reinterpret_cast<const float4*>(p.x + (int64_t)m * p.x_ps + p.x_c0 + k);
          if (p.ascale) {
            const int b = fdiv(m, dv.ohw);
            const float4 s4 = *reinterpret_cast<const float4*>(p.ascale + (int64_t)b * p.ascale_bs + k);
            v.x *= s4.x; v.y *= s4.y; v.z *= s4.z; v.w *= s4.w;
          }
        } else {
          const int b = fdiv(m, dv.ohw), rr = m - b * OHW;
          const int oh = fdiv(rr, dv.ow), ow = rr - oh * p.OW;
          const int tap = fdiv(k, dv.cin), ci = k - tap * p.Cin;
          const int kh = fdiv(tap, dv.kw), kw = tap - kh * p.KW;
          const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
          if (ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) {
            v = *reinterpret_cast<const float4*>(p.x + (int64_t)b * p.x_bs +
                                                 ((int64_t)ih * p.W + iw) * p.x_ps + p.x_c0 + ci);
            if (p.ascale) {
              const float4 s4 =
                  *reinterpret_cast<const float4*>(p.ascale + (int64_t)b * p.ascale_bs + ci);
              v.x *= s4.x; v.y *= s4.y; v.z *= s4.z; v.w *= s4.w;
            }
          }
        }
      }
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      const int idx = q * 256 + t;
      const int px = idx / (NT / 4), c4 = (idx % (NT / 4)) * 4;
      const int m = px0 + px;
      const int n = n0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < mend && n < p.Cout)
        v = *reinterpret_cast<const float4*>(p.y + (int64_t)m * p.y_ps + p.y_c0 + n);
      rd[q] = v;
    }
  };

  f32x4 acc[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // this wave's blocks: NB >= 4 -> blocks wave*BPW + j; else block wave % NB
  const int sub = NB >= 4 ? 0 : wave / NB;  // pixel-group residue (NB < 4)

  load_stage(mbeg);
  for (int px0 = mbeg; px0 < mend; px0 += kWvP) {
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int idx = q * 256 + t;
      const int px = idx / (KT / 4), c4 = (idx % (KT / 4)) * 4;
      *reinterpret_cast<float4*>(Xs + px * LDA + c4) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      const int idx = q * 256 + t;
      const int px = idx / (NT / 4), c4 = (idx % (NT / 4)) * 4;
      *reinterpret_cast<float4*>(Ds + px * LDN + c4) = rd[q];
    }
    __syncthreads();
    if (px0 + kWvP < mend) load_stage(px0 + kWvP);
#pragma unroll
    for (int S = 0; S < kWvP / 16; ++S) {
      if (NB < 4 && (S % WPB) != sub) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * S + g + 4 * e;
#pragma unroll
        for (int j = 0; j < BPW; ++j) {
          const int blk = NB >= 4 ? wave * BPW + j : wave % NB;
          const int bk = blk / NBN, bn = blk % NBN;
          const float a = Xs[row * LDA + 16 * bk + i];
          const float b = Ds[row * LDN + 16 * bn + i];
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  if (NB < 4) {  // combine the WPB waves of each block (fixed order), via LDS
    f32x4* red = reinterpret_cast<f32x4*>(Xs);  // 4 waves x 64 lanes x f32x4 = 4 KB
    red[wave * 64 + lane] = acc[0];
    __syncthreads();
    if (wave >= NB) return;
    f32x4 s4 = red[wave * 64 + lane];
    for (int w2 = 1; w2 < WPB; ++w2) {
      const f32x4 o = red[(wave + w2 * NB) * 64 + lane];
      s4[0] += o[0]; s4[1] += o[1]; s4[2] += o[2]; s4[3] += o[3];
    }
    acc[0] = s4;
  }
  float* pc = part + (int64_t)chunk * K * p.Cout;
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int blk = NB >= 4 ? wave * BPW + j : wave % NB;
    const int bk = blk / NBN, bn = blk % NBN;
    const int n = n0 + 16 * bn + i;
    if (n >= p.Cout) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 16 * bk + 4 * g + r;
      if (k < K) pc[(int64_t)k * p.Cout + n] = acc[j][r];
    }
  }
}

// dW[n][ci][tap] = sum over chunks of part[chunk][k = tap*Cin + ci][n]:
// workgroup = `lanes` consecutive outputs x (256/lanes) chunk stripes, fixed
// order combine (deterministic).
__global__ __launch_bounds__(256) void wgrad_reduce2_kernel(const float* __restrict__ part,
                                                            int64_t nchunk, int K, int Cout,
                                                            int Cin, int KHW, int lanes,
                                                            float* __restrict__ dw) {
  __shared__ float red[256];
  const int t = threadIdx.x;
  const int rows = 256 / lanes, r = t / lanes;
  const int64_t KN = (int64_t)K * Cout;
  const int64_t o = (int64_t)blockIdx.x * lanes + t % lanes;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (r < rows && o < KN) {
    int64_t c = r;
    // two iterations' loads in flight (same accumulation order; 10.2 -> 8.4
    // us per call over C4's 71 calls per step)
#pragma unroll 2
    for (; c + 3 * rows < nchunk; c += 4 * rows) {
      s0 += part[c * KN + o];
      s1 += part[(c + rows) * KN + o];
      s2 += part[(c + 2 * rows) * KN + o];
      s3 += part[(c + 3 * rows) * KN + o];
    }
    for (; c < nchunk; c += rows) s0 += part[c * KN + o];
  }
  red[t] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (t >= lanes || o >= KN) return;
  float s = 0.f;
  for (int k = 0; k < rows; ++k) s += red[k * lanes + t];
  const int k = (int)(o / Cout), n = (int)(o - (int64_t)k * Cout);
  const int tap = k / Cin, ci = k - tap * Cin;
  dw[((int64_t)n * Cin + ci) * KHW + tap] = s;
}

// Weight gradient of a conv over the NCHW network input with a small im2col
// depth (the MobileNetV3 stem, 3x3/s2, 3 -> 16: K = 27, Cout = 16), where the
// tiled kernels above would run 64x64 tiles at ~10% occupancy of the MFMA
// block and gather x element by element.  Each wave takes segments of 64
// consecutive output pixels of one output row: it stages the segment's input
// window (Cin x KH rows x (63*stride + KW) columns, zero-padded) into its own
// LDS slice with coalesced row loads, then runs 16 steps of two 16x16x4 MFMAs
// (A = im2col rows k = 16t + i, B = dY[pixel][co], 4 pixels per step) — the
// reduction index is the pixel.  Per-wave partials [wave][K][Cout] are summed
// by wgrad_reduce2_kernel in a fixed order.
constexpr int kSwPx = 64;

static bool stem_wgrad_ok(const ConvArgs& a) {
  return a.nchw_in && !a.ascale && a.KH * a.KW * a.Cin <= 32 && a.Cout <= 16 && a.stride <= 2 &&
         a.KW <= 7 && a.Cin * a.KH * ((kSwPx - 1) * a.stride + a.KW) <= 1536;
}

static int64_t stem_wgrad_waves(const ConvArgs& a) {
  const int64_t ntask = (int64_t)a.B * a.OH * cdiv(a.OW, kSwPx);
  return 4 * std::min<int64_t>(2048, cdiv(ntask, 4 * 8));
}

__global__ __launch_bounds__(256) void stem_wgrad_kernel(const ConvArgs p, int64_t ntask,
                                                         float* __restrict__ part) {
  extern __shared__ float sw_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int WC = (kSwPx - 1) * p.stride + p.KW;
  const int WS = p.Cin * p.KH * WC;
  float* win = sw_lds + wave * WS;
  const int K = p.Cin * p.KH * p.KW;
  int aoff[2];
  bool aval[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kk = 16 * t + i;  // k = tap * Cin + ci, tap = kh * KW + kw
    aval[t] = kk < K;
    const int tap = kk / p.Cin, ci = kk - tap * p.Cin;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
    aoff[t] = aval[t] ? (ci * p.KH + kh) * WC + kw : 0;
  }
  f32x4 acc0 = (f32x4){0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const int nseg = (p.OW + kSwPx - 1) / kSwPx;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave, nw = (int64_t)gridDim.x * 4;
  for (int64_t task = gw; task < ntask; task += nw) {
    const int seg = (int)(task % nseg);
    const int64_t row = task / nseg;
    const int oy = (int)(row % p.OH);
    const int b = (int)(row / p.OH);
    const int ox0 = seg * kSwPx;
    const int iy0 = oy * p.stride - p.pad, ix0 = ox0 * p.stride - p.pad;
    const float* xb = p.x + (int64_t)b * p.x_bs;
    for (int e = lane; e < WS; e += 64) {
      const int r = e / WC, col = e - r * WC;
      const int ci = r / p.KH, kh = r - ci * p.KH;
      const int iy = iy0 + kh, ix = ix0 + col;
      float v = 0.f;
      if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
        v = xb[((int64_t)ci * p.H + iy) * p.W + ix];
      win[e] = v;
    }
    // the window is wave-private: LDS writes -> reads need only this wave
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const float* dyr = p.y + (int64_t)b * p.y_bs + ((int64_t)oy * p.OW) * p.y_ps + p.y_c0 + i;
#pragma unroll 4
    for (int q = 0; q < kSwPx / 4; ++q) {
      const int px = 4 * q + g, ox = ox0 + px;
      const bool v = ox < p.OW;
      const float d = (v && i < p.Cout) ? dyr[(int64_t)ox * p.y_ps] : 0.f;
      const float a0 = aval[0] && v ? win[aoff[0] + px * p.stride] : 0.f;
      const float a1 = aval[1] && v ? win[aoff[1] + px * p.stride] : 0.f;
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, d, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, d, acc1, 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // every lane's reads done before the next staging
  }
  // acc_t[r] = dW[k = 16t + 4g + r][n = i]
  float* pc = part + gw * K * p.Cout;
  if (i < p.Cout) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k0 = 4 * g + r, k1 = 16 + 4 * g + r;
      if (k0 < K) pc[(int64_t)k0 * p.Cout + i] = acc0[r];
      if (k1 < K) pc[(int64_t)k1 * p.Cout + i] = acc1[r];
    }
  }
}

static int wv_tile(int64_t n) { return n <= 16 ? 16 : (n <= 32 ? 32 : 64); }

// ---------------------------------------------------------------------------
// Weight gradient on the 32x32x2 fp32 MFMA: dW[k][n] = sum_m A[m][k] dY[m][n]
// (A = im2col(x) on the fly, k = tap * Cin + ci).  Workgroup tile KT x NT
// (4 waves as 2 x 2, wave tile KT/2 x NT/2 of 32x32 blocks) over a chunk of
// pixels; each stage stages kWg32Px pixels of A and dY in LDS in their
// natural [pixel][channel] layout (float4 global loads and LDS stores); the
// MFMA contracts the 2 pixels of a lane half (lane l: pixel 2pp + (l >> 5),
// row/col l & 31), so every operand read is a conflict-free ds_read_b32 of 32
// consecutive floats.  2x the FLOPs per LDS operand of the 16x16x4 kernel.
// Global loads of stage s+1 are in registers while stage s computes.
// ---------------------------------------------------------------------------
constexpr int kWg32Px = 32;  // pixels per stage


template <int KT, int NT, bool DB>
__global__ __launch_bounds__(256, 2) void conv_wgrad32_kernel(const ConvArgs p, int px_per_wg,
                                                              int fast1x1,
                                                              float* __restrict__ part,
                                                              const WgDivs dv) {
  constexpr int TK = KT / 64, TNn = NT / 64;          // 32x32 blocks per wave (k, n)
  constexpr int QA = kWg32Px * KT / 4 / 256, QD = kWg32Px * NT / 4 / 256;
  // DB: two LDS stage buffers — stage s+1 is stored while no wave can still
  // be reading its buffer (read in stage s-1, before the last barrier): one
  // barrier per stage instead of two
  __shared__ float XsA[(DB ? 2 : 1) * kWg32Px * KT];
  __shared__ float DsA[(DB ? 2 : 1) * kWg32Px * NT];
  const int K = p.KH * p.KW * p.Cin;
  const int k0 = blockIdx.x * KT, n0 = blockIdx.y * NT;
  const int chunk = blockIdx.z;
  const int mbeg = chunk * px_per_wg;
  const int mend = min(mbeg + px_per_wg, (int)p.M);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int wk = (wave >> 1) * (KT / 2), wn = (wave & 1) * (NT / 2);
  const int OHW = p.OH * p.OW;

  float4 ra[QA], rd[QD];
  // the A elements' im2col k decomposition is fixed for the launch (this
  // thread's channel column does not move between stages): decoded once here,
  // not per stage (a runtime-divisor division inside the stage loop's guarded
  // block cannot be hoisted by the compiler)
  int a_ci[QA], a_kh[QA], a_kw[QA];
#pragma unroll
  for (int q = 0; q < QA; ++q) {
    const int k = k0 + ((q * 256 + t) % (KT / 4)) * 4;
    a_ci[q] = k;
    a_kh[q] = a_kw[q] = 0;
    if (!fast1x1 && k < K) {
      const int tap = fdiv(k, dv.cin);
      a_ci[q] = k - tap * p.Cin;
      a_kh[q] = fdiv(tap, dv.kw);
      a_kw[q] = tap - a_kh[q] * p.KW;
    }
  }
  auto load_stage = [&](int px0) {
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int idx = q * 256 + t;
      const int px = idx / (KT / 4), c4 = (idx % (KT / 4)) * 4;
      const int m = px0 + px, k = k0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < mend && k < K) {
        int b = 0;
        const int ci = a_ci[q];
        int64_t off;
        bool ok = true;
        if (fast1x1) {
          off = (int64_t)m * p.x_ps + p.x_c0 + k;
          if (p.ascale) b = fdiv(m, dv.ohw);
        } else {
          b = fdiv(m, dv.ohw);
          const int rr = m - b * OHW;
          const int oh = fdiv(rr, dv.ow), ow = rr - oh * p.OW;
          const int kh = a_kh[q], kw = a_kw[q];
          const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
          ok = ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
          off = (int64_t)b * p.x_bs + ((int64_t)ih * p.W + iw) * p.x_ps + p.x_c0 + ci;
        }
        if (ok) {
          v = *reinterpret_cast<const float4*>(p.x + off);
          if (p.ascale) {
            const float4 s4 =
                *reinterpret_cast<const float4*>(p.ascale + (int64_t)b * p.ascale_bs + ci);
            v.x *= s4.x; v.y *= s4.y; v.z *= s4.z; v.w *= s4.w;
          }
        }
      }
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      const int idx = q * 256 + t;
      const int px = idx / (NT / 4), c4 = (idx % (NT / 4)) * 4;
      const int m = px0 + px, n = n0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < mend && n < p.Cout)
        v = *reinterpret_cast<const float4*>(p.y + (int64_t)m * p.y_ps + p.y_c0 + n);
      rd[q] = v;
    }
  };

  f32x16 acc[TK][TNn];
#pragma unroll
  for (int u = 0; u < TK; ++u)
#pragma unroll
    for (int v = 0; v < TNn; ++v)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][v][r] = 0.f;

  if constexpr (DB) {
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int q = 0; q < QA; ++q)
      reinterpret_cast<float4*>(XsA + buf * kWg32Px * KT)[q * 256 + t] = ra[q];
#pragma unroll
    for (int q = 0; q < QD; ++q)
      reinterpret_cast<float4*>(DsA + buf * kWg32Px * NT)[q * 256 + t] = rd[q];
  };
  load_stage(mbeg);
  store_stage(0);
  __syncthreads();
  int cb = 0;
  for (int px0 = mbeg; px0 < mend; px0 += kWg32Px, cb ^= 1) {
    const bool more = px0 + kWg32Px < mend;
    if (more) load_stage(px0 + kWg32Px);
    const float* Xs = XsA + cb * kWg32Px * KT;
    const float* Ds = DsA + cb * kWg32Px * NT;
#pragma unroll 4
    for (int pp = 0; pp < kWg32Px / 2; ++pp) {
      const int row = 2 * pp + h;
      float a[TK], b[TNn];
#pragma unroll
      for (int u = 0; u < TK; ++u) a[u] = Xs[row * KT + wk + 32 * u + j];
#pragma unroll
      for (int v = 0; v < TNn; ++v) b[v] = Ds[row * NT + wn + 32 * v + j];
#pragma unroll
      for (int u = 0; u < TK; ++u)
#pragma unroll
        for (int v = 0; v < TNn; ++v)
          acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[v], acc[u][v], 0, 0, 0);
    }
    if (more) store_stage(cb ^ 1);
    __syncthreads();
  }
  } else {
  float* Xs = XsA;
  float* Ds = DsA;
  load_stage(mbeg);
  for (int px0 = mbeg; px0 < mend; px0 += kWg32Px) {
#pragma unroll
    for (int q = 0; q < QA; ++q)
      reinterpret_cast<float4*>(Xs)[q * 256 + t] = ra[q];
#pragma unroll
    for (int q = 0; q < QD; ++q)
      reinterpret_cast<float4*>(Ds)[q * 256 + t] = rd[q];
    __syncthreads();
    if (px0 + kWg32Px < mend) load_stage(px0 + kWg32Px);
#pragma unroll 4
    for (int pp = 0; pp < kWg32Px / 2; ++pp) {
      const int row = 2 * pp + h;
      float a[TK], b[TNn];
#pragma unroll
      for (int u = 0; u < TK; ++u) a[u] = Xs[row * KT + wk + 32 * u + j];
#pragma unroll
      for (int v = 0; v < TNn; ++v) b[v] = Ds[row * NT + wn + 32 * v + j];
#pragma unroll
      for (int u = 0; u < TK; ++u)
#pragma unroll
        for (int v = 0; v < TNn; ++v)
          acc[u][v] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[v], acc[u][v], 0, 0, 0);
    }
    __syncthreads();
  }
  }
  // acc[u][v][r]: k = k0 + wk + 32u + 8(r>>2) + 4h + (r&3), n = n0 + wn + 32v + j
  float* pc = part + (int64_t)chunk * K * p.Cout;
#pragma unroll
  for (int u = 0; u < TK; ++u)
#pragma unroll
    for (int v = 0; v < TNn; ++v) {
      const int n = n0 + wn + 32 * v + j;
      if (n >= p.Cout) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = k0 + wk + 32 * u + 8 * (r >> 2) + 4 * h + (r & 3);
        if (k < K) pc[(int64_t)k * p.Cout + n] = acc[u][v][r];
      }
    }
}

// The 32x32 wgrad kernel takes NHWC/vector shapes with K, Cout >= 64;
// JABD_WGRAD32=0 forces the 16x16x4 kernels (A/B).
static bool wgrad32_ok(const ConvArgs& a) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JABD_WGRAD32");
    v = e && e[0] == '0' ? 0 : 1;
  }
  const int64_t K = (int64_t)a.KH * a.KW * a.Cin;
  return v == 1 && K >= 64 && a.Cout >= 64;
}
// 128-wide tiles unless they pad more than 1/8 beyond what 64-wide ones do
static int wg32_tile(int64_t n) { return cdiv(n, 128) * 128 - n <= n / 8 ? 128 : 64; }


static bool wgrad_vec_ok(const ConvArgs& a) {
  return !a.nchw_in && a.Cin % 4 == 0 && a.x_ps % 4 == 0 && a.x_c0 % 4 == 0 && a.Cout % 4 == 0 &&
         a.y_ps % 4 == 0 && a.y_c0 % 4 == 0 && a.y_bs == (int64_t)a.OH * a.OW * a.y_ps &&
         a.x_bs == (int64_t)a.H * a.W * a.x_ps && (!a.ascale || a.ascale_bs % 4 == 0);
}

static int64_t wgrad_chunks(const ConvArgs& a) {
  const int64_t K = (int64_t)a.KH * a.KW * a.Cin;
  const bool vec = wgrad_vec_ok(a);
  const bool w32 = vec && wgrad32_ok(a);
  const int64_t tk = w32 ? wg32_tile(K) : (vec ? wv_tile(K) : kWgT);
  const int64_t tn = w32 ? wg32_tile(a.Cout) : (vec ? wv_tile(a.Cout) : kWgT);
  const int64_t tiles = cdiv(K, tk) * cdiv(a.Cout, tn);
  int64_t nchunk = cdiv(2048, tiles);
  const int64_t maxchunk = cdiv(a.M, kWgPx);
  if (nchunk > maxchunk) nchunk = maxchunk;
  // keep the partial buffer <= 64M floats
  const int64_t cap = ((int64_t)64 << 20) / (K * a.Cout);
  if (nchunk > cap) nchunk = cap;
  return nchunk < 1 ? 1 : nchunk;
}

// ---------------------------------------------------------------------------
// Depthwise gradients: dgrad is a gather (no atomics), wgrad per-block
// partials reduced in a fixed order.  Register-strip kernels (3x3/5x5, stride 1/2, pad k/2).  A
// thread owns one float4 channel group of a strip of PW consecutive pixels
// of one row; workgroup = `lanes` channel groups x (256/lanes) strips.  Row
// segments are loaded once per kernel row and reused across the k taps in
// registers; no per-element index division.
__device__ __forceinline__ void fma4(float4& a, const float4 x, const float4 y) {
  a = fma4pk(x, y, a);
}

__host__ __device__ constexpr int floordiv_c(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// dx strip iw0..iw0+PW-1 of input row ih: dx = sum_{kh,kw} dy[(ih+pad-kh)/S][(iw+pad-kw)/S] w[kh][kw]
template <int K, int S, int PW>
__global__ __launch_bounds__(256) void dw_dgrad_strip_kernel(
    const float* __restrict__ dy, const float* __restrict__ w, int H, int W, int C, int OH, int OW,
    int nstrip, int64_t items, int lanes, float* __restrict__ dx) {
  constexpr int PAD = K / 2;
  constexpr int OFF = floordiv_c(PAD - K + 1, S);   // ow0 = iw0/S + OFF
  constexpr int L = (PW - 1 + PAD - S * OFF) / S + 1;
  const int C4 = C >> 2;
  const int t = threadIdx.x;
  const int rows_pass = 256 / lanes;
  if (t / lanes >= rows_pass) return;
  const int cg = blockIdx.y * lanes + t % lanes;
  if (cg >= C4) return;
  const int64_t it = (int64_t)blockIdx.x * rows_pass + t / lanes;
  if (it >= items) return;
  const int row = (int)(it / nstrip), strip = (int)(it - (int64_t)row * nstrip);
  const int b = row / H, ih = row - b * H;
  const int iw0 = strip * PW;
  const int ow0 = iw0 / S + OFF;
  float4 acc[PW];
#pragma unroll
  for (int q = 0; q < PW; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
    const int nh = ih + PAD - kh;
    if (nh < 0 || (S == 2 && (nh & 1))) continue;
    const int oh = nh / S;
    if (oh >= OH) continue;
    const float4* drow = reinterpret_cast<const float4*>(dy + (((int64_t)b * OH + oh) * OW) * C) + cg;
    float4 seg[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int ow = ow0 + j;
      seg[j] = (ow >= 0 && ow < OW) ? drow[(int64_t)ow * C4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 wk[K];
#pragma unroll
    for (int kw = 0; kw < K; ++kw) wk[kw] = reinterpret_cast<const float4*>(w + (kh * K + kw) * C)[cg];
#pragma unroll
    for (int q = 0; q < PW; ++q)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        if (((q + PAD - kw) % S + S) % S) continue;  // parity (iw0 % S == 0)
        const int j = (q + PAD - kw - S * OFF) / S;
        fma4(acc[q], seg[j], wk[kw]);
      }
  }
  float4* xrow = reinterpret_cast<float4*>(dx + (((int64_t)b * H + ih) * W) * C) + cg;
#pragma unroll
  for (int q = 0; q < PW; ++q)
    if (iw0 + q < W) xrow[(int64_t)(iw0 + q) * C4] = acc[q];
}

// Depthwise data gradient with the following BatchNorm's backward partials
// fused in (MNv3 Block_eca: e = act(bn1(e_pre)) feeds the depthwise conv, so
// its data gradient de is bn1's output gradient).  Each thread computes the
// de strip as dw_dgrad_strip_kernel does (same tap order: bit-identical de),
// stores it, loads e_pre at the same pixels and accumulates dz = de *
// act'(xhat * gamma + beta), sum dz and sum dz * xhat (as bn_bwd_part_kernel);
// a workgroup walks `spb` strip rows and writes part[blockIdx.x][0|1][c] for
// its channels, rows added in a fixed order (deterministic).  Saves
// bn_bwd_part's pass over de and e_pre (the block's largest tensors).
// MODE 0: store de to dx + partials; 1: partials only (de not stored);
// 2: the apply pass with de recomputed: dx = gamma * invstd * (dz - sdz / M -
// xhat * sdzx / M) (bn_bwd_apply_kernel's expression) stored, no partials.
// 1 + 2 replace 0 + bn_bwd_apply: de is never written nor read back, at the
// price of a second read of dy (a quarter of de's size at stride 2).
template <int K, int S, int PW, int MODE = 0>
__global__ __launch_bounds__(256) void dw_dgrad_bn_kernel(
    const float* __restrict__ dy, const float* __restrict__ w, int H, int W, int C, int OH, int OW,
    int nstrip, int64_t items, int lanes, int spb, float* __restrict__ dx,
    const float* __restrict__ xb, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int act, float slope,
    float* __restrict__ part, const float* __restrict__ sdz = nullptr,
    const float* __restrict__ sdzx = nullptr, int64_t M = 1) {
  constexpr int PAD = K / 2;
  constexpr int OFF = floordiv_c(PAD - K + 1, S);
  constexpr int L = (PW - 1 + PAD - S * OFF) / S + 1;
  __shared__ float4 rs[256], rq[256];
  const int C4 = C >> 2;
  const int t = threadIdx.x;
  const int rows_pass = 256 / lanes;
  const int r0 = t / lanes;
  const int cg = blockIdx.y * lanes + t % lanes;
  const bool tv = r0 < rows_pass && cg < C4;
  float4 sS = make_float4(0.f, 0.f, 0.f, 0.f), sQ = sS;
  if (tv) {
    const int c = cg * 4;
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
    const float4 bt = *reinterpret_cast<const float4*>(beta + c);
    float a1[4] = {}, a2[4] = {};
    if (MODE == 2) {
      const float invM = 1.f / (float)M;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a1[e] = sdz[c + e] * invM;
        a2[e] = sdzx[c + e] * invM;
      }
    }
    // groups band-major (image, band of rows_pass strips, row): a workgroup
    // walks spb consecutive rows of one band, so the dy rows a row shares
    // with its neighbours are re-read from this CU's L2 instead of by
    // workgroups on other XCDs (PMC: 1.70x the algorithmic bytes row-major)
    const int nbands = (nstrip + rows_pass - 1) / rows_pass;
    for (int sp = 0; sp < spb; ++sp) {
      const int64_t grp = (int64_t)blockIdx.x * spb + sp;
      if (grp >= items) break;
      const int64_t bb = grp / H;
      const int ih = (int)(grp - bb * H);
      const int b = (int)(bb / nbands), band = (int)(bb - (int64_t)b * nbands);
      const int strip = band * rows_pass + r0;
      if (strip >= nstrip) continue;
      const int iw0 = strip * PW;
      const int ow0 = iw0 / S + OFF;
      float4 acc[PW];
#pragma unroll
      for (int q = 0; q < PW; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        const int nh = ih + PAD - kh;
        if (nh < 0 || (S == 2 && (nh & 1))) continue;
        const int oh = nh / S;
        if (oh >= OH) continue;
        const float4* drow =
            reinterpret_cast<const float4*>(dy + (((int64_t)b * OH + oh) * OW) * C) + cg;
        float4 seg[L];
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const int ow = ow0 + j;
          seg[j] = (ow >= 0 && ow < OW) ? drow[(int64_t)ow * C4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float4 wk[K];
#pragma unroll
        for (int kw = 0; kw < K; ++kw) wk[kw] = reinterpret_cast<const float4*>(w + (kh * K + kw) * C)[cg];
#pragma unroll
        for (int q = 0; q < PW; ++q)
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            if (((q + PAD - kw) % S + S) % S) continue;
            const int j = (q + PAD - kw - S * OFF) / S;
            fma4(acc[q], seg[j], wk[kw]);
          }
      }
      const int64_t rb = (((int64_t)b * H + ih) * W) * C4 + cg;
      float4* xrow = reinterpret_cast<float4*>(dx) + rb;
      const float4* brow = reinterpret_cast<const float4*>(xb) + rb;
#pragma unroll
      for (int q = 0; q < PW; ++q) {
        if (iw0 + q >= W) break;
        if (MODE == 0) xrow[(int64_t)(iw0 + q) * C4] = acc[q];
        const float4 xv = brow[(int64_t)(iw0 + q) * C4];
        const float xh[4] = {(xv.x - mu.x) * is.x, (xv.y - mu.y) * is.y, (xv.z - mu.z) * is.z,
                             (xv.w - mu.w) * is.w};
        const float gg[4] = {acc[q].x, acc[q].y, acc[q].z, acc[q].w};
        const float gmm[4] = {gm.x, gm.y, gm.z, gm.w}, btt[4] = {bt.x, bt.y, bt.z, bt.w};
        const float iss[4] = {is.x, is.y, is.z, is.w};
        float dz[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) dz[e] = gg[e] * act_d(fmaf(xh[e], gmm[e], btt[e]), act, slope);
        if (MODE == 2) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = gmm[e] * iss[e] * (dz[e] - a1[e] - xh[e] * a2[e]);
          xrow[(int64_t)(iw0 + q) * C4] = make_float4(o[0], o[1], o[2], o[3]);
          continue;
        }
        sS.x += dz[0]; sS.y += dz[1]; sS.z += dz[2]; sS.w += dz[3];
        sQ.x = fmaf(dz[0], xh[0], sQ.x); sQ.y = fmaf(dz[1], xh[1], sQ.y);
        sQ.z = fmaf(dz[2], xh[2], sQ.z); sQ.w = fmaf(dz[3], xh[3], sQ.w);
      }
    }
  }
  if (MODE == 2) return;
  rs[t] = sS;
  rq[t] = sQ;
  __syncthreads();
  if (t < lanes && cg < C4) {
    float4 S_ = make_float4(0.f, 0.f, 0.f, 0.f), Q_ = S_;
    for (int r = 0; r < rows_pass; ++r) {
      const float4 a = rs[r * lanes + t], q = rq[r * lanes + t];
      S_.x += a.x; S_.y += a.y; S_.z += a.z; S_.w += a.w;
      Q_.x += q.x; Q_.y += q.y; Q_.z += q.z; Q_.w += q.w;
    }
    reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C)[cg] = S_;
    reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C + C)[cg] = Q_;
  }
}

// dw_dgrad_bn_kernel for 3x3 as a row walker: a thread owns PW input (dx)
// columns x 4 channels and a chunk of R dx rows and keeps the dy rows it
// still needs in registers (stride 1: the three rows around the current dx
// row, rotated by unrolling; stride 2: the row an even dx row shares with the
// next odd one), so each dy row is read once per chunk instead of once per
// dx row it feeds.  The taps are accumulated in dw_dgrad_bn_kernel's order
// (kh ascending, rows outside dy skipped; kw ascending per column): dx / de
// and the partials' terms are that kernel's bit for bit.  Workgroup
// blockIdx.x = (image, band, chunk) < nwork; the remaining blocks of the
// partial-row count write zero rows.
template <int S, int PW, int MODE>
__global__ __launch_bounds__(256) void dw_dgrad_bn_rows_kernel(
    const float* __restrict__ dy, const float* __restrict__ w, int H, int W, int C, int OH, int OW,
    int nstrip, int nbands, int nchunks, int R, int nwork, int lanes, float* __restrict__ dx,
    const float* __restrict__ xb, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int act, float slope,
    float* __restrict__ part, const float* __restrict__ sdz = nullptr,
    const float* __restrict__ sdzx = nullptr, int64_t M = 1) {
  constexpr int K = 3, PAD = 1;
  constexpr int OFF = floordiv_c(PAD - K + 1, S);
  constexpr int L = (PW - 1 + PAD - S * OFF) / S + 1;
  __shared__ float4 rs[256], rq[256];
  const int C4 = C >> 2;
  const int t = threadIdx.x;
  const int rows_pass = 256 / lanes;
  const int r0 = t / lanes;
  const int cg = blockIdx.y * lanes + t % lanes;
  const int chunk = blockIdx.x % nchunks;
  const int bb = blockIdx.x / nchunks;
  const int b = bb / nbands, band = bb % nbands;
  const int strip = band * rows_pass + r0;
  const bool tv = r0 < rows_pass && cg < C4 && (int)blockIdx.x < nwork && strip < nstrip;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sS = z, sQ = z;
  if (tv) {
    const int c = cg * 4;
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
    const float4 is = *reinterpret_cast<const float4*>(invstd + c);
    const float4 gm = *reinterpret_cast<const float4*>(gamma + c);
    const float4 bt = *reinterpret_cast<const float4*>(beta + c);
    float a1[4] = {}, a2[4] = {};
    if (MODE == 2) {
      const float invM = 1.f / (float)M;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a1[e] = sdz[c + e] * invM;
        a2[e] = sdzx[c + e] * invM;
      }
    }
    float4 wk[K * K];
#pragma unroll
    for (int q = 0; q < K * K; ++q) wk[q] = reinterpret_cast<const float4*>(w + q * C)[cg];
    const int iw0 = strip * PW;
    const int ow0 = iw0 / S + OFF;
    const int ih0 = chunk * R, ih1 = min(H, ih0 + R);
    auto load_dy = [&](int oh, float4 (&seg)[L]) {
      const bool rv = oh >= 0 && oh < OH;
      const float4* drow =
          reinterpret_cast<const float4*>(dy + (((int64_t)b * OH + (rv ? oh : 0)) * OW) * C) + cg;
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int ow = ow0 + j;
        seg[j] = (rv && ow >= 0 && ow < OW) ? drow[(int64_t)ow * C4] : z;
      }
    };
    // one dx row from the dy rows of taps kh (valid ones only, kh ascending)
    auto finish = [&](int ih, float4 (&acc)[PW]) {
      const int64_t rb = (((int64_t)b * H + ih) * W) * C4 + cg;
      float4* xrow = reinterpret_cast<float4*>(dx) + rb;
      const float4* brow = reinterpret_cast<const float4*>(xb) + rb;
#pragma unroll
      for (int q = 0; q < PW; ++q) {
        if (iw0 + q >= W) break;
        if (MODE == 0) xrow[(int64_t)(iw0 + q) * C4] = acc[q];
        const float4 xv = brow[(int64_t)(iw0 + q) * C4];
        const float xh[4] = {(xv.x - mu.x) * is.x, (xv.y - mu.y) * is.y, (xv.z - mu.z) * is.z,
                             (xv.w - mu.w) * is.w};
        const float gg[4] = {acc[q].x, acc[q].y, acc[q].z, acc[q].w};
        const float gmm[4] = {gm.x, gm.y, gm.z, gm.w}, btt[4] = {bt.x, bt.y, bt.z, bt.w};
        const float iss[4] = {is.x, is.y, is.z, is.w};
        float dzv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) dzv[e] = gg[e] * act_d(fmaf(xh[e], gmm[e], btt[e]), act, slope);
        if (MODE == 2) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = gmm[e] * iss[e] * (dzv[e] - a1[e] - xh[e] * a2[e]);
          xrow[(int64_t)(iw0 + q) * C4] = make_float4(o[0], o[1], o[2], o[3]);
          continue;
        }
        sS.x += dzv[0]; sS.y += dzv[1]; sS.z += dzv[2]; sS.w += dzv[3];
        sQ.x = fmaf(dzv[0], xh[0], sQ.x); sQ.y = fmaf(dzv[1], xh[1], sQ.y);
        sQ.z = fmaf(dzv[2], xh[2], sQ.z); sQ.w = fmaf(dzv[3], xh[3], sQ.w);
      }
    };
    auto tap = [&](int kh, const float4 (&seg)[L], float4 (&acc)[PW]) {
#pragma unroll
      for (int q = 0; q < PW; ++q)
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          if (((q + PAD - kw) % S + S) % S) continue;  // parity (iw0 % S == 0)
          const int j = (q + PAD - kw - S * OFF) / S;
          fma4(acc[q], seg[j], wk[kh * K + kw]);
        }
    };
    if (ih0 < ih1) {
      if constexpr (S == 1) {
        // dx row ih: kh 0, 1, 2 read dy rows ih+1, ih, ih-1
        float4 gA[L], gB[L], gC[L];
        load_dy(ih0 - 1, gA);
        load_dy(ih0, gB);
        auto row = [&](int ih, const float4 (&gm1)[L], const float4 (&g0)[L],
                       const float4 (&gp1)[L]) {
          float4 acc[PW];
#pragma unroll
          for (int q = 0; q < PW; ++q) acc[q] = z;
          if (ih + 1 < OH) tap(0, gp1, acc);
          if (ih < OH) tap(1, g0, acc);
          if (ih >= 1 && ih - 1 < OH) tap(2, gm1, acc);
          finish(ih, acc);
        };
        for (int ih = ih0; ih < ih1; ih += 3) {
          load_dy(ih + 1, gC);
          row(ih, gA, gB, gC);
          if (ih + 1 >= ih1) break;
          load_dy(ih + 2, gA);
          row(ih + 1, gB, gC, gA);
          if (ih + 2 >= ih1) break;
          load_dy(ih + 3, gB);
          row(ih + 2, gC, gA, gB);
        }
      } else {
        // even dx row 2m: kh 1 reads dy row m; odd row 2m+1: kh 0 reads m+1,
        // kh 2 reads m
        float4 gP[L], gN[L];
        int have = -1;  // dy row held in gP
        for (int ih = ih0; ih < ih1; ++ih) {
          float4 acc[PW];
#pragma unroll
          for (int q = 0; q < PW; ++q) acc[q] = z;
          const int m = ih >> 1;
          if ((ih & 1) == 0) {
            if (have != m) load_dy(m, gP);
            have = m;
            if (m < OH) tap(1, gP, acc);
          } else {
            if (have != m) load_dy(m, gP);
            load_dy(m + 1, gN);
            if (m + 1 < OH) tap(0, gN, acc);
            if (m < OH) tap(2, gP, acc);
#pragma unroll
            for (int j = 0; j < L; ++j) gP[j] = gN[j];
            have = m + 1;
          }
          finish(ih, acc);
        }
      }
    }
  }
  if (MODE == 2) return;
  rs[t] = sS;
  rq[t] = sQ;
  __syncthreads();
  if (t < lanes && cg < C4) {
    float4 S_ = z, Q_ = z;
    for (int r = 0; r < rows_pass; ++r) {
      const float4 a = rs[r * lanes + t], q = rq[r * lanes + t];
      S_.x += a.x; S_.y += a.y; S_.z += a.z; S_.w += a.w;
      Q_.x += q.x; Q_.y += q.y; Q_.z += q.z; Q_.w += q.w;
    }
    reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C)[cg] = S_;
    reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C + C)[cg] = Q_;
  }
}

// part[blk][tap][c] = sum over this block's output strips of dy * x(tap)
// IT: x(tap) = act(bn(xs)) of the stored pre-BN tensor xs, recomputed on load
// with dwconv.hip's BN-input forward expression (common.h dw_bn_in; in-bounds
// taps only, padding stays zero).
template <int K, int S, int PW, bool IT = false>
__global__ __launch_bounds__(256) void dw_wgrad_strip_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, int H, int W, int C, int OH,
    int OW, int nstrip, int64_t items, int64_t items_per_blk, int lanes,
    float* __restrict__ part, const float* __restrict__ bmean = nullptr,
    const float* __restrict__ binvstd = nullptr, const float* __restrict__ bgamma = nullptr,
    const float* __restrict__ bbeta = nullptr, int bact = 0, float bslope = 0.f) {
  constexpr int PAD = K / 2;
  constexpr int L = (PW - 1) * S + K;
  __shared__ float4 red[256];
  const int C4 = C >> 2;
  const int t = threadIdx.x;
  const int rows_pass = 256 / lanes;
  const int r0 = t / lanes;
  const int cg = blockIdx.y * lanes + t % lanes;
  const bool active = r0 < rows_pass && cg < C4;
  float4 acc[K * K];
#pragma unroll
  for (int q = 0; q < K * K; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  DwBnCoef bc{};
  if (IT && active) bc = dw_bn_coef(bmean, binvstd, bgamma, bbeta, cg);
  auto tf = [&](float4 v) -> float4 { return IT ? dw_bn_in(v, bc, bact, bslope) : v; };
  // items band-major (image, band of rows_pass strips, row, strip in band):
  // a pass of the workgroup is one row of a band and its passes walk down the
  // band, so an input row is re-read by the next K/S output rows from this
  // CU's L2 (row-major items re-read whole rows across XCDs: PMC 2.7x the
  // algorithmic bytes)
  const int nbands = (nstrip + rows_pass - 1) / rows_pass;
  const int64_t i0 = (int64_t)blockIdx.x * items_per_blk;
  const int64_t i1 = min(i0 + items_per_blk, items);
  for (int64_t it = i0 + r0; active && it < i1; it += rows_pass) {
    const int64_t grp = it / rows_pass;  // it % rows_pass == r0 (items_per_blk % rows_pass == 0)
    const int64_t bb = grp / OH;
    const int oh = (int)(grp - bb * OH);
    const int b = (int)(bb / nbands), band = (int)(bb - (int64_t)b * nbands);
    const int strip = band * rows_pass + r0;
    if (strip >= nstrip) continue;
    const int ow0 = strip * PW;
    const float4* drow = reinterpret_cast<const float4*>(dy + (((int64_t)b * OH + oh) * OW) * C) + cg;
    float4 g[PW];
#pragma unroll
    for (int q = 0; q < PW; ++q)
      g[q] = (ow0 + q < OW) ? drow[(int64_t)(ow0 + q) * C4] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int iw0 = ow0 * S - PAD;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - PAD + kh;
      if (ih < 0 || ih >= H) continue;
      const float4* xrow = reinterpret_cast<const float4*>(x + (((int64_t)b * H + ih) * W) * C) + cg;
      float4 seg[L];
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int iw = iw0 + j;
        seg[j] = (iw >= 0 && iw < W) ? tf(xrow[(int64_t)iw * C4]) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int kw = 0; kw < K; ++kw)
#pragma unroll
        for (int q = 0; q < PW; ++q) fma4(acc[kh * K + kw], g[q], seg[q * S + kw]);
    }
  }
#pragma unroll
  for (int q = 0; q < K * K; ++q) {
    __syncthreads();
    red[t] = acc[q];
    __syncthreads();
    if (t < lanes && cg < C4) {
      float4 Sm = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < rows_pass; ++r) {
        const float4 a = red[r * lanes + t];
        Sm.x += a.x; Sm.y += a.y; Sm.z += a.z; Sm.w += a.w;
      }
      reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * K * K + q) * C)[cg] = Sm;
    }
  }
}


// 3x3 depthwise weight gradient with every input row read once per chunk of
// R output rows: a thread owns one strip of PW output columns and one channel
// quad and walks its chunk's rows; the rows it still needs stay in registers
// (stride 1: the three dy rows around the current input row; stride 2: the
// shared input row between consecutive output rows), so x and dy cross HBM
// once per chunk (+2 / +1 halo rows) instead of once per tap row.
// Workgroup blockIdx.x = (image, band of rows_pass strips, row chunk); the
// partials are part[blk][tap][c] as dw_wgrad_strip_kernel's.
template <int S, int PW, bool IT = false>
__global__ __launch_bounds__(256) void dw_wgrad_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, int H, int W, int C, int OH,
    int OW, int nstrip, int nbands, int nchunks, int R, int lanes, float* __restrict__ part,
    const float* __restrict__ bmean = nullptr, const float* __restrict__ binvstd = nullptr,
    const float* __restrict__ bgamma = nullptr, const float* __restrict__ bbeta = nullptr,
    int bact = 0, float bslope = 0.f) {
  constexpr int K = 3;
  constexpr int L = (PW - 1) * S + K;
  __shared__ float4 red[256];
  const int C4 = C >> 2;
  const int t = threadIdx.x;
  const int rows_pass = 256 / lanes;
  const int r0 = t / lanes;
  const int cg = blockIdx.y * lanes + t % lanes;
  const int chunk = blockIdx.x % nchunks;
  const int bb = blockIdx.x / nchunks;
  const int b = bb / nbands, band = bb % nbands;
  const int strip = band * rows_pass + r0;
  const bool active = r0 < rows_pass && cg < C4 && strip < nstrip;
  float4 acc[K * K];
#pragma unroll
  for (int q = 0; q < K * K; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  DwBnCoef bc{};
  if (IT && active) bc = dw_bn_coef(bmean, binvstd, bgamma, bbeta, cg);
  const int oh0 = chunk * R, oh1 = min(OH, oh0 + R);
  const int ow0 = strip * PW, iw0 = ow0 * S - 1;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load_x = [&](int ih, float4 (&xs)[L]) {
    const bool rv = ih >= 0 && ih < H;
    const float4* xrow = reinterpret_cast<const float4*>(x + (((int64_t)b * H + (rv ? ih : 0)) * W) * C) + cg;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int iw = iw0 + j;
      xs[j] = (rv && iw >= 0 && iw < W) ? (IT ? dw_bn_in(xrow[(int64_t)iw * C4], bc, bact, bslope)
                                              : xrow[(int64_t)iw * C4])
                                        : z;
    }
  };
  auto load_g = [&](int oh, float4 (&g)[PW]) {
    const bool rv = oh >= oh0 && oh < oh1;
    const float4* drow = reinterpret_cast<const float4*>(dy + (((int64_t)b * OH + (rv ? oh : oh0)) * OW) * C) + cg;
#pragma unroll
    for (int q = 0; q < PW; ++q) g[q] = (rv && ow0 + q < OW) ? drow[(int64_t)(ow0 + q) * C4] : z;
  };
  // acc[kh*3 + kw] += g[q] * xs[q*S + kw]
  auto tap_row = [&](int kh, const float4 (&g)[PW], const float4 (&xs)[L]) {
#pragma unroll
    for (int kw = 0; kw < K; ++kw)
#pragma unroll
      for (int q = 0; q < PW; ++q) fma4(acc[kh * K + kw], g[q], xs[q * S + kw]);
  };
  if (active && oh0 < oh1) {
    if constexpr (S == 1) {
      // input row ih meets dy rows ih+1 (kh 0), ih (kh 1), ih-1 (kh 2); the
      // three dy rows rotate through gA/gB/gC (unrolled by 3: no copies)
      float4 gA[PW], gB[PW], gC[PW], xs[L];
#pragma unroll
      for (int q = 0; q < PW; ++q) gA[q] = gB[q] = z;
      auto step = [&](int ih, const float4 (&gm1)[PW], const float4 (&g0)[PW], const float4 (&gp1)[PW]) {
        load_x(ih, xs);
        tap_row(0, gp1, xs);
        tap_row(1, g0, xs);
        tap_row(2, gm1, xs);
      };
      for (int ih = oh0 - 1; ih <= oh1; ih += 3) {
        load_g(ih + 1, gC);
        step(ih, gA, gB, gC);
        if (ih + 1 > oh1) break;
        load_g(ih + 2, gA);
        step(ih + 1, gB, gC, gA);
        if (ih + 2 > oh1) break;
        load_g(ih + 3, gB);
        step(ih + 2, gC, gA, gB);
      }
    } else {
      // output row oh reads input rows 2oh-1, 2oh, 2oh+1; 2oh+1 is the next
      // row's 2oh'-1 (unrolled by 2: no copies)
      float4 xp[L], xa[L], xb[L], g[PW];
      load_x(2 * oh0 - 1, xp);
      for (int oh = oh0; oh < oh1; oh += 2) {
        load_g(oh, g);
        load_x(2 * oh, xa);
        load_x(2 * oh + 1, xb);
        tap_row(0, g, xp);
        tap_row(1, g, xa);
        tap_row(2, g, xb);
        if (oh + 1 >= oh1) break;
        load_g(oh + 1, g);
        load_x(2 * oh + 2, xa);
        load_x(2 * oh + 3, xp);
        tap_row(0, g, xb);
        tap_row(1, g, xa);
        tap_row(2, g, xp);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < K * K; ++q) {
    __syncthreads();
    red[t] = acc[q];
    __syncthreads();
    if (t < lanes && cg < C4) {
      float4 Sm = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < rows_pass; ++r) {
        const float4 a = red[r * lanes + t];
        Sm.x += a.x; Sm.y += a.y; Sm.z += a.z; Sm.w += a.w;
      }
      reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * K * K + q) * C)[cg] = Sm;
    }
  }
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
        if (dx)  // (jabd_eca_bwd_f32 writes dx in its final pass instead)
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
    // blocks in order (up to 64 partials per channel: the unroll keeps 8 of
    // the loads in flight instead of one L2 round trip per add)
#pragma unroll 8
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
    // (in-order fma chain; the unroll only lets the LDS reads run ahead of
    // it: up to C = 960 iterations, each waiting on its read otherwise)
#pragma unroll 8
    for (int c = 0; c < C; ++c) {
      const int cc = c + t - h;
      if (cc >= 0 && cc < C) acc = fmaf(dz[c], mu[cc], acc);
    }
    dw1d_img[(int64_t)b * k + t] = acc;
  }
}

// dx = da * s[b][c] + v[b][c]: the gate-scaled gradient plus the ECA mean
// term in one pass (replaces writing da*s in scale_bwd and a read-modify-write
// add_bc pass: 4 tensor passes instead of 5).
__global__ void scale_add_kernel(const float* __restrict__ da, const float* __restrict__ s,
                                 const float* __restrict__ v, int64_t HW, int C, int64_t total4,
                                 float* __restrict__ dx) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int C4 = C >> 2;
  const int64_t m = i / C4;
  const int c4 = (int)(i - m * C4);
  const int64_t bc = (m / HW) * C4 + c4;
  const float4 sc = reinterpret_cast<const float4*>(s)[bc];
  const float4 a = reinterpret_cast<const float4*>(v)[bc];
  const float4 g = reinterpret_cast<const float4*>(da)[i];
  reinterpret_cast<float4*>(dx)[i] =
      make_float4(fmaf(g.x, sc.x, a.x), fmaf(g.y, sc.y, a.y), fmaf(g.z, sc.z, a.z),
                  fmaf(g.w, sc.w, a.w));
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
// Channel-vectorised form (C % 4 == 0): one thread per (input pixel, 4
// channels), 32-bit index math, only the windows that contain the pixel, the
// argmax of each recomputed with the same first-max / last-NaN rule per
// channel.  Deterministic gather (no atomics).
__global__ __launch_bounds__(256) void maxpool_bwd4_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ dy, int H,
                                                          int W, int C4, int OH, int OW, int k,
                                                          int s, int pad, int total,
                                                          float* __restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c4 = i % C4;
  int r = i / C4;
  const int iw = r % W;
  r /= W;
  const int ih = r % H;
  const int b = r / H;
  const float4* xb = reinterpret_cast<const float4*>(x) + (int64_t)b * H * W * C4 + c4;
  const float4* dyb = reinterpret_cast<const float4*>(dy) + (int64_t)b * OH * OW * C4 + c4;
  // windows (oh, ow) with oh*s - pad <= ih <= oh*s - pad + k - 1
  const int oh0 = max(0, (ih + pad - k + s) / s), oh1 = min(OH - 1, (ih + pad) / s);
  const int ow0 = max(0, (iw + pad - k + s) / s), ow1 = min(OW - 1, (iw + pad) / s);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int me = ih * W + iw;
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      float best[4];
      int arg[4] = {-1, -1, -1, -1};
      for (int a = 0; a < k; ++a) {
        const int yh = oh * s - pad + a;
        if (yh < 0 || yh >= H) continue;
        for (int q = 0; q < k; ++q) {
          const int yw = ow * s - pad + q;
          if (yw < 0 || yw >= W) continue;
          const int pos = yh * W + yw;
          const float4 v4 = xb[(int64_t)pos * C4];
          const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (arg[e] < 0 || v[e] > best[e] || v[e] != v[e]) {
              best[e] = v[e];
              arg[e] = pos;
            }
        }
      }
      const float4 g = dyb[(int64_t)(oh * OW + ow) * C4];
      if (arg[0] == me) acc[0] += g.x;
      if (arg[1] == me) acc[1] += g.y;
      if (arg[2] == me) acc[2] += g.z;
      if (arg[3] == me) acc[3] += g.w;
    }
  reinterpret_cast<float4*>(dx)[i] = make_float4(acc[0], acc[1], acc[2], acc[3]);
}

// Training form of the stem max-pool (F.max_pool2d(3, 2, 1) in the R50 body,
// nets/resnet_pytorch_r.py:174-178): the forward also keeps each output's
// argmax as its window position (kh * k + kw, uint8 per channel; the first
// maximum in scan order, a NaN taking the place — the rule the
// recomputing backward above uses), so the backward gathers idx + dy
// instead of re-reading and re-reducing every window that contains a pixel
// (which ran from L2 at ~1.2 TB/s).  One thread per (output pixel, 4 channels).
__global__ __launch_bounds__(256) void maxpool_idx4_kernel(const float* __restrict__ x, int H, int W,
                                                           int C4, int OH, int OW, int k, int s,
                                                           int pad, int total,
                                                           float* __restrict__ y,
                                                           uchar4* __restrict__ idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c4 = i % C4;
  int r = i / C4;
  const int ow = r % OW;
  r /= OW;
  const int oh = r % OH;
  const int b = r / OH;
  const float4* xb = reinterpret_cast<const float4*>(x) + (int64_t)b * H * W * C4 + c4;
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  float best[4] = {0.f, 0.f, 0.f, 0.f};
  int arg[4] = {-1, -1, -1, -1};
  for (int a = 0; a < k; ++a) {
    const int ih = oh * s - pad + a;
    if (ih < 0 || ih >= H) continue;
    for (int q = 0; q < k; ++q) {
      const int iw = ow * s - pad + q;
      if (iw < 0 || iw >= W) continue;
      const float4 v4 = xb[(int64_t)(ih * W + iw) * C4];
      const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        m[e] = (v[e] > m[e] || v[e] != v[e]) ? v[e] : m[e];   // the eval maxpool_kernel's value
        if (arg[e] < 0 || v[e] > best[e] || v[e] != v[e]) {
          best[e] = v[e];
          arg[e] = a * k + q;
        }
      }
    }
  }
  reinterpret_cast<float4*>(y)[i] = make_float4(m[0], m[1], m[2], m[3]);
  idx[i] = make_uchar4((unsigned char)arg[0], (unsigned char)arg[1], (unsigned char)arg[2],
                       (unsigned char)arg[3]);
}

// dx[pixel] = sum over the windows holding it (oh, then ow ascending — the
// recomputing kernel's order) of dy where the window's argmax is this pixel
__global__ __launch_bounds__(256) void maxpool_bwd_idx4_kernel(const uchar4* __restrict__ idx,
                                                               const float* __restrict__ dy, int H,
                                                               int W, int C4, int OH, int OW, int k,
                                                               int s, int pad, int total,
                                                               float* __restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c4 = i % C4;
  int r = i / C4;
  const int iw = r % W;
  r /= W;
  const int ih = r % H;
  const int b = r / H;
  const int64_t ob = (int64_t)b * OH * OW * C4 + c4;
  const int oh0 = max(0, (ih + pad - k + s) / s), oh1 = min(OH - 1, (ih + pad) / s);
  const int ow0 = max(0, (iw + pad - k + s) / s), ow1 = min(OW - 1, (iw + pad) / s);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int me = (ih - (oh * s - pad)) * k + (iw - (ow * s - pad));
      const int64_t o = ob + (int64_t)(oh * OW + ow) * C4;
      const uchar4 a = idx[o];
      const float4 g = reinterpret_cast<const float4*>(dy)[o];
      if (a.x == me) acc[0] += g.x;
      if (a.y == me) acc[1] += g.y;
      if (a.z == me) acc[2] += g.z;
      if (a.w == me) acc[3] += g.w;
    }
  reinterpret_cast<float4*>(dx)[i] = make_float4(acc[0], acc[1], acc[2], acc[3]);
}

// Same gather with the index math per workgroup: block (x, ih, b) covers
// 256 / C4 input columns of one input row, thread t -> channel quad
// t % C4 (C4 a power of two), column t / C4 — no per-thread division of the
// flat index (three 32-bit divisions per float4 of dx were the kernel's
// bound at the R50 stem's 64 channels).  Same sums in the same order.
__global__ __launch_bounds__(256) void maxpool_bwd_idx4_row_kernel(
    const uchar4* __restrict__ idx, const float* __restrict__ dy, int H, int W, int c4s, int OH,
    int OW, int k, int s, int pad, float* __restrict__ dx) {
  const int C4 = 1 << c4s;
  const int t = threadIdx.x;
  const int c4 = t & (C4 - 1);
  const int iw = blockIdx.x * (256 >> c4s) + (t >> c4s);
  const int ih = blockIdx.y, b = blockIdx.z;
  if (iw >= W) return;
  const int64_t ob = (int64_t)b * OH * OW * C4 + c4;
  const int oh0 = max(0, (ih + pad - k + s) / s), oh1 = min(OH - 1, (ih + pad) / s);
  const int ow0 = max(0, (iw + pad - k + s) / s), ow1 = min(OW - 1, (iw + pad) / s);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int oh = oh0; oh <= oh1; ++oh)
    for (int ow = ow0; ow <= ow1; ++ow) {
      const int me = (ih - (oh * s - pad)) * k + (iw - (ow * s - pad));
      const int64_t o = ob + (int64_t)(oh * OW + ow) * C4;
      const uchar4 a = idx[o];
      const float4 g = reinterpret_cast<const float4*>(dy)[o];
      if (a.x == me) acc[0] += g.x;
      if (a.y == me) acc[1] += g.y;
      if (a.z == me) acc[2] += g.z;
      if (a.w == me) acc[3] += g.w;
    }
  const int64_t i = (((int64_t)b * H + ih) * W + iw) * C4 + c4;
  reinterpret_cast<float4*>(dx)[i] = make_float4(acc[0], acc[1], acc[2], acc[3]);
}

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

// The final half of jabd_bn_stats_f32 for partials a producer wrote in
// bn_stats_part's format (shift[c] = the value the partials were taken
// around): mean, invstd and the running-statistics update.
extern "C" int jabd_bn_stats_final_f32(const float* shift, const float* part, int64_t nblk,
                                       int64_t M, int32_t C, float* mean, float* invstd,
                                       float* running_mean, float* running_var, float momentum,
                                       float eps, jabd_stream_t stream) {
  JABD_REQUIRE(shift && part && mean && invstd && nblk > 0 && M > 0 && C > 0,
               "bn_stats_final: bad args");
  bn_stats_final_kernel<float><<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, as_stream(stream)>>>(
      shift, part, nblk, M, C, momentum, eps, mean, invstd, running_mean, running_var);
  return check_launch("bn_stats_final");
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
  bn_stats_final_kernel<float><<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, st>>>(
      x, part, nblk, M, C, momentum, eps, mean, invstd, running_mean, running_var);
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
  if (M == 0 || C == 0) return JABD_OK;
  int lanes;
  const dim3 grid = ew_grid(M, C, lanes);
  (res ? bn_act_fwd_kernel<true> : bn_act_fwd_kernel<false>)<<<grid, kRedThreads, 0,
                                                                as_stream(stream)>>>(
      x, ldx, M, C, mean, invstd, gamma, beta, res, ldr, act, slope, y, ldy, yc0, lanes);
  return check_launch("bn_act_fwd");
}

// Rows per channel-sum block of jabd_bn_act_fwd_sum_f32 for C channels:
// rp (a power of two, rp * lanes <= 256) times kEwIters.
static int bn_sum_rp(int C) {
  const int C4 = C / 4, lanes = C4 < 64 ? C4 : 64;
  int rp = 1;
  while (rp * 2 * lanes <= kRedThreads) rp *= 2;
  return rp;
}

extern "C" int64_t jabd_bn_sum_nblk(int64_t hw, int32_t C) {
  if (hw <= 0 || C <= 0 || C % 4) return 0;
  const int64_t rb = (int64_t)bn_sum_rp(C) * kEwIters;
  return hw % rb ? 0 : hw / rb;
}

extern "C" int jabd_bn_act_fwd_sum_f32(const float* x, int64_t M, int32_t C, const float* mean,
                                       const float* invstd, const float* gamma,
                                       const float* beta, int32_t act, float slope, float* y,
                                       int64_t hw, float* part, jabd_stream_t stream) {
  JABD_REQUIRE(x && mean && invstd && gamma && beta && y && part && C % 4 == 0 && hw > 0 &&
                   M % hw == 0,
               "bn_act_fwd_sum: bad args");
  JABD_REQUIRE(jabd_bn_sum_nblk(hw, C) > 0, "bn_act_fwd_sum: hw %lld not a multiple of the %d-row "
               "block (jabd_bn_sum_nblk = 0)", (long long)hw, bn_sum_rp(C) * kEwIters);
  if (M == 0) return JABD_OK;
  const int C4 = C / 4, lanes = C4 < 64 ? C4 : 64, rp = bn_sum_rp(C);
  const dim3 grid((unsigned)(M / ((int64_t)rp * kEwIters)), (unsigned)cdiv(C4, lanes), 1);
  bn_act_fwd_sum_kernel<<<grid, kRedThreads, 0, as_stream(stream)>>>(
      x, M, C, mean, invstd, gamma, beta, act, slope, y, lanes, rp, part);
  return check_launch("bn_act_fwd_sum");
}

extern "C" int jabd_bn_act_bwd_f32(const float* dy, int32_t lddy, int32_t dyc0, const float* x,
                                   int32_t ldx, const float* res, int32_t ldr, int64_t M,
                                   int32_t C, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, int32_t act,
                                   float slope, float* part, float* dgamma, float* dbeta,
                                   float* dx, float* dres, jabd_stream_t stream) {
  return jabd_bn_act_bwd_ex_f32(dy, lddy, dyc0, x, ldx, res, ldr, M, C, mean, invstd, gamma,
                                beta, act, slope, nullptr, nullptr, 0, part, dgamma, dbeta, dx,
                                dres, stream);
}

extern "C" int jabd_bn_act_bwd_ex_f32(const float* dy, int32_t lddy, int32_t dyc0,
                                      const float* x, int32_t ldx, const float* res, int32_t ldr,
                                      int64_t M, int32_t C, const float* mean,
                                      const float* invstd, const float* gamma, const float* beta,
                                      int32_t act, float slope, const float* dys,
                                      const float* dya, int64_t hw, float* part, float* dgamma,
                                      float* dbeta, float* dx, float* dres,
                                      jabd_stream_t stream) {
  JABD_REQUIRE(dy && x && mean && invstd && gamma && beta && part && dgamma && dbeta && dx &&
                   C % 4 == 0 && lddy % 4 == 0 && dyc0 % 4 == 0 && ldx % 4 == 0,
               "bn_act_bwd: bad args");
  JABD_REQUIRE(!dys || (dya && hw > 0 && M % hw == 0), "bn_act_bwd: dy transform needs dya, hw");
  hipStream_t st = as_stream(stream);
  const int64_t per = bn_rows_per_blk(M, C), nblk = cdiv(M, per);
  auto part_k = res ? (dys ? bn_bwd_part_kernel<true, true> : bn_bwd_part_kernel<true, false>)
                    : (dys ? bn_bwd_part_kernel<false, true> : bn_bwd_part_kernel<false, false>);
  part_k<<<(unsigned)nblk, kRedThreads, 0, st>>>(dy, lddy, dyc0, x, ldx, res, ldr, M, C, mean,
                                                invstd, gamma, beta, act, slope, per, part, dys,
                                                dya, hw);
  if (int e = check_launch("bn_bwd_part")) return e;
  bn_bwd_final_kernel<float><<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, st>>>(
      part, nblk, C, dbeta, dgamma);
  if (int e = check_launch("bn_bwd_final")) return e;
  int lanes;
  const dim3 grid = ew_grid(M, C, lanes);
  auto apply_k = res ? (dys ? bn_bwd_apply_kernel<true, true> : bn_bwd_apply_kernel<true, false>)
                     : (dys ? bn_bwd_apply_kernel<false, true> : bn_bwd_apply_kernel<false, false>);
  apply_k<<<grid, kRedThreads, 0, st>>>(dy, lddy, dyc0, x, ldx, res, ldr, M, C, mean, invstd,
                                        gamma, beta, act, slope, dbeta, dgamma, dx, dres, lanes,
                                        dys, dya, hw);
  return check_launch("bn_bwd_apply");
}

// The tiled weight-gradient kernels over chunks of `per` output pixels
// (chunk c covers pixels [c*per, min((c+1)*per, M))), partials part[chunk][K][Cout].
static void wgrad_launch_parts(const ConvArgs& a, int64_t per, int64_t nch, float* part,
                               hipStream_t st) {
  const int K = a.KH * a.KW * a.Cin;
  const WgDivs dv{make_fastdiv((uint32_t)((int64_t)a.OH * a.OW)), make_fastdiv((uint32_t)a.OW),
                  make_fastdiv((uint32_t)a.Cin), make_fastdiv((uint32_t)a.KW)};
  if (wgrad_vec_ok(a) && wgrad32_ok(a)) {
    const int tk = wg32_tile(K), tn = wg32_tile(a.Cout);
    const int fast = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && a.H == a.OH &&
                     a.W == a.OW;
    dim3 g((unsigned)cdiv(K, tk), (unsigned)cdiv(a.Cout, tn), (unsigned)nch);
    // double-buffered stages for the 1x1 layers (tools/wgdb_ab.sh: 1x1 shapes
    // +0-19%, the 3x3 ones 5% slower with the doubled LDS)
#define W32_CASE(KT_, NT_)                                                              \
  if (tk == KT_ && tn == NT_) {                                                         \
    if (fast)                                                                           \
      conv_wgrad32_kernel<KT_, NT_, true><<<g, 256, 0, st>>>(a, (int)per, fast, part, dv);  \
    else                                                                                \
      conv_wgrad32_kernel<KT_, NT_, false><<<g, 256, 0, st>>>(a, (int)per, fast, part, dv); \
  }
    W32_CASE(64, 64) W32_CASE(64, 128) W32_CASE(128, 64) W32_CASE(128, 128)
#undef W32_CASE
  } else if (wgrad_vec_ok(a)) {
    const int tk = wv_tile(K), tn = wv_tile(a.Cout);
    const int fast = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && a.H == a.OH &&
                     a.W == a.OW;
    dim3 g((unsigned)cdiv(K, tk), (unsigned)cdiv(a.Cout, tn), (unsigned)nch);
#define WV_CASE(KT_, NT_)                                                         \
  if (tk == KT_ && tn == NT_)                                                     \
    conv_wgrad_v_kernel<KT_, NT_><<<g, 256, 0, st>>>(a, (int)per, fast, part, dv);
    WV_CASE(16, 16) WV_CASE(16, 32) WV_CASE(16, 64)
    WV_CASE(32, 16) WV_CASE(32, 32) WV_CASE(32, 64)
    WV_CASE(64, 16) WV_CASE(64, 32) WV_CASE(64, 64)
#undef WV_CASE
  } else {
    dim3 g((unsigned)cdiv(K, kWgT), (unsigned)cdiv(a.Cout, kWgT), (unsigned)nch);
    conv_wgrad_kernel<<<g, 256, 0, st>>>(a, per, part);
  }
}

namespace jabd {
bool stem7_ok(const ConvArgs& a);
int64_t stem7_wgrad_groups(const ConvArgs& a);
int stem7_wgrad_launch(const ConvArgs& a, float* part, hipStream_t st);
}  // namespace jabd

// ResNet-50 7x7/s2 stem (stem7.hip); JABD_STEM7=0 -> the tiled kernels
static bool stem7_wgrad_on(const ConvArgs& a) {
  static const bool on = [] {
    const char* e = getenv("JABD_STEM7");
    return !(e && e[0] == '0');
  }();
  return on && stem7_ok(a) && a.y_ps % 4 == 0 && a.y_c0 % 4 == 0 && a.y_bs % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(a.y) & 15) == 0;
}

extern "C" int64_t jabd_conv_wgrad_part_floats(const jabd_conv_args* args) {
  if (!args) return -1;
  ConvArgs a = *args;
  a.M = (int64_t)a.B * a.OH * a.OW;
  const int64_t KN = (int64_t)a.KH * a.KW * a.Cin * a.Cout;
  if (stem_wgrad_ok(a)) return stem_wgrad_waves(a) * KN;
  if (stem7_wgrad_on(a)) return stem7_wgrad_groups(a) * KN;
  return wgrad_chunks(a) * KN;
}

// BatchNorm + act backward from the sums a data-gradient GEMM took in its
// epilogue (jabd_conv_bn_bwd_sums_f32's part: rows then the fp64 chunks):
// fixed-order fp64 sums -> dbeta = sum dz, dgamma = sum dz * xhat, then the
// apply pass dx = gamma invstd (dz - dbeta/M - xhat dgamma/M), as
// jabd_bn_act_bwd_f32 without its reduction pass.
extern "C" int jabd_bn_act_bwd_rows_f32(float* part, const float* dy, const float* x,
                                        int64_t M, int32_t C, const float* mean,
                                        const float* invstd, const float* gamma,
                                        const float* beta, int32_t act, float slope,
                                        float* dgamma, float* dbeta, float* dx,
                                        jabd_stream_t stream) {
  JABD_REQUIRE(part && dy && x && mean && invstd && gamma && beta && dgamma && dbeta && dx &&
                   M > 0 && C > 0 && C % 32 == 0 && ((uintptr_t)part & 15) == 0,
               "bn_act_bwd_rows: bad args");
  hipStream_t st = as_stream(stream);
  const int64_t nrow = cdiv(M, (int64_t)32), nch = cdiv(nrow, (int64_t)kRowChunk);
  double* chunks = reinterpret_cast<double*>(part + nrow * 2 * C);
  bn_rows_sum_kernel<<<(unsigned)cdiv(nch * C, (int64_t)256), 256, 0, st>>>(part, nrow, C, chunks);
  if (int e = check_launch("bn_rows_sum")) return e;
  bn_bwd_final_kernel<double><<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, st>>>(
      chunks, nch, C, dbeta, dgamma);
  if (int e = check_launch("bn_bwd_final (rows)")) return e;
  int lanes;
  const dim3 grid = ew_grid(M, C, lanes);
  bn_bwd_apply_kernel<false, false><<<grid, kRedThreads, 0, st>>>(
      dy, C, 0, x, C, nullptr, C, M, C, mean, invstd, gamma, beta, act, slope, dbeta, dgamma, dx,
      nullptr, lanes, nullptr, nullptr, 0);
  return check_launch("bn_bwd_apply (rows)");
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
  if (stem_wgrad_ok(a)) {
    const int64_t nwv = stem_wgrad_waves(a);
    const int64_t ntask = (int64_t)a.B * a.OH * cdiv(a.OW, kSwPx);
    const size_t lds = 4 * sizeof(float) * a.Cin * a.KH * ((kSwPx - 1) * a.stride + a.KW);
    stem_wgrad_kernel<<<(unsigned)(nwv / 4), 256, lds, st>>>(a, ntask, part);
    if (int e = check_launch("stem_wgrad")) return e;
    const int64_t tot = (int64_t)K * a.Cout;
    wgrad_reduce2_kernel<<<(unsigned)cdiv(tot, 16), 256, 0, st>>>(part, nwv, K, a.Cout, a.Cin,
                                                                  a.KH * a.KW, 16, dw);
    return check_launch("wgrad_reduce");
  }
  if (stem7_wgrad_on(a)) {
    const int64_t ng = stem7_wgrad_groups(a);
    if (int e = stem7_wgrad_launch(a, part, st)) return e;
    const int64_t tot = (int64_t)K * a.Cout;
    wgrad_reduce2_kernel<<<(unsigned)cdiv(tot, 64), 256, 0, st>>>(part, ng, K, a.Cout, a.Cin,
                                                                  a.KH * a.KW, 64, dw);
    return check_launch("wgrad_reduce");
  }
  wgrad_launch_parts(a, per, nch, part, st);
  if (int e = check_launch("conv_wgrad")) return e;
  const int64_t tot = (int64_t)K * a.Cout;
  const int lanes = tot >= 64 * 512 ? 64 : 16;
  wgrad_reduce2_kernel<<<(unsigned)cdiv(tot, lanes), 256, 0, st>>>(part, nch, K, a.Cout, a.Cin,
                                                                   a.KH * a.KW, lanes, dw);
  return check_launch("wgrad_reduce");
}

// ---------------------------------------------------------------------------
// ECA-gated project conv (nets/mobilenetV3.py:343-348 then conv3 at :145):
// p = conv3(d * s[b][c]).  Its weight gradient and the gate's input sum
//   dW[n][c]  = sum_b s[b][c] G_b[c][n],
//   ds[b][c]  = sum_hw da * d = sum_n W[n][c] G_b[c][n],   da = dgrad(dp),
// with G_b[c][n] = sum over image b's pixels of d[c] dp[n], share one GEMM:
// the weight-gradient kernels run on the ungated d over pixel chunks that
// never straddle an image, and one reduction forms both.  This replaces the
// separate sum(da * d) pass over two full tensors (scale_bwd).
// ---------------------------------------------------------------------------
// Workgroup per gated channel c: lane n sums image b's chunks in a fixed
// order (cpi = 1 after wgrad_img_reduce_kernel); the W-weighted terms are
// reduced per image from LDS in n order.
__global__ __launch_bounds__(256) void wgrad_eca_reduce_kernel(
    const float* __restrict__ part, int cpi, int B, int E, int Cout,
    const float* __restrict__ scale, const float* __restrict__ w, float* __restrict__ dw,
    float* __restrict__ ds) {
  extern __shared__ float prod[];  // [B][Cout]
  const int c = blockIdx.x, t = threadIdx.x;
  const int64_t EN = (int64_t)E * Cout;
  for (int n = t; n < Cout; n += blockDim.x) {
    const float wn = w[(int64_t)n * E + c];
    float acc = 0.f;
    // images in order (the unroll lets their loads run ahead of the chain)
#pragma unroll 8
    for (int b = 0; b < B; ++b) {
      const float* pb = part + (int64_t)b * cpi * EN + (int64_t)c * Cout + n;
      float g0 = 0.f, g1 = 0.f;
      int j = 0;
      for (; j + 1 < cpi; j += 2) {
        g0 += pb[(int64_t)j * EN];
        g1 += pb[(int64_t)(j + 1) * EN];
      }
      if (j < cpi) g0 += pb[(int64_t)j * EN];
      const float g = g0 + g1;
      acc = fmaf(scale[(int64_t)b * E + c], g, acc);
      prod[b * Cout + n] = wn * g;
    }
    dw[(int64_t)n * E + c] = acc;
  }
  __syncthreads();
  for (int b = t; b < B; b += blockDim.x) {
    float sm = 0.f;
#pragma unroll 8
    for (int n = 0; n < Cout; ++n) sm += prod[b * Cout + n];
    ds[(int64_t)b * E + c] = sm;
  }
}

// G[b][i] = sum_j part[b * cpi + j][i] (i < EN, EN % 4 == 0): the per-image
// sum of the chunk partials, float4 per thread, j in order (deterministic).
__global__ __launch_bounds__(256) void wgrad_img_reduce_kernel(const float* __restrict__ part,
                                                               int cpi, int64_t EN,
                                                               float* __restrict__ G) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (i4 * 4 >= EN) return;
  const float4* pb = reinterpret_cast<const float4*>(part + (int64_t)b * cpi * EN) + i4;
  const int64_t st = EN / 4;
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  int j = 0;
  for (; j + 3 < cpi; j += 4) {
    const float4 v0 = pb[j * st], v1 = pb[(j + 1) * st], v2 = pb[(j + 2) * st],
                 v3 = pb[(j + 3) * st];
    a0.x += v0.x; a0.y += v0.y; a0.z += v0.z; a0.w += v0.w;
    a1.x += v1.x; a1.y += v1.y; a1.z += v1.z; a1.w += v1.w;
    a2.x += v2.x; a2.y += v2.y; a2.z += v2.z; a2.w += v2.w;
    a3.x += v3.x; a3.y += v3.y; a3.z += v3.z; a3.w += v3.w;
  }
  for (; j < cpi; ++j) {
    const float4 v = pb[j * st];
    a0.x += v.x; a0.y += v.y; a0.z += v.z; a0.w += v.w;
  }
  reinterpret_cast<float4*>(G + (int64_t)b * EN)[i4] =
      make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                  (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
}

// Image-aligned chunk length: the largest per = HW / 2^j (a multiple of the
// kernels' 64-pixel stage) that is still >= the normal chunk length, or 0 if
// the shape does not qualify (1x1 / stride 1, HW % 64, LDS for [B][Cout]).
static int64_t wgrad_eca_per(const ConvArgs& a) {
  const int64_t HW = (int64_t)a.OH * a.OW;
  if (a.KH != 1 || a.KW != 1 || a.stride != 1 || a.pad != 0 || a.H != a.OH || a.W != a.OW ||
      HW % kWgPx || (int64_t)a.B * a.Cout * 4 > 64 * 1024 || !wgrad_vec_ok(a) || a.ascale ||
      ((int64_t)a.Cin * a.Cout) % 4)
    return 0;
  const int64_t target = cdiv(a.M, wgrad_chunks(a));
  int64_t per = HW;
  while (per % (2 * kWgPx) == 0 && per / 2 >= target) per /= 2;
  if ((cdiv(a.M, per) + a.B) * a.Cin * a.Cout > ((int64_t)64 << 20)) return 0;
  return per;
}

extern "C" int64_t jabd_conv_wgrad_eca_part_floats(const jabd_conv_args* args) {
  if (!args) return -1;
  ConvArgs a = *args;
  a.M = (int64_t)a.B * a.OH * a.OW;
  const int64_t per = wgrad_eca_per(a);
  return per ? (cdiv(a.M, per) + a.B) * a.Cin * a.Cout : 0;  // chunk partials + per-image sums
}

extern "C" int jabd_conv_wgrad_eca_f32(const jabd_conv_args* args, const float* scale,
                                       const float* w, float* part, float* dw, float* ds,
                                       jabd_stream_t stream) {
  JABD_REQUIRE(args && scale && w && part && dw && ds, "conv_wgrad_eca: null");
  ConvArgs a = *args;
  JABD_REQUIRE(a.x && a.y && !a.x2 && !a.tconv && !a.ascale, "conv_wgrad_eca: bad args");
  a.M = (int64_t)a.B * a.OH * a.OW;
  JABD_REQUIRE(a.M < (int64_t)0x7fffffff, "conv_wgrad_eca: M too large");
  const int64_t per = wgrad_eca_per(a);
  JABD_REQUIRE(per > 0, "conv_wgrad_eca: unsupported shape (jabd_conv_wgrad_eca_part_floats = 0)");
  const int64_t nch = cdiv(a.M, per);
  const int cpi = (int)(((int64_t)a.OH * a.OW) / per);
  hipStream_t st = as_stream(stream);
  wgrad_launch_parts(a, per, nch, part, st);
  if (int e = check_launch("conv_wgrad")) return e;
  const int64_t EN = (int64_t)a.Cin * a.Cout;
  float* G = part + nch * EN;
  wgrad_img_reduce_kernel<<<dim3((unsigned)cdiv(EN / 4, 256), (unsigned)a.B), 256, 0, st>>>(
      part, cpi, EN, G);
  if (int e = check_launch("wgrad_img_reduce")) return e;
  wgrad_eca_reduce_kernel<<<(unsigned)a.Cin, 256, (size_t)a.B * a.Cout * sizeof(float), st>>>(
      G, 1, a.B, a.Cin, a.Cout, scale, w, dw, ds);
  return check_launch("wgrad_eca_reduce");
}

extern "C" int jabd_dw_dgrad_f32(const float* dy, const float* w, int32_t B, int32_t H, int32_t W,
                                 int32_t C, int32_t OH, int32_t OW, int32_t k, int32_t stride,
                                 int32_t pad, float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(dy && w && dx && C % 4 == 0 && B > 0 && H > 0 && W > 0, "dw_dgrad: bad args");
  JABD_REQUIRE((k == 3 || k == 5) && pad == k / 2 && (stride == 1 || stride == 2) &&
                   OH == (H + 2 * pad - k) / stride + 1 && OW == (W + 2 * pad - k) / stride + 1,
               "dw_dgrad: unsupported geometry");
  const int C4 = C / 4, lanes = C4 < 64 ? C4 : 64, rows_pass = 256 / lanes;
  hipStream_t st = as_stream(stream);
#define DG_CASE(K_, S_, PW_)                                                                   \
  if (k == K_ && stride == S_) {                                                               \
    const int nstrip = (int)cdiv(W, PW_);                                                      \
    const int64_t items = (int64_t)B * H * nstrip;                                             \
    dim3 g((unsigned)cdiv(items, rows_pass), (unsigned)cdiv(C4, lanes));                       \
    dw_dgrad_strip_kernel<K_, S_, PW_><<<g, 256, 0, st>>>(dy, w, H, W, C, OH, OW, nstrip, items, \
                                                          lanes, dx);                          \
  }
  DG_CASE(3, 1, 8) DG_CASE(3, 2, 8) DG_CASE(5, 1, 8) DG_CASE(5, 2, 8)
#undef DG_CASE
  return check_launch("dw_dgrad");
}

// Workgroups of dw_dgrad_bn_kernel along the strip rows: ~8192 (each walks
// spb rows of rows_pass strips), so bn_bwd_final reads few partial rows.
static int64_t dgbn_groups(int B, int H, int W, int C) {
  const int C4 = C / 4, lanes = C4 < 64 ? C4 : 64, rows_pass = 256 / lanes;
  return (int64_t)B * cdiv(cdiv(W, 8), rows_pass) * H;  // (image, band, row)
}
static void dgbn_plan(int B, int H, int W, int C, int& nblk, int& spb) {
  const int64_t groups = dgbn_groups(B, H, W, C);
  spb = (int)cdiv(groups, 8192);
  nblk = (int)cdiv(groups, spb);
}

extern "C" int64_t jabd_dw_dgrad_bn_part_floats(int32_t B, int32_t H, int32_t W, int32_t C) {
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4) return -1;
  int nblk, spb;
  dgbn_plan(B, H, W, C, nblk, spb);
  return (int64_t)nblk * 2 * C;
}

extern "C" int jabd_dw_dgrad_bn_bwd_f32(const float* dy, const float* w, int32_t B, int32_t H,
                                        int32_t W, int32_t C, int32_t OH, int32_t OW, int32_t k,
                                        int32_t stride, int32_t pad, const float* x,
                                        const float* mean, const float* invstd,
                                        const float* gamma, const float* beta, int32_t act,
                                        float slope, float* part, float* dgamma, float* dbeta,
                                        float* dz, float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(dy && w && x && mean && invstd && gamma && beta && part && dgamma && dbeta &&
                   dx && C % 4 == 0 && B > 0 && H > 0 && W > 0,
               "dw_dgrad_bn_bwd: bad args");
  JABD_REQUIRE((k == 3 || k == 5) && pad == k / 2 && (stride == 1 || stride == 2) &&
                   OH == (H + 2 * pad - k) / stride + 1 && OW == (W + 2 * pad - k) / stride + 1,
               "dw_dgrad_bn_bwd: unsupported geometry");
  const int C4 = C / 4, lanes = C4 < 64 ? C4 : 64;
  int nblk, spb;
  dgbn_plan(B, H, W, C, nblk, spb);
  hipStream_t st = as_stream(stream);
  const int nstrip = (int)cdiv(W, 8);
  const int64_t items = dgbn_groups(B, H, W, C);  // (image, band, row) groups
  const dim3 g((unsigned)nblk, (unsigned)cdiv(C4, lanes));
  const int64_t M = (int64_t)B * H * W;
  // dz == NULL: the two-pass form (partials, then the apply with de
  // recomputed; MODE 1 + 2), else de is stored to dz and applied (MODE 0)
  // 3x3 row walker, opt-in (JABD_DW_DGRAD_ROWS=1): measured slower than the
  // strip-row kernel at every C4 shape (b1 s2 1803 -> 2640 us, b3 647 -> 1017,
  // b7 181 -> 205: ~200 VGPRs, two waves per SIMD, where the strip-row
  // kernel's dy re-reads hit L2)
  static const bool rows_on = [] {
    const char* e = getenv("JABD_DW_DGRAD_ROWS");
    return e && e[0] == '1';
  }();
  const int rows_pass = 256 / lanes;
#define DGR_CASE(S_, PW_)                                                                      \
  if (rows_on && k == 3 && stride == S_) {                                                     \
    const int ns = (int)cdiv(W, PW_);                                                          \
    const int nbands = (int)cdiv(ns, rows_pass);                                               \
    if ((int64_t)B * nbands <= nblk) {                                                         \
      const int want = (int)std::max<int64_t>(1, std::min<int64_t>(H, nblk / ((int64_t)B * nbands))); \
      const int R = (int)cdiv(H, want);                                                        \
      const int nch = (int)cdiv(H, R);                                                         \
      const int nwork = B * nbands * nch;                                                      \
      if (dz)                                                                                  \
        dw_dgrad_bn_rows_kernel<S_, PW_, 0><<<g, 256, 0, st>>>(                                \
            dy, w, H, W, C, OH, OW, ns, nbands, nch, R, nwork, lanes, dz, x, mean, invstd,     \
            gamma, beta, act, slope, part);                                                    \
      else                                                                                     \
        dw_dgrad_bn_rows_kernel<S_, PW_, 1><<<g, 256, 0, st>>>(                                \
            dy, w, H, W, C, OH, OW, ns, nbands, nch, R, nwork, lanes, nullptr, x, mean, invstd, \
            gamma, beta, act, slope, part);                                                    \
      if (int e = check_launch("dw_dgrad_bn_rows")) return e;                                  \
      bn_bwd_final_kernel<<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, st>>>(part, nblk, C, \
                                                                                dbeta, dgamma); \
      if (int e = check_launch("bn_bwd_final")) return e;                                      \
      if (!dz) {                                                                               \
        dw_dgrad_bn_rows_kernel<S_, PW_, 2><<<g, 256, 0, st>>>(                                \
            dy, w, H, W, C, OH, OW, ns, nbands, nch, R, nwork, lanes, dx, x, mean, invstd,     \
            gamma, beta, act, slope, nullptr, dbeta, dgamma, M);                               \
        return check_launch("dw_dgrad_bn_rows_apply");                                         \
      }                                                                                        \
      goto apply;                                                                              \
    }                                                                                          \
  }
  DGR_CASE(1, 4) DGR_CASE(2, 8)
#undef DGR_CASE
#define DGB_CASE(K_, S_)                                                                       \
  if (k == K_ && stride == S_) {                                                               \
    if (dz)                                                                                    \
      dw_dgrad_bn_kernel<K_, S_, 8><<<g, 256, 0, st>>>(dy, w, H, W, C, OH, OW, nstrip, items,  \
                                                       lanes, spb, dz, x, mean, invstd, gamma,  \
                                                       beta, act, slope, part);                 \
    else                                                                                       \
      dw_dgrad_bn_kernel<K_, S_, 8, 1><<<g, 256, 0, st>>>(dy, w, H, W, C, OH, OW, nstrip,      \
                                                          items, lanes, spb, nullptr, x, mean,  \
                                                          invstd, gamma, beta, act, slope,      \
                                                          part);                                \
    if (int e = check_launch("dw_dgrad_bn")) return e;                                         \
    bn_bwd_final_kernel<<<(unsigned)cdiv(C, kFinLanes), kFinThreads, 0, st>>>(part, nblk, C,   \
                                                                              dbeta, dgamma);  \
    if (int e = check_launch("bn_bwd_final")) return e;                                        \
    if (!dz) {                                                                                 \
      dw_dgrad_bn_kernel<K_, S_, 8, 2><<<g, 256, 0, st>>>(dy, w, H, W, C, OH, OW, nstrip,      \
                                                          items, lanes, spb, dx, x, mean,       \
                                                          invstd, gamma, beta, act, slope,      \
                                                          nullptr, dbeta, dgamma, M);           \
      return check_launch("dw_dgrad_bn_apply");                                                \
    }                                                                                          \
  }
  DGB_CASE(3, 1) DGB_CASE(3, 2) DGB_CASE(5, 1) DGB_CASE(5, 2)
#undef DGB_CASE
apply:
  int elanes;
  const dim3 grid = ew_grid(M, C, elanes);
  bn_bwd_apply_kernel<false, false><<<grid, kRedThreads, 0, st>>>(dz, C, 0, x, C, nullptr, 0, M, C,
                                                                  mean, invstd,
                                                    gamma, beta, act, slope, dbeta, dgamma, dx,
                                                    nullptr, elanes, nullptr, nullptr, 1);
  return check_launch("bn_bwd_apply");
}

extern "C" int64_t jabd_dw_wgrad_part_floats(int64_t M, int32_t C, int32_t k) {
  return 1024 * (int64_t)k * k * C;
}

static int dw_wgrad(const float* x, const float* dy, int32_t B, int32_t H, int32_t W, int32_t C,
                    int32_t OH, int32_t OW, int32_t k, int32_t stride, int32_t pad,
                    const float* bmean, const float* binvstd, const float* bgamma,
                    const float* bbeta, int32_t bact, float bslope, float* part, float* dw,
                    jabd_stream_t stream) {
  JABD_REQUIRE(x && dy && part && dw && C % 4 == 0 && B > 0, "dw_wgrad: bad args");
  const bool it = bmean != nullptr;
  JABD_REQUIRE(!it || (binvstd && bgamma && bbeta), "dw_wgrad: null BN input");
  JABD_REQUIRE((k == 3 || k == 5) && pad == k / 2 && (stride == 1 || stride == 2) &&
                   OH == (H + 2 * pad - k) / stride + 1 && OW == (W + 2 * pad - k) / stride + 1,
               "dw_wgrad: unsupported geometry");
  const int C4 = C / 4, lanes = C4 < 64 ? C4 : 64, rows_pass = 256 / lanes;
  hipStream_t st = as_stream(stream);
  int64_t nblk = 0;
  // 3x3: the row-walking kernel when (image, band) pairs leave room for row
  // chunks within the 1024 partial blocks (JABD_DW_WGRAD_ROWS=0: strip kernel)
  static const bool rows_on = [] {
    const char* e = getenv("JABD_DW_WGRAD_ROWS");
    return !(e && e[0] == '0');
  }();
#define WR_CASE(S_, PW_)                                                                        \
  if (rows_on && k == 3 && stride == S_) {                                                      \
    const int nstrip = (int)cdiv(OW, PW_);                                                      \
    const int nbands = (int)cdiv(nstrip, rows_pass);                                            \
    if ((int64_t)B * nbands <= 1024) {                                                          \
      const int want = (int)std::max<int64_t>(1, std::min<int64_t>(OH, 1024 / ((int64_t)B * nbands))); \
      const int R = (int)cdiv(OH, want);                                                        \
      const int nch = (int)cdiv(OH, R);                                                         \
      nblk = (int64_t)B * nbands * nch;                                                         \
      dim3 g((unsigned)nblk, (unsigned)cdiv(C4, lanes));                                        \
      if (it)                                                                                   \
        dw_wgrad_rows_kernel<S_, PW_, true><<<g, 256, 0, st>>>(                                 \
            x, dy, H, W, C, OH, OW, nstrip, nbands, nch, R, lanes, part, bmean, binvstd, bgamma, \
            bbeta, bact, bslope);                                                               \
      else                                                                                      \
        dw_wgrad_rows_kernel<S_, PW_><<<g, 256, 0, st>>>(x, dy, H, W, C, OH, OW, nstrip, nbands, \
                                                          nch, R, lanes, part);                 \
    }                                                                                           \
  }
  WR_CASE(1, 4) WR_CASE(2, 2)
#undef WR_CASE
#define WG_CASE(K_, S_, PW_)                                                                    \
  if (nblk == 0 && k == K_ && stride == S_) {                                                   \
    const int nstrip = (int)cdiv(OW, PW_);                                                      \
    const int64_t items = (int64_t)B * OH * cdiv(nstrip, rows_pass) * rows_pass;               \
    int64_t per = cdiv(items, 1024);                                                            \
    per = cdiv(per, rows_pass) * rows_pass;                                                     \
    nblk = cdiv(items, per);                                                                    \
    dim3 g((unsigned)nblk, (unsigned)cdiv(C4, lanes));                                          \
    if (it)                                                                                     \
      dw_wgrad_strip_kernel<K_, S_, PW_, true><<<g, 256, 0, st>>>(                               \
          x, dy, H, W, C, OH, OW, nstrip, items, per, lanes, part, bmean, binvstd, bgamma, bbeta, \
          bact, bslope);                                                                        \
    else                                                                                        \
      dw_wgrad_strip_kernel<K_, S_, PW_><<<g, 256, 0, st>>>(x, dy, H, W, C, OH, OW, nstrip,      \
                                                            items, per, lanes, part);           \
  }
  WG_CASE(3, 1, 8) WG_CASE(3, 2, 4) WG_CASE(5, 1, 4) WG_CASE(5, 2, 4)
#undef WG_CASE
  if (int e = check_launch("dw_wgrad")) return e;
  const int64_t tot = (int64_t)k * k * C;
  const int rl = tot >= 64 * 512 ? 64 : 16;
  wgrad_reduce2_kernel<<<(unsigned)cdiv(tot, rl), 256, 0, st>>>(part, nblk, k * k, C, 1, k * k, rl,
                                                                dw);
  return check_launch("dw_wgrad_reduce");
}

extern "C" int jabd_dw_wgrad_f32(const float* x, const float* dy, int32_t B, int32_t H, int32_t W,
                                 int32_t C, int32_t OH, int32_t OW, int32_t k, int32_t stride,
                                 int32_t pad, float* part, float* dw, jabd_stream_t stream) {
  return dw_wgrad(x, dy, B, H, W, C, OH, OW, k, stride, pad, nullptr, nullptr, nullptr, nullptr,
                  0, 0.f, part, dw, stream);
}

extern "C" int jabd_dw_wgrad_bnin_f32(const float* x_bn, const float* dy, int32_t B, int32_t H,
                                      int32_t W, int32_t C, int32_t OH, int32_t OW, int32_t k,
                                      int32_t stride, int32_t pad, const float* mean,
                                      const float* invstd, const float* gamma, const float* beta,
                                      int32_t act, float slope, float* part, float* dw,
                                      jabd_stream_t stream) {
  JABD_REQUIRE(mean, "dw_wgrad_bnin: null mean");
  return dw_wgrad(x_bn, dy, B, H, W, C, OH, OW, k, stride, pad, mean, invstd, gamma, beta, act,
                  slope, part, dw, stream);
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
  scale_bwd_kernel<<<g, 256, 0, st>>>(da, x, scale, HW, C, per, nblk, nullptr, part);
  if (int e = check_launch("scale_bwd")) return e;
  eca_gate_bwd_kernel<<<(unsigned)B, 256, 2 * C * sizeof(float), st>>>(
      part, nblk, C, mean, scale, w1d, k, gate, 1.f / (float)HW, dmean_ws, dw1d_ws);
  if (int e = check_launch("eca_gate_bwd")) return e;
  const int64_t total4 = B * HW * (C / 4);
  scale_add_kernel<<<(unsigned)cdiv(total4, 256), 256, 0, st>>>(da, scale, dmean_ws, HW, C, total4,
                                                                dx);
  if (int e = check_launch("eca_scale_add")) return e;
  eca_w_reduce_kernel<<<1, 64, 0, st>>>(dw1d_ws, (int)B, k, dw1d);
  return check_launch("eca_w_reduce");
}

// The ECA backward without its dx pass: the per-image partials of sum(da * x),
// the gate backward (dmean term [B][C], the Conv1d weight gradient).  The
// caller folds dx = da * scale + dmean_ws into the next consumer
// (jabd_bn_act_bwd_ex_f32's dy transform).
extern "C" int jabd_eca_bwd_terms_f32(const float* da, const float* x, int64_t B, int64_t HW,
                                      int32_t C, const float* scale, const float* mean,
                                      const float* w1d, int32_t k, int32_t gate, float* part,
                                      int32_t nblk, float* dmean_ws, float* dw1d_ws, float* dw1d,
                                      jabd_stream_t stream) {
  JABD_REQUIRE(da && x && scale && mean && w1d && part && dmean_ws && dw1d_ws && dw1d &&
                   C % 4 == 0 && nblk > 0,
               "eca_bwd_terms: bad args");
  hipStream_t st = as_stream(stream);
  const int64_t per = cdiv(HW, nblk);
  scale_bwd_kernel<<<dim3((unsigned)nblk, (unsigned)B), 256, 0, st>>>(da, x, scale, HW, C, per,
                                                                      nblk, nullptr, part);
  if (int e = check_launch("scale_bwd")) return e;
  eca_gate_bwd_kernel<<<(unsigned)B, 256, 2 * C * sizeof(float), st>>>(
      part, nblk, C, mean, scale, w1d, k, gate, 1.f / (float)HW, dmean_ws, dw1d_ws);
  if (int e = check_launch("eca_gate_bwd")) return e;
  eca_w_reduce_kernel<<<1, 64, 0, st>>>(dw1d_ws, (int)B, k, dw1d);
  return check_launch("eca_w_reduce");
}

// The gate half of jabd_eca_bwd_terms_f32 from precomputed sums
// part[b][blk][c] of da * x (e.g. jabd_conv_wgrad_eca_f32's ds, nblk = 1).
extern "C" int jabd_eca_gate_bwd_f32(const float* part, int32_t nblk, int64_t B, int64_t HW,
                                     int32_t C, const float* scale, const float* mean,
                                     const float* w1d, int32_t k, int32_t gate, float* dmean_ws,
                                     float* dw1d_ws, float* dw1d, jabd_stream_t stream) {
  JABD_REQUIRE(part && scale && mean && w1d && dmean_ws && dw1d_ws && dw1d && nblk > 0 && HW > 0,
               "eca_gate_bwd: bad args");
  hipStream_t st = as_stream(stream);
  eca_gate_bwd_kernel<<<(unsigned)B, 256, 2 * C * sizeof(float), st>>>(
      part, nblk, C, mean, scale, w1d, k, gate, 1.f / (float)HW, dmean_ws, dw1d_ws);
  if (int e = check_launch("eca_gate_bwd")) return e;
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

extern "C" int jabd_maxpool_idx_nhwc_f32(const float* x, int32_t B, int32_t H, int32_t W,
                                         int32_t C, int32_t k, int32_t stride, int32_t pad,
                                         float* y, uint8_t* idx, jabd_stream_t stream) {
  JABD_REQUIRE(x && y && idx && B > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && k > 0 &&
                   k * k <= 255 && stride > 0,
               "maxpool_idx: bad args");
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  const int64_t t4 = (int64_t)B * OH * OW * (C / 4);
  JABD_REQUIRE(t4 < ((int64_t)1 << 31) && (int64_t)B * H * W * (C / 4) < ((int64_t)1 << 31),
               "maxpool_idx: too large");
  maxpool_idx4_kernel<<<(unsigned)cdiv(t4, 256), 256, 0, as_stream(stream)>>>(
      x, H, W, C / 4, OH, OW, k, stride, pad, (int)t4, y, reinterpret_cast<uchar4*>(idx));
  return check_launch("maxpool_idx");
}

extern "C" int jabd_maxpool_bwd_idx_f32(const uint8_t* idx, const float* dy, int32_t B, int32_t H,
                                        int32_t W, int32_t C, int32_t k, int32_t stride,
                                        int32_t pad, float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(idx && dy && dx && C % 4 == 0, "maxpool_bwd_idx: bad args");
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  const int64_t t4 = (int64_t)B * H * W * (C / 4);
  JABD_REQUIRE(t4 < ((int64_t)1 << 31), "maxpool_bwd_idx: too large");
  const int C4 = C / 4;
  if ((C4 & (C4 - 1)) == 0 && C4 <= 64 && H <= 65535 && B <= 65535) {
    int c4s = 0;
    while ((1 << c4s) < C4) ++c4s;
    dim3 g((unsigned)cdiv(W, 256 >> c4s), (unsigned)H, (unsigned)B);
    maxpool_bwd_idx4_row_kernel<<<g, 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const uchar4*>(idx), dy, H, W, c4s, OH, OW, k, stride, pad, dx);
    return check_launch("maxpool_bwd_idx");
  }
  maxpool_bwd_idx4_kernel<<<(unsigned)cdiv(t4, 256), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const uchar4*>(idx), dy, H, W, C / 4, OH, OW, k, stride, pad, (int)t4, dx);
  return check_launch("maxpool_bwd_idx");
}

extern "C" int jabd_maxpool_bwd_f32(const float* x, const float* dy, int32_t B, int32_t H,
                                    int32_t W, int32_t C, int32_t k, int32_t stride, int32_t pad,
                                    float* dx, jabd_stream_t stream) {
  JABD_REQUIRE(x && dy && dx, "maxpool_bwd: null");
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  const int64_t total = (int64_t)B * H * W * C;
  if (C % 4 == 0 && total / 4 < ((int64_t)1 << 31) &&
      (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) |
       reinterpret_cast<uintptr_t>(dx)) % 16 == 0) {
    const int t4 = (int)(total / 4);
    maxpool_bwd4_kernel<<<(unsigned)cdiv(t4, 256), 256, 0, as_stream(stream)>>>(
        x, dy, H, W, C / 4, OH, OW, k, stride, pad, t4, dx);
    return check_launch("maxpool_bwd4");
  }
  maxpool_bwd_kernel<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      x, dy, H, W, C, OH, OW, k, stride, pad, total, dx);
  return check_launch("maxpool_bwd");
}
