// A2-A4 attention and head kernels on gfx950: ECA pooling + gate, the CSAF
// non-local block (PSP-pooled keys/values, per-pixel softmax over S bins)
// fused with the FPN's nearest up-sample and lateral add, and the three
// detection heads written straight into the anchor-major output layout.
// All HBM/latency-bound: one pass over each activation, fixed-order sums.
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "conv_args.h"

namespace jabd {

// ---------------------------------------------------------------- ECA
constexpr int kSumThreads = 256;

// part[b][blk][c] = sum over this block's pixels of x[b, pix, c]
__device__ __forceinline__ void channel_sum_body(const float* __restrict__ x, int64_t x_bs,
                                                 int x_ps, int64_t HW, int C, int64_t per_blk,
                                                 int64_t nblk, float* __restrict__ part,
                                                 float* red) {
  const int b = blockIdx.y;
  const int64_t p0 = blockIdx.x * per_blk;
  const int64_t p1 = min(p0 + per_blk, HW);
  const float* xb = x + (int64_t)b * x_bs;
  const int rows = kSumThreads / C > 0 ? kSumThreads / C : 1;
  for (int c0 = 0; c0 < C; c0 += kSumThreads) {
    const int c = c0 + (threadIdx.x % min(C, kSumThreads));
    const int r = threadIdx.x / min(C, kSumThreads);
    const int nrows = C >= kSumThreads ? 1 : rows;
    float s = 0.f;
    if (r < nrows && c < C) {
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      int64_t q = p0 + r;
      for (; q + 3 * nrows < p1; q += 4 * nrows) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s4[u] += xb[(q + u * nrows) * x_ps + c];
      }
      for (; q < p1; q += nrows) s4[0] += xb[q * x_ps + c];
      s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
    __syncthreads();
    if (r < nrows && c < C) red[r * min(C, kSumThreads) + (c - c0)] = s;
    __syncthreads();
    if (threadIdx.x < min(C - c0, kSumThreads)) {
      float t = 0.f;
      for (int q = 0; q < nrows; ++q) t += red[q * min(C, kSumThreads) + threadIdx.x];
      part[((int64_t)b * nblk + blockIdx.x) * C + c0 + threadIdx.x] = t;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kSumThreads) void channel_sum_kernel(
    const float* __restrict__ x, int64_t x_bs, int x_ps, int64_t HW, int C, int64_t per_blk,
    int64_t nblk, float* __restrict__ part) {
  __shared__ float red[kSumThreads];  // [rows][min(C, kSumThreads)]
  channel_sum_body(x, x_bs, x_ps, HW, C, per_blk, nblk, part, red);
}

// Several independent channel sums in one launch (blockIdx.z picks the
// tensor): the head's ECA pools of the three pyramid levels.
struct CsumMulti {
  const float* x[4];
  int64_t x_bs[4], HW[4], per[4], nblk[4];
  int x_ps[4], C[4];
  float* part[4];
};
__global__ __launch_bounds__(kSumThreads) void channel_sum_multi_kernel(const CsumMulti d) {
  __shared__ float red[kSumThreads];
  const int z = blockIdx.z;
  if (blockIdx.x >= d.nblk[z]) return;  // whole workgroup
  channel_sum_body(d.x[z], d.x_bs[z], d.x_ps[z], d.HW[z], d.C[z], d.per[z], d.nblk[z], d.part[z],
                   red);
}

// scale[b][c] = gate( sum_t w[t] * mean[b][c + t - (k-1)/2] )   (zero padded)
// One thread per channel of a block's window [c0 - h, c0 - h + blockDim):
// mean over the partial rows in row order, then the Conv1d over the window
// and the gate for the blockDim - 2h channels whose taps are all inside it.
// Grid (channel windows, B); one barrier.
__global__ __launch_bounds__(256) void eca_gate_kernel(const float* __restrict__ part,
                                                       int64_t nblk, int C, float inv_hw,
                                                       const float* __restrict__ w1d, int k,
                                                       int gate, float* __restrict__ scale,
                                                       float* __restrict__ mean_out) {
  __shared__ float mean[256];
  const int h = (k - 1) / 2;
  const int oc = blockDim.x - 2 * h;  // output channels per block
  const int b = blockIdx.y, t = threadIdx.x;
  const int c = blockIdx.x * oc - h + t;
  float m = 0.f;
  if (c >= 0 && c < C) {
    const float* pb = part + (int64_t)b * nblk * C + c;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // 4 loads in flight, fixed order
    int64_t r = 0;
    for (; r + 3 < nblk; r += 4) {
      s0 += pb[r * C];
      s1 += pb[(r + 1) * C];
      s2 += pb[(r + 2) * C];
      s3 += pb[(r + 3) * C];
    }
    for (; r < nblk; ++r) s0 += pb[r * C];
    m = ((s0 + s1) + (s2 + s3)) * inv_hw;
  }
  mean[t] = m;  // zero outside [0, C): the Conv1d's zero padding
  __syncthreads();
  if (t >= h && t < h + oc && c < C) {
    float y = 0.f;
    for (int q = 0; q < k; ++q) y = fmaf(w1d[q], mean[t - h + q], y);
    const float g = gate == ACT_SIGMOID ? 1.f / (1.f + expf(-y))
                                        : fminf(fmaxf(y + 3.f, 0.f), 6.f) * (1.f / 6.f);
    scale[(int64_t)b * C + c] = g;
    if (mean_out) mean_out[(int64_t)b * C + c] = m;
  }
}

// Same result for C % 4 == 0 with the row reduction spread over the whole
// workgroup: thread (row group rg, channel quad q) sums rows rg, rg + RG, ...
// with float4 loads (8 in flight), the RG partial quads are summed in row-group
// order through LDS (fixed order: deterministic), then the Conv1d + gate.  A
// window covers channels [cs - 4, cs + 248 + 4) (k <= 9), cs = 248 * blockIdx.x.
// The one-thread-per-channel form walks all nblk rows serially (up to 1024
// dependent L2 round trips for the 512^2 gates).
constexpr int kGateOC = 248;
__device__ __forceinline__ void eca_gate4_body(const float* __restrict__ part, int nblk, int C,
                                               float inv_hw, const float* __restrict__ w1d,
                                               int k, int gate, float* __restrict__ scale,
                                               float* __restrict__ mean_out, float4* red,
                                               float* mean) {
  const int b = blockIdx.y, t = threadIdx.x;
  const int cs = blockIdx.x * kGateOC;
  const int ce = min(C, cs + kGateOC);
  const int nq = (ce - cs + 8) >> 2;  // quads of [cs - 4, ce + 4)
  const int RG = 256 / nq;
  const int rg = t / nq, q = t - rg * nq;
  const int c = cs - 4 + 4 * q;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rg < RG && c >= 0 && c < C) {
    const float* pb = part + (int64_t)b * nblk * C + c;
    float4 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    int r = rg;
    for (; r + 7 * RG < nblk; r += 8 * RG) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(pb + (int64_t)(r + u * RG) * C);
        a[u].x += v.x; a[u].y += v.y; a[u].z += v.z; a[u].w += v.w;
      }
    }
    for (; r < nblk; r += RG) {
      const float4 v = *reinterpret_cast<const float4*>(pb + (int64_t)r * C);
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s.x += a[u].x; s.y += a[u].y; s.z += a[u].z; s.w += a[u].w;
    }
  }
  red[t] = s;
  __syncthreads();
  if (t < nq) {
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int g = 0; g < RG; ++g) {
      const float4 v = red[g * nq + t];
      m.x += v.x; m.y += v.y; m.z += v.z; m.w += v.w;
    }
    // zero outside [0, C): the Conv1d's zero padding
    const bool in = c >= 0 && c < C;
    mean[4 * t + 0] = in ? m.x * inv_hw : 0.f;
    mean[4 * t + 1] = in ? m.y * inv_hw : 0.f;
    mean[4 * t + 2] = in ? m.z * inv_hw : 0.f;
    mean[4 * t + 3] = in ? m.w * inv_hw : 0.f;
  }
  __syncthreads();
  const int h = (k - 1) / 2;
  const int co = cs + t;
  if (co < ce) {
    float y = 0.f;
    for (int j = 0; j < k; ++j) y = fmaf(w1d[j], mean[t + 4 - h + j], y);
    const float g = gate == ACT_SIGMOID ? 1.f / (1.f + expf(-y))
                                        : fminf(fmaxf(y + 3.f, 0.f), 6.f) * (1.f / 6.f);
    scale[(int64_t)b * C + co] = g;
    if (mean_out) mean_out[(int64_t)b * C + co] = mean[t + 4];
  }
}

__global__ __launch_bounds__(256) void eca_gate4_kernel(const float* __restrict__ part,
                                                        int nblk, int C, float inv_hw,
                                                        const float* __restrict__ w1d, int k,
                                                        int gate, float* __restrict__ scale,
                                                        float* __restrict__ mean_out) {
  __shared__ float4 red[256];
  __shared__ float mean[kGateOC + 8];
  eca_gate4_body(part, nblk, C, inv_hw, w1d, k, gate, scale, mean_out, red, mean);
}

// Several gates in one launch (blockIdx.z picks the tensor).
struct GateMulti {
  const float* part[4];
  const float* w1d[4];
  float* scale[4];
  int nblk[4], C[4], k[4];
  float inv_hw[4];
  int gate;
};
__global__ __launch_bounds__(256) void eca_gate4_multi_kernel(const GateMulti d) {
  __shared__ float4 red[256];
  __shared__ float mean[kGateOC + 8];
  const int z = blockIdx.z;
  if ((int)blockIdx.x * kGateOC >= d.C[z]) return;  // whole workgroup
  eca_gate4_body(d.part[z], d.nblk[z], d.C[z], d.inv_hw[z], d.w1d[z], d.k[z], d.gate,
                 d.scale[z], nullptr, red, mean);
}

// First level of the ECA pool for many partial rows: block (s, b) sums rows
// [s*R, min(nblk, (s+1)*R)) of part[b] in row order into out[b][s] — a
// deterministic two-level sum that spreads the read of nblk x C partials over
// nsplit x B workgroups instead of B.
__global__ __launch_bounds__(256) void partial_reduce_kernel(const float* __restrict__ part,
                                                             int nblk, int C, int R,
                                                             float* __restrict__ out) {
  const int s = blockIdx.x, b = blockIdx.y, nsplit = gridDim.x;
  const int r0 = s * R, r1 = min(nblk, r0 + R);
  const float* pb = part + (int64_t)b * nblk * C;
  float* ob = out + ((int64_t)b * nsplit + s) * C;
  if ((C & 3) == 0) {
    const int C4 = C >> 2;
    for (int c4 = threadIdx.x; c4 < C4; c4 += blockDim.x) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = r0; r < r1; ++r) {
        const float4 v = reinterpret_cast<const float4*>(pb + (int64_t)r * C)[c4];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      reinterpret_cast<float4*>(ob)[c4] = a;
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float a = 0.f;
      for (int r = r0; r < r1; ++r) a += pb[(int64_t)r * C + c];
      ob[c] = a;
    }
  }
}

// ---------------------------------------------------------------- NLM
// F.interpolate(mode='nearest', size=...) source index (ATen nearest_idx).
__device__ __forceinline__ int nearest_src(int dst, int in, int out) {
  if (out == in) return dst;
  if (out == 2 * in) return dst >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}

struct NlmSizes {
  int n;
  int v[8];
};

// kv[b][pix][0:CH] = f_key(x), [CH:2CH] = f_value(x) on the SOURCE grid (the
// nearest up-sample only repeats source pixels, so projecting before the
// gather gives identical values at 1/4 of the work).
template <int CH>
__global__ __launch_bounds__(256) void nlm_kv_kernel(const float* __restrict__ src, int64_t src_bs,
                                                     int src_ps, int hsws, int C,
                                                     const float* __restrict__ wk,
                                                     const float* __restrict__ bk,
                                                     const float* __restrict__ wv,
                                                     const float* __restrict__ bv,
                                                     float* __restrict__ kv) {
  extern __shared__ float sw[];  // [2CH][C]
  for (int t = threadIdx.x; t < CH * C; t += blockDim.x) {
    sw[t] = wk[t];
    sw[CH * C + t] = wv[t];
  }
  __syncthreads();
  const int b = blockIdx.y;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= hsws) return;
  const float* xp = src + (int64_t)b * src_bs + (int64_t)pix * src_ps;
  float o[2 * CH];
#pragma unroll
  for (int q = 0; q < CH; ++q) { o[q] = bk[q]; o[CH + q] = bv[q]; }
  for (int c = 0; c < C; c += 4) {
    const float4 x = *reinterpret_cast<const float4*>(xp + c);
#pragma unroll
    for (int q = 0; q < 2 * CH; ++q) {
      const float* w = sw + q * C + c;
      o[q] = fmaf(w[0], x.x, o[q]);
      o[q] = fmaf(w[1], x.y, o[q]);
      o[q] = fmaf(w[2], x.z, o[q]);
      o[q] = fmaf(w[3], x.w, o[q]);
    }
  }
  float* dst = kv + ((int64_t)b * hsws + pix) * (2 * CH);
#pragma unroll
  for (int q = 0; q < 2 * CH; ++q) dst[q] = o[q];
}

// One workgroup per (bin s, image b): adaptive-avg-pool bin of the
// up-sampled kv map -> kpool/vpool [B][S][CH].
template <int CH>
__global__ __launch_bounds__(256) void nlm_pool_kernel(const float* __restrict__ kv, int hs, int ws,
                                                       int h, int w, const NlmSizes sizes, int S,
                                                       float* __restrict__ kpool,
                                                       float* __restrict__ vpool) {
  const int s = blockIdx.x, b = blockIdx.y;
  int base = 0, lvl = 0;
  for (; lvl < sizes.n; ++lvl) {
    const int n = sizes.v[lvl] * sizes.v[lvl];
    if (s < base + n) break;
    base += n;
  }
  const int sz = sizes.v[lvl];
  const int bi = (s - base) / sz, bj = (s - base) % sz;
  const int h0 = (bi * h) / sz, h1 = ((bi + 1) * h + sz - 1) / sz;  // AdaptiveAvgPool2d bins
  const int w0 = (bj * w) / sz, w1 = ((bj + 1) * w + sz - 1) / sz;
  const int rw = w1 - w0;
  const int npix = (h1 - h0) * rw;
  const float* kb = kv + (int64_t)b * hs * ws * (2 * CH);
  float a[2 * CH];
#pragma unroll
  for (int q = 0; q < 2 * CH; ++q) a[q] = 0.f;
  for (int p = threadIdx.x; p < npix; p += blockDim.x) {
    const int i = h0 + p / rw, jx = w0 + p % rw;
    const float* v = kb + ((int64_t)nearest_src(i, hs, h) * ws + nearest_src(jx, ws, w)) * (2 * CH);
#pragma unroll
    for (int q = 0; q < 2 * CH; ++q) a[q] += v[q];
  }
  // fixed-shape reduction: wave butterflies, then the 4 wave sums in order
  // (a 256-long serial LDS sum per channel was most of this kernel's time)
#pragma unroll
  for (int q = 0; q < 2 * CH; ++q)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) a[q] += __shfl_xor(a[q], m);
  __shared__ float red[4][2 * CH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane < 2 * CH) {
    float v = a[0];
#pragma unroll
    for (int q = 1; q < 2 * CH; ++q) v = lane == q ? a[q] : v;
    red[wave][lane] = v;
  }
  __syncthreads();
  if (threadIdx.x < 2 * CH) {
    const int q = threadIdx.x;
    const float t = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
    const float avg = t / (float)npix;
    if (q < CH) kpool[((int64_t)b * S + s) * CH + q] = avg;
    else vpool[((int64_t)b * S + s) * CH + (q - CH)] = avg;
  }
}

// Per pixel: out = lateral + (W · softmax_S(q·K) V + bW + x).
// A quad of lanes per pixel: lane r of the quad computes q[r] (then the quad
// exchanges them), scores and softmax partials for every 4th bin s = r, r+4,
// ... (max, then exp-sum and the V-weighted sum, rescaled to the quad's max
// and combined by butterfly), and writes every 4th float4 channel group of
// the output.  One lane per pixel ran the 225-bin chain serially at two waves
// per SIMD (latency-bound, ~10% of its HBM floor).
template <int CH, int PX>
__global__ __launch_bounds__(256) void nlm_apply_kernel(
    const float* __restrict__ src, int64_t src_bs, int src_ps, int hs, int ws, int C, int h,
    int w, const float* __restrict__ wq, const float* __restrict__ bq,
    const float* __restrict__ kpool, const float* __restrict__ vpool, int S,
    const float* __restrict__ wW, const float* __restrict__ bW, const float* __restrict__ lateral,
    float* __restrict__ out, float* __restrict__ q_out, float* __restrict__ ctx_out) {
  // PX pixels per quad: every K / V bin read from LDS serves PX pixels (the
  // bin loops were LDS-read bound at one pixel per quad).
  static_assert(CH == 4, "one q channel per quad lane");
  extern __shared__ float sm[];  // K [S][CH], V [S][CH], wq [CH][C], wW [C][CH], bW [C]
  const int b = blockIdx.y;
  float* sK = sm;
  float* sV = sK + S * CH;
  float* sWq = sV + S * CH;
  float* sWW = sWq + CH * C;
  float* sbW = sWW + C * CH;
  for (int t = threadIdx.x; t < S * CH; t += blockDim.x) {
    sK[t] = kpool[(int64_t)b * S * CH + t];
    sV[t] = vpool[(int64_t)b * S * CH + t];
  }
  for (int t = threadIdx.x; t < CH * C; t += blockDim.x) {
    sWq[t] = wq[t];
    sWW[t] = wW[t];
  }
  for (int t = threadIdx.x; t < C; t += blockDim.x) sbW[t] = bW[t];
  __syncthreads();
  const int r = threadIdx.x & 3;
  const int qb = threadIdx.x & ~3;  // quad base lane
  // quad's pixels: pix0 + i * 64 (consecutive quads -> consecutive pixels)
  const int pix0 = blockIdx.x * (blockDim.x >> 2) * PX + (threadIdx.x >> 2);
  int pix[PX];
  bool pv[PX];
  const float* xp[PX];
  float q[PX][CH];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    pix[i] = pix0 + i * (blockDim.x >> 2);
    pv[i] = pix[i] < h * w;
    const int pc = pv[i] ? pix[i] : 0;  // the quad stays whole for the shuffles
    const int yy = pc / w, xx = pc - yy * w;
    xp[i] = src + (int64_t)b * src_bs +
            ((int64_t)nearest_src(yy, hs, h) * ws + nearest_src(xx, ws, w)) * src_ps;
    float qr = bq[r];
    for (int c = 0; c < C; c += 4) {
      const float4 x = *reinterpret_cast<const float4*>(xp[i] + c);
      const float* wr = sWq + r * C + c;
      qr = fmaf(wr[0], x.x, qr);
      qr = fmaf(wr[1], x.y, qr);
      qr = fmaf(wr[2], x.z, qr);
      qr = fmaf(wr[3], x.w, qr);
    }
#pragma unroll
    for (int o = 0; o < CH; ++o) q[i][o] = __shfl(qr, (qb + o) & 63);
  }
  const float4* K4 = reinterpret_cast<const float4*>(sK);
  const float4* V4 = reinterpret_cast<const float4*>(sV);
  float mx[PX];
#pragma unroll
  for (int i = 0; i < PX; ++i) mx[i] = -INFINITY;
#pragma unroll 4
  for (int s = r; s < S; s += 4) {
    const float4 k = K4[s];
#pragma unroll
    for (int i = 0; i < PX; ++i)
      mx[i] = fmaxf(mx[i], fmaf(q[i][0], k.x, fmaf(q[i][1], k.y, fmaf(q[i][2], k.z, q[i][3] * k.w))));
  }
  float den[PX], cx[PX][CH];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    den[i] = 0.f;
#pragma unroll
    for (int o = 0; o < CH; ++o) cx[i][o] = 0.f;
  }
#pragma unroll 4
  for (int s = r; s < S; s += 4) {
    const float4 k = K4[s], v = V4[s];
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      const float e = __expf(
          fmaf(q[i][0], k.x, fmaf(q[i][1], k.y, fmaf(q[i][2], k.z, q[i][3] * k.w))) - mx[i]);
      den[i] += e;
      cx[i][0] = fmaf(e, v.x, cx[i][0]);
      cx[i][1] = fmaf(e, v.y, cx[i][1]);
      cx[i][2] = fmaf(e, v.z, cx[i][2]);
      cx[i][3] = fmaf(e, v.w, cx[i][3]);
    }
  }
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    // combine the quad's partials at the quad max (fixed butterfly order)
    float M = fmaxf(mx[i], __shfl_xor(mx[i], 1));
    M = fmaxf(M, __shfl_xor(M, 2));
    const float sc = mx[i] == -INFINITY ? 0.f : __expf(mx[i] - M);  // lane with no bins (S < 4)
    den[i] *= sc;
#pragma unroll
    for (int o = 0; o < CH; ++o) cx[i][o] *= sc;
#pragma unroll
    for (int m = 1; m <= 2; m <<= 1) {
      den[i] += __shfl_xor(den[i], m);
#pragma unroll
      for (int o = 0; o < CH; ++o) cx[i][o] += __shfl_xor(cx[i][o], m);
    }
  }
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    if (!pv[i]) continue;
    const float inv = 1.f / den[i];
    float c4[CH];
#pragma unroll
    for (int o = 0; o < CH; ++o) c4[o] = cx[i][o] * inv;
    if (q_out && r == 0) {  // training: saved for the backward
      const int64_t mq = ((int64_t)b * h * w + pix[i]) * CH;
      *reinterpret_cast<float4*>(q_out + mq) = make_float4(q[i][0], q[i][1], q[i][2], q[i][3]);
      *reinterpret_cast<float4*>(ctx_out + mq) = make_float4(c4[0], c4[1], c4[2], c4[3]);
    }
    const int64_t opix = ((int64_t)b * h * w + pix[i]) * C;
    for (int c = 4 * r; c < C; c += 16) {
      const float4 x = *reinterpret_cast<const float4*>(xp[i] + c);
      const float4 lt = lateral ? *reinterpret_cast<const float4*>(lateral + opix + c)
                                : make_float4(0.f, 0.f, 0.f, 0.f);  // standalone NLM
      float v[4] = {x.x, x.y, x.z, x.w};
      float lv[4] = {lt.x, lt.y, lt.z, lt.w};
      float rr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = sbW[c + e];
#pragma unroll
        for (int o = 0; o < CH; ++o) a = fmaf(sWW[(c + e) * CH + o], c4[o], a);
        rr[e] = lv[e] + (a + v[e]);
      }
      *reinterpret_cast<float4*>(out + opix + c) = make_float4(rr[0], rr[1], rr[2], rr[3]);
    }
  }
}

// ---------------------------------------------------------------- heads
constexpr int kHeadOut = 32;  // 8 bbox + 4 class + 20 landmark channels

__global__ __launch_bounds__(256) void heads_kernel(const float* __restrict__ x, int64_t x_bs,
                                                    int x_ps, int HW, int C,
                                                    const float* __restrict__ wt,
                                                    const float* __restrict__ bias, int64_t A,
                                                    int64_t a_off, int softmax,
                                                    float* __restrict__ loc,
                                                    float* __restrict__ conf,
                                                    float* __restrict__ landm) {
  // Weights [32][C] are read at wave-uniform addresses (scalar loads, SGPR
  // FMA operands), 16 outputs x 4 channels at a time; the empty asm with a
  // memory clobber keeps the compiler from hoisting all 32*C of them into the
  // scalar file.  An LDS copy costs a broadcast ds_read per 4 FMAs, and the
  // LDS port was this kernel's bound.
  const int b = blockIdx.y;
  const int64_t pix0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool pv = pix0 < HW;
  const int64_t pix = pv ? pix0 : 0;
  const float* xp = x + (int64_t)b * x_bs + pix * x_ps;
  float o[kHeadOut];
#pragma unroll
  for (int n = 0; n < kHeadOut; ++n) o[n] = bias[n];
  // the pixel's channels in chunks of kHeadChunk float4, all loads of a chunk
  // issued before its FMAs: one HBM round trip per 32 channels instead of one
  // per 4 (a 40-channel pixel was 10 dependent load -> FMA steps)
  constexpr int kHeadChunk = 8;
#pragma unroll 1
  for (int c0 = 0; c0 < C; c0 += 4 * kHeadChunk) {
    float4 xv[kHeadChunk];
#pragma unroll
    for (int q = 0; q < kHeadChunk; ++q)
      xv[q] = c0 + 4 * q < C ? *reinterpret_cast<const float4*>(xp + c0 + 4 * q)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < kHeadChunk; ++q) {
      const int c = c0 + 4 * q;
      if (c >= C) break;  // wave-uniform
      const float4 v = xv[q];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int n = 16 * h; n < 16 * h + 16; ++n) {
          const float4 wr = *reinterpret_cast<const float4*>(wt + n * C + c);
          o[n] = fmaf(wr.x, v.x, o[n]);
          o[n] = fmaf(wr.y, v.y, o[n]);
          o[n] = fmaf(wr.z, v.z, o[n]);
          o[n] = fmaf(wr.w, v.w, o[n]);
        }
      }
    }
  }
  float c0 = o[8], c1 = o[9], c2 = o[10], c3 = o[11];
  if (softmax) {  // F.softmax over each anchor's 2 logits
    float m = fmaxf(c0, c1), e0 = expf(c0 - m), e1 = expf(c1 - m), s = e0 + e1;
    c0 = e0 / s; c1 = e1 / s;
    m = fmaxf(c2, c3); e0 = expf(c2 - m); e1 = expf(c3 - m); s = e0 + e1;
    c2 = e0 / s; c3 = e1 / s;
  }
  o[8] = c0; o[9] = c1; o[10] = c2; o[11] = c3;
  // The wave's 64 positions own contiguous runs of loc (8 floats each), conf
  // (4) and landm (20): transpose through wave-private LDS so every store
  // instruction writes consecutive 16 B per lane (a per-position store of 20
  // landmark floats is 20 instructions at an 80 B lane stride).
  constexpr int P = kHeadOut + 4;  // row pitch (float4-aligned)
  __shared__ float4 st4[4][64 * P / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4* sw = st4[wave];
#pragma unroll
  for (int q = 0; q < kHeadOut / 4; ++q)
    sw[lane * (P / 4) + q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region
  const int64_t p0 = pix0 - lane;
  const int npx = (int)min<int64_t>(64, HW - p0);
  if (npx <= 0) return;
  const int64_t row0 = (int64_t)b * A + a_off + p0 * 2;  // 2 anchors per position
  float4* lp = reinterpret_cast<float4*>(loc + row0 * 4);
  float4* cp = reinterpret_cast<float4*>(conf + row0 * 2);
  float4* mp = reinterpret_cast<float4*>(landm + row0 * 10);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = k * 64 + lane;
    if (i < 2 * npx) lp[i] = sw[(i >> 1) * (P / 4) + (i & 1)];
  }
  if (lane < npx) cp[lane] = sw[lane * (P / 4) + 2];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int i = k * 64 + lane;
    const int px = i / 5;
    if (i < 5 * npx) mp[i] = sw[px * (P / 4) + 3 + (i - 5 * px)];
  }
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_channel_sum_f32(const float* x, int64_t x_bs, int32_t x_ps, int64_t B,
                                    int64_t HW, int64_t C, int64_t nblk, float* part,
                                    jabd_stream_t stream) {
  JABD_REQUIRE(x && part && B > 0 && HW > 0 && C > 0 && nblk > 0, "channel_sum: bad args");
  const int64_t per = cdiv(HW, nblk);
  const int cw = (int)(C < kSumThreads ? C : kSumThreads);
  const int rows = C >= kSumThreads ? 1 : kSumThreads / (int)C;
  dim3 g((unsigned)nblk, (unsigned)B);
  (void)rows;
  (void)cw;
  channel_sum_kernel<<<g, kSumThreads, 0, as_stream(stream)>>>(x, x_bs, x_ps, HW, (int)C, per,
                                                               nblk, part);
  return check_launch("channel_sum");
}

// Up to 4 channel sums and their ECA gates in two launches (the head's
// per-level pools: nets/retinaface_r.py:219-224 applied to the three FPN
// inputs, or to the three SSH inputs).  Arrays of n entries; every tensor
// has B images, C % 4 == 0, k <= 9; part[i] holds B x nblk[i] x C[i] floats.
extern "C" int jabd_eca_pool_gate_multi_f32(int32_t n, int64_t B, const float* const* x,
                                            const int64_t* x_bs, const int32_t* x_ps,
                                            const int64_t* HW, const int32_t* C,
                                            const int64_t* nblk, float* const* part,
                                            const float* const* w1d, const int32_t* k,
                                            int32_t gate, float* const* scale,
                                            jabd_stream_t stream) {
  JABD_REQUIRE(n >= 1 && n <= 4 && B > 0 && B <= 65535 && x && x_bs && x_ps && HW && C && nblk &&
                   part && w1d && k && scale,
               "eca_pool_gate_multi: bad args");
  JABD_REQUIRE(gate == ACT_SIGMOID || gate == ACT_HSIGMOID, "eca_pool_gate_multi: gate");
  CsumMulti cs{};
  GateMulti gm{};
  int64_t maxblk = 1, maxc = 1;
  for (int i = 0; i < n; ++i) {
    JABD_REQUIRE(x[i] && part[i] && w1d[i] && scale[i] && C[i] > 0 && C[i] % 4 == 0 &&
                     HW[i] > 0 && nblk[i] > 0 && k[i] > 0 && k[i] <= 9 && (k[i] & 1) &&
                     nblk[i] * C[i] < ((int64_t)1 << 31),
                 "eca_pool_gate_multi: bad entry %d", i);
    cs.x[i] = x[i];
    cs.x_bs[i] = x_bs[i];
    cs.x_ps[i] = x_ps[i];
    cs.HW[i] = HW[i];
    cs.C[i] = C[i];
    cs.nblk[i] = nblk[i];
    cs.per[i] = cdiv(HW[i], nblk[i]);
    cs.part[i] = part[i];
    gm.part[i] = part[i];
    gm.w1d[i] = w1d[i];
    gm.scale[i] = scale[i];
    gm.nblk[i] = (int)nblk[i];
    gm.C[i] = C[i];
    gm.k[i] = k[i];
    gm.inv_hw[i] = 1.f / (float)HW[i];
    maxblk = std::max<int64_t>(maxblk, nblk[i]);
    maxc = std::max<int64_t>(maxc, C[i]);
  }
  gm.gate = gate;
  hipStream_t st = as_stream(stream);
  channel_sum_multi_kernel<<<dim3((unsigned)maxblk, (unsigned)B, (unsigned)n), kSumThreads, 0,
                             st>>>(cs);
  if (int e = check_launch("channel_sum_multi")) return e;
  eca_gate4_multi_kernel<<<dim3((unsigned)cdiv(maxc, kGateOC), (unsigned)B, (unsigned)n), 256, 0,
                           st>>>(gm);
  return check_launch("eca_gate_multi");
}

extern "C" int jabd_partial_reduce_f32(const float* part, int64_t nblk, int64_t B, int64_t C,
                                       int64_t nsplit, float* out, jabd_stream_t stream) {
  JABD_REQUIRE(part && out && B > 0 && C > 0 && nblk > 0 && nsplit > 0 && nsplit <= nblk &&
                   nblk * C < ((int64_t)1 << 31) && B <= 65535,
               "partial_reduce: bad args");
  const int64_t R = cdiv(nblk, nsplit);
  dim3 g((unsigned)nsplit, (unsigned)B);
  const int threads = C >= 1024 ? 256 : (int)std::max<int64_t>(64, cdiv(cdiv(C, 4), 64) * 64);
  partial_reduce_kernel<<<g, threads, 0, as_stream(stream)>>>(part, (int)nblk, (int)C, (int)R,
                                                             out);
  return check_launch("partial_reduce");
}

extern "C" int jabd_eca_gate_f32(const float* part, int64_t nblk, int64_t B, int64_t C,
                                 int64_t hw, const float* w1d, int32_t k, int32_t gate,
                                 float* scale, float* mean_out, jabd_stream_t stream) {
  JABD_REQUIRE(part && w1d && scale && B > 0 && C > 0 && hw > 0 && k > 0 && (k & 1),
               "eca_gate: bad args");
  JABD_REQUIRE(gate == ACT_SIGMOID || gate == ACT_HSIGMOID, "eca_gate: gate must be (h)sigmoid");
  JABD_REQUIRE(C * sizeof(float) <= 64 * 1024, "eca_gate: C too large");
  JABD_REQUIRE(k <= 31, "eca_gate: k too large");
  if (C % 4 == 0 && k <= 9 && nblk * C < ((int64_t)1 << 31) && B <= 65535) {
    dim3 g4((unsigned)cdiv(C, kGateOC), (unsigned)B);
    eca_gate4_kernel<<<g4, 256, 0, as_stream(stream)>>>(part, (int)nblk, (int)C,
                                                       1.f / (float)hw, w1d, k, gate, scale,
                                                       mean_out);
    return check_launch("eca_gate");
  }
  const int oc = 256 - 2 * ((k - 1) / 2);
  dim3 g((unsigned)cdiv(C, oc), (unsigned)B);
  eca_gate_kernel<<<g, 256, 0, as_stream(stream)>>>(part, nblk, (int)C, 1.f / (float)hw, w1d, k,
                                                    gate, scale, mean_out);
  return check_launch("eca_gate");
}

extern "C" int jabd_nlm_pool_f32(const float* src, int64_t src_bs, int32_t src_ps, int32_t B,
                                 int32_t hs, int32_t ws, int32_t C, int32_t h, int32_t w,
                                 const float* wk, const float* bk, const float* wv,
                                 const float* bv, int32_t ch, const int32_t* sizes,
                                 int32_t nsizes, float* kpool, float* vpool, float* kv_ws,
                                 jabd_stream_t stream) {
  JABD_REQUIRE(src && wk && bk && wv && bv && sizes && kpool && vpool && kv_ws,
               "nlm_pool: null pointer");
  JABD_REQUIRE(ch == 4, "nlm_pool: only ch=4 (the JABD NLM) is built");
  JABD_REQUIRE(C > 0 && C % 4 == 0 && src_ps % 4 == 0, "nlm_pool: C must be a multiple of 4");
  JABD_REQUIRE(nsizes > 0 && nsizes <= 8, "nlm_pool: nsizes");
  NlmSizes sz;
  sz.n = nsizes;
  int S = 0;
  for (int i = 0; i < 8; ++i) {
    sz.v[i] = i < nsizes ? sizes[i] : 0;
    if (i < nsizes) {
      JABD_REQUIRE(sizes[i] > 0, "nlm_pool: bad PSP size");
      S += sizes[i] * sizes[i];
    }
  }
  hipStream_t st = as_stream(stream);
  const size_t smem = 2 * (size_t)ch * C * sizeof(float);
  JABD_REQUIRE(smem <= 64 * 1024, "nlm_pool: C too large");
  dim3 g1((unsigned)cdiv((int64_t)hs * ws, 256), (unsigned)B);
  nlm_kv_kernel<4><<<g1, 256, smem, st>>>(src, src_bs, src_ps, hs * ws, C, wk, bk, wv, bv, kv_ws);
  if (int e = check_launch("nlm_kv")) return e;
  dim3 g2((unsigned)S, (unsigned)B);
  nlm_pool_kernel<4><<<g2, 256, 0, st>>>(kv_ws, hs, ws, h, w, sz, S, kpool, vpool);
  return check_launch("nlm_pool");
}

extern "C" int jabd_nlm_apply_f32(const float* src, int64_t src_bs, int32_t src_ps, int32_t B,
                                  int32_t hs, int32_t ws, int32_t C, int32_t h, int32_t w,
                                  const float* wq, const float* bq, const float* kpool,
                                  const float* vpool, int32_t S, int32_t ch, const float* wW,
                                  const float* bW, const float* lateral, float* out,
                                  float* q_out, float* ctx_out, jabd_stream_t stream) {
  JABD_REQUIRE(src && wq && bq && kpool && vpool && wW && bW && out, "nlm_apply: null pointer");
  JABD_REQUIRE(ch == 4, "nlm_apply: only ch=4 (the JABD NLM) is built");
  JABD_REQUIRE(C > 0 && C % 4 == 0 && src_ps % 4 == 0 && S > 0, "nlm_apply: bad sizes");
  const size_t smem = (2 * (size_t)S * ch + 2 * (size_t)ch * C + C) * sizeof(float);
  JABD_REQUIRE(smem <= 64 * 1024, "nlm_apply: LDS %zu > 64KiB", smem);
  // JABD_NLM_PX=1: one pixel per quad (A/B)
  static int px = -1;
  if (px < 0) {
    const char* e = getenv("JABD_NLM_PX");
    px = e && e[0] == '1' ? 1 : 2;
  }
  if (px == 2) {
    dim3 g((unsigned)cdiv((int64_t)h * w, 128), (unsigned)B);  // a quad of lanes per 2 pixels
    nlm_apply_kernel<4, 2><<<g, 256, smem, as_stream(stream)>>>(src, src_bs, src_ps, hs, ws, C, h,
                                                                w, wq, bq, kpool, vpool, S, wW, bW,
                                                                lateral, out, q_out, ctx_out);
  } else {
    dim3 g((unsigned)cdiv((int64_t)h * w, 64), (unsigned)B);  // a quad of lanes per pixel
    nlm_apply_kernel<4, 1><<<g, 256, smem, as_stream(stream)>>>(src, src_bs, src_ps, hs, ws, C, h,
                                                                w, wq, bq, kpool, vpool, S, wW, bW,
                                                                lateral, out, q_out, ctx_out);
  }
  return check_launch("nlm_apply");
}

namespace jabd {
__global__ void heads_scatter_kernel(const float4* __restrict__ y, int64_t HW, int64_t A,
                                     int64_t a_off, int softmax, float4* __restrict__ loc,
                                     float4* __restrict__ conf, float4* __restrict__ landm);
}

extern "C" int jabd_heads_scatter_f32(const float* y, int32_t B, int64_t HW, int64_t A,
                                      int64_t a_off, int32_t softmax, float* loc, float* conf,
                                      float* landm, jabd_stream_t stream) {
  JABD_REQUIRE(y && loc && conf && landm && B > 0 && HW > 0, "heads_scatter: bad args");
  JABD_REQUIRE(A % 2 == 0 && a_off % 2 == 0 && a_off + 2 * HW <= A, "heads_scatter: anchor range");
  JABD_REQUIRE(((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(loc) |
                 reinterpret_cast<uintptr_t>(conf) | reinterpret_cast<uintptr_t>(landm)) & 15) == 0,
               "heads_scatter: buffers must be 16-byte aligned");
  dim3 g((unsigned)cdiv(HW * 8, 256), (unsigned)B);
  heads_scatter_kernel<<<g, 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const float4*>(y), HW, A, a_off, softmax, reinterpret_cast<float4*>(loc),
      reinterpret_cast<float4*>(conf), reinterpret_cast<float4*>(landm));
  return check_launch("heads_scatter");
}

extern "C" int jabd_heads_f32(const float* x, int64_t x_bs, int32_t x_ps, int32_t B, int32_t HW,
                              int32_t C, const float* wt, const float* bias, int64_t A,
                              int64_t a_off, int32_t softmax, float* loc, float* conf,
                              float* landm, jabd_stream_t stream) {
  JABD_REQUIRE(x && wt && bias && loc && conf && landm, "heads: null pointer");
  JABD_REQUIRE(C % 4 == 0 && x_ps % 4 == 0, "heads: C and pixel stride must be multiples of 4");
  JABD_REQUIRE(a_off + 2 * (int64_t)HW <= A, "heads: anchor range out of bounds");
  dim3 g((unsigned)cdiv(HW, 256), (unsigned)B);
  heads_kernel<<<g, 256, 0, as_stream(stream)>>>(
      x, x_bs, x_ps, HW, C, wt, bias, A, a_off, softmax, loc, conf, landm);
  return check_launch("heads");
}

namespace jabd {
// One thread per (position, float4 of the 32 head channels): q 0-1 loc (the
// position's 2 anchor rows), q 2 conf (softmax per anchor pair), q 3-7 landm.
// A and a_off are even, so every destination float4 is 16-byte aligned.
__global__ __launch_bounds__(256) void heads_scatter_kernel(const float4* __restrict__ y,
                                                            int64_t HW, int64_t A,
                                                            int64_t a_off, int softmax,
                                                            float4* __restrict__ loc,
                                                            float4* __restrict__ conf,
                                                            float4* __restrict__ landm) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= HW * 8) return;
  const int64_t p = i >> 3;
  const int q = (int)(i & 7);
  float4 v = y[((int64_t)b * HW) * 8 + i];
  const int64_t row0 = (int64_t)b * A + a_off + 2 * p;  // the position's first anchor row
  if (q < 2) {
    loc[row0 + q] = v;
  } else if (q == 2) {
    if (softmax) {  // F.softmax over each anchor's 2 logits, as heads_kernel
      float m = fmaxf(v.x, v.y), e0 = expf(v.x - m), e1 = expf(v.y - m), s = e0 + e1;
      v.x = e0 / s; v.y = e1 / s;
      m = fmaxf(v.z, v.w); e0 = expf(v.z - m); e1 = expf(v.w - m); s = e0 + e1;
      v.z = e0 / s; v.w = e1 / s;
    }
    conf[row0 >> 1] = v;
  } else {
    landm[(row0 >> 1) * 5 + (q - 3)] = v;
  }
}

// torchvision resnet50 stem maxpool (F.max_pool2d(3, 2, 1)) on NHWC, float4 lanes.
__global__ void maxpool_kernel(const float* __restrict__ x, int H, int W, int C, int OH, int OW,
                               int k, int s, int pad, int64_t total4, float* __restrict__ y) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int C4 = C >> 2;
  const int c4 = (int)(i % C4);
  int64_t r = i / C4;
  const int ow = (int)(r % OW);
  r /= OW;
  const int oh = (int)(r % OH);
  const int b = (int)(r / OH);
  float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  for (int kh = 0; kh < k; ++kh) {
    const int ih = oh * s - pad + kh;
    if (ih < 0 || ih >= H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int iw = ow * s - pad + kw;
      if (iw < 0 || iw >= W) continue;
      const float4 v =
          reinterpret_cast<const float4*>(x + (((int64_t)b * H + ih) * W + iw) * C)[c4];
      // max_pool2d propagates NaN
      m.x = (v.x > m.x || v.x != v.x) ? v.x : m.x;
      m.y = (v.y > m.y || v.y != v.y) ? v.y : m.y;
      m.z = (v.z > m.z || v.z != v.z) ? v.z : m.z;
      m.w = (v.w > m.w || v.w != v.w) ? v.w : m.w;
    }
  }
  reinterpret_cast<float4*>(y)[i] = m;
}
}  // namespace jabd

extern "C" int jabd_maxpool_nhwc_f32(const float* x, int32_t B, int32_t H, int32_t W, int32_t C,
                                     int32_t k, int32_t stride, int32_t pad, float* y,
                                     jabd_stream_t stream) {
  JABD_REQUIRE(x && y && B > 0 && H > 0 && W > 0 && C > 0 && C % 4 == 0 && k > 0 && stride > 0,
               "maxpool: bad args");
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  const int64_t total4 = (int64_t)B * OH * OW * (C / 4);
  maxpool_kernel<<<(unsigned)cdiv(total4, 256), 256, 0, as_stream(stream)>>>(
      x, H, W, C, OH, OW, k, stride, pad, total4, y);
  return check_launch("maxpool");
}
