// A3/A11 CSAF non-local block backward (nets/retinaface_r.py:124-152 and the
// FPN's nearest up-sample :192-203).  Forward (training) saves q and ctx per
// pixel and the pooled K/V; backward recomputes the attention row per pixel:
//   dctx = W^T dOut;  dP = dctx . V;  dL = P (dP - sum P dP);  dq = dL K
//   dK[s] += dL_s q,  dV[s] += P_s dctx      (wave shuffles -> block partials)
//   dx_up = dOut + Wq^T dq + Wk^T dkproj + Wv^T dvproj,
//   dkproj(pix) = sum over PSP bins containing pix of dK[bin] / |bin|
// then the up-sample backward gathers dx_up onto the source grid.  Weight
// gradients are 1x1-conv weight gradients (jabd_conv_wgrad_f32) of the saved
// per-pixel tensors.
#include "common.h"
#include "conv_args.h"

namespace jabd {

__device__ __forceinline__ int nsrc(int dst, int in, int out) {
  if (out == in) return dst;
  if (out == 2 * in) return dst >> 1;
  const float scale = (float)in / (float)out;
  const int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}

constexpr int CH = 4;

// A quad of lanes per up-sampled pixel (64 pixels per workgroup); lane r of
// a quad takes the PSP bins s = r, r+4, ...  Softmax max / sums combine over
// the quad; the per-bin dK/dV sums over the wave's 16 pixels reduce across
// the 16 lanes that share r (4 butterfly steps for 4 bins at once, where one
// lane per pixel needed 6 steps per bin).  Block partials of dK/dV:
// part[b][blk][S][8].
__global__ __launch_bounds__(256) void nlm_bwd_attn_kernel(
    const float* __restrict__ dout, int h, int w, int C, const float* __restrict__ q,
    const float* __restrict__ kpool, const float* __restrict__ vpool, int S,
    const float* __restrict__ wW, const float* __restrict__ wq, float* __restrict__ dq_out,
    float* __restrict__ dxup, float* __restrict__ part, int nblk) {
  extern __shared__ float sm[];  // K[S][4], V[S][4], wW[C][4], wq[4][C], red[4 waves][S][8]
  const int b = blockIdx.y;
  float* sK = sm;
  float* sV = sK + S * CH;
  float* sWW = sV + S * CH;
  float* sWq = sWW + C * CH;
  float* red = sWq + CH * C;
  for (int t = threadIdx.x; t < S * CH; t += blockDim.x) {
    sK[t] = kpool[(int64_t)b * S * CH + t];
    sV[t] = vpool[(int64_t)b * S * CH + t];
  }
  for (int t = threadIdx.x; t < C * CH; t += blockDim.x) {
    sWW[t] = wW[t];
    sWq[t] = wq[t];
  }
  __syncthreads();
  const int r = threadIdx.x & 3;
  const int pix = blockIdx.x * (blockDim.x >> 2) + (threadIdx.x >> 2);
  const bool ok = pix < h * w;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t m = (int64_t)b * h * w + (ok ? pix : 0);
  float qv[CH];
  {
    const float4 q4 = *reinterpret_cast<const float4*>(q + m * CH);
    qv[0] = ok ? q4.x : 0.f; qv[1] = ok ? q4.y : 0.f;
    qv[2] = ok ? q4.z : 0.f; qv[3] = ok ? q4.w : 0.f;
  }
  // dctx[r] by lane r, then exchanged within the quad
  const float* dop = dout + m * C;
  float dr = 0.f;
  if (ok)
    for (int c = 0; c < C; c += 4) {
      const float4 g = *reinterpret_cast<const float4*>(dop + c);
      dr = fmaf(g.x, sWW[(c + 0) * CH + r], dr);
      dr = fmaf(g.y, sWW[(c + 1) * CH + r], dr);
      dr = fmaf(g.z, sWW[(c + 2) * CH + r], dr);
      dr = fmaf(g.w, sWW[(c + 3) * CH + r], dr);
    }
  const int qb = lane & ~3;
  float dctx[CH];
#pragma unroll
  for (int o = 0; o < CH; ++o) dctx[o] = __shfl(dr, qb + o);
  const float4* K4 = reinterpret_cast<const float4*>(sK);
  const float4* V4 = reinterpret_cast<const float4*>(sV);
  auto logit = [&](const float4 k) {
    return fmaf(qv[0], k.x, fmaf(qv[1], k.y, fmaf(qv[2], k.z, qv[3] * k.w)));
  };
  auto dprod = [&](const float4 v) {
    return fmaf(dctx[0], v.x, fmaf(dctx[1], v.y, fmaf(dctx[2], v.z, dctx[3] * v.w)));
  };
  // recompute the softmax row (max, then sums, each combined over the quad)
  float mx = -INFINITY;
  for (int s = r; s < S; s += 4) mx = fmaxf(mx, logit(K4[s]));
  mx = fmaxf(mx, __shfl_xor(mx, 1));
  mx = fmaxf(mx, __shfl_xor(mx, 2));
  float den = 0.f, sdp = 0.f;
  for (int s = r; s < S; s += 4) {
    const float e = __expf(logit(K4[s]) - mx);
    den += e;
    sdp = fmaf(e, dprod(V4[s]), sdp);
  }
  den += __shfl_xor(den, 1);
  den += __shfl_xor(den, 2);
  sdp += __shfl_xor(sdp, 1);
  sdp += __shfl_xor(sdp, 2);
  const float inv = 1.f / den;
  sdp *= inv;
  float dq[CH] = {0.f, 0.f, 0.f, 0.f};
  const int nk = (S + 3) >> 2;  // uniform trip count (shuffles inside)
  for (int k = 0; k < nk; ++k) {
    const int s = 4 * k + r;
    const bool sv = s < S;
    const float4 kk = K4[sv ? s : 0], vv = V4[sv ? s : 0];
    const float P = (ok && sv) ? __expf(logit(kk) - mx) * inv : 0.f;
    const float dL = P * (dprod(vv) - sdp);
    dq[0] = fmaf(dL, kk.x, dq[0]);
    dq[1] = fmaf(dL, kk.y, dq[1]);
    dq[2] = fmaf(dL, kk.z, dq[2]);
    dq[3] = fmaf(dL, kk.w, dq[3]);
    float v[2 * CH];
#pragma unroll
    for (int o = 0; o < CH; ++o) {
      v[o] = dL * qv[o];
      v[CH + o] = P * dctx[o];
    }
#pragma unroll
    for (int o = 0; o < 2 * CH; ++o) {
      float a = v[o];
#pragma unroll
      for (int off = 4; off < 64; off <<= 1) a += __shfl_xor(a, off);
      v[o] = a;
    }
    if (lane < 4 && sv) {
      float4* rd = reinterpret_cast<float4*>(red + (wave * S + s) * 2 * CH);
      rd[0] = make_float4(v[0], v[1], v[2], v[3]);
      rd[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
#pragma unroll
  for (int o = 0; o < CH; ++o) {
    dq[o] += __shfl_xor(dq[o], 1);
    dq[o] += __shfl_xor(dq[o], 2);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < S * 2 * CH; t += blockDim.x) {
    float a = 0.f;
    for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) a += red[wv * S * 2 * CH + t];
    part[((int64_t)b * nblk + blockIdx.x) * S * 2 * CH + t] = a;
  }
  if (!ok) return;
  if (r == 0) *reinterpret_cast<float4*>(dq_out + m * CH) = make_float4(dq[0], dq[1], dq[2], dq[3]);
  float* dx = dxup + m * C;
  for (int c = 4 * r; c < C; c += 16) {
    const float4 g = *reinterpret_cast<const float4*>(dop + c);
    float rr[4] = {g.x, g.y, g.z, g.w};  // the "+ x" path
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 0; o < CH; ++o) rr[e] = fmaf(sWq[o * C + c + e], dq[o], rr[e]);
    *reinterpret_cast<float4*>(dx + c) = make_float4(rr[0], rr[1], rr[2], rr[3]);
  }
}

// One thread per up-sampled pixel (256 pixels per workgroup): the softmax row
// is recomputed over all S bins in registers (K/V broadcast from LDS), and
// the bin sums dK[s] = sum_p dL[p][s] q[p], dV[s] = sum_p P[p][s] dctx[p] go
// through LDS in chunks of kNb bins: the pixels write their dL / P columns,
// then thread (bin, group of 16 pixels) accumulates 16 pixels and the 16
// groups are added in a fixed order.  No cross-lane shuffles (the quad form
// spent its time in 32 LDS-routed butterflies per bin and wave).
// part[b][blk][S][8] as nlm_bwd_attn_kernel's, blk = 256-pixel block.
constexpr int kNb = 8;             // bins per LDS chunk
constexpr int kNg = 256 / kNb;     // reducer pixel groups (of 256 / kNg pixels)
constexpr int kNbP = 256 + 1;      // padded pixel stride of the chunk columns
__global__ __launch_bounds__(256) void nlm_bwd_attn256_kernel(
    const float* __restrict__ dout, int h, int w, int C, const float* __restrict__ q,
    const float* __restrict__ kpool, const float* __restrict__ vpool, int S,
    const float* __restrict__ wW, const float* __restrict__ wq, float* __restrict__ dq_out,
    float* __restrict__ dxup, float* __restrict__ part, int nblk) {
  // wW[C][4], wq[4][C], qs[256][4], dcs[256][4], dLs[kNb][kNbP], Ps[kNb][kNbP],
  // red[kNg][kNb][8]
  extern __shared__ float sm[];
  const int b = blockIdx.y, t = threadIdx.x;
  float* sWW = sm;
  float* sWq = sWW + C * CH;
  float* qs = sWq + CH * C;
  float* dcs = qs + 256 * CH;
  float* dLs = dcs + 256 * CH;
  float* Ps = dLs + kNb * kNbP;
  float* red = Ps + kNb * kNbP;
  for (int i = t; i < C * CH; i += 256) {
    sWW[i] = wW[i];
    sWq[i] = wq[i];
  }
  const int pix = blockIdx.x * 256 + t;
  const bool ok = pix < h * w;
  const int64_t m = (int64_t)b * h * w + (ok ? pix : 0);
  float qv[CH] = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    const float4 q4 = *reinterpret_cast<const float4*>(q + m * CH);
    qv[0] = q4.x; qv[1] = q4.y; qv[2] = q4.z; qv[3] = q4.w;
  }
  __syncthreads();
  const float* dop = dout + m * C;
  float dctx[CH] = {0.f, 0.f, 0.f, 0.f};
  if (ok)
    for (int c = 0; c < C; c += 4) {
      const float4 g = *reinterpret_cast<const float4*>(dop + c);
#pragma unroll
      for (int o = 0; o < CH; ++o)
        dctx[o] = fmaf(g.x, sWW[(c + 0) * CH + o],
                  fmaf(g.y, sWW[(c + 1) * CH + o],
                  fmaf(g.z, sWW[(c + 2) * CH + o], fmaf(g.w, sWW[(c + 3) * CH + o], dctx[o]))));
    }
  *reinterpret_cast<float4*>(qs + t * CH) = make_float4(qv[0], qv[1], qv[2], qv[3]);
  *reinterpret_cast<float4*>(dcs + t * CH) = make_float4(dctx[0], dctx[1], dctx[2], dctx[3]);
  // K / V rows straight from global memory at wave-uniform addresses: scalar
  // loads into SGPR operands (an LDS broadcast of a float4 costs the LDS a
  // 1 KiB return per wave and bin)
  const float4* __restrict__ K4 = reinterpret_cast<const float4*>(kpool + (int64_t)b * S * CH);
  const float4* __restrict__ V4 = reinterpret_cast<const float4*>(vpool + (int64_t)b * S * CH);
  auto logit = [&](const float4 k) {
    return fmaf(qv[0], k.x, fmaf(qv[1], k.y, fmaf(qv[2], k.z, qv[3] * k.w)));
  };
  auto dprod = [&](const float4 v) {
    return fmaf(dctx[0], v.x, fmaf(dctx[1], v.y, fmaf(dctx[2], v.z, dctx[3] * v.w)));
  };
  // four independent partial chains per reduction (two waves per SIMD do not
  // hide a serial max / sum chain's latency)
  float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  int s = 0;
  for (; s + 4 <= S; s += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) m4[u] = fmaxf(m4[u], logit(K4[s + u]));
  for (; s < S; ++s) m4[0] = fmaxf(m4[0], logit(K4[s]));
  const float mx = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
  float d4[4] = {0.f, 0.f, 0.f, 0.f}, p4[4] = {0.f, 0.f, 0.f, 0.f};
  for (s = 0; s + 4 <= S; s += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float e = __expf(logit(K4[s + u]) - mx);
      d4[u] += e;
      p4[u] = fmaf(e, dprod(V4[s + u]), p4[u]);
    }
  for (; s < S; ++s) {
    const float e = __expf(logit(K4[s]) - mx);
    d4[0] += e;
    p4[0] = fmaf(e, dprod(V4[s]), p4[0]);
  }
  const float den = (d4[0] + d4[1]) + (d4[2] + d4[3]);
  const float inv = 1.f / den;
  const float sdp = ((p4[0] + p4[1]) + (p4[2] + p4[3])) * inv;
  float dq[CH] = {0.f, 0.f, 0.f, 0.f};
  constexpr int ppg = 256 / kNg;
  const int rb = t % kNb, rg = t / kNb;  // reducer: bin rb of the chunk, pixels ppg rg .. ppg rg + ppg - 1
  for (int s0 = 0; s0 < S; s0 += kNb) {
#pragma unroll 8
    for (int j = 0; j < kNb; ++j) {  // (K4 / V4 rows: scalar loads batched by the unroll)
      const int sj = s0 + j;
      const bool sv = sj < S;
      const float4 kk = K4[sv ? sj : 0], vv = V4[sv ? sj : 0];
      const float P = (ok && sv) ? __expf(logit(kk) - mx) * inv : 0.f;
      const float dL = P * (dprod(vv) - sdp);
      dq[0] = fmaf(dL, kk.x, dq[0]);
      dq[1] = fmaf(dL, kk.y, dq[1]);
      dq[2] = fmaf(dL, kk.z, dq[2]);
      dq[3] = fmaf(dL, kk.w, dq[3]);
      dLs[j * kNbP + t] = dL;
      Ps[j * kNbP + t] = P;
    }
    __syncthreads();
    float acc[2 * CH] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int i = 0; i < ppg; ++i) {
      const int p = rg * ppg + i;
      const float dl = dLs[rb * kNbP + p], pp = Ps[rb * kNbP + p];
      const float4 qq = *reinterpret_cast<const float4*>(qs + p * CH);
      const float4 dc = *reinterpret_cast<const float4*>(dcs + p * CH);
      acc[0] = fmaf(dl, qq.x, acc[0]); acc[1] = fmaf(dl, qq.y, acc[1]);
      acc[2] = fmaf(dl, qq.z, acc[2]); acc[3] = fmaf(dl, qq.w, acc[3]);
      acc[4] = fmaf(pp, dc.x, acc[4]); acc[5] = fmaf(pp, dc.y, acc[5]);
      acc[6] = fmaf(pp, dc.z, acc[6]); acc[7] = fmaf(pp, dc.w, acc[7]);
    }
    float4* rr = reinterpret_cast<float4*>(red + (rg * kNb + rb) * 2 * CH);
    rr[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    rr[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    __syncthreads();
    if (t < kNb * 2 * CH) {  // (bin, component): the kNg groups in order
      const int j = t / (2 * CH), o = t % (2 * CH);
      float a = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < kNg; ++g2) a += red[(g2 * kNb + j) * 2 * CH + o];
      if (s0 + j < S) part[(((int64_t)b * nblk + blockIdx.x) * S + s0 + j) * 2 * CH + o] = a;
    }
    // (the next chunk's dLs / Ps writes come after this barrier; red is
    // rewritten only after the next chunk's first barrier)
    __syncthreads();
  }
  if (!ok) return;
  *reinterpret_cast<float4*>(dq_out + m * CH) = make_float4(dq[0], dq[1], dq[2], dq[3]);
  float* dx = dxup + m * C;
  for (int c = 0; c < C; c += 4) {
    const float4 g = *reinterpret_cast<const float4*>(dop + c);
    float rr2[4] = {g.x, g.y, g.z, g.w};  // the "+ x" path
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 0; o < CH; ++o) rr2[e] = fmaf(sWq[o * C + c + e], dq[o], rr2[e]);
    *reinterpret_cast<float4*>(dx + c) = make_float4(rr2[0], rr2[1], rr2[2], rr2[3]);
  }
}

// dk/dv[b][s][o] = sum over the nblk block partials (four block ranges per
// output, added in a fixed order)
__global__ __launch_bounds__(256) void nlm_bwd_kv_reduce4_kernel(const float* __restrict__ part,
                                                                 int nblk, int S,
                                                                 float* __restrict__ dk,
                                                                 float* __restrict__ dv) {
  __shared__ float red[4][64];
  const int b = blockIdx.y;
  const int o = blockIdx.x * 64 + (threadIdx.x & 63), qq = threadIdx.x >> 6;
  const int tot = S * 2 * CH;
  float a = 0.f;
  if (o < tot)
    for (int k = qq; k < nblk; k += 4) a += part[((int64_t)b * nblk + k) * tot + o];
  red[qq][threadIdx.x & 63] = a;
  __syncthreads();
  if (qq == 0 && o < tot) {
    a = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    const int s = o / (2 * CH), c = o % (2 * CH);
    if (c < CH) dk[((int64_t)b * S + s) * CH + c] = a;
    else dv[((int64_t)b * S + s) * CH + (c - CH)] = a;
  }
}

__global__ void nlm_bwd_kv_reduce_kernel(const float* __restrict__ part, int nblk, int S,
                                         float* __restrict__ dk, float* __restrict__ dv) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= S * 2 * CH) return;
  float a = 0.f;
  for (int q = 0; q < nblk; ++q) a += part[((int64_t)b * nblk + q) * S * 2 * CH + t];
  const int s = t / (2 * CH), o = t % (2 * CH);
  if (o < CH) dk[((int64_t)b * S + s) * CH + o] = a;
  else dv[((int64_t)b * S + s) * CH + (o - CH)] = a;
}

struct PspSizes {
  int n;
  int v[8];
};

// Per up-sampled pixel: dkproj/dvproj from every PSP bin containing it, then
// dx_up += Wk^T dkproj + Wv^T dvproj.  dkv [M][8] is kept for the weight grads.
__global__ __launch_bounds__(256) void nlm_bwd_proj_kernel(
    const float* __restrict__ dk, const float* __restrict__ dv, int S, const PspSizes ps, int h,
    int w, int C, const float* __restrict__ wk, const float* __restrict__ wv,
    float* __restrict__ dkv, float* __restrict__ dxup) {
  extern __shared__ float sm[];  // dK[S][4], dV[S][4], wk[4][C], wv[4][C]
  const int b = blockIdx.y;
  float* sK = sm;
  float* sV = sK + S * CH;
  float* sWk = sV + S * CH;
  float* sWv = sWk + CH * C;
  for (int t = threadIdx.x; t < S * CH; t += blockDim.x) {
    sK[t] = dk[(int64_t)b * S * CH + t];
    sV[t] = dv[(int64_t)b * S * CH + t];
  }
  for (int t = threadIdx.x; t < CH * C; t += blockDim.x) {
    sWk[t] = wk[t];
    sWv[t] = wv[t];
  }
  __syncthreads();
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= h * w) return;
  const int i = pix / w, j = pix - (pix / w) * w;
  float gk[CH] = {0.f, 0.f, 0.f, 0.f}, gv[CH] = {0.f, 0.f, 0.f, 0.f};
  int base = 0;
  for (int l = 0; l < ps.n; ++l) {
    const int sz = ps.v[l];
    // bins bi with floor(bi*h/sz) <= i < ceil((bi+1)*h/sz)
    // bins containing row i: floor(bi*h/sz) <= i < ceil((bi+1)*h/sz); when
    // sz > h several consecutive bins share a row, so scan the full range
    const int bi_lo = max(0, ((i - 1) * sz) / h - 1), bi_hi = min(sz - 1, ((i + 1) * sz) / h);
    for (int bi = bi_lo; bi <= bi_hi; ++bi) {
      const int h0 = (bi * h) / sz, h1 = ((bi + 1) * h + sz - 1) / sz;
      if (i < h0 || i >= h1) continue;
      const int bj_lo = max(0, ((j - 1) * sz) / w - 1), bj_hi = min(sz - 1, ((j + 1) * sz) / w);
      for (int bj = bj_lo; bj <= bj_hi; ++bj) {
        const int w0 = (bj * w) / sz, w1 = ((bj + 1) * w + sz - 1) / sz;
        if (j < w0 || j >= w1) continue;
        const float invn = 1.f / (float)((h1 - h0) * (w1 - w0));
        const int s = base + bi * sz + bj;
#pragma unroll
        for (int o = 0; o < CH; ++o) {
          gk[o] = fmaf(sK[s * CH + o], invn, gk[o]);
          gv[o] = fmaf(sV[s * CH + o], invn, gv[o]);
        }
      }
    }
    base += sz * sz;
  }
  const int64_t m = (int64_t)b * h * w + pix;
#pragma unroll
  for (int o = 0; o < CH; ++o) {
    dkv[m * 2 * CH + o] = gk[o];
    dkv[m * 2 * CH + CH + o] = gv[o];
  }
  float* dx = dxup + m * C;
  for (int c = 0; c < C; c += 4) {
    float4 r = *reinterpret_cast<float4*>(dx + c);
    float rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 0; o < CH; ++o)
        rr[e] = fmaf(sWk[o * C + c + e], gk[o], fmaf(sWv[o * C + c + e], gv[o], rr[e]));
    *reinterpret_cast<float4*>(dx + c) = make_float4(rr[0], rr[1], rr[2], rr[3]);
  }
}

// Nearest up-sample backward: dsrc[si][sj] += sum of dx_up over its preimage
// (a contiguous index range per axis; gather, no atomics).  dsrc may hold a
// gradient already (accumulate=1).
__global__ void upsample_bwd_kernel(const float* __restrict__ dxup, int h, int w, int hs, int ws,
                                    int C, int accumulate, float* __restrict__ dsrc) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int C4 = C >> 2;
  const int b = blockIdx.y;
  if (idx >= (int64_t)hs * ws * C4) return;
  const int c4 = (int)(idx % C4);
  const int sp = (int)(idx / C4);
  const int si = sp / ws, sj = sp - (sp / ws) * ws;
  // preimage rows: dst i with nsrc(i) == si (monotone in i)
  int i0 = (int)((int64_t)si * h / hs) - 2, j0 = (int)((int64_t)sj * w / ws) - 2;
  if (i0 < 0) i0 = 0;
  if (j0 < 0) j0 = 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = i0; i < h; ++i) {
    const int ni = nsrc(i, hs, h);
    if (ni < si) continue;
    if (ni > si) break;
    for (int j = j0; j < w; ++j) {
      const int nj = nsrc(j, ws, w);
      if (nj < sj) continue;
      if (nj > sj) break;
      const float4 g = reinterpret_cast<const float4*>(dxup + (((int64_t)b * h + i) * w + j) * C)[c4];
      acc.x += g.x; acc.y += g.y; acc.z += g.z; acc.w += g.w;
    }
  }
  float4* d = reinterpret_cast<float4*>(dsrc + (((int64_t)b * hs + si) * ws + sj) * C) + c4;
  if (accumulate) {
    const float4 o = *d;
    acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
  }
  *d = acc;
}

// Training forward helper: x_up = nearest(src) materialised (the NLM weight
// gradients need it per pixel).
__global__ void upsample_fwd_kernel(const float* __restrict__ src, int hs, int ws, int h, int w,
                                    int C, float* __restrict__ dst) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int C4 = C >> 2;
  const int b = blockIdx.y;
  if (idx >= (int64_t)h * w * C4) return;
  const int c4 = (int)(idx % C4);
  const int p = (int)(idx / C4);
  const int i = p / w, j = p - (p / w) * w;
  reinterpret_cast<float4*>(dst + (((int64_t)b * h + i) * w + j) * C)[c4] =
      reinterpret_cast<const float4*>(src + (((int64_t)b * hs + nsrc(i, hs, h)) * ws + nsrc(j, ws, w)) * C)[c4];
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_nlm_bwd_attn_f32(const float* dout, int32_t B, int32_t h, int32_t w,
                                     int32_t C, const float* q, const float* kpool,
                                     const float* vpool, int32_t S, const float* wW,
                                     const float* wq, float* dq, float* dxup, float* part,
                                     float* dk, float* dv, jabd_stream_t stream) {
  JABD_REQUIRE(dout && q && kpool && vpool && wW && wq && dq && dxup && part && dk && dv &&
                   C % 4 == 0,
               "nlm_bwd_attn: bad args");
  hipStream_t st = as_stream(stream);
  // JABD_NLM_BWD_QUAD=1: the lane-quad kernel (A/B)
  static const bool quad = [] {
    const char* e = getenv("JABD_NLM_BWD_QUAD");
    return e && e[0] == '1';
  }();
  if (!quad) {
    const int nblk = (int)cdiv((int64_t)h * w, 256);  // within jabd.h's part size (64-pixel blocks)
    const size_t smem = (2 * (size_t)C * CH + 2 * 256 * CH + 2 * (size_t)kNb * kNbP +
                         kNg * (size_t)kNb * 2 * CH) * 4;
    JABD_REQUIRE(smem <= 160 * 1024, "nlm_bwd_attn: LDS %zu > 160KiB", smem);
    if (smem > 64 * 1024)
      JABD_HIP(hipFuncSetAttribute((const void*)nlm_bwd_attn256_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    dim3 g((unsigned)nblk, (unsigned)B);
    nlm_bwd_attn256_kernel<<<g, 256, smem, st>>>(dout, h, w, C, q, kpool, vpool, S, wW, wq, dq,
                                                 dxup, part, nblk);
    if (int e = check_launch("nlm_bwd_attn")) return e;
    dim3 g2((unsigned)cdiv(S * 2 * CH, 64), (unsigned)B);
    nlm_bwd_kv_reduce4_kernel<<<g2, 256, 0, st>>>(part, nblk, S, dk, dv);
    return check_launch("nlm_bwd_kv_reduce");
  }
  const int nblk = (int)cdiv((int64_t)h * w, 64);  // a lane quad per pixel
  const size_t smem = (2 * (size_t)S * CH + 2 * (size_t)C * CH + 4 * (size_t)S * 2 * CH) * 4;
  JABD_REQUIRE(smem <= 64 * 1024, "nlm_bwd_attn: LDS %zu > 64KiB", smem);
  dim3 g((unsigned)nblk, (unsigned)B);
  nlm_bwd_attn_kernel<<<g, 256, smem, st>>>(dout, h, w, C, q, kpool, vpool, S, wW, wq, dq, dxup,
                                            part, nblk);
  if (int e = check_launch("nlm_bwd_attn")) return e;
  dim3 g2((unsigned)cdiv(S * 2 * CH, 256), (unsigned)B);
  nlm_bwd_kv_reduce_kernel<<<g2, 256, 0, st>>>(part, nblk, S, dk, dv);
  return check_launch("nlm_bwd_kv_reduce");
}

extern "C" int jabd_nlm_bwd_proj_f32(const float* dk, const float* dv, int32_t B, int32_t S,
                                     const int32_t* sizes, int32_t nsizes, int32_t h, int32_t w,
                                     int32_t C, const float* wk, const float* wv, float* dkv,
                                     float* dxup, jabd_stream_t stream) {
  JABD_REQUIRE(dk && dv && sizes && wk && wv && dkv && dxup && nsizes > 0 && nsizes <= 8 &&
                   C % 4 == 0,
               "nlm_bwd_proj: bad args");
  PspSizes ps;
  ps.n = nsizes;
  for (int i = 0; i < 8; ++i) ps.v[i] = i < nsizes ? sizes[i] : 0;
  const size_t smem = (2 * (size_t)S * CH + 2 * (size_t)C * CH) * 4;
  dim3 g((unsigned)cdiv((int64_t)h * w, 256), (unsigned)B);
  nlm_bwd_proj_kernel<<<g, 256, smem, as_stream(stream)>>>(dk, dv, S, ps, h, w, C, wk, wv, dkv,
                                                           dxup);
  return check_launch("nlm_bwd_proj");
}

extern "C" int jabd_upsample_nearest_bwd_f32(const float* dxup, int32_t B, int32_t h, int32_t w,
                                             int32_t hs, int32_t ws, int32_t C, int32_t accumulate,
                                             float* dsrc, jabd_stream_t stream) {
  JABD_REQUIRE(dxup && dsrc && C % 4 == 0 && hs <= h && ws <= w, "upsample_bwd: bad args");
  dim3 g((unsigned)cdiv((int64_t)hs * ws * (C / 4), 256), (unsigned)B);
  upsample_bwd_kernel<<<g, 256, 0, as_stream(stream)>>>(dxup, h, w, hs, ws, C, accumulate, dsrc);
  return check_launch("upsample_bwd");
}

extern "C" int jabd_upsample_nearest_f32(const float* src, int32_t B, int32_t hs, int32_t ws,
                                         int32_t h, int32_t w, int32_t C, float* dst,
                                         jabd_stream_t stream) {
  JABD_REQUIRE(src && dst && C % 4 == 0, "upsample: bad args");
  dim3 g((unsigned)cdiv((int64_t)h * w * (C / 4), 256), (unsigned)B);
  upsample_fwd_kernel<<<g, 256, 0, as_stream(stream)>>>(src, hs, ws, h, w, C, dst);
  return check_launch("upsample");
}
