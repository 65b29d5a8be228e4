// A1/A4/A5 dense convolutions on gfx950 as NHWC implicit GEMM on the exact
// fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
//   Y[m, n] = act( sum_k A[m, k] * W[k, n] + bias[n] (+ R[m, n]) )
//   m = (image, oh, ow) output pixel, n = output channel,
//   k = (kh, kw, ci) tap-major, channel-minor (1x1: k = ci).
//
// Operand mapping.  The MFMA sums over its 4-wide k index (lane>>4).  Each
// lane loads 16 contiguous bytes — channels 4g..4g+3 of its pixel (g = lane>>4)
// — and feeds element e to MFMA step e, so one 16-channel K chunk is four
// MFMAs whose logical k order is (4g + e).  Weights are pre-packed on the host
// in exactly that order: Wp[kc][ntile][lane] = float4{W[16kc+4g+e][16nt+j]},
// j = lane&15, so every B fragment is one coalesced float4 per lane.
// Accumulator layout (16x16 f32): col = lane&15, row = 4*(lane>>4) + reg.
//
// Fusions: BN folded into W/bias (eval) or applied by the caller's BN
// kernels (train); optional per-(image, k) A-scale (ECA gate of the
// producing block, applied on load exactly as the reference's x*y);
// optional K-concatenated second source (the block's skip branch folded into
// the same GEMM); residual add; activation; channel-offset / strided output
// (SSH concat, head layout).
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "conv_args.h"

namespace jabd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return relu_f(v);
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: return hswish_f(v);
    case ACT_HSIGMOID: return hsigmoid_f(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// The epilogue staging regions are wave-private: ordering a wave's own LDS
// writes before its reads needs lgkmcnt(0), not a workgroup barrier (which
// would also align the four waves and drain their outstanding loads).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float4 load_x2(const ConvArgs& p, int b, int oh, int ow, int c) {
  const float* src = p.x2 + (int64_t)b * p.x2_bs +
                     ((int64_t)oh * p.x2_stride * p.x2_W + (int64_t)ow * p.x2_stride) * p.x2_ps;
  return *reinterpret_cast<const float4*>(src + c);
}

// Load the float4 of A for one lane: pixel (b, oh, ow) and k4 = first of 4 ks.
template <bool VEC4>
__device__ __forceinline__ float4 load_a(const ConvArgs& p, int b, int oh, int ow, bool mvalid,
                                         int k4) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!mvalid) return r;
  if (p.KH == 1 && p.KW == 1 && p.stride == 1 && p.pad == 0 && !p.tconv) {
    if (k4 < p.Cin) {
      const float* src = p.x + (int64_t)b * p.x_bs + ((int64_t)oh * p.W + ow) * p.x_ps + p.x_c0;
      if (VEC4) {
        r = *reinterpret_cast<const float4*>(src + k4);
      } else {
        r.x = src[k4];
        if (k4 + 1 < p.Cin) r.y = src[k4 + 1];
        if (k4 + 2 < p.Cin) r.z = src[k4 + 2];
        if (k4 + 3 < p.Cin) r.w = src[k4 + 3];
      }
      if (p.ascale) {
        const float* s = p.ascale + (int64_t)b * p.ascale_bs + k4;
        r.x *= s[0]; r.y *= s[1]; r.z *= s[2]; r.w *= s[3];
      }
    } else if (p.x2 && k4 < p.Cin + p.Cin2) {
      r = load_x2(p, b, oh, ow, k4 - p.Cin);
    }
    return r;
  }
  // k x k taps (tap-major, channel-minor)
  const int Ktot = p.KH * p.KW * p.Cin;
  if (p.x2 && k4 >= Ktot) {
    if (k4 < Ktot + p.Cin2) r = load_x2(p, b, oh, ow, k4 - Ktot);
    return r;
  }
  if (VEC4) {
    if (k4 >= Ktot) return r;
    const int tap = k4 / p.Cin, ci = k4 - tap * p.Cin;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
    int ih, iw;
    if (p.tconv) {
      const int nh = oh + p.pad - kh, nw = ow + p.pad - kw;
      if (nh < 0 || nw < 0 || nh % p.stride || nw % p.stride) return r;
      ih = nh / p.stride;
      iw = nw / p.stride;
    } else {
      ih = oh * p.stride - p.pad + kh;
      iw = ow * p.stride - p.pad + kw;
    }
    if (ih < 0 || ih >= p.H || iw < 0 || iw >= p.W) return r;
    const float* src = p.x + (int64_t)b * p.x_bs + ((int64_t)ih * p.W + iw) * p.x_ps + p.x_c0 + ci;
    r = *reinterpret_cast<const float4*>(src);
    if (p.ascale) {
      const float* s = p.ascale + (int64_t)b * p.ascale_bs + ci;
      r.x *= s[0]; r.y *= s[1]; r.z *= s[2]; r.w *= s[3];
    }
    return r;
  }
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = 0.f;
    const int k = k4 + e;
    if (k >= Ktot) continue;
    const int tap = k / p.Cin, ci = k - tap * p.Cin;
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
    int ih, iw;
    if (p.tconv) {
      const int nh = oh + p.pad - kh, nw = ow + p.pad - kw;
      if (nh < 0 || nw < 0 || nh % p.stride || nw % p.stride) continue;
      ih = nh / p.stride;
      iw = nw / p.stride;
    } else {
      ih = oh * p.stride - p.pad + kh;
      iw = ow * p.stride - p.pad + kw;
    }
    if (ih < 0 || ih >= p.H || iw < 0 || iw >= p.W) continue;
    float x;
    if (p.nchw_in)
      x = p.x[(int64_t)b * p.x_bs + ((int64_t)ci * p.H + ih) * p.W + iw];
    else
      x = p.x[(int64_t)b * p.x_bs + ((int64_t)ih * p.W + iw) * p.x_ps + p.x_c0 + ci];
    if (p.ascale) x *= p.ascale[(int64_t)b * p.ascale_bs + ci];
    v[e] = x;
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

template <int TM, int TN, bool VEC4>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const ConvArgs p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int nblk_n = p.Ntiles / TN;
  // blocks of the same M range are adjacent -> share A through L2
  const int bid = blockIdx.x;
  const int nb = bid % nblk_n;
  const int mb = bid / nblk_n;
  const int m_wave = (mb * 4 + wave) * (16 * TM);
  const int OHW = p.OH * p.OW;  // host guarantees M < 2^31

  // per-lane pixel of each 16-pixel subtile (column j of the MFMA tile)
  int pb[TM], poh[TM], pow_[TM];
  bool pv[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int m = m_wave + t * 16 + j;
    pv[t] = m < p.M;
    const int mm = pv[t] ? m : 0;
    pb[t] = mm / OHW;
    const int r = mm - pb[t] * OHW;
    poh[t] = r / p.OW;
    pow_[t] = r - poh[t] * p.OW;
  }

  // acc[t][u] = MFMA tile with rows = output channels, columns = pixels:
  // operand A = packed weights (row n = lane&15), operand B = activations
  // (column m = lane&15), so each lane ends up holding 4 consecutive output
  // channels of one pixel -> one 16-byte store per tile.
  f32x4 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const float4* wbase = reinterpret_cast<const float4*>(p.w) + ((int64_t)nb * TN) * 64 + lane;
  const int64_t wstride_k = (int64_t)p.Ntiles * 64;

  // k x k taps walked incrementally (no per-load integer division): the
  // lane's next float4 is channel tci of tap (tkh, tkw); each K chunk
  // advances it by 16 channels.  Used for plain forward k x k convs.
  const bool taps = VEC4 && !p.tconv && !p.x2 && p.KH * p.KW > 1;
  int tci = 4 * g, tkh = 0, tkw = 0;
  auto tap_advance = [&](int by) {
    tci += by;
    while (tci >= p.Cin) {
      tci -= p.Cin;
      if (++tkw == p.KW) { tkw = 0; ++tkh; }
    }
  };
  auto load_tap = [&](int t) -> float4 {
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    const int ih = poh[t] * p.stride - p.pad + tkh, iw = pow_[t] * p.stride - p.pad + tkw;
    if (pv[t] && tkh < p.KH && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) {
      r = *reinterpret_cast<const float4*>(p.x + (int64_t)pb[t] * p.x_bs +
                                           ((int64_t)ih * p.W + iw) * p.x_ps + p.x_c0 + tci);
      if (p.ascale) {
        const float4 s4 =
            *reinterpret_cast<const float4*>(p.ascale + (int64_t)pb[t] * p.ascale_bs + tci);
        r.x *= s4.x; r.y *= s4.y; r.z *= s4.z; r.w *= s4.w;
      }
    }
    return r;
  };
  if (taps) tap_advance(0);

  float4 a_cur[TM], b_cur[TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
    a_cur[t] = taps ? load_tap(t) : load_a<VEC4>(p, pb[t], poh[t], pow_[t], pv[t], 4 * g);
  if (taps) tap_advance(16);
#pragma unroll
  for (int u = 0; u < TN; ++u) b_cur[u] = wbase[u * 64];

  for (int kc = 0; kc < p.Kc; ++kc) {
    float4 a_nxt[TM], b_nxt[TN];
    const bool more = kc + 1 < p.Kc;
    if (more) {
      const int k4 = (kc + 1) * 16 + 4 * g;
      if (taps) {
#pragma unroll
        for (int t = 0; t < TM; ++t) a_nxt[t] = load_tap(t);
        tap_advance(16);
      } else {
#pragma unroll
        for (int t = 0; t < TM; ++t) a_nxt[t] = load_a<VEC4>(p, pb[t], poh[t], pow_[t], pv[t], k4);
      }
#pragma unroll
      for (int u = 0; u < TN; ++u) b_nxt[u] = wbase[(kc + 1) * wstride_k + u * 64];
    }
    // k-step outermost: consecutive MFMAs update independent accumulators
    // (16x16x4 f32: 32-cycle issue, 40-cycle dependent latency)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].x, a_cur[t].x, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].y, a_cur[t].y, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].z, a_cur[t].z, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].w, a_cur[t].w, acc[t][u], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int t = 0; t < TM; ++t) a_cur[t] = a_nxt[t];
#pragma unroll
      for (int u = 0; u < TN; ++u) b_cur[u] = b_nxt[u];
    }
  }

  // epilogue: acc[t][u][r] = Y[pixel m_wave + 16t + j][channel 16(nb*TN+u) + 4g + r]
  const bool v4 = (p.flags & 1) != 0;  // host: every channel offset/stride % 4 == 0
  if (v4) {
    // Stage each 16-pixel x 16*TN-channel subtile through LDS so every store
    // instruction writes whole 16*TN-float pixel rows (1 KB contiguous when
    // the tile spans the full channel range) instead of 16 scattered 64-B pieces.
    constexpr int LDW = 16 * TN + 4;
    __shared__ float s_epi[4 * 16 * LDW];
    float* sm = s_epi + wave * 16 * LDW;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
#pragma unroll
      for (int u = 0; u < TN; ++u)
        *reinterpret_cast<f32x4*>(sm + j * LDW + 16 * u + 4 * g) = acc[t][u];
      const int64_t pix = (int64_t)poh[t] * p.OW + pow_[t];
      const long long yoff = pv[t] ? (long long)((int64_t)pb[t] * p.y_bs + pix * p.y_ps + p.y_c0) : -1;
      const long long roff =
          p.res ? (long long)((int64_t)pb[t] * p.res_bs + pix * p.res_ps + p.res_c0) : 0;
      const long long y2off =
          p.y2 ? (long long)((int64_t)pb[t] * p.y2_bs + pix * p.y2_ps + p.y2_c0) : 0;
      wave_lds_sync();  // wave-private LDS region
#pragma unroll
      for (int f0 = 0; f0 < 16 * 4 * TN; f0 += 64) {
        const int f = f0 + lane;
        const int q = f / (4 * TN), c4 = f - q * (4 * TN);
        // shuffles stay outside the divergent branch (an inactive source lane reads as 0)
        const long long yo = __shfl(yoff, q);
        const long long ro = __shfl(roff, q);
        const long long y2o = __shfl(y2off, q);
        const int n0 = nb * TN * 16 + 4 * c4;
        if (yo >= 0 && n0 < p.Cout) {
          float4 v = *reinterpret_cast<const float4*>(sm + q * LDW + 4 * c4);
          if (p.bias) {
            const float4 bb = *reinterpret_cast<const float4*>(p.bias + n0);
            v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
          }
          if (p.res) {
            const float4 rr = *reinterpret_cast<const float4*>(p.res + ro + n0);
            v.x += rr.x; v.y += rr.y; v.z += rr.z; v.w += rr.w;
          }
          if (p.y2 && n0 >= p.nsplit) {  // second fused convolution's channels
            v.x = act_apply(v.x, p.act2, p.slope2);
            v.y = act_apply(v.y, p.act2, p.slope2);
            v.z = act_apply(v.z, p.act2, p.slope2);
            v.w = act_apply(v.w, p.act2, p.slope2);
            *reinterpret_cast<float4*>(p.y2 + y2o + (n0 - p.nsplit)) = v;
          } else {
            v.x = act_apply(v.x, p.act, p.slope);
            v.y = act_apply(v.y, p.act, p.slope);
            v.z = act_apply(v.z, p.act, p.slope);
            v.w = act_apply(v.w, p.act, p.slope);
            *reinterpret_cast<float4*>(p.y + yo + n0) = v;
          }
        }
      }
      wave_lds_sync();  // wave-private LDS region
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    if (!pv[t]) continue;
    const int64_t pix = (int64_t)poh[t] * p.OW + pow_[t];
    float* yrow = p.y + (int64_t)pb[t] * p.y_bs + pix * p.y_ps + p.y_c0;
    const float* rrow =
        p.res ? p.res + (int64_t)pb[t] * p.res_bs + pix * p.res_ps + p.res_c0 : nullptr;
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int n0 = (nb * TN + u) * 16 + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + r;
        if (n >= p.Cout) break;
        float v = acc[t][u][r] + (p.bias ? p.bias[n] : 0.f);
        if (rrow) v += rrow[n];
        yrow[n] = act_apply(v, p.act, p.slope);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 1x1 / stride-1 fast path.  Same MFMA mapping as conv_gemm_kernel, but the
// A operand of pixel m is the contiguous row x + m*x_ps (no im2col index
// math, no generic-path registers), so the kernel holds ~half the VGPRs and
// runs at twice the occupancy — the layers it serves (MobileNetV3 project
// convs, FPN laterals, ResNet 1x1s) are memory-bound and latency-limited.
//   X2: 0 = no second source, 1 = same-resolution K-concat source (MNv3
//   skip), 2 = strided K-concat source (ResNet downsample).
// Host guarantees: Cin, x_ps, x_c0, Cin2, x2_ps % 4 == 0; batch-contiguous
// x / y / res (bs == pixels * ps); M * max(ps) < 2^31; v4 epilogue.
// ---------------------------------------------------------------------------
template <int TM, int TN, int X2, bool ASCALE>
__global__ __launch_bounds__(256) void conv1x1_kernel(const ConvArgs p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int nblk_n = p.Ntiles / TN;
  const int bid = blockIdx.x;
  const int nb = bid % nblk_n;
  const int mb = bid / nblk_n;
  const int m_wave = (mb * 4 + wave) * (16 * TM);
  const int OHW = p.OH * p.OW;
  const int M = (int)p.M;

  int pm[TM];  // pixel index (clamped), -1 when out of range
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int m = m_wave + t * 16 + j;
    pm[t] = m < M ? m : -1;
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const float4* wbase = reinterpret_cast<const float4*>(p.w) + ((int64_t)nb * TN) * 64 + lane;
  const int wstride_k = p.Ntiles * 64;
  const float* xg = p.x + p.x_c0 + 4 * g;
  const int x2_pix = X2 == 2 ? (int)(p.x2_bs / p.x2_ps) : 0;  // x2 pixels per image

  auto load = [&](int kc, float4 (&a)[TM]) {
    const int k4 = kc * 16 + 4 * g;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
      const int m = pm[t];
      if (m >= 0 && !(p.reserved1 & 1)) {
        if (k4 < p.Cin) {
          r = *reinterpret_cast<const float4*>(xg + m * p.x_ps + kc * 16);
          if (ASCALE) {
            const int b = m / OHW;
            const float4 s4 = *reinterpret_cast<const float4*>(p.ascale + b * (int)p.ascale_bs + k4);
            r.x *= s4.x; r.y *= s4.y; r.z *= s4.z; r.w *= s4.w;
          }
        } else if (X2 != 0 && k4 < p.Cin + p.Cin2) {
          int q;
          if (X2 == 1) {
            q = m;
          } else {
            const int b = m / OHW, rr = m - b * OHW;
            const int oh = rr / p.OW, ow = rr - oh * p.OW;
            q = b * x2_pix + (oh * p.x2_stride) * p.x2_W + ow * p.x2_stride;
          }
          r = *reinterpret_cast<const float4*>(p.x2 + q * p.x2_ps + (k4 - p.Cin));
        }
      }
      a[t] = r;
    }
  };

  float4 a_cur[TM], b_cur[TN];
  load(0, a_cur);
#pragma unroll
  for (int u = 0; u < TN; ++u) b_cur[u] = wbase[u * 64];

  for (int kc = 0; kc < p.Kc; ++kc) {
    float4 a_nxt[TM], b_nxt[TN];
    const bool more = kc + 1 < p.Kc;
    if (more) {
      load(kc + 1, a_nxt);
#pragma unroll
      for (int u = 0; u < TN; ++u) b_nxt[u] = wbase[(kc + 1) * wstride_k + u * 64];
    }
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].x, a_cur[t].x, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].y, a_cur[t].y, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].z, a_cur[t].z, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].w, a_cur[t].w, acc[t][u], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int t = 0; t < TM; ++t) a_cur[t] = a_nxt[t];
#pragma unroll
      for (int u = 0; u < TN; ++u) b_cur[u] = b_nxt[u];
    }
  }

  // epilogue (LDS-staged whole-row stores), acc[t][u][r] = Y[pixel][16(nb*TN+u) + 4g + r]
  constexpr int LDW = 16 * TN + 4;
  __shared__ float s_epi[4 * 16 * LDW];
  float* sm = s_epi + wave * 16 * LDW;
#pragma unroll
  for (int t = 0; t < TM; ++t) {
#pragma unroll
    for (int u = 0; u < TN; ++u)
      *reinterpret_cast<f32x4*>(sm + j * LDW + 16 * u + 4 * g) = acc[t][u];
    wave_lds_sync();  // wave-private LDS region
#pragma unroll
    for (int f0 = 0; f0 < 16 * 4 * TN; f0 += 64) {
      const int f = f0 + lane;
      const int q = f / (4 * TN), c4 = f - q * (4 * TN);
      const int m = __shfl(pm[t], q);  // outside the branch (inactive lanes read 0)
      const int n0 = nb * TN * 16 + 4 * c4;
      if (m >= 0 && n0 < p.Cout) {
        float4 v = *reinterpret_cast<const float4*>(sm + q * LDW + 4 * c4);
        if (p.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + n0);
          v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
        }
        if (p.res) {
          const float4 rr = *reinterpret_cast<const float4*>(p.res + m * p.res_ps + p.res_c0 + n0);
          v.x += rr.x; v.y += rr.y; v.z += rr.z; v.w += rr.w;
        }
        v.x = act_apply(v.x, p.act, p.slope);
        v.y = act_apply(v.y, p.act, p.slope);
        v.z = act_apply(v.z, p.act, p.slope);
        v.w = act_apply(v.w, p.act, p.slope);
        if (!(p.reserved1 & 2)) *reinterpret_cast<float4*>(p.y + m * p.y_ps + p.y_c0 + n0) = v;
      }
    }
    wave_lds_sync();  // wave-private LDS region
  }
}

// ---------------------------------------------------------------------------
// 3x3 / stride-1 / pad-1 convs with few input channels (Cin <= 64: the SSH
// branches and FPN merges, Cin 40 / 12 at 128^2 and 64^2).  The generic
// kernel re-reads every input pixel 9x per K chunk through L1; here a
// workgroup stages its (8+2) x (16+2) x Cin input window once into LDS
// (ECA gate applied while staging, zero padding written explicitly) and the
// four waves — two output rows of 16 pixels each — take every A fragment
// from LDS.  Same packed weights, MFMA mapping and vector epilogue (split
// output for the fused SSH branches) as conv_gemm_kernel.  tconv = 1 (the
// stride-1 data gradient, transposed weights) reads the window flipped.
// ---------------------------------------------------------------------------
constexpr int k3Cols = 16, k3IC = k3Cols + 2;

template <int TN, int TM>
__global__ __launch_bounds__(256) void conv3x3_tile_kernel(const ConvArgs p, int tiles_w,
                                                           int tiles_img) {
  constexpr int k3Rows = 4 * TM, k3IR = k3Rows + 2;  // TM output rows per wave
  extern __shared__ float c3_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int nblk_n = p.Ntiles / TN;
  const int nb = blockIdx.x % nblk_n;
  const int tile = blockIdx.x / nblk_n;
  const int b = tile / tiles_img;
  const int tr = tile - b * tiles_img;
  const int oh0 = (tr / tiles_w) * k3Rows, ow0 = (tr % tiles_w) * k3Cols;
  const int C4 = p.Cin >> 2;
  const int PIT = p.Cin + 4;  // pixel pitch in LDS (floats)
  // stage the input window: (k3IR x k3IC pixels) x Cin channels
  {
    const float* xb = p.x + (int64_t)b * p.x_bs + p.x_c0;
    const float* sb = p.ascale ? p.ascale + (int64_t)b * p.ascale_bs : nullptr;
    for (int i = threadIdx.x; i < k3IR * k3IC * C4; i += 256) {
      const int px = i / C4, c4 = i - px * C4;
      const int r = px / k3IC, c = px - r * k3IC;
      const int ih = oh0 - 1 + r, iw = ow0 - 1 + c;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) {
        v = *reinterpret_cast<const float4*>(xb + ((int64_t)ih * p.W + iw) * p.x_ps + 4 * c4);
        if (sb) {
          const float4 s4 = *reinterpret_cast<const float4*>(sb + 4 * c4);
          v.x *= s4.x; v.y *= s4.y; v.z *= s4.z; v.w *= s4.w;
        }
      }
      *reinterpret_cast<float4*>(c3_lds + px * PIT + 4 * c4) = v;
    }
  }
  __syncthreads();

  f32x4 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const float4* wbase = reinterpret_cast<const float4*>(p.w) + ((int64_t)nb * TN) * 64 + lane;
  const int64_t wstride_k = (int64_t)p.Ntiles * 64;
  const int Ktot = 9 * p.Cin;
  // this lane's k4 = 16 kc + 4g walks (tap, channel) incrementally
  int tci = 4 * g, tap = 0;
  while (tci >= p.Cin) { tci -= p.Cin; ++tap; }
  float4 b_cur[TN];
#pragma unroll
  for (int u = 0; u < TN; ++u) b_cur[u] = wbase[u * 64];
  for (int kc = 0; kc < p.Kc; ++kc) {
    float4 b_nxt[TN];
    const bool more = kc + 1 < p.Kc;
    if (more) {
#pragma unroll
      for (int u = 0; u < TN; ++u) b_nxt[u] = wbase[(kc + 1) * wstride_k + u * 64];
    }
    float4 a[TM];
    const bool kv = 16 * kc + 4 * g < Ktot;
    // forward: tap (kh, kw) reads window offset (kh, kw); the stride-1 data
    // gradient (tconv) reads dy at (oh + 1 - kh, ow + 1 - kw): offset (2-kh, 2-kw)
    int kh = tap / 3, kw = tap - 3 * (tap / 3);
    if (p.tconv) {
      kh = 2 - kh;
      kw = 2 - kw;
    }
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int r = wave * TM + t + kh;  // window row
      a[t] = kv ? *reinterpret_cast<const float4*>(c3_lds + (r * k3IC + j + kw) * PIT + tci)
                : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].x, a[t].x, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].y, a[t].y, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].z, a[t].z, acc[t][u], 0, 0, 0);
        acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b_cur[u].w, a[t].w, acc[t][u], 0, 0, 0);
      }
    tci += 16;
    while (tci >= p.Cin) { tci -= p.Cin; ++tap; }
    if (more) {
#pragma unroll
      for (int u = 0; u < TN; ++u) b_cur[u] = b_nxt[u];
    }
  }
  __syncthreads();  // the input window is dead: its LDS becomes the epilogue's

  // epilogue: acc[t][u][r] = Y[pixel (oh0 + wave*TM + t, ow0 + j)][16(nb*TN+u) + 4g + r]
  constexpr int LDW = 16 * TN + 4;
  float* sm = c3_lds + wave * 16 * LDW;
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int oh = oh0 + wave * TM + t, ow = ow0 + j;
    const bool pv = oh < p.OH && ow < p.OW;
#pragma unroll
    for (int u = 0; u < TN; ++u)
      *reinterpret_cast<f32x4*>(sm + j * LDW + 16 * u + 4 * g) = acc[t][u];
    const int64_t pix = (int64_t)oh * p.OW + ow;
    const long long yoff = pv ? (long long)((int64_t)b * p.y_bs + pix * p.y_ps + p.y_c0) : -1;
    const long long y2off = p.y2 ? (long long)((int64_t)b * p.y2_bs + pix * p.y2_ps + p.y2_c0) : 0;
    wave_lds_sync();
#pragma unroll
    for (int f0 = 0; f0 < 16 * 4 * TN; f0 += 64) {
      const int f = f0 + lane;
      const int q = f / (4 * TN), c4 = f - q * (4 * TN);
      const long long yo = __shfl(yoff, q);
      const long long y2o = __shfl(y2off, q);
      const int n0 = nb * TN * 16 + 4 * c4;
      if (yo >= 0 && n0 < p.Cout) {
        float4 v = *reinterpret_cast<const float4*>(sm + q * LDW + 4 * c4);
        if (p.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + n0);
          v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
        }
        if (p.y2 && n0 >= p.nsplit) {
          v.x = act_apply(v.x, p.act2, p.slope2);
          v.y = act_apply(v.y, p.act2, p.slope2);
          v.z = act_apply(v.z, p.act2, p.slope2);
          v.w = act_apply(v.w, p.act2, p.slope2);
          *reinterpret_cast<float4*>(p.y2 + y2o + (n0 - p.nsplit)) = v;
        } else {
          v.x = act_apply(v.x, p.act, p.slope);
          v.y = act_apply(v.y, p.act, p.slope);
          v.z = act_apply(v.z, p.act, p.slope);
          v.w = act_apply(v.w, p.act, p.slope);
          *reinterpret_cast<float4*>(p.y + yo + n0) = v;
        }
      }
    }
    wave_lds_sync();
  }
}

// JABD_CONV3X3_TILE=0 disables the LDS-tiled 3x3 kernel, =2 keeps it for
// forward convs only (A/B).
static bool conv3x3_tile_on(bool tconv) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JABD_CONV3X3_TILE");
    v = e && e[0] == '0' ? 0 : (e && e[0] == '2' ? 2 : 1);
  }
  return v == 1 || (v == 2 && !tconv);
}

static int conv3x3_rows_per_wave() {  // JABD_CONV3X3_TM=2|4 (A/B; 4 measured 5% slower)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JABD_CONV3X3_TM");
    v = e && e[0] == '4' ? 4 : 2;
  }
  return v;
}

static int launch_conv3x3_tile(const ConvArgs& a, hipStream_t st) {
  const int tn = a.tn;
  int tm = conv3x3_rows_per_wave();
  if (tm == 4 && (int64_t)a.B * cdiv(a.OH, 16) * cdiv(a.OW, k3Cols) < 1024) tm = 2;
  const int rows = 4 * tm;
  const int tiles_w = (int)cdiv(a.OW, k3Cols), tiles_h = (int)cdiv(a.OH, rows);
  const int tiles_img = tiles_w * tiles_h;
  const int64_t grid = (int64_t)a.B * tiles_img * (a.Ntiles / tn);
  JABD_REQUIRE(grid < (int64_t)0x7fffffff, "conv3x3: grid too large");
  const size_t lds_in = (size_t)(rows + 2) * k3IC * (a.Cin + 4) * sizeof(float);
  const size_t lds_epi = (size_t)4 * 16 * (16 * tn + 4) * sizeof(float);
  const size_t lds = std::max(lds_in, lds_epi);
  if (lds > 64 * 1024) return -1;
#define C3_CASE(TN_, TM_)                                                                    \
  if (tn == TN_ && tm == TM_) {                                                              \
    conv3x3_tile_kernel<TN_, TM_><<<(unsigned)grid, 256, lds, st>>>(a, tiles_w, tiles_img);  \
    return check_launch("conv3x3_tile");                                                     \
  }
  C3_CASE(1, 2) C3_CASE(2, 2) C3_CASE(3, 2) C3_CASE(1, 4) C3_CASE(2, 4) C3_CASE(3, 4)
#undef C3_CASE
  return -1;
}

template <int TM, int TN>
static int launch_1x1(const ConvArgs& a, hipStream_t st) {
  const int64_t grid = cdiv(a.M, (int64_t)4 * 16 * TM) * (a.Ntiles / TN);
  JABD_REQUIRE(grid < (int64_t)0x7fffffff, "conv: grid too large");
  const int x2 = !a.x2 ? 0 : (a.x2_stride == 1 ? 1 : 2);
  const bool as = a.ascale != nullptr;
#define C1_CASE(X2_, AS_)                                                    \
  if (x2 == X2_ && as == AS_) {                                              \
    conv1x1_kernel<TM, TN, X2_, AS_><<<(unsigned)grid, 256, 0, st>>>(a);     \
    return check_launch("conv1x1");                                          \
  }
  C1_CASE(0, false) C1_CASE(0, true) C1_CASE(1, false) C1_CASE(1, true)
  C1_CASE(2, false) C1_CASE(2, true)
#undef C1_CASE
  return JABD_EINVAL;
}

template <int TM, int TN>
static int launch_conv(const ConvArgs& a, bool vec4, hipStream_t st) {
  const int64_t rows_per_blk = 4 * 16 * TM;
  const int64_t mblk = cdiv(a.M, rows_per_blk);
  const int64_t nblk = a.Ntiles / TN;
  const int64_t grid = mblk * nblk;
  JABD_REQUIRE(grid < (int64_t)0x7fffffff, "conv: grid too large");
  if (vec4)
    conv_gemm_kernel<TM, TN, true><<<(unsigned)grid, 256, 0, st>>>(a);
  else
    conv_gemm_kernel<TM, TN, false><<<(unsigned)grid, 256, 0, st>>>(a);
  return check_launch("conv_gemm");
}

}  // namespace jabd

using namespace jabd;

namespace jabd {
// (tn, tm) -> kernel instance; -1 when not instantiated.
template <bool FAST>
static int dispatch_conv(const ConvArgs& a, int tn, int tm, bool vec4, hipStream_t st) {
#define DC(TM_, TN_)                                                         \
  if (tm == TM_ && tn == TN_)                                                \
    return FAST ? launch_1x1<TM_, TN_>(a, st) : launch_conv<TM_, TN_>(a, vec4, st);
  DC(4, 1) DC(2, 1) DC(1, 1) DC(4, 2) DC(2, 2) DC(1, 2) DC(4, 3) DC(2, 3) DC(1, 3)
  DC(4, 4) DC(2, 4) DC(1, 4) DC(4, 5) DC(2, 5) DC(1, 5) DC(2, 8) DC(1, 8)
#undef DC
  return -1;
}
}  // namespace jabd

extern "C" int jabd_conv_pack_tn(int cout) {
  // N-tile group per launch: minimise padded columns, cap accumulators.
  int tiles = (cout + 15) / 16;
  if (tiles <= 5) return tiles;
  int best = 4, waste = 1 << 30;
  for (int tn : {4, 5, 8}) {
    int grp = (tiles + tn - 1) / tn;
    int w = grp * tn - tiles;
    if (w < waste || (w == waste && tn > best)) { waste = w; best = tn; }
  }
  return best;
}

// JABD_CONV_GENERIC=1 forces the generic implicit-GEMM kernel (A/B tests).
static bool conv_generic_only() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JABD_CONV_GENERIC");
    v = e && e[0] == '1' ? 1 : 0;
  }
  return v == 1;
}

namespace jabd {
bool stem7_ok(const ConvArgs& a);
int stem7_fwd_launch(const ConvArgs& a, hipStream_t st);
int conv1x1_m32_dispatch(const ConvArgs& a, hipStream_t st, bool kxk);
int conv_m32_stats_dispatch(const ConvArgs& a, bool kxk, float* part, const BnEpi& bb,
                            hipStream_t st);
int64_t bn_rows_sum_doubles(int64_t M, int C);
int64_t bn_rows_chunk_doubles(int64_t M, int C);
int bn_rows_final_launch(const float* rows, int ldc, int64_t M, int C, double* chunks,
                         float* mean, float* invstd, float* rmean, float* rvar, float momentum,
                         float eps, hipStream_t st);
int conv1x1_stream_dispatch(const ConvArgs& a, hipStream_t st, StreamStats* ss = nullptr);
}

// Which 1x1 kernel: the 32x32x2 LDS-weight kernel (conv32.hip) pays off when
// the GEMM is compute-heavy.  JABD_CONV32=0 / 1 forces it off / on (A/B).
static bool use_conv32(const ConvArgs& a) {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("JABD_CONV32");
    v = e && e[0] == '0' ? 0 : (e && e[0] == '1' ? 1 : -1);
  }
  if (!a.w32 || a.tn32 <= 0 || a.ntiles32 % a.tn32 || a.ntiles32 * 32 < a.Cout) return false;
  if (v >= 0) return v == 1;
  // K 64 / 128 1x1s into >= 64 channels: the 32x32 kernel's streaming form
  // (conv1x1_m32s_kernel; R50 l1.c3-shaped GEMM 2190 -> 2005 us vs conv.hip)
  if (a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && !a.x2 && !a.ascale && !a.y2 &&
      !a.tconv && (a.Cin == 64 || a.Cin == 128) && a.Cout >= 64)
    return true;
  const int K = a.KH * a.KW * a.Cin + (a.x2 ? a.Cin2 : 0);
  if (a.KH * a.KW > 1) return a.Cout >= 64 && K >= 288;
  return a.Cout >= 96 && K >= 96;
}

// Argument checks shared by the conv entry points; fills a (M, flags) and
// reports whether the fast 1x1 kernels take the layout.
static int conv_setup(const jabd_conv_args* args, ConvArgs& a, bool& fast1x1, bool& vec4) {
  JABD_REQUIRE(args, "conv: null args");
  a = *args;
  JABD_REQUIRE(a.x && a.w && a.y, "conv: null pointer");
  JABD_REQUIRE(a.B > 0 && a.Cin > 0 && a.Cout > 0 && a.KH > 0 && a.KW > 0 && a.stride > 0,
               "conv: bad shape");
  if (a.tconv) {  // data gradient: (OH, OW) is the forward input size, (H, W) its output
    JABD_REQUIRE(a.H == (a.OH + 2 * a.pad - a.KH) / a.stride + 1 &&
                     a.W == (a.OW + 2 * a.pad - a.KW) / a.stride + 1 && !a.nchw_in && !a.x2,
                 "conv: transposed-conv size mismatch");
  } else {
    JABD_REQUIRE(a.OH == (a.H + 2 * a.pad - a.KH) / a.stride + 1 &&
                     a.OW == (a.W + 2 * a.pad - a.KW) / a.stride + 1,
                 "conv: output size mismatch");
  }
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
  JABD_REQUIRE(!a.y2 || (a.nsplit > 0 && a.nsplit % 4 == 0 && a.nsplit < a.Cout &&
                         a.y2_ps % 4 == 0 && a.y2_c0 % 4 == 0 && a.y2_bs % 4 == 0 &&
                         (reinterpret_cast<uintptr_t>(a.y2) & 15) == 0 && !a.res && !a.tconv),
               "conv: split output needs nsplit %% 4 == 0, 16-byte aligned y2, no residual");
  JABD_REQUIRE(!a.x2 || ((a.KH * a.KW * a.Cin) % 4 == 0 && a.Cin2 % 4 == 0 && a.x2_ps % 4 == 0 &&
                         a.x2_stride > 0 && !a.nchw_in),
               "conv: K-concat needs K and Cin2 multiples of 4");
  (void)is1x1;
  const int Ktot = a.KH * a.KW * a.Cin + (a.x2 ? a.Cin2 : 0);
  JABD_REQUIRE(a.Kc == (Ktot + 15) / 16, "conv: Kc=%d, expected %d", a.Kc, (Ktot + 15) / 16);
  const int tiles = (a.Cout + 15) / 16;
  JABD_REQUIRE(a.Ntiles >= tiles, "conv: Ntiles=%d < %d", a.Ntiles, tiles);
  a.M = (int64_t)a.B * a.OH * a.OW;
  JABD_REQUIRE(a.M < (int64_t)0x7fffffff, "conv: B*OH*OW must be < 2^31");
  {
    const uintptr_t al = reinterpret_cast<uintptr_t>(a.y) | reinterpret_cast<uintptr_t>(a.bias) |
                         reinterpret_cast<uintptr_t>(a.res);
    const bool v4 = a.Cout % 4 == 0 && a.y_ps % 4 == 0 && a.y_c0 % 4 == 0 && a.y_bs % 4 == 0 &&
                    (!a.res || (a.res_ps % 4 == 0 && a.res_c0 % 4 == 0 && a.res_bs % 4 == 0)) &&
                    (al & 15) == 0;
    a.flags = v4 ? 1 : 0;
    JABD_REQUIRE(!a.y2 || v4, "conv: split output needs the vector epilogue layout");
  }
  vec4 = !a.nchw_in && a.Cin % 4 == 0 && a.x_ps % 4 == 0 && a.x_c0 % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(a.x) & 15) == 0;
  JABD_REQUIRE(a.tn > 0 && a.Ntiles % a.tn == 0, "conv: Ntiles %% tn != 0");
  const int64_t OHW = (int64_t)a.OH * a.OW;
  const int64_t maxps = std::max<int64_t>(std::max<int64_t>(a.x_ps, a.y_ps),
                                          std::max<int64_t>(a.res ? a.res_ps : 0,
                                                            a.x2 ? a.x2_ps : 0));
  fast1x1 =
      is1x1 && !a.tconv && vec4 && (a.flags & 1) && !a.y2 && a.x_bs == OHW * a.x_ps &&
      a.y_bs == OHW * a.y_ps && (!a.res || a.res_bs == OHW * a.res_ps) &&
      (!a.ascale || a.ascale_bs % 4 == 0) &&
      (!a.x2 || (a.x2_stride == 1 ? (a.x2_W == a.OW && a.x2_bs == OHW * a.x2_ps)
                                  : (a.x2_stride > 1 && a.x2_bs % a.x2_ps == 0 &&
                                     a.x2_bs * a.B < ((int64_t)1 << 31)))) &&
      (a.M + 64) * (maxps + 16) < ((int64_t)1 << 31) && !conv_generic_only();
  return 0;
}

// The statistics form of the streaming 1x1 conv serves the layer iff the
// plain entry point would route it to the streaming kernel and it carries no
// gate, second source or residual.
static bool conv_stats_form(const ConvArgs& a, bool fast1x1) {
  return fast1x1 && !use_conv32(a) && !a.reserved1 && !a.ascale && !a.x2 && !a.res;
}

extern "C" int64_t jabd_conv1x1_bn_stats_nblk(const jabd_conv_args* args) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false;
  if (conv_setup(args, a, fast1x1, vec4) != JABD_OK || !conv_stats_form(a, fast1x1)) return 0;
  jabd::StreamStats ss{nullptr, nullptr, 0, true};
  if (jabd::conv1x1_stream_dispatch(a, nullptr, &ss) != 0) return 0;
  return ss.nblk;
}

extern "C" int jabd_conv1x1_bn_stats_f32(const jabd_conv_args* args, float* part, int64_t nblk,
                                         float* shift, jabd_stream_t stream) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false;
  const int e = conv_setup(args, a, fast1x1, vec4);
  if (e != JABD_OK) return e;
  JABD_REQUIRE(conv_stats_form(a, fast1x1),
               "conv1x1_bn_stats: layer not served by the streaming statistics form");
  jabd::StreamStats ss{part, shift, nblk, false};
  const int r = jabd::conv1x1_stream_dispatch(a, as_stream(stream), &ss);
  JABD_REQUIRE(r >= 0, "conv1x1_bn_stats: no streaming kernel for this shape");
  return r;
}

// The 32x32 GEMM's statistics form (conv32.hip, ST): a bias-free,
// activation-free forward conv with no gate, residual, second source or
// split output whose BatchNorm follows — the ResNet-50 bottleneck convs
// (nets/resnet_pytorch_r.py:122-143).  The GEMM takes the shape even where
// use_conv32's throughput heuristic would pick another kernel (the saved
// statistics pass outweighs it); JABD_CONV_STATS32=0 turns the form off.
static bool conv_m32_stats_form(const ConvArgs& a, bool fast1x1, bool vec4, bool& kxk) {
  static const bool on = [] {
    const char* e = getenv("JABD_CONV_STATS32");
    return !(e && e[0] == '0');
  }();
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
  kxk = !is1x1;
  const int64_t OHW = (int64_t)a.OH * a.OW;
  if (!on || conv_generic_only() || a.bias || a.res || a.ascale || a.x2 || a.y2 ||
      a.act != ACT_NONE || a.tconv || a.nchw_in || !(a.flags & 1) || a.Cout % 4)
    return false;
  if (!a.w32 || a.tn32 < 1 || a.tn32 > 4 || a.ntiles32 % a.tn32 || a.ntiles32 * 32 < a.Cout)
    return false;
  if (is1x1) return fast1x1;
  return vec4 && a.Cin % 32 == 0 && a.x_bs % 4 == 0 && a.y_bs == OHW * a.y_ps;
}

// floats of the statistics rows (ceil(M / 32) x 2 x ntiles32 * 32) followed
// by the fp64 chunk sums (8-byte aligned)
static int64_t conv_stats_rows_floats(const ConvArgs& a) {
  return cdiv(a.M, (int64_t)32) * 2 * a.ntiles32 * 32;
}

extern "C" int64_t jabd_conv_bn_stats_part_floats(const jabd_conv_args* args) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false, kxk = false;
  if (conv_setup(args, a, fast1x1, vec4) != JABD_OK || !conv_m32_stats_form(a, fast1x1, vec4, kxk))
    return 0;
  const int64_t rows = (conv_stats_rows_floats(a) + 1) & ~(int64_t)1;
  return rows + 2 * bn_rows_chunk_doubles(a.M, a.Cout);
}

extern "C" int jabd_conv_bn_stats_f32(const jabd_conv_args* args, float* part, int64_t part_floats,
                                      float* mean, float* invstd, float* running_mean,
                                      float* running_var, float momentum, float eps,
                                      jabd_stream_t stream) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false, kxk = false;
  {
    const int e = conv_setup(args, a, fast1x1, vec4);
    if (e != JABD_OK) return e;
  }
  JABD_REQUIRE(conv_m32_stats_form(a, fast1x1, vec4, kxk),
               "conv_bn_stats: layer not served by the 32x32 statistics form");
  const int64_t rows = (conv_stats_rows_floats(a) + 1) & ~(int64_t)1;
  JABD_REQUIRE(part && mean && invstd && part_floats >= rows + 2 * bn_rows_chunk_doubles(a.M, a.Cout),
               "conv_bn_stats: part holds %lld floats, %lld needed", (long long)part_floats,
               (long long)(rows + 2 * bn_rows_chunk_doubles(a.M, a.Cout)));
  JABD_REQUIRE(((uintptr_t)part & 15) == 0, "conv_bn_stats: part must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const int r = conv_m32_stats_dispatch(a, kxk, part, BnEpi{}, st);
  if (r != JABD_OK) return r < 0 ? JABD_EINVAL : r;
  return bn_rows_final_launch(part, a.ntiles32 * 32, a.M, a.Cout,
                              reinterpret_cast<double*>(part + rows), mean, invstd, running_mean,
                              running_var, momentum, eps, st);
}

// The BatchNorm-backward form (BB): a bias-free data gradient (1x1 plain,
// or k x k transposed at stride 1) whose output is the dy of a BatchNorm +
// ReLU / LeakyReLU / identity with Cout % 32 == 0 (the R50 bottleneck's bn1 /
// bn2 backward, nets/resnet_pytorch_r.py:122-143).
static bool conv_m32_bb_form(const ConvArgs& a, bool fast1x1, bool vec4, bool& kxk) {
  static const bool on = [] {
    const char* e = getenv("JABD_CONV_BNBWD32");
    return !(e && e[0] == '0');
  }();
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && !a.tconv;
  kxk = !is1x1;
  const int64_t OHW = (int64_t)a.OH * a.OW;
  if (!on || conv_generic_only() || a.bias || a.res || a.ascale || a.x2 || a.y2 ||
      a.act != ACT_NONE || a.nchw_in || !(a.flags & 1) || a.Cout % 32)
    return false;
  if (!a.w32 || a.tn32 < 1 || a.tn32 > 4 || a.ntiles32 % a.tn32 || a.ntiles32 * 32 != a.Cout)
    return false;
  if (is1x1) return fast1x1;
  return vec4 && a.Cin % 32 == 0 && a.x_bs % 4 == 0 && a.y_bs == OHW * a.y_ps &&
         (!a.tconv || a.stride == 1);
}

extern "C" int64_t jabd_conv_bn_bwd_part_floats(const jabd_conv_args* args) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false, kxk = false;
  if (conv_setup(args, a, fast1x1, vec4) != JABD_OK || !conv_m32_bb_form(a, fast1x1, vec4, kxk))
    return 0;
  return cdiv(a.M, (int64_t)32) * 2 * a.Cout + 2 * bn_rows_sum_doubles(a.M, a.Cout);
}

extern "C" int jabd_conv_bn_bwd_sums_f32(const jabd_conv_args* args, const float* x, int32_t x_ps,
                                         const float* mean, const float* invstd,
                                         const float* gamma, const float* beta, int32_t act,
                                         float slope, float* part, int64_t part_floats,
                                         jabd_stream_t stream) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false, kxk = false;
  {
    const int e = conv_setup(args, a, fast1x1, vec4);
    if (e != JABD_OK) return e;
  }
  JABD_REQUIRE(conv_m32_bb_form(a, fast1x1, vec4, kxk),
               "conv_bn_bwd_sums: layer not served by the 32x32 BatchNorm-backward form");
  JABD_REQUIRE(x && mean && invstd && gamma && beta && part && x_ps % 4 == 0 && x_ps >= a.Cout &&
                   (act == ACT_NONE || act == ACT_RELU || act == ACT_LEAKY),
               "conv_bn_bwd_sums: bad BatchNorm arguments");
  const int64_t need = cdiv(a.M, (int64_t)32) * 2 * a.Cout + 2 * bn_rows_sum_doubles(a.M, a.Cout);
  JABD_REQUIRE(part_floats >= need && ((uintptr_t)part & 15) == 0,
               "conv_bn_bwd_sums: part holds %lld floats, %lld needed (16-byte aligned)",
               (long long)part_floats, (long long)need);
  BnEpi bb{x, mean, invstd, gamma, beta, part, x_ps, act, slope};
  const int r = conv_m32_stats_dispatch(a, kxk, nullptr, bb, as_stream(stream));
  return r < 0 ? JABD_EINVAL : r;
}

// The residual-ReLU form (R50 bn3): a bias-free 1x1 data gradient y = dx +
// args->res whose output is the dy of out = relu(bn(x) + identity); the
// GEMM writes dz = y * [out > 0] (out = mask, the block output saved by the
// forward) and the per-32-pixel-tile sums of dz and dz * xhat into part, in
// jabd_conv_bn_bwd_sums_f32's layout (jabd_bn_act_bwd_rows_f32 with act none
// finishes the BatchNorm backward from them).
extern "C" int jabd_conv_bn_bwd_sums_res_f32(const jabd_conv_args* args, const float* x,
                                             int32_t x_ps, const float* mask, int32_t mask_ps,
                                             const float* mean, const float* invstd, float* part,
                                             int64_t part_floats, jabd_stream_t stream) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false, kxk = false;
  {
    const int e = conv_setup(args, a, fast1x1, vec4);
    if (e != JABD_OK) return e;
  }
  ConvArgs ab = a;  // the form check without the residual
  ab.res = nullptr;
  JABD_REQUIRE(conv_m32_bb_form(ab, fast1x1, vec4, kxk) && !kxk,
               "conv_bn_bwd_sums_res: layer not served (1x1 / stride-1 32x32 form only)");
  JABD_REQUIRE(!a.res || (a.res_ps % 4 == 0 && a.res_c0 % 4 == 0),
               "conv_bn_bwd_sums_res: residual rows must be float4-aligned");
  JABD_REQUIRE(x && mask && mean && invstd && part && x_ps % 4 == 0 && x_ps >= a.Cout &&
                   mask_ps % 4 == 0 && mask_ps >= a.Cout,
               "conv_bn_bwd_sums_res: bad BatchNorm arguments");
  const int64_t need = cdiv(a.M, (int64_t)32) * 2 * a.Cout + 2 * bn_rows_sum_doubles(a.M, a.Cout);
  JABD_REQUIRE(part_floats >= need && ((uintptr_t)part & 15) == 0,
               "conv_bn_bwd_sums_res: part holds %lld floats, %lld needed (16-byte aligned)",
               (long long)part_floats, (long long)need);
  BnEpi bb{x, mean, invstd, nullptr, nullptr, part, x_ps, ACT_NONE, 0.f, mask, mask_ps};
  const int r = conv_m32_stats_dispatch(a, false, nullptr, bb, as_stream(stream));
  return r < 0 ? JABD_EINVAL : r;
}

extern "C" int jabd_conv2d_nhwc_f32(const jabd_conv_args* args, jabd_stream_t stream) {
  ConvArgs a;
  bool fast1x1 = false, vec4 = false;
  {
    const int e = conv_setup(args, a, fast1x1, vec4);
    if (e != JABD_OK) return e;
  }
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
  hipStream_t st = as_stream(stream);
  const int tn = a.tn;
  const int64_t OHW = (int64_t)a.OH * a.OW;
  // ResNet-50 7x7/s2 stem over the NCHW input (stem7.hip); JABD_STEM7=0 -> generic
  static const bool stem7_on = [] {
    const char* e = getenv("JABD_STEM7");
    return !(e && e[0] == '0');
  }();
  if (stem7_on && stem7_ok(a) && (a.flags & 1) && (a.act == ACT_NONE || a.act == ACT_RELU) &&
      a.Ntiles >= 4 && !conv_generic_only())
    return stem7_fwd_launch(a, st);
  if (fast1x1 && use_conv32(a)) {
    const int r = conv1x1_m32_dispatch(a, st, false);
    if (r >= 0) return r;
  }
  if (fast1x1 && !a.reserved1) {  // short-K / narrow-N: streaming kernel (conv_stream.hip)
    const int r = conv1x1_stream_dispatch(a, st);
    if (r >= 0) return r;
  }
  // k x k implicit GEMM on the 32x32 kernel: 32-channel stages inside one tap
  if (!is1x1 && vec4 && (a.flags & 1) && !a.x2 && !a.y2 && a.Cin % 32 == 0 &&
      (!a.tconv || a.stride == 1 || (a.stride == 2 && !a.ascale)) && a.x_bs % 4 == 0 &&
      a.y_bs == OHW * a.y_ps && (!a.res || a.res_bs == OHW * a.res_ps) && use_conv32(a)) {
    const int r = conv1x1_m32_dispatch(a, st, true);
    if (r >= 0) return r;
  }
  if (!is1x1 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && !a.nchw_in &&
      !a.x2 && !a.res && vec4 && (a.flags & 1) && a.Cin <= 64 && a.tn <= 3 &&
      (!a.ascale || a.ascale_bs % 4 == 0) && conv3x3_tile_on(a.tconv)) {
    const int r = launch_conv3x3_tile(a, st);
    if (r >= 0) return r;
  }
  // Pixel tiles per wave: 4 x 16 by default; small-M layers (the SSH / FPN
  // convs at 32x32 and 64x64) drop to 2 or 1 so the grid still fills the
  // 256 CUs several times over.
  const int64_t nblk_n = a.Ntiles / tn;
  auto grid_for = [&](int tm) { return cdiv(a.M, (int64_t)64 * tm) * nblk_n; };
  // Short-K GEMMs are load-latency bound with few k-steps per wave: fewer
  // pixel tiles per wave (fewer VGPRs, more resident waves) overlap more
  // loads with MFMAs (measured on the C2 layers: tools/convbench.py).
  const int Kall = a.KH * a.KW * a.Cin + (a.x2 ? a.Cin2 : 0);
  const int tm_max = tn == 8 ? 2 : (Kall <= 32 ? 2 : (Kall <= 160 ? 1 : (Kall <= 400 ? 2 : 4)));
  int tm = tm_max;
  while (tm > 1 && grid_for(tm) < 1024) tm >>= 1;
  {  // JABD_CONV_TM=1|2|4 forces the pixel tiles per wave (A/B experiments)
    static int ftm = -1;
    if (ftm < 0) {
      const char* e = getenv("JABD_CONV_TM");
      ftm = e ? atoi(e) : 0;
    }
    if (ftm == 1 || ftm == 2 || (ftm == 4 && tn != 8)) tm = ftm;
  }
  const int r = fast1x1 ? dispatch_conv<true>(a, tn, tm, vec4, st) : -1;
  if (r >= 0) return r;
  const int r2 = dispatch_conv<false>(a, tn, tm, vec4, st);
  if (r2 >= 0) return r2;
  set_error("conv: unsupported tn=%d", tn);
  return JABD_EINVAL;
}

// ---------------------------------------------------------------------------
// MobileNetV3 stem: conv3x3/s2/p1, 3 -> 16 channels, read straight from the
// NCHW network input (layout conversion fused), folded BN + activation,
// NHWC output.  One thread per output column, kStemRows output rows.
//  - all (2 kStemRows + 1) x 9 input values are loaded up front (the input
//    row shared by two output rows once: 45 loads for 2 pixels instead of
//    54; 2 rows per thread measured 245 -> 226 us at bs32 1024^2);
//  - the 27x16 weights and the bias are read at wave-uniform addresses, so
//    they arrive through scalar loads and feed the FMAs as SGPR operands; an
//    empty asm with a memory clobber between taps keeps the compiler from
//    hoisting all 432 of them at once (that spills the scalar file);
//  - the 64 B per pixel go out through a wave-private LDS transpose, so each
//    store instruction writes one contiguous 1 KiB run of the wave's 4 KiB
//    NHWC block instead of 64 lanes at a 64 B stride.
// Reference: nets/mobilenetV3.py:455-457,511 (conv1 + bn1 + hs1).
// ---------------------------------------------------------------------------
namespace jabd {
constexpr int kStemOut = 16;
constexpr int kStemThreads = 128;
#ifndef STEM_ROWS
#define STEM_ROWS 2
#endif
constexpr int kStemRows = STEM_ROWS;  // output rows per thread

template <int ACT>
__global__ __launch_bounds__(kStemThreads) void stem_kernel(const float* __restrict__ x, int H,
                                                            int W, int OH, int OW,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            float* __restrict__ y) {
  __shared__ float4 st[kStemThreads / 64][64 * kStemOut / 4 + 64 / 8];  // +1 float4 per 8 px
  const int b = blockIdx.z, oh0 = blockIdx.y * kStemRows;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ow0 = blockIdx.x * kStemThreads + wave * 64;  // this wave's first pixel
  const int ow = ow0 + lane;
  const bool pv = ow < OW;
  const float* xb = x + (int64_t)b * 3 * H * W;
  const int64_t HW = (int64_t)H * W;
  // the 2 kStemRows + 1 input rows of this thread's kStemRows output rows
  // (rows shared by neighbouring output rows are loaded once)
  constexpr int IR = 2 * kStemRows + 1;
  float v[IR][9];
#pragma unroll
  for (int r = 0; r < IR; ++r) {
    const int ih = 2 * oh0 - 1 + r;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int iw = 2 * ow - 1 + kw;
      const bool ok = pv && ih >= 0 && ih < H && iw >= 0 && iw < W;
      const float* xp = xb + (ok ? (int64_t)ih * W + iw : 0);
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        const float t = xp[ci * HW];
        v[r][kw * 3 + ci] = ok ? t : 0.f;
      }
    }
  }
  auto f = [](float u) {
    return ACT == ACT_HSWISH ? hswish_f(u) : ACT == ACT_RELU ? relu_f(u) : u;
  };
  float4* sw = st[wave];
#pragma unroll
  for (int ro = 0; ro < kStemRows; ++ro) {
    const int oh = oh0 + ro;
    if (oh >= OH) break;
    float o[kStemOut];
#pragma unroll
    for (int n = 0; n < kStemOut; ++n) o[n] = bias[n];
#pragma unroll
    for (int tp = 0; tp < 27; ++tp) {
      asm volatile("" ::: "memory");
      const float* wr = w + tp * kStemOut;
      const float xv = v[2 * ro + tp / 9][tp % 9];   // tap (kh, kw, ci) = tp
#pragma unroll
      for (int n = 0; n < kStemOut; ++n) o[n] = fmaf(wr[n], xv, o[n]);
    }
    // pixel p's 4 float4 at st[4p + p/8 + q]: the pad keeps the 16 B writes of
    // 8 consecutive lanes on distinct banks
#pragma unroll
    for (int q = 0; q < kStemOut / 4; ++q)
      sw[4 * lane + (lane >> 3) + q] =
          make_float4(f(o[4 * q]), f(o[4 * q + 1]), f(o[4 * q + 2]), f(o[4 * q + 3]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region
    float4* yw = reinterpret_cast<float4*>(y + (((int64_t)b * OH + oh) * OW + ow0) * kStemOut);
    const int npx = min(64, OW - ow0);
#pragma unroll
    for (int q = 0; q < kStemOut / 4; ++q) {
      const int i = q * 64 + lane;  // float4 index in the wave's block
      const int p = i >> 2;
      if (p < npx) yw[i] = sw[i + (p >> 3)];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next row's writes
  }
}
}  // namespace jabd

extern "C" int jabd_stem_nchw_f32(const float* x, int32_t B, int32_t H, int32_t W,
                                  const float* w, const float* bias, int32_t act, float* y,
                                  jabd_stream_t stream) {
  JABD_REQUIRE(x && w && bias && y && B > 0 && H > 0 && W > 0, "stem: bad args");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  dim3 g((unsigned)cdiv(OW, kStemThreads), (unsigned)cdiv(OH, kStemRows), (unsigned)B);
  JABD_REQUIRE(act == ACT_HSWISH || act == ACT_RELU || act == ACT_NONE, "stem: act %d", act);
  hipStream_t st = as_stream(stream);
  if (act == ACT_HSWISH)
    stem_kernel<ACT_HSWISH><<<g, kStemThreads, 0, st>>>(x, H, W, OH, OW, w, bias, y);
  else if (act == ACT_RELU)
    stem_kernel<ACT_RELU><<<g, kStemThreads, 0, st>>>(x, H, W, OH, OW, w, bias, y);
  else
    stem_kernel<ACT_NONE><<<g, kStemThreads, 0, st>>>(x, H, W, OH, OW, w, bias, y);
  return check_launch("stem");
}
