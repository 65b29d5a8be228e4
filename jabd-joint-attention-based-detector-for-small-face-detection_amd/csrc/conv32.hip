// 1x1 stride-1 convolutions (A1 project/expand convs, A4 FPN laterals, A5
// ResNet 1x1s) on the 32x32x2 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
//   Y[m, n] = act( sum_k X[m, k] * W[k, n] + bias[n] (+ R[m, n]) )
//
// Why a second GEMM kernel next to conv.hip's 16x16x4 one: the 32x32 tile
// does 2x the FLOPs per operand register, so a wave's 64-pixel x 128-channel
// tile needs 6 float4 operands per 8 k (16x16x4: 12), and the weights of a
// K stage are staged ONCE per workgroup in LDS (shared by the 4 waves)
// instead of being re-read from L2 by every wave.  This serves the
// compute-heavy layers (K >= ~100, Cout >= ~96), where conv.hip sat at
// 30-45% of the fp32 MFMA peak.
//
// Operand mapping (swapped, as conv.hip): MFMA A = weights (row i = output
// channel), MFMA B = pixels (column j = pixel), so lane l ends up holding, for
// pixel j = l & 31, the channels 8*(r>>2) + 4*(l>>5) + (r&3): four float4
// runs of 4 consecutive channels.  The MFMA contracts k over the lane half
// (l >> 5); each lane loads a float4 of 4 consecutive channels and feeds
// component e to MFMA e, so within an 8-channel group the logical k order is
// (4h + e).  Weights are pre-packed in exactly that order (PackedConv.w32):
//   w32[k8][nt][lane] = float4{ W[8k8 + 4(lane>>5) + e][32nt + (lane&31)] }.
// One K stage is BK = 32 channels = 4 groups.
//
// Fusions: ECA gate (per-(image, input channel) scale) folded into the
// weights while staging them (a workgroup's pixels lie in one image);
// K-concatenated second source (MNv3 skip / ResNet downsample); bias;
// residual; activation; channel-offset / strided output.
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "conv_args.h"

namespace jabd {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float act32(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return relu_f(v);
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: return hswish_f(v);
    case ACT_HSIGMOID: return hsigmoid_f(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

constexpr int kBK = 32;          // K channels per stage

// LDS hand-off inside one wave (its private epilogue slice): the stores must
// land before the other lanes read them; no workgroup barrier needed.
__device__ __forceinline__ void wave_lds_sync32() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
constexpr int kG = kBK / 8;      // 8-channel groups per stage
constexpr int kGateLds = 1024;   // ECA gate channels staged in LDS

// The TM = 1 epilogue of one 32-pixel x 32*TN-channel wave tile (shared by
// conv1x1_m32_kernel and the streaming form conv1x1_m32s_kernel, so both
// produce the same bits): lane (h, j) holds pixel pm / output pixel om (-1:
// past M) and the accumulators acc[u][4c + e] of channels
// (nb*TN + u)*32 + 8c + 4h + e; ep is the wave's private LDS slice
// (32 x kEpiPitch floats); srow the tile's statistics row (ST / BB).
constexpr int kEpiPitch = 36;
// EPI: what the host guarantees about the plain epilogue terms — kEpiRt
// reads bias / residual / activation from p at run time; kEpiNone: no bias,
// no residual, identity activation (the statistics / BatchNorm-backward forms
// and plain data gradients); kEpiRes: the residual only.  The run-time form
// inlines every activation (incl. the sigmoid's division) at each of the 64
// element sites: ~5.6k instructions per kernel instead of ~1.5k.
enum { kEpiRt = 0, kEpiNone = 1, kEpiRes = 2 };
template <int TN, bool ST, bool BB, int EPI = kEpiRt>
__device__ __forceinline__ void m32_epilogue_tm1(const ConvArgs& p, const f32x16 (&acc)[TN],
                                                 int pm, int om, int nb, int srow, float* ep,
                                                 float* __restrict__ part, const BnEpi& bb,
                                                 int lane) {
  const bool has_bias = EPI == kEpiRt && p.bias;
  const bool has_res = EPI == kEpiRes || (EPI == kEpiRt && p.res);
  const int h = lane >> 5, j = lane & 31;
  const int ep_px = lane >> 3, ep_q = lane & 7;
  // the tile's pixel rows (pm < 0: past M) for the 8-pixel store groups
  int mrow[4], prow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    prow[r] = __shfl(pm, ep_px + 8 * r);
    mrow[r] = __shfl(om, ep_px + 8 * r);
  }
#pragma unroll
  for (int u = 0; u < TN; ++u) {
    const int nb0 = (nb * TN + u) * 32;
    if (nb0 >= p.Cout) break;  // wave-uniform
    const int n = nb0 + 4 * ep_q;
    float4 ss = make_float4(0.f, 0.f, 0.f, 0.f), sq = ss, sh = ss;
    float4 bmu = sh, bis = sh, bgm = sh, bbt = sh;
    float4 bx[4], bmk[4];
    if constexpr (BB) {  // issued before the LDS round trip: in flight across it
      if (n < p.Cout) {
        bmu = *reinterpret_cast<const float4*>(bb.mean + n);
        bis = *reinterpret_cast<const float4*>(bb.invstd + n);
        if (!bb.mask) {  // (the mask form takes no gamma / beta)
          bgm = *reinterpret_cast<const float4*>(bb.gamma + n);
          bbt = *reinterpret_cast<const float4*>(bb.beta + n);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)   // the BatchNorm input at the tile's pixels, in flight
        bx[r] = (prow[r] >= 0 && n < p.Cout)
                    ? *reinterpret_cast<const float4*>(bb.x + (int64_t)mrow[r] * bb.x_ps + n)
                    : sh;
      if (bb.mask) {  // mask form: the act's saved output, in flight as well
#pragma unroll
        for (int r = 0; r < 4; ++r)
          bmk[r] = (prow[r] >= 0 && n < p.Cout)
                       ? *reinterpret_cast<const float4*>(bb.mask + (int64_t)mrow[r] * bb.mask_ps + n)
                       : sh;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      *reinterpret_cast<float4*>(ep + j * kEpiPitch + 8 * c + 4 * h) =
          make_float4(acc[u][4 * c], acc[u][4 * c + 1], acc[u][4 * c + 2],
                      acc[u][4 * c + 3]);
    wave_lds_sync32();
    if constexpr (ST) sh = *reinterpret_cast<const float4*>(ep + 4 * ep_q);  // pixel 0
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int px = ep_px + 8 * r;
      if (prow[r] < 0 || n >= p.Cout) continue;
      float4 v = *reinterpret_cast<const float4*>(ep + px * kEpiPitch + 4 * ep_q);
      if (BB && bb.mask) {
        // dz = (y + res) * [mask > 0], written instead of y; as bn_bwd_part's
        // sums of dz and dz * xhat
        if (p.res) {
          const float4 rr = *reinterpret_cast<const float4*>(p.res + (int64_t)mrow[r] * p.res_ps +
                                                             p.res_c0 + n);
          v.x += rr.x; v.y += rr.y; v.z += rr.z; v.w += rr.w;
        }
        v.x *= bmk[r].x > 0.f ? 1.f : 0.f;
        v.y *= bmk[r].y > 0.f ? 1.f : 0.f;
        v.z *= bmk[r].z > 0.f ? 1.f : 0.f;
        v.w *= bmk[r].w > 0.f ? 1.f : 0.f;
        const float xh0 = (bx[r].x - bmu.x) * bis.x, xh1 = (bx[r].y - bmu.y) * bis.y;
        const float xh2 = (bx[r].z - bmu.z) * bis.z, xh3 = (bx[r].w - bmu.w) * bis.w;
        ss.x += v.x; ss.y += v.y; ss.z += v.z; ss.w += v.w;
        sq.x += v.x * xh0; sq.y += v.y * xh1; sq.z += v.z * xh2; sq.w += v.w * xh3;
        *reinterpret_cast<float4*>(p.y + (int64_t)mrow[r] * p.y_ps + p.y_c0 + n) = v;
        continue;
      }
      if constexpr (BB) {
        // as bn_bwd_part / bn_bwd_apply (train.hip): xhat, act'(xhat gamma + beta)
        const float xv[4] = {bx[r].x, bx[r].y, bx[r].z, bx[r].w};
        const float mu[4] = {bmu.x, bmu.y, bmu.z, bmu.w}, is[4] = {bis.x, bis.y, bis.z, bis.w};
        const float gm[4] = {bgm.x, bgm.y, bgm.z, bgm.w}, bt[4] = {bbt.x, bbt.y, bbt.z, bbt.w};
        const float gv[4] = {v.x, v.y, v.z, v.w};
        float dzs[4], dzx[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[e] - mu[e]) * is[e];
          const float z = fmaf(xh, gm[e], bt[e]);
          const float d = bb.act == ACT_RELU ? (z > 0.f ? 1.f : 0.f)
                          : bb.act == ACT_LEAKY ? (z > 0.f ? 1.f : bb.slope) : 1.f;
          dzs[e] = gv[e] * d;
          dzx[e] = dzs[e] * xh;
        }
        ss.x += dzs[0]; ss.y += dzs[1]; ss.z += dzs[2]; ss.w += dzs[3];
        sq.x += dzx[0]; sq.y += dzx[1]; sq.z += dzx[2]; sq.w += dzx[3];
      }
      if constexpr (ST) {
        const float dx = v.x - sh.x, dy = v.y - sh.y, dz = v.z - sh.z, dw = v.w - sh.w;
        ss.x += dx; ss.y += dy; ss.z += dz; ss.w += dw;
        sq.x = fmaf(dx, dx, sq.x); sq.y = fmaf(dy, dy, sq.y);
        sq.z = fmaf(dz, dz, sq.z); sq.w = fmaf(dw, dw, sq.w);
      }
      if (has_bias) {
        const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
      }
      if (has_res) {
        const float4 rr = *reinterpret_cast<const float4*>(p.res + (int64_t)mrow[r] * p.res_ps +
                                                           p.res_c0 + n);
        v.x += rr.x; v.y += rr.y; v.z += rr.z; v.w += rr.w;
      }
      if constexpr (EPI == kEpiRt) {
        v.x = act32(v.x, p.act, p.slope);
        v.y = act32(v.y, p.act, p.slope);
        v.z = act32(v.z, p.act, p.slope);
        v.w = act32(v.w, p.act, p.slope);
      }
      *reinterpret_cast<float4*>(p.y + (int64_t)mrow[r] * p.y_ps + p.y_c0 + n) = v;
    }
    if constexpr (BB) {
#pragma unroll
      for (int off = 8; off <= 32; off <<= 1) {
        ss.x += __shfl_xor(ss.x, off); ss.y += __shfl_xor(ss.y, off);
        ss.z += __shfl_xor(ss.z, off); ss.w += __shfl_xor(ss.w, off);
        sq.x += __shfl_xor(sq.x, off); sq.y += __shfl_xor(sq.y, off);
        sq.z += __shfl_xor(sq.z, off); sq.w += __shfl_xor(sq.w, off);
      }
      if (ep_px == 0 && (int64_t)srow * 32 < p.M && n < p.Cout) {
        const int ldc = p.Ntiles * 32;
        float* pr = bb.rows + (int64_t)srow * 2 * ldc + n;
        *reinterpret_cast<float4*>(pr) = ss;
        *reinterpret_cast<float4*>(pr + ldc) = sq;
      }
    }
    if constexpr (ST) {
      // the 8 lanes of one channel quad (lane xor 8, 16, 32), fixed order
#pragma unroll
      for (int off = 8; off <= 32; off <<= 1) {
        ss.x += __shfl_xor(ss.x, off); ss.y += __shfl_xor(ss.y, off);
        ss.z += __shfl_xor(ss.z, off); ss.w += __shfl_xor(ss.w, off);
        sq.x += __shfl_xor(sq.x, off); sq.y += __shfl_xor(sq.y, off);
        sq.z += __shfl_xor(sq.z, off); sq.w += __shfl_xor(sq.w, off);
      }
      const int64_t cnt = min<int64_t>(32, p.M - (int64_t)srow * 32);
      if (ep_px == 0 && cnt > 0 && n < p.Cout) {
        const float inv = 1.f / (float)cnt;
        const int ldc = p.Ntiles * 32;
        float* pr = part + (int64_t)srow * 2 * ldc + n;
        *reinterpret_cast<float4*>(pr) =
            make_float4(fmaf(ss.x, inv, sh.x), fmaf(ss.y, inv, sh.y), fmaf(ss.z, inv, sh.z),
                        fmaf(ss.w, inv, sh.w));
        *reinterpret_cast<float4*>(pr + ldc) =
            make_float4(fmaxf(sq.x - ss.x * ss.x * inv, 0.f), fmaxf(sq.y - ss.y * ss.y * inv, 0.f),
                        fmaxf(sq.z - ss.z * ss.z * inv, 0.f), fmaxf(sq.w - ss.w * ss.w * inv, 0.f));
      }
    }
    wave_lds_sync32();
  }
}

// Workgroup = 4 waves stacked along M (BM = 128*TM pixels) x BN = 32*TN
// channels.  Tiles never straddle an image when `per_img` (ECA gate folded
// into the staged weights), else M is tiled flat.
// KXK: k x k implicit GEMM (tap-major K; every 32-channel stage lies inside
// one tap, host guarantees Cin % 32 == 0, no K-concat source); stride-1
// transposed form (tconv) for the data gradient.
template <int TM, int TN, bool KXK, bool AS, bool ST = false, bool BB = false, int EPI = kEpiRt>
// AS: the ECA gate (ascale) is set — staged in LDS, applied at the weight store.
// ST (TM = 1, training forward, no bias / residual / act): the epilogue also
// writes the following BatchNorm's statistics per 32-pixel wave tile, row
// r = 4 mb + wave of part[r][0|1][Ntiles*32]: the tile's mean and sum of
// squared deviations (Sum (y - sh) and Sum (y - sh)^2 around the tile's first
// pixel, then mean = sh + S/n, M2 = Q - S^2/n); jabd_bn_stats_final_rows_f32
// combines the rows exactly (Chan) in a fixed order.
// BB (TM = 1, a data gradient whose output is the dy of a BatchNorm + act):
// the epilogue also reads that BatchNorm's input x at the tile's pixels and
// writes per 32-pixel wave tile the sums of dz = dy * act'(bn(x)) and of
// dz * xhat (bn_bwd_part's terms) to bb.rows[r][0|1][Ntiles*32] — the
// reduction pass over dy and x the BatchNorm backward would otherwise make.
// phase >= 0 (KXK, stride-2 tconv): this launch covers only the output
// pixels (2i + ph, 2j + pw), phase = 2 ph + pw, and only the taps that reach
// them — the sub-pixel decomposition of a strided data gradient (the other
// 3/4 of a naive transposed conv's taps read structural zeros).
// ks > 1 (split K): blockIdx.y takes K stages [y * ceil(S/ks), ...) and writes
// its raw sums to part[y][m][n] (n < Ntiles32 * 32); m32_ksplit_reduce adds
// the ks partials in order and applies the epilogue.
__global__ __launch_bounds__(256, 2) void conv1x1_m32_kernel(const ConvArgs p, int mtiles_img,
                                                             int per_img, int phase, int ks,
                                                             float* __restrict__ part,
                                                             const BnEpi bb) {
  constexpr int BM = 4 * 32 * TM;
  constexpr int NB4 = kG * TN * 64;            // float4 of one weight stage
  constexpr int NBT = (NB4 + 255) / 256;       // ... per thread
  // the TM = 1 epilogue reuses the weight buffers: per wave a 32-pixel x
  // 32-channel block, pitch 36 floats (kEpiPitch)
  constexpr int kEpi4 = 4 * 32 * kEpiPitch / 4;
  constexpr int SB4 = (TM == 1 && kEpi4 > 2 * NB4) ? kEpi4 : 2 * NB4;
  __shared__ float4 sB_[SB4];
  float4 (*sB)[NB4] = reinterpret_cast<float4 (*)[NB4]>(sB_);
  __shared__ __attribute__((aligned(16))) float sGate[AS ? kGateLds : 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, j = lane & 31;
  const int nblk_n = p.Ntiles / TN;  // Ntiles counts 32-channel tiles here
  const int bid = blockIdx.x;
  const int nb = bid % nblk_n, mb = bid / nblk_n;
  const int OHW = p.OH * p.OW;
  // phase geometry: sub-grid SH x SW of output pixels, taps kh0 + 2i, kw0 + 2j
  const int ph = phase >> 1, pw = phase & 1;
  const int SH = phase >= 0 ? (p.OH - ph + 1) >> 1 : p.OH;
  const int SW = phase >= 0 ? (p.OW - pw + 1) >> 1 : p.OW;
  const int kh0 = phase >= 0 ? (ph + p.pad) & 1 : 0, kw0 = phase >= 0 ? (pw + p.pad) & 1 : 0;
  const int nkh = phase >= 0 ? (p.KH - kh0 + 1) >> 1 : p.KH;
  const int nkw = phase >= 0 ? (p.KW - kw0 + 1) >> 1 : p.KW;
  const int M = phase >= 0 ? p.B * SH * SW : (int)p.M;
  int img = 0, m_lo, m_hi;
  if (per_img) {
    img = mb / mtiles_img;
    m_lo = img * OHW + (mb - img * mtiles_img) * BM;
    m_hi = min(img * OHW + OHW, M);
  } else {
    m_lo = mb * BM;
    m_hi = M;
  }
  int pm[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int m = m_lo + wave * 32 * TM + t * 32 + j;
    pm[t] = m < m_hi ? m : -1;
  }
  const int Kt = KXK ? nkh * nkw * p.Cin : p.Cin + (p.x2 ? p.Cin2 : 0);
  const int S_all = (Kt + kBK - 1) / kBK;
  const int kchunk = (S_all + ks - 1) / ks;
  const int s_beg = ks > 1 ? (int)blockIdx.y * kchunk : 0;
  const int S = ks > 1 ? min(S_all, s_beg + kchunk) : S_all;  // stages [s_beg, S)
  // KXK: per-lane output coordinates (oh, ow), image base of each pixel tile,
  // and the flat output pixel om (differs from m in phase mode)
  int poh[TM], pow_[TM], om[TM];
  int64_t pbase[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) om[t] = pm[t];
  if constexpr (KXK) {
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int m = pm[t] >= 0 ? pm[t] : 0;
      const int SHW = SH * SW;
      const int b = m / SHW, r = m - b * SHW;
      const int i = r / SW, jj = r - i * SW;
      poh[t] = phase >= 0 ? 2 * i + ph : i;
      pow_[t] = phase >= 0 ? 2 * jj + pw : jj;
      pbase[t] = (int64_t)b * p.x_bs + p.x_c0;
      if (pm[t] >= 0) om[t] = (b * p.OH + poh[t]) * p.OW + pow_[t];
    }
  }
  const int cps = p.Cin / kBK;  // KXK: stages per tap
  const int x2_pix = (p.x2 && p.x2_stride != 1) ? (int)(p.x2_bs / p.x2_ps) : 0;
  const float4* wg = reinterpret_cast<const float4*>(p.w);
  const float* sc = AS ? p.ascale + (int64_t)img * p.ascale_bs : nullptr;

  auto load_a = [&](int s, float4 (&a)[TM][kG]) {
    if constexpr (KXK) {
      const int tl = s / cps, ci0 = (s - tl * cps) * kBK;
      const int khi = tl / nkw;
      const int kh = kh0 + (phase >= 0 ? 2 : 1) * khi;
      const int kw = kw0 + (phase >= 0 ? 2 : 1) * (tl - khi * nkw);
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        // tconv: stride 1, or stride 2 in phase mode (the division is exact)
        const int ih = p.tconv ? (poh[t] + p.pad - kh) >> (phase >= 0 ? 1 : 0)
                               : poh[t] * p.stride - p.pad + kh;
        const int iw = p.tconv ? (pow_[t] + p.pad - kw) >> (phase >= 0 ? 1 : 0)
                               : pow_[t] * p.stride - p.pad + kw;
        const bool ok = pm[t] >= 0 && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        const float* src = p.x + pbase[t] + ((int64_t)ih * p.W + iw) * p.x_ps + ci0 + 4 * h;
#pragma unroll
        for (int q = 0; q < kG; ++q)
          a[t][q] = ok ? *reinterpret_cast<const float4*>(src + 8 * q)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      return;
    }
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const int k4 = s * kBK + 8 * q + 4 * h;
        const int m = pm[t];
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m >= 0) {
          if (k4 < p.Cin) {
            r = *reinterpret_cast<const float4*>(p.x + (int64_t)m * p.x_ps + p.x_c0 + k4);
          } else if (k4 < Kt) {
            int qq = m;
            if (p.x2_stride != 1) {
              const int b = m / OHW, rr = m - b * OHW;
              const int oh = rr / p.OW, ow = rr - oh * p.OW;
              qq = b * x2_pix + (oh * p.x2_stride) * p.x2_W + ow * p.x2_stride;
            }
            r = *reinterpret_cast<const float4*>(p.x2 + (int64_t)qq * p.x2_ps + (k4 - p.Cin));
          }
        }
        a[t][q] = r;
      }
  };
  // ECA gate of this workgroup's image staged in LDS once (Cin <= kGateLds):
  // store_b applies it on the way to LDS.  Applied in load_b (from global) the
  // multiply makes the wave wait for the weight and gate loads before the
  // stage's MFMAs instead of behind them (b12 project 312 -> see DESIGN).
  const bool gate_lds = AS && p.Cin <= kGateLds;
  // weight stage s -> registers (ECA gate applied to the rows k < Cin when it
  // is not staged in LDS)
  auto load_b = [&](int s, float4 (&b)[NBT]) {
    // phase mode: local stage -> the global tap's weight stage
    if (KXK && phase >= 0) {
      const int tl = s / cps, khi = tl / nkw;
      const int tap = (kh0 + 2 * khi) * p.KW + kw0 + 2 * (tl - khi * nkw);
      s = tap * cps + (s - tl * cps);
    }
#pragma unroll
    for (int i = 0; i < NBT; ++i) {
      const int f = i * 256 + threadIdx.x;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < NB4) {
        const int g = f / (TN * 64), rem = f - g * (TN * 64);
        const int u = rem >> 6, l = rem & 63;
        const int k8 = s * kG + g;
        v = wg[((int64_t)k8 * p.Ntiles + nb * TN + u) * 64 + l];
        if (sc && !gate_lds) {
          int k0 = 8 * k8 + 4 * (l >> 5);
          if (KXK) k0 -= (s / cps) * p.Cin;  // channel within the stage's tap
          if (k0 < p.Cin) {
            const float4 s4 = *reinterpret_cast<const float4*>(sc + k0);
            v.x *= s4.x; v.y *= s4.y; v.z *= s4.z; v.w *= s4.w;
          }
        }
      }
      b[i] = v;
    }
  };
  auto store_b = [&](int buf, int s, const float4 (&b)[NBT]) {
    if (KXK && phase >= 0) {  // as load_b: the global tap's weight stage
      const int tl = s / cps, khi = tl / nkw;
      const int tap = (kh0 + 2 * khi) * p.KW + kw0 + 2 * (tl - khi * nkw);
      s = tap * cps + (s - tl * cps);
    }
#pragma unroll
    for (int i = 0; i < NBT; ++i) {
      const int f = i * 256 + threadIdx.x;
      if (f < NB4) {
        float4 v = b[i];
        if (gate_lds) {
          const int g = f / (TN * 64), l = f & 63;
          int k0 = 8 * (s * kG + g) + 4 * (l >> 5);
          if (KXK) k0 -= (s / cps) * p.Cin;
          if (k0 < p.Cin) {
            const float4 s4 = *reinterpret_cast<const float4*>(sGate + k0);
            v.x *= s4.x; v.y *= s4.y; v.z *= s4.z; v.w *= s4.w;
          }
        }
        sB[buf][f] = v;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

  float4 a_cur[TM][kG], a_nxt[TM][kG], b_nxt[NBT];
  if (gate_lds) {
    for (int i = threadIdx.x; i < p.Cin; i += 256) sGate[i] = sc[i];
    __syncthreads();
  }
  if (S > s_beg) {  // (a phase of a 1x1 stride-2 data gradient has no taps: zeros)
    load_a(s_beg, a_cur);
    load_b(s_beg, b_nxt);
    store_b(s_beg & 1, s_beg, b_nxt);
  }
  __syncthreads();
  for (int s = s_beg; s < S; ++s) {
    const bool more = s + 1 < S;
    if (more) {
      load_a(s + 1, a_nxt);
      load_b(s + 1, b_nxt);
    }
    const float4* bs = sB[s & 1];
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      float4 bw[TN];
#pragma unroll
      for (int u = 0; u < TN; ++u) bw[u] = bs[(q * TN + u) * 64 + lane];
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].x, a_cur[t][q].x, acc[t][u], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].y, a_cur[t][q].y, acc[t][u], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].z, a_cur[t][q].z, acc[t][u], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].w, a_cur[t][q].w, acc[t][u], 0, 0, 0);
    }
    if (more) {
      store_b((s + 1) & 1, s + 1, b_nxt);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int q = 0; q < kG; ++q) a_cur[t][q] = a_nxt[t][q];
    }
    __syncthreads();
  }

  if (ks > 1) {  // raw partial sums of this K range
    const int npad = p.Ntiles * 32;
    float* pb = part + (int64_t)blockIdx.y * p.M * npad;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      if (pm[t] < 0) continue;
      float* prow = pb + (int64_t)om[t] * npad;
#pragma unroll
      for (int u = 0; u < TN; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int n = (nb * TN + u) * 32 + 8 * c + 4 * h;
          *reinterpret_cast<float4*>(prow + n) = make_float4(
              acc[t][u][4 * c], acc[t][u][4 * c + 1], acc[t][u][4 * c + 2], acc[t][u][4 * c + 3]);
        }
    }
    return;
  }
  // TM = 1 (32-pixel wave tiles, the large-M ungated layers): each
  // 32-pixel x 32-channel block goes through the wave's LDS slice so that a
  // store instruction covers 8 pixels x 128 contiguous bytes (lane l: pixel
  // l / 8, channel quad l % 8) instead of 32 pixels x 32 bytes (the
  // accumulator layout): R50 l1.c3 920 -> 795 us, l2.c3 613 -> 565, l2.c1
  // 391 -> 359; the TM = 2 shapes (N 1024 / 2048 at small M, the gated MNv3
  // project convs) measured neutral to 10% slower with it and keep the
  // direct stores.  Same values and operations either way, so the same bits.
  if constexpr (TM == 1) {
    float* ep = reinterpret_cast<float*>(sB_) + wave * 32 * kEpiPitch;
    const int srow = mb * 4 + wave;  // ST: this wave tile's statistics row (flat M tiling)
    m32_epilogue_tm1<TN, ST, BB, (ST || BB) ? kEpiNone : EPI>(p, acc[0], pm[0], om[0], nb, srow,
                                                                ep, part, bb, lane);
    return;
  }
  // TM = 2: acc[t][u][4c + e] = Y[pixel pm[t]][nb*BN + 32u + 8c + 4h + e]
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int m = om[t];
    if (pm[t] < 0) continue;
    float* yrow = p.y + (int64_t)m * p.y_ps + p.y_c0;
    const float* rrow = p.res ? p.res + (int64_t)m * p.res_ps + p.res_c0 : nullptr;
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int n = (nb * TN + u) * 32 + 8 * c + 4 * h;
        if (n >= p.Cout) continue;
        float4 v = make_float4(acc[t][u][4 * c], acc[t][u][4 * c + 1], acc[t][u][4 * c + 2],
                               acc[t][u][4 * c + 3]);
        if (p.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
          v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
        }
        if (rrow) {
          const float4 rr = *reinterpret_cast<const float4*>(rrow + n);
          v.x += rr.x; v.y += rr.y; v.z += rr.z; v.w += rr.w;
        }
        v.x = act32(v.x, p.act, p.slope);
        v.y = act32(v.y, p.act, p.slope);
        v.z = act32(v.z, p.act, p.slope);
        v.w = act32(v.w, p.act, p.slope);
        *reinterpret_cast<float4*>(yrow + n) = v;
      }
  }

}

// Y[m][n] = act(sum_y part[y][m][n] + bias[n] (+ R[m][n])), partials added in
// y order (deterministic); one thread per (pixel, 4 channels).
__global__ __launch_bounds__(256) void m32_ksplit_reduce(const ConvArgs p, int ks,
                                                         const float* __restrict__ part) {
  const int npad = p.Ntiles * 32, c4n = (p.Cout + 3) >> 2;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= p.M * c4n) return;
  const int64_t m = i / c4n;
  const int n = (int)(i - m * c4n) * 4;
  float4 v = *reinterpret_cast<const float4*>(part + m * npad + n);
  for (int y = 1; y < ks; ++y) {
    const float4 q = *reinterpret_cast<const float4*>(part + ((int64_t)y * p.M + m) * npad + n);
    v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
  }
  if (p.bias) {
    const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
    v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
  }
  if (p.res) {
    const float4 rr = *reinterpret_cast<const float4*>(p.res + m * p.res_ps + p.res_c0 + n);
    v.x += rr.x; v.y += rr.y; v.z += rr.z; v.w += rr.w;
  }
  v.x = act32(v.x, p.act, p.slope);
  v.y = act32(v.y, p.act, p.slope);
  v.z = act32(v.z, p.act, p.slope);
  v.w = act32(v.w, p.act, p.slope);
  *reinterpret_cast<float4*>(p.y + m * p.y_ps + p.y_c0 + n) = v;
}

// Streaming form of the 1x1 / stride-1 GEMM for short K (Cin = 32 KS, KS 2
// or 4): the R50 bottleneck convs with K 64 / 128 (l1.c3 64 -> 256 and its
// statistics form, l1.c1 of block 1, the data gradients into 256 / 512
// channels, l2.c3 128 -> 512).  A conv1x1_m32_kernel workgroup of such a
// layer lives through only 2-4 K stages, so its pixel loads, the weight
// staging and its barrier, and the epilogue's stores run back to back with
// little MFMA work to hide them: those layers sat at 40-57% of the MFMA peak
// while moving 2-3 TB/s.  Here a persistent workgroup copies its N block's
// weights (all of K: KS x TN x 4 KiB) into LDS once; each wave then walks
// 32-pixel tiles (tile = 4 wgm + wave + k * 4 gm) with no workgroup barrier,
// refilling a K group's registers with the next tile's pixels as soon as its
// MFMAs are issued, so a whole tile of loads is in flight behind the current
// tile's MFMAs and epilogue.  Same MFMA order and the same epilogue
// (m32_epilogue_tm1) as conv1x1_m32_kernel<1, TN>: bit-identical outputs and
// statistics / BatchNorm-backward rows.
template <int TN, int KS, bool ST, bool BB, int EPI>
__global__ __launch_bounds__(256) void conv1x1_m32s_kernel(const ConvArgs p, int nblk_n,
                                                            float* __restrict__ part,
                                                            const BnEpi bb) {
  constexpr int NW4 = KS * kG * TN * 64;  // float4 of the resident weights
  extern __shared__ __attribute__((aligned(16))) float4 m32s_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, j = lane & 31;
  // XCD-paired N blocks: workgroups bid, bid + 8, ... (one XCD) take the
  // nblk_n N blocks of the same pixel tiles (gridDim = gm * nblk_n, gm a
  // multiple of 8), so a tile's pixels are read through one L2 and its
  // output rows are written from one XCD
  const int xcd = blockIdx.x & 7, rr = blockIdx.x >> 3;
  const int nb = rr % nblk_n, wgm = (rr / nblk_n) * 8 + xcd;
  const int gm = gridDim.x / nblk_n;
  {
    const float4* wg = reinterpret_cast<const float4*>(p.w);
    for (int f = threadIdx.x; f < NW4; f += 256) {
      const int k8 = f / (TN * 64), rem = f - k8 * (TN * 64);
      m32s_lds[f] = wg[((int64_t)k8 * p.Ntiles + nb * TN + (rem >> 6)) * 64 + (rem & 63)];
    }
  }
  __syncthreads();
  float* ep = reinterpret_cast<float*>(m32s_lds + NW4) + wave * 32 * kEpiPitch;
  const int64_t ntiles = (p.M + 31) >> 5;
  const int64_t step = (int64_t)gm * 4;
  const float* xb = p.x + p.x_c0 + 4 * h;
  auto load = [&](int64_t T, int s, int q) {
    const int64_t m = T * 32 + j;
    return m < p.M ? *reinterpret_cast<const float4*>(xb + m * p.x_ps + s * kBK + 8 * q)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float4 a[KS][kG];
  int64_t T = (int64_t)wgm * 4 + wave;
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int q = 0; q < kG; ++q) a[s][q] = load(T, s, q);
  for (; T < ntiles; T += step) {
    const int64_t Tn = T + step;
    f32x16 acc[TN];
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        float4 bw[TN];
#pragma unroll
        for (int u = 0; u < TN; ++u) bw[u] = m32s_lds[((s * kG + q) * TN + u) * 64 + lane];
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].x, a[s][q].x, acc[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].y, a[s][q].y, acc[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].z, a[s][q].z, acc[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw[u].w, a[s][q].w, acc[u], 0, 0, 0);
        a[s][q] = load(Tn, s, q);  // the next tile's pixels, in flight from here
      }
    const int64_t m = T * 32 + j;
    const int pm = m < p.M ? (int)m : -1;
    m32_epilogue_tm1<TN, ST, BB, EPI>(p, acc, pm, pm, nb, (int)T, ep, part, bb, lane);
  }
}

// K split of a forward launch (k x k, or 1x1 with its K-concatenated second
// source) whose grid (`grid` workgroups) cannot fill the device — R50 layer3/4
// at bs1: enough splits for ~512 workgroups, each keeping >= 4 stages of 32
// channels; 1 = no split.  Needs a caller workspace (args.ws).
static int m32_ksplit(const ConvArgs& a, bool kxk, int64_t grid) {
  if (a.tconv || a.Cout % 4 || grid >= 256) return 1;
  const int Kt = kxk ? a.KH * a.KW * a.Cin : a.Cin + (a.x2 ? a.Cin2 : 0);
  const int S = (Kt + kBK - 1) / kBK;
  int ks = (int)std::min<int64_t>(8, (512 + grid - 1) / grid);
  ks = std::min(ks, S / 4);
  return ks >= 2 ? ks : 1;
}
static int64_t m32_ksplit_bytes(const ConvArgs& a, int ks) {
  return ks > 1 ? (int64_t)ks * a.B * a.OH * a.OW * a.ntiles32 * 32 * (int64_t)sizeof(float) : 0;
}

template <int TM, int TN, bool KXK, bool AS>
static int launch_m32_as(const ConvArgs& a, hipStream_t st);

template <int TM, int TN, bool KXK>
static int launch_m32(const ConvArgs& a, hipStream_t st) {
  if (a.ascale) return launch_m32_as<TM, TN, KXK, true>(a, st);
  return launch_m32_as<TM, TN, KXK, false>(a, st);
}

template <int TM, int TN, bool KXK, bool AS>
static int launch_m32_as(const ConvArgs& a, hipStream_t st) {
  constexpr int BM = 4 * 32 * TM;
  const int64_t OHW = (int64_t)a.OH * a.OW;
  const int per_img = a.ascale != nullptr;
  const int64_t mt_img = cdiv(OHW, BM);
  if (KXK && a.tconv && a.stride == 2) {  // sub-pixel phases, one launch each
    JABD_REQUIRE(!per_img, "conv32: phase mode without ascale");
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        const int64_t Mp = (int64_t)a.B * ((a.OH - ph + 1) / 2) * ((a.OW - pw + 1) / 2);
        if (Mp <= 0) continue;
        const int64_t grid = cdiv(Mp, BM) * (a.Ntiles / TN);
        JABD_REQUIRE(grid < (int64_t)0x7fffffff, "conv32: grid too large");
        conv1x1_m32_kernel<TM, TN, KXK, AS><<<(unsigned)grid, 256, 0, st>>>(a, (int)mt_img, 0,
                                                                        2 * ph + pw, 1, nullptr,
                                                                        BnEpi{});
        if (int e = check_launch("conv1x1_m32")) return e;
      }
    return JABD_OK;
  }
  const int64_t mtiles = per_img ? mt_img * a.B : cdiv(a.M, BM);
  const int64_t grid = mtiles * (a.Ntiles / TN);
  JABD_REQUIRE(grid < (int64_t)0x7fffffff, "conv32: grid too large");
  const int ks = a.ws ? m32_ksplit(a, KXK, grid) : 1;
  if (ks > 1 && a.ws_bytes >= m32_ksplit_bytes(a, ks)) {
    float* part = static_cast<float*>(a.ws);
    conv1x1_m32_kernel<TM, TN, KXK, AS><<<dim3((unsigned)grid, (unsigned)ks), 256, 0, st>>>(
        a, (int)mt_img, per_img, -1, ks, part, BnEpi{});
    if (int e = check_launch("conv1x1_m32 (split K)")) return e;
    const int64_t n4 = a.M * ((a.Cout + 3) / 4);
    m32_ksplit_reduce<<<(unsigned)cdiv(n4, 256), 256, 0, st>>>(a, ks, part);
    return check_launch("m32_ksplit_reduce");
  }
  if constexpr (TM == 1 && !AS) {  // the epilogue terms specialised (m32_epilogue_tm1)
    if (!a.bias && a.act == ACT_NONE) {
      if (a.res)
        conv1x1_m32_kernel<1, TN, KXK, false, false, false, kEpiRes>
            <<<(unsigned)grid, 256, 0, st>>>(a, (int)mt_img, per_img, -1, 1, nullptr, BnEpi{});
      else
        conv1x1_m32_kernel<1, TN, KXK, false, false, false, kEpiNone>
            <<<(unsigned)grid, 256, 0, st>>>(a, (int)mt_img, per_img, -1, 1, nullptr, BnEpi{});
      return check_launch("conv1x1_m32");
    }
  }
  conv1x1_m32_kernel<TM, TN, KXK, AS><<<(unsigned)grid, 256, 0, st>>>(a, (int)mt_img, per_img, -1,
                                                                     1, nullptr, BnEpi{});
  return check_launch("conv1x1_m32");
}

// conv1x1_m32s_kernel launch: a persistent grid of (CUs x resident
// workgroups) rounded to whole N blocks.  JABD_M32S=0 keeps every layer on
// conv1x1_m32_kernel (A/B).
static bool m32s_on() {
  static const bool on = [] {
    const char* e = getenv("JABD_M32S");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int TN, int KS, bool ST, bool BB, int EPI>
static int launch_m32s(const ConvArgs& a, float* part, const BnEpi& bb, hipStream_t st) {
  auto kern = conv1x1_m32s_kernel<TN, KS, ST, BB, EPI>;
  const size_t lds = (size_t)KS * kG * TN * 64 * 16 + (size_t)4 * 32 * kEpiPitch * 4;
  static int slots = 0;  // CUs x resident workgroups of this instance
  if (slots <= 0) {
    int dev = 0, ncu = 0, occ = 0;
    JABD_HIP(hipGetDevice(&dev));
    JABD_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    JABD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, lds));
    JABD_REQUIRE(occ >= 1, "conv32 stream: no resident workgroup (%zu B LDS)", lds);
    slots = ncu * occ;
  }
  const int nblk_n = a.Ntiles / TN;
  const int64_t ntiles = cdiv(a.M, (int64_t)32);
  int64_t gm = std::min<int64_t>(cdiv(ntiles, 4), slots / nblk_n);
  gm = std::max<int64_t>(8, gm / 8 * 8);  // whole XCD rounds (see the kernel)
  kern<<<(unsigned)(gm * nblk_n), 256, lds, st>>>(a, nblk_n, part, bb);
  return check_launch("conv1x1_m32s");
}

// The streaming form for a 1x1 / stride-1 layer with K = 64 or 128 (a: the
// w32 view, Ntiles = ntiles32); form 0 plain, 1 statistics (ST), 2
// BatchNorm-backward sums (BB).  -1: not served.
static int m32s_dispatch(const ConvArgs& a, int tn32, float* part, const BnEpi& bb, int form,
                         hipStream_t st) {
  if (!m32s_on() || a.KH != 1 || a.KW != 1 || a.stride != 1 || a.pad != 0 || a.tconv ||
      a.nchw_in || a.x2 || a.ascale || a.y2 || a.Cin % kBK || a.M >= ((int64_t)1 << 31) - 64)
    return -1;
  const int KS = a.Cin / kBK;
  if (KS != 2 && KS != 4) return -1;
  // K = 128: the plain form only by default (JABD_M32S_KS4 = mask of forms: bit 0 plain, 1
  // statistics, 2 BatchNorm-backward).  There TN = 2 (32 KiB of resident weights) re-reads the
  // pixels N / 64 times; the statistics form measured 463 (tile kernel) vs 479 us (l2.c3 at
  // bs16) and the C3 step 517.0-517.6 (plain only) vs 517.9-518.7 ms (all forms), r06/ab/ks4
  {
    static const int ks4 = [] {
      const char* e = getenv("JABD_M32S_KS4");
      return e ? atoi(e) : 1;
    }();
    static const int ks2 = [] {  // the same mask for K = 64 (all forms by default)
      const char* e = getenv("JABD_M32S_KS2");
      return e ? atoi(e) : 7;
    }();
    if (!(((KS == 4 ? ks4 : ks2) >> form) & 1)) return -1;
  }
  int TN = tn32;
  while (KS * TN > 8 && TN % 2 == 0) TN /= 2;  // resident weights <= 32 KiB
  if (TN < 1 || KS * TN > 8 || a.Ntiles % TN) return -1;
  // the plain form's epilogue terms, specialised when the layer has none or
  // only a residual (the R50 data gradients)
  const bool plain_none = !a.bias && !a.res && a.act == ACT_NONE;
  const bool plain_res = !a.bias && a.res && a.act == ACT_NONE;
#define M32S(TN_, KS_)                                                                 \
  return form == 1   ? launch_m32s<TN_, KS_, true, false, kEpiNone>(a, part, bb, st)   \
         : form == 2 ? launch_m32s<TN_, KS_, false, true, kEpiNone>(a, part, bb, st)   \
         : plain_none ? launch_m32s<TN_, KS_, false, false, kEpiNone>(a, part, bb, st) \
         : plain_res  ? launch_m32s<TN_, KS_, false, false, kEpiRes>(a, part, bb, st)  \
                      : launch_m32s<TN_, KS_, false, false, kEpiRt>(a, part, bb, st);
  if (KS == 2) {
    switch (TN) {
      case 1: M32S(1, 2)
      case 2: M32S(2, 2)
      case 3: M32S(3, 2)
      case 4: M32S(4, 2)
      default: return -1;
    }
  }
  switch (TN) {
    case 1: M32S(1, 4)
    case 2: M32S(2, 4)
    default: return -1;
  }
#undef M32S
}

// Forward conv on the 32x32 kernel with the BatchNorm statistics rows (ST):
// 32-pixel wave tiles, no gate / split / bias / residual / activation.
// (bb.rows set: the BatchNorm-backward sums form instead)
template <int TN, bool KXK>
static int launch_m32_stats(const ConvArgs& a, float* part, const BnEpi& bb, hipStream_t st) {
  const int64_t grid = cdiv(a.M, (int64_t)128) * (a.Ntiles / TN);
  JABD_REQUIRE(grid < (int64_t)0x7fffffff, "conv32 stats: grid too large");
  if (bb.rows) {
    conv1x1_m32_kernel<1, TN, KXK, false, false, true><<<(unsigned)grid, 256, 0, st>>>(
        a, (int)cdiv((int64_t)a.OH * a.OW, 128), 0, -1, 1, nullptr, bb);
    return check_launch("conv1x1_m32 (BN backward sums)");
  }
  conv1x1_m32_kernel<1, TN, KXK, false, true><<<(unsigned)grid, 256, 0, st>>>(
      a, (int)cdiv((int64_t)a.OH * a.OW, 128), 0, -1, 1, part, BnEpi{});
  return check_launch("conv1x1_m32 (BN statistics)");
}

int conv_m32_stats_dispatch(const ConvArgs& a0, bool kxk, float* part, const BnEpi& bb,
                            hipStream_t st) {
  ConvArgs a = a0;
  a.w = a0.w32;
  a.Ntiles = a0.ntiles32;
  if (!kxk) {
    const int r = m32s_dispatch(a, a0.tn32, part, bb, bb.rows ? 2 : 1, st);
    if (r >= 0) return r;
  }
#define MS(TN_) return kxk ? launch_m32_stats<TN_, true>(a, part, bb, st) : launch_m32_stats<TN_, false>(a, part, bb, st);
  switch (a0.tn32) {
    case 1: MS(1)
    case 2: MS(2)
    case 3: MS(3)
    case 4: MS(4)
    default: return -1;
  }
#undef MS
}

}  // namespace jabd

using namespace jabd;

// Pixel tiles per wave of the 32x32 kernel (1: 32-pixel wave tiles, more and
// shorter workgroups; 2: 64).  1 measured faster on GEMMs without a folded
// ECA gate (R50 at bs16-64: 5-10%; at bs1, where the grid cannot fill the
// device, R50 640^2 predict 230 -> 313 fps) and on small gated ones (bs1
// MNv3 +3%); the gate's per-workgroup weight scaling makes them slower on
// the large gated GEMMs (C2's project convs).  JABD_M32_TM=1|2 forces one.
static int m32_tm(const ConvArgs& a) {
  static int ftm = -1;
  if (ftm < 0) {
    const char* e = getenv("JABD_M32_TM");
    ftm = e ? atoi(e) : 0;
  }
  if (a.tn32 > 4) return 1;
  if (ftm == 1 || ftm == 2) return ftm;
  return (!a.ascale || a.M < 65536) ? 1 : 2;
}

// N-tiles per workgroup to launch: the packing's tn32, or 1 for a gated GEMM
// whose grid with tn32 could not fill the device (bs1 MNv3 projects at
// 20^2-40^2: the 960 -> 160 ones ran 4 workgroups of 5 N-tiles; one N-tile
// each gives 5x the workgroups: MNv3 640^2 predict 1005 -> 1070 fps).  Not
// for the ungated R50 GEMMs: layer4 at 32^2 lost 220 -> 189 fps (1024^2
// predict; its K-split already fills the device and 4x the workgroups each
// re-read the pixel tile).  JABD_M32_TN1=0 keeps tn32 (A/B).
static int m32_tn_launch(const ConvArgs& a) {
  static const bool off = [] {
    const char* e = getenv("JABD_M32_TN1");
    return e && e[0] == '0';
  }();
  if (off || a.tn32 <= 1 || a.tconv || !a.ascale) return a.tn32;
  const int64_t BM = 4 * 32 * m32_tm(a);
  const int64_t OHW = (int64_t)a.OH * a.OW;
  const int64_t mtiles = a.ascale ? cdiv(OHW, BM) * a.B : cdiv((int64_t)a.B * OHW, BM);
  return mtiles * (a.ntiles32 / a.tn32) >= 256 ? a.tn32 : 1;
}

// N-tiles (32 output channels each) per workgroup for the 32x32 kernel.
// Prefers a 64x128 wave tile (TM=2, TN<=4), else the exact-fit wide tile.
extern "C" int64_t jabd_conv_workspace_size(const jabd_conv_args* args) {
  if (!args) return 0;
  const ConvArgs& a = *args;
  if (!a.w32 || a.Cin % 32 || a.tconv || a.nchw_in || a.tn32 <= 0) return 0;
  // 1x1 / stride 1 / pad 0 takes the 32x32 kernel's 1x1 form, anything else its k x k form
  const bool kxk = !(a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0);
  ConvArgs am = a;
  am.M = (int64_t)a.B * a.OH * a.OW;
  const int tn = m32_tn_launch(am);
  const int TM = tn == a.tn32 ? m32_tm(am) : 1;
  const int64_t BM = 4 * 32 * TM;
  const int64_t OHW = (int64_t)a.OH * a.OW;
  const int64_t mtiles = a.ascale ? cdiv(OHW, BM) * a.B : cdiv((int64_t)a.B * OHW, BM);
  const int64_t grid = mtiles * (a.ntiles32 / tn);
  return m32_ksplit_bytes(a, m32_ksplit(a, kxk, grid));
}

extern "C" int jabd_conv_pack_tn32(int cout) {
  const int nt = (cout + 31) / 32;
  if (nt <= 4) return nt;
  if (nt % 4 == 0) return 4;
  int best = 4, waste = (nt + 3) / 4 * 4 - nt;
  for (int tn : {5, 6, 7}) {
    const int w = (nt + tn - 1) / tn * tn - nt;
    if (w < waste) { waste = w; best = tn; }
  }
  return best;
}

namespace jabd {
// Called by jabd_conv2d_nhwc_f32 for 1x1 / stride-1 convs when the caller
// supplied the 32x32 packing (args->w32).  Returns -1 when this kernel does
// not take the shape (the caller then uses conv.hip).
int conv1x1_m32_dispatch(const ConvArgs& a0, hipStream_t st, bool kxk) {
  ConvArgs a = a0;
  a.w = a0.w32;
  a.Ntiles = a0.ntiles32;
  if (!kxk) {  // K 64 / 128: the streaming form (no K split at <= 4 stages)
    const int r = m32s_dispatch(a, a0.tn32, nullptr, BnEpi{}, 0, st);
    if (r >= 0) return r;
  }
#define M32(TM_, TN_) \
  return kxk ? launch_m32<TM_, TN_, true>(a, st) : launch_m32<TM_, TN_, false>(a, st);
  if (m32_tn_launch(a0) == 1 && a0.tn32 > 1) M32(1, 1)
  if (m32_tm(a0) == 1) {
    switch (a0.tn32) {
      case 1: M32(1, 1)
      case 2: M32(1, 2)
      case 3: M32(1, 3)
      case 4: M32(1, 4)
      default: break;
    }
  }
  switch (a0.tn32) {
    case 1: M32(2, 1)
    case 2: M32(2, 2)
    case 3: M32(2, 3)
    case 4: M32(2, 4)
    case 5: M32(1, 5)
    case 6: M32(1, 6)
    case 7: M32(1, 7)
    default: return -1;
  }
#undef M32
}
}  // namespace jabd

// ---------------------------------------------------------------------------
// Weight packing on the device (the training convs repack after every
// optimizer step): straight from the torch weight [Cout][Cin][KH][KW] (or,
// transposed = 1, the data-gradient form W'[ci][co] = W[co][ci]) to
//   wp   float4 [Kc][Ntiles][64]:  lane 16g + j, element e = W2d[16kc+4g+e][16nt+j]
//   wp32 float4 [K8][NT32][64]:    lane 32h + j, element e = W2d[8k8+4h+e][32nt+j]
// with W2d[k][n], k = tap * Cin' + ci' (tap = kh * KW + kw), zero outside
// K x N — the layouts jabd_amd.functional.PackedConv builds on the host.
namespace jabd {

__device__ __forceinline__ float w2d_at(const float* __restrict__ w, int cout, int cin, int khw,
                                        int transposed, int k, int n) {
  const int cinp = transposed ? cout : cin;  // the packed GEMM's input channels
  const int ncols = transposed ? cin : cout;
  if (k >= khw * cinp || n >= ncols) return 0.f;
  const int tap = k / cinp, c = k - tap * cinp;
  const int co = transposed ? c : n, ci = transposed ? n : c;
  return w[((int64_t)co * cin + ci) * khw + tap];
}

__global__ __launch_bounds__(256) void pack_w_kernel(const float* __restrict__ w, int cout,
                                                     int cin, int khw, int transposed, int Kc,
                                                     int Ntiles, float* __restrict__ wp, int K8,
                                                     int NT32, float* __restrict__ wp32) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t n16 = (int64_t)Kc * Ntiles * 64;
  if (i < n16) {
    const int lane = (int)(i & 63);
    const int64_t r = i >> 6;
    const int nt = (int)(r % Ntiles), kc = (int)(r / Ntiles);
    const int g = lane >> 4, j = lane & 15;
    float4 v;
    v.x = w2d_at(w, cout, cin, khw, transposed, 16 * kc + 4 * g + 0, 16 * nt + j);
    v.y = w2d_at(w, cout, cin, khw, transposed, 16 * kc + 4 * g + 1, 16 * nt + j);
    v.z = w2d_at(w, cout, cin, khw, transposed, 16 * kc + 4 * g + 2, 16 * nt + j);
    v.w = w2d_at(w, cout, cin, khw, transposed, 16 * kc + 4 * g + 3, 16 * nt + j);
    reinterpret_cast<float4*>(wp)[i] = v;
    return;
  }
  const int64_t i2 = i - n16;
  if (!wp32 || i2 >= (int64_t)K8 * NT32 * 64) return;
  const int lane = (int)(i2 & 63);
  const int64_t r = i2 >> 6;
  const int nt = (int)(r % NT32), k8 = (int)(r / NT32);
  const int h = lane >> 5, j = lane & 31;
  float4 v;
  v.x = w2d_at(w, cout, cin, khw, transposed, 8 * k8 + 4 * h + 0, 32 * nt + j);
  v.y = w2d_at(w, cout, cin, khw, transposed, 8 * k8 + 4 * h + 1, 32 * nt + j);
  v.z = w2d_at(w, cout, cin, khw, transposed, 8 * k8 + 4 * h + 2, 32 * nt + j);
  v.w = w2d_at(w, cout, cin, khw, transposed, 8 * k8 + 4 * h + 3, 32 * nt + j);
  reinterpret_cast<float4*>(wp32)[i2] = v;
}

// Batched pack: one launch for every weight an optimizer step changed.  Job
// rows {w, wp, wp32, cout, cin, khw, transposed, Kc, Ntiles, K8, NT32};
// starts[i] = float4 outputs of jobs < i, staged in LDS for a binary search.
constexpr int kPackMaxJobs = 1024;
__global__ __launch_bounds__(256) void pack_w_multi_kernel(const int64_t* __restrict__ jobs,
                                                           const int64_t* __restrict__ starts,
                                                           int njobs, int64_t total) {
  __shared__ int64_t st[kPackMaxJobs + 1];
  for (int t = threadIdx.x; t <= njobs; t += blockDim.x) st[t] = starts[t];
  __syncthreads();
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  int lo = 0, hi = njobs - 1;  // last job with st[job] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (st[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const int64_t* jb = jobs + (int64_t)lo * 11;
  const float* w = reinterpret_cast<const float*>(jb[0]);
  float* wp = reinterpret_cast<float*>(jb[1]);
  float* wp32 = reinterpret_cast<float*>(jb[2]);
  const int cout = (int)jb[3], cin = (int)jb[4], khw = (int)jb[5], tr = (int)jb[6];
  const int Kc = (int)jb[7], Ntiles = (int)jb[8], NT32 = (int)jb[10];
  const int64_t r0 = i - st[lo];
  const int64_t n16 = (int64_t)Kc * Ntiles * 64;
  if (r0 < n16) {
    const int lane = (int)(r0 & 63);
    const int64_t r = r0 >> 6;
    const int nt = (int)(r % Ntiles), kc = (int)(r / Ntiles);
    const int g = lane >> 4, j = lane & 15;
    float4 v;
    v.x = w2d_at(w, cout, cin, khw, tr, 16 * kc + 4 * g + 0, 16 * nt + j);
    v.y = w2d_at(w, cout, cin, khw, tr, 16 * kc + 4 * g + 1, 16 * nt + j);
    v.z = w2d_at(w, cout, cin, khw, tr, 16 * kc + 4 * g + 2, 16 * nt + j);
    v.w = w2d_at(w, cout, cin, khw, tr, 16 * kc + 4 * g + 3, 16 * nt + j);
    reinterpret_cast<float4*>(wp)[r0] = v;
    return;
  }
  const int64_t i2 = r0 - n16;
  const int lane = (int)(i2 & 63);
  const int64_t r = i2 >> 6;
  const int nt = (int)(r % NT32), k8 = (int)(r / NT32);
  const int h = lane >> 5, j = lane & 31;
  float4 v;
  v.x = w2d_at(w, cout, cin, khw, tr, 8 * k8 + 4 * h + 0, 32 * nt + j);
  v.y = w2d_at(w, cout, cin, khw, tr, 8 * k8 + 4 * h + 1, 32 * nt + j);
  v.z = w2d_at(w, cout, cin, khw, tr, 8 * k8 + 4 * h + 2, 32 * nt + j);
  v.w = w2d_at(w, cout, cin, khw, tr, 8 * k8 + 4 * h + 3, 32 * nt + j);
  reinterpret_cast<float4*>(wp32)[i2] = v;
}

}  // namespace jabd

extern "C" int jabd_conv_pack_multi_f32(const int64_t* jobs, const int64_t* starts,
                                        int32_t njobs, int64_t total, jabd_stream_t stream) {
  using namespace jabd;
  if (njobs <= 0 || total <= 0) return JABD_OK;
  JABD_REQUIRE(jobs && starts && njobs <= kPackMaxJobs, "conv_pack_multi: bad args (njobs %d)",
               njobs);
  pack_w_multi_kernel<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(jobs, starts,
                                                                                njobs, total);
  return check_launch("conv_pack_multi");
}

extern "C" int jabd_conv_pack_f32(const float* w, int32_t cout, int32_t cin, int32_t kh,
                                  int32_t kw, int32_t transposed, int32_t Kc, int32_t Ntiles,
                                  float* wp, int32_t K8, int32_t NT32, float* wp32,
                                  jabd_stream_t stream) {
  using namespace jabd;
  JABD_REQUIRE(w && wp && cout > 0 && cin > 0 && kh > 0 && kw > 0 && Kc > 0 && Ntiles > 0 &&
                   (!wp32 || (K8 > 0 && NT32 > 0)),
               "conv_pack: bad args");
  const int cinp = transposed ? cout : cin, ncols = transposed ? cin : cout;
  JABD_REQUIRE(16 * Kc >= kh * kw * cinp && 16 * Ntiles >= ncols &&
                   (!wp32 || (8 * K8 >= kh * kw * cinp && 32 * NT32 >= ncols)),
               "conv_pack: tile counts do not cover the weight");
  const int64_t tot = (int64_t)Kc * Ntiles * 64 + (wp32 ? (int64_t)K8 * NT32 * 64 : 0);
  pack_w_kernel<<<(unsigned)cdiv(tot, 256), 256, 0, as_stream(stream)>>>(
      w, cout, cin, kh * kw, transposed, Kc, Ntiles, wp, K8, NT32, wp32);
  return check_launch("conv_pack");
}
