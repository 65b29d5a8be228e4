// A1 fused MobileNetV3 block front half, eval mode (nets/mobilenetV3.py:
// 141-142): expand 1x1 conv + folded BN + act  ->  depthwise k x k + folded BN
// + act  ->  ECA average-pool partial sums.  The expanded tensor never
// touches HBM: it is the largest activation of the network (e.g. 64 channels
// at 512x512 for block 2) and the unfused path writes it once and reads it
// back (plus halo) once.
//
// Workgroup = one TH x TW output tile x EC expanded channels of one image.
//  phase 1: the input tile (plus the k-1 halo, all Cin channels, 16 at a
//           time) is staged in LDS; the expand GEMM runs on the fp32 MFMA
//           with swapped operands (A = packed weights, B = pixels) so each
//           lane ends up holding 4 consecutive expanded channels of one
//           pixel; bias + act + zero outside the image (the depthwise conv
//           zero-pads the *activated* map), written to LDS as [pixel][EC].
//  phase 2: depthwise register strips (4 outputs along W per thread) read
//           the LDS tile, add bias, activate, store NHWC and accumulate the
//           ECA sums, reduced per workgroup in a fixed order into
//           part[b][tile][E] (deterministic, no atomics).
// The LDS buffer is shared by the two phases (the expand accumulators live
// in registers across the switch).  Workgroup ids are decoded XCD-aware: the
// EC-chunks of one tile land on the same XCD (id % 8), so their re-reads of
// the input tile hit that XCD's L2.
#include "expdw_shared.h"

namespace jabd {

// Resident workgroups the register allocation must allow: 2, or 4 for the
// skip form when its LDS leaves room for 4 (its extra live registers
// otherwise cost a resident workgroup: 142 vs 114 VGPRs on the 3x3/s2 tile).
template <int K, int S, int TH, int TW, int EC, bool SKIP, int NW, int SKC>
constexpr int xd1_min_wg() {
  using C = XdCfg<K, S, TH, TW, EC>;
  constexpr int bytes = C::LDS * 4 + K * K * (EC / 4) * 16 + (SKIP ? 10 * (SKC / 4) * 16 : 16);
  return (SKIP && NW == 4 && 4 * bytes <= 160 * 1024) ? 4 : 2;
}

// KCC: the number of 16-channel input stages when known at compile time
// (Cin <= 32: the stage loop unrolls away with its next-stage addressing),
// 0 = p.Kc at run time.  Taken where it measured faster (tools/ab_xd.sh,
// two rounds): Cin 16 E16 k3 s1 246 vs 258 us, the Cin 24 k5 s2 skip form
// 305-313 vs 324-327 us; the Cin 16 k3 s2 skip form measured 506-514 vs
// 491-498 us with it and keeps the run-time count.
// PRE (KCC == 1, Cin <= 16): the previous block's project in front of the
// expand (jabd_expdw_args.pw): the staged tile is that block's depthwise
// output d; its 1x1 GEMM (the ECA gate folded into the packed weights, one
// 16-channel stage, one n-tile: 4 MFMAs per 16-pixel block), bias, the
// identity residual and the activation turn it into the block output in LDS,
// which the expand (and the skip branch) then read.  The block output never
// goes to HBM: its project launch (a write + a read of it) disappears, for a
// second input read (the residual) and a quarter more MFMAs here.
template <int K, int S, int TH, int TW, int EC, int ACT, int KP, bool SKIP = false, int NW = 4,
          int SKC = 160, int KCC = 0, bool PRE = false>
__global__ __launch_bounds__(64 * NW, (xd1_min_wg<K, S, TH, TW, EC, SKIP, NW, SKC>())) void expdw1_kernel(const jabd_expdw_args p, const XdDivs dv,
                                                       int nitems) {
  static_assert(!PRE || (KCC == 1 && KP == 1), "PRE: one input stage");
  const int Kc = KCC ? KCC : p.Kc;
  using C = XdCfg<K, S, TH, TW, EC>;
  constexpr int T = 64 * NW;                  // threads
  constexpr int NPF = (C::IPAD * 4 + T - 1) / T;
  constexpr int BPW = (C::NBLK + NW - 1) / NW;  // MFMA blocks per wave
  static_assert(NW % C::NNT == 0, "waves split evenly over the 16-channel tiles");
  constexpr int NWD = K * K * C::NC4;  // depthwise taps staged in LDS (bias: registers)
  // skip-branch taps staged in LDS (SKC >= Cin), none without the skip branch
  __shared__ __attribute__((aligned(16))) float lds[C::LDS];
  __shared__ float4 wsh[K * K][C::NC4];
  __shared__ float4 sws[SKIP ? 10 : 1][SKIP ? SKC / 4 : 1];  // 9 taps + bias of the skip dw
  XdItem it;
  XD_RT(0);
  XD_T(1);
  if (!xd_item<K, S, TH, TW, EC>(p, blockIdx.x, dv, nitems, it)) return;
  const bool skip = SKIP && it.c0 == 0;
  if (skip) {  // tap q (9 = bias) by wave, channel quad by lane: no division (Cin <= 256)
    const int c4 = threadIdx.x & 63;
    if (c4 < (p.Cin >> 2))
      for (int q = threadIdx.x >> 6; q < 10; q += NW)
        sws[q][c4] = *reinterpret_cast<const float4*>((q < 9 ? p.sw + q * p.Cin : p.sb) + 4 * c4);
  }
  // the whole input tile (halo included) inside the image: no per-pixel
  // bounds in the loads or the expanded-tile epilogue (most tiles)
  const bool interior =
      it.ih0 >= 0 && it.iw0 >= 0 && it.ih0 + C::IH <= p.H && it.iw0 + C::IW <= p.W;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, j = lane & 15, g = lane >> 4;
  const int ntw = wave % C::NNT;
  const int nt = it.c0 / 16 + ntw;
  const bool ntv = nt < p.Ntiles;
  const int ntc = ntv ? nt : 0;
  const f32x4* wpk = reinterpret_cast<const f32x4*>(p.we);
  // small operands first (consumed after the expand phase)
  // padded expanded channels (chb >= E) start from a zero bias and see zero
  // packed weights (or no MFMAs at all past Ntiles), so act(acc) is already
  // the 0 the depthwise tile needs there: no per-element select
  const int chb = it.c0 + 16 * ntw + 4 * g;
  const bool chok = chb < p.E;
  float4 pbi = *reinterpret_cast<const float4*>(p.be + (chok ? chb : 0));
  if (!chok) pbi = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 pwd = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < NWD) {
    const int tp = t / C::NC4, cc = it.c0 + 4 * (t - tp * C::NC4);
    const float4 w = *reinterpret_cast<const float4*>(p.wd + tp * p.E + (cc < p.E ? cc : 0));
    pwd = cc < p.E ? w : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // depthwise lane map and its bias (consumed after the expand phase)
  int c4, sl;
  dw_lane<C::NC4>(lane, c4, sl);
  const int chl = 4 * c4;
  const bool chv = it.c0 + chl < p.E;
  const float4 bias2 = *reinterpret_cast<const float4*>(p.bd + (chv ? it.c0 + chl : 0));
  // PRE: packed project weights of lane (j, g) (component e: input channel
  // 4g + e, output channel j) scaled by this image's gate; bias of output
  // channels 4g .. 4g + 3 (the lane's accumulator rows)
  f32x4 apre = (f32x4){0.f, 0.f, 0.f, 0.f};
  float4 bpre = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (PRE) {
    const f32x4 w = reinterpret_cast<const f32x4*>(p.pw)[lane];
    const float4 gt = *reinterpret_cast<const float4*>(p.pg + (int64_t)it.b * p.pg_bs + 4 * g);
    apre = (f32x4){w.x * gt.x, w.y * gt.y, w.z * gt.z, w.w * gt.w};
    bpre = *reinterpret_cast<const float4*>(p.pb + 4 * g);
  }
  // input stage loads through a buffer descriptor: an out-of-range slot gets
  // voffset 0xFFFFFFF0 and reads zeros (host: x < 4 GiB)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x), (short)0, (int)(uint32_t)((int64_t)p.B * p.x_bs * 4), 0x00020000);
  // stage slot u of this thread: pixel u*16*NW + (t>>6)*16 + (t&15), channel quad (t>>4)&3
  const int cq = ((t >> 4) & 3) * 4;
  const int spx0 = (t >> 6) * 16 + (t & 15);
  // KP-deep register ring of input stages: stage kc + KP is issued as soon
  // as stage kc has been written to LDS, and the raw LDS barriers below keep
  // it in flight across the MFMA phase (a __syncthreads() would drain it).
  float4 pf[KP][NPF];
  auto load_stage = [&](int kc, float4 (&dst)[NPF]) {
    const int cofs = 16 * kc + cq;
    const uint32_t base = (uint32_t)(it.b * p.x_bs + cofs);
    const bool cok = cofs < p.Cin;
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int px = u * 16 * NW + spx0;
      const int r = px / C::IW, c = px - r * C::IW;
      const int ih = it.ih0 + r, iw = it.iw0 + c;
      const bool ok = px < C::IPX && cok &&
                      (interior || ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W));
      const uint32_t off = ok ? (base + (uint32_t)((ih * p.W + iw) * p.x_ps)) * 4u : 0xFFFFFFF0u;
      if (XD_SKIP & 16) dst[u] = make_float4(0.f, 0.f, 0.f, (float)off);
      else dst[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  // accumulators start at the expand bias (no epilogue add)
  f32x4 acc[BPW];
  const f32x4 bias4 = (f32x4){pbi.x, pbi.y, pbi.z, pbi.w};
#pragma unroll
  for (int u = 0; u < BPW; ++u) acc[u] = bias4;
#pragma unroll
  for (int s = 0; s < KP; ++s)
    if (s < Kc) load_stage(s, pf[s]);
  // Cin 24 (two input stages, KCC == 2): the last stage holds 8 channels.
  // The packed fragments put channel 4g + e of a stage in MFMA e (lane group
  // g), so each of its four MFMAs would contract 2 real channels and 2 zeros;
  // the tail stage instead runs 2 MFMAs over channels 4e + g (e = 0, 1): A
  // from the packed array's lane group e, component g (two scalar loads), B
  // one float of quad plane e per lane.  A quarter of the layer's MFMAs; the
  // sum over k is taken in another order.  (Cin 40 with a run-time stage
  // count measured +5% on the 3x3/s2 skip form: not taken there.)
  const bool tail8 = KCC == 2 && (p.Cin & 15) == 8;
  for (int kc0 = 0; kc0 < Kc; kc0 += KP) {
#pragma unroll
    for (int s = 0; s < KP; ++s) {
      const int kc = kc0 + s;
      if (kc >= Kc) break;
      const bool tl = tail8 && kc == Kc - 1;
      f32x4 a;
      if (tl) {
        const float* wf = reinterpret_cast<const float*>(p.we) +
                          ((int64_t)(kc * p.Ntiles + ntc) * 64 + j) * 4 + g;
        a = (f32x4){wf[0], wf[64], 0.f, 0.f};
      } else {
        a = wpk[(kc * p.Ntiles + ntc) * 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        if (u * 16 * NW + spx0 < C::IPAD)
          *reinterpret_cast<float4*>(lds + (cq / 4 * C::IPAD + u * 16 * NW + spx0) * 4) = pf[s][u];
      }
      // retire the weight load here, before the next stage's loads are in
      // flight: the compiler's vmcnt tracking cannot count through the
      // predicated prefetch and would otherwise wait vmcnt(0) (draining the
      // prefetch) at the first MFMA
      if (!ntv) a = (f32x4){0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+v"(a));
      lds_barrier();
      if (kc == 0) XD_T(2);
      if constexpr (PRE) {
        // block output = pact(Wp (g d) + pb + res) on the staged tile, back into
        // the same quad planes (lane (j, g) of block pb: pixel 16 pb + j,
        // channels 4g .. 4g + 3); zero outside the image (the expand input's
        // padding) and on the pad pixels past IPX
        constexpr int BPP = (C::NPB + NW - 1) / NW;
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(p.pres), (short)0, (int)(uint32_t)((int64_t)p.B * p.x_bs * 4),
            0x00020000);
        f32x4 pacc[BPP];
        float4 res[BPP];
        bool pin[BPP];
#pragma unroll
        for (int u = 0; u < BPP; ++u) {
          const int pb = wave + NW * u;
          const int px = pb * 16 + j;
          const int r = px / C::IW, c = px - r * C::IW;
          const int ih = it.ih0 + r, iw = it.iw0 + c;
          pin[u] = pb < C::NPB && px < C::IPX &&
                   (interior || ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W));
          const uint32_t off =
              pin[u] ? (uint32_t)(it.b * p.x_bs + (ih * p.W + iw) * p.x_ps + 4 * g) * 4u : 0xFFFFFFF0u;
          res[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
          pacc[u] = (f32x4){bpre.x, bpre.y, bpre.z, bpre.w};
          if (pb < C::NPB) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(lds + (g * C::IPAD + px) * 4);
            pacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(apre.x, bv.x, pacc[u], 0, 0, 0);
            pacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(apre.y, bv.y, pacc[u], 0, 0, 0);
            pacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(apre.z, bv.z, pacc[u], 0, 0, 0);
            pacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(apre.w, bv.w, pacc[u], 0, 0, 0);
          }
        }
        lds_barrier();  // every wave's reads of d done
#pragma unroll
        for (int u = 0; u < BPP; ++u) {
          const int pb = wave + NW * u;
          if (pb >= C::NPB) continue;
          float4 v = make_float4(pacc[u][0] + res[u].x, pacc[u][1] + res[u].y,
                                 pacc[u][2] + res[u].z, pacc[u][3] + res[u].w);
          if (p.pact == ACT_RELU) v = xd_act4<ACT_RELU>(v);
          else if (p.pact == ACT_HSWISH) v = xd_act4<ACT_HSWISH>(v);
          if (!pin[u]) v = make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(lds + (g * C::IPAD + pb * 16 + j) * 4) = v;
        }
        lds_barrier();
      }
      if (kc + KP < Kc) load_stage(kc + KP, pf[s]);
      // fused skip branch (stride 2, first chunk's workgroups): this stage's
      // 16 channels for output pixel t & 63, channel quad t >> 6 (waves 0-3), taps from LDS
      const int sc = 16 * kc + 4 * (t >> 6);
      if (skip && wave < 4 && sc < p.Cin) {
        // output (orow, ocol) of the TH x TW tile reads tile pixels
        // (2 orow + kh + PAD - 1, 2 ocol + kw + PAD - 1): the dw3x3/s2/p1 window
        const int op = t & 63, orow = op / TW, ocol = op - orow * TW;
        const int oh = it.oh0 + orow, ow = it.ow0 + ocol;
        if (orow < TH && oh < p.OH && ow < p.OW) {
          const int sq = sc >> 2;
          float4 v = sws[9][sq];
          const float* xq = lds + ((t >> 6) * C::IPAD) * 4;
#pragma unroll 1
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              const int px = (2 * orow + kh + C::PAD - 1) * C::IW + 2 * ocol + kw + C::PAD - 1;
              const float4 xv = *reinterpret_cast<const float4*>(xq + px * 4);
              const float4 wv = sws[kh * 3 + kw][sq];
              v = fma4pk(xv, wv, v);
            }
          *reinterpret_cast<float4*>(p.sy + (int64_t)it.b * p.sy_bs +
                                     ((int64_t)oh * p.OW + ow) * p.sy_ps + sc) = v;
        }
      }
      // a wave whose 16-channel tile lies past E skips its MFMAs (wave-uniform;
      // its accumulators are masked in the epilogue)
      if (ntv && !(XD_SKIP & 1) && tl) {
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
          const int blk = wave + NW * u;
          if (blk < C::NBLK) {
            const int pb = blk / C::NNT;
            const float b0 = lds[(pb * 16 + j) * 4 + g];
            const float b1 = lds[(C::IPAD + pb * 16 + j) * 4 + g];
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b1, acc[u], 0, 0, 0);
          }
        }
      } else if (ntv && !(XD_SKIP & 1)) {
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
          const int blk = wave + NW * u;
          if (blk < C::NBLK) {
            const int pb = blk / C::NNT;
            const f32x4 bv = *reinterpret_cast<const f32x4*>(lds + (g * C::IPAD + pb * 16 + j) * 4);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bv.x, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bv.y, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bv.z, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bv.w, acc[u], 0, 0, 0);
          }
        }
      }
      lds_barrier();
    }
  }
  XD_T(3);
  // expanded tile: act, zero outside the image / on padded channels
  if (XD_SKIP & 2) {
  } else if (interior) {
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
      const int blk = wave + NW * u;
      if (blk < C::NBLK) {
        const int pb = blk / C::NNT;
        const int px = pb * 16 + j, q = 4 * ntw + g;
        const float4 o = xd_act4<ACT>(make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]));
        if (pb * 16 + 16 <= C::IPX || px < C::IPX)
          *reinterpret_cast<float4*>(lds + (q * C::QP + px) * 4) = o;
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
      const int blk = wave + NW * u;
      if (blk < C::NBLK) {
        const int pb = blk / C::NNT;
        const int px = pb * 16 + j, q = 4 * ntw + g;
        const int r = px / C::IW, c = px - r * C::IW;
        const int ih = it.ih0 + r, iw = it.iw0 + c;
        const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        float4 o = xd_act4<ACT>(make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]));
        if (!ok) o = make_float4(0.f, 0.f, 0.f, 0.f);
        if (px < C::IPX) *reinterpret_cast<float4*>(lds + (q * C::QP + px) * 4) = o;
      }
    }
  }
  if (t < NWD) wsh[t / C::NC4][t % C::NC4] = pwd;
  __syncthreads();
  XD_T(4);

  // depthwise phase
  constexpr int SPW = 64 / C::NC4;  // strips per wave per pass
  float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
  if (chv && !(XD_SKIP & 4)) {
    float* yb = p.y + (int64_t)it.b * p.y_bs + it.c0 + chl;
#pragma unroll 1
    for (int pass = 0; pass * T < C::ITEMS; ++pass) {
      const int strip = (pass * NW + wave) * SPW + sl;
      if (strip >= TH * C::NSTRIP) break;
      const int orow = strip / C::NSTRIP, st = strip - orow * C::NSTRIP;
      const int oh = it.oh0 + orow, owb = it.ow0 + st * C::PW;
      if (oh >= p.OH || owb >= p.OW) continue;
      float4 a2[C::PW];
#pragma unroll
      for (int o = 0; o < C::PW; ++o) a2[o] = bias2;
#pragma unroll 1
      for (int kh = 0; kh < K; ++kh) {
        const float* rowp = lds + (c4 * C::QP + (orow * S + kh) * C::IW + st * C::PW * S) * 4;
        float4 row[C::SPAN];
#pragma unroll
        for (int c = 0; c < C::SPAN; ++c)
          row[c] = *reinterpret_cast<const float4*>(rowp + c * 4);
        float4 wk[K];
#pragma unroll
        for (int kw = 0; kw < K; ++kw) wk[kw] = wsh[kh * K + kw][c4];
#pragma unroll
        for (int o = 0; o < C::PW; ++o)
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            const float4 xv = row[o * S + kw], wv = wk[kw];
            a2[o] = fma4pk(xv, wv, a2[o]);
          }
      }
#pragma unroll
      for (int o = 0; o < C::PW; ++o) {
        if (owb + o >= p.OW) break;
        const float4 v = xd_act4<ACT>(a2[o]);
        *reinterpret_cast<float4*>(yb + ((int64_t)oh * p.OW + owb + o) * p.y_ps) = v;
        psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
      }
    }
  }
  XD_T(5);
  if (p.part && !(XD_SKIP & 8)) {
    // sum the lanes holding the same channel quad (dw_lane): EC = 32 -> lane
    // xor 12, 20 (the even-popcount quad permutations) and 32; EC = 16 ->
    // xor 4, 8, 16, 32.  Fixed order: deterministic.  Lanes 0..NC4-1 then
    // hold channel quads 0..NC4-1.
    constexpr int NX = C::NC4 == 16 ? 2 : C::NC4 == 8 ? 3 : 4;
    constexpr int X8[3] = {12, 20, 32}, X4[4] = {4, 8, 16, 32}, X16[2] = {16, 32};
#pragma unroll
    for (int r = 0; r < NX; ++r) {
      const int off = C::NC4 == 16 ? X16[r] : C::NC4 == 8 ? X8[r] : X4[r];
      psum.x += __shfl_xor(psum.x, off);
      psum.y += __shfl_xor(psum.y, off);
      psum.z += __shfl_xor(psum.z, off);
      psum.w += __shfl_xor(psum.w, off);
    }
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(lds);
    if (lane < C::NC4) red[wave * C::NC4 + lane] = psum;
    __syncthreads();
    if (t < C::NC4 && it.c0 + 4 * t < p.E) {
      // pairwise over the waves in a fixed order
      float4 v[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) v[w] = red[w * C::NC4 + t];
#pragma unroll
      for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
        for (int w = 0; w < h; ++w) {
          v[w].x += v[w + h].x;
          v[w].y += v[w + h].y;
          v[w].z += v[w + h].z;
          v[w].w += v[w + h].w;
        }
      const float4 sm = v[0];
      *reinterpret_cast<float4*>(p.part + ((int64_t)it.b * (int)dv.tiles_img.d + it.t_in) * p.E +
                                 it.c0 + 4 * t) = sm;
    }
  }
  XD_T(6);
  XD_RT(7);
}


// ---------------------------------------------------------------------------
// Stride-1 strip form: a workgroup owns one column strip (NPX = 16 NB input
// columns, NPX - 2 PAD output columns) of a band of rows of one image, for EC
// expanded channels, and walks down the band R rows at a time.  The expanded
// rows live in an LDS ring of R + 2 PAD rows, so each expanded row is
// computed once (no vertical halo recompute) and the band's fixed costs (item
// decode, weight and bias loads, ECA reduction) are paid once per band, not
// per 16x16 tile.  The input stages form one flat software pipeline over
// (row step, 16-channel stage): the next stage's global loads are in flight
// while the current stage's MFMAs, and at a step's end the epilogue and the
// depthwise phase, run.
// ---------------------------------------------------------------------------
template <int K, int EC, int NB, int R>
struct XsCfg {
  static constexpr int PAD = K / 2;
  static constexpr int NPX = 16 * NB, OWS = NPX - 2 * PAD;
  static constexpr int NR = R + 2 * PAD;
  static constexpr int EP = EC + 4;
  static constexpr int NT = EC / 16, NC4 = EC / 4;
  static constexpr int SPX = R * NPX;             // staged pixels per step
  static constexpr int NPF = SPX * 4 / 256;       // float4 stage slots per thread
  static constexpr int NBLK = R * NB * NT, BPW = NBLK / 4;
  static constexpr int PW = 2, NSTRIP = OWS / PW;
  static constexpr int ITEMS = R * NSTRIP * NC4;
  static constexpr int SPAN = PW + K - 1;
  static constexpr int LDS_X = 16 * SPX, LDS_E = NR * NPX * EP;
  static_assert(SPX * 4 % 256 == 0 && NBLK % 4 == 0 && 4 % NT == 0, "strip shape");
  static_assert(OWS % PW == 0, "strip width");
  static_assert((LDS_X + LDS_E) * 4 + (K * K + 1) * EC * 4 <= 80 * 1024, "LDS");
  static_assert(LDS_X >= 4 * 256, "ECA reduction buffer aliases the stage buffer");
};

template <int K, int EC, int NB, int R, int ACT>
__global__ __launch_bounds__(256, 2) void expdw_strip_kernel(const jabd_expdw_args p,
                                                             const XdDivs dv, int nitems,
                                                             int nstrip, int hb) {
  using C = XsCfg<K, EC, NB, R>;
  __shared__ __attribute__((aligned(16))) float xs[C::LDS_X];
  __shared__ __attribute__((aligned(16))) float er[C::LDS_E];
  __shared__ float4 wsh[K * K + 1][C::NC4];
  float4* red = reinterpret_cast<float4*>(xs);  // ECA reduction after the last step
  // item -> (image, band, strip, channel chunk); the chunks of one strip on
  // one XCD (blockIdx % 8), as in xd_item
  const int i = blockIdx.x;
  if (i >= nitems) return;
  const int xcd = i & 7, q = i >> 3;
  const int qn = fdiv(q, dv.nch);
  const int chunk = q - qn * (int)dv.nch.d;
  const int tile = qn * 8 + xcd;
  if (tile >= p.B * (int)dv.tiles_img.d) return;
  const int b = fdiv(tile, dv.tiles_img);
  const int t_in = tile - b * (int)dv.tiles_img.d;
  const int band = t_in / nstrip, strip = t_in - band * nstrip;
  const int hb0 = band * hb, hb1 = min(hb0 + hb, p.OH);
  const int ow0 = strip * C::OWS, iw0 = ow0 - C::PAD;
  const int c0 = chunk * EC;
  const int t = threadIdx.x, lane = t & 63, j = lane & 15, g = lane >> 4;
  const int wave = t >> 6;
  const int ntw = wave % C::NT;
  const int nt = c0 / 16 + ntw;
  const bool ntv = nt < p.Ntiles;
  const int ntc = ntv ? nt : 0;
  const f32x4* wpk = reinterpret_cast<const f32x4*>(p.we);
  const int chb = c0 + 16 * ntw + 4 * g;
  const bool chok = chb < p.E;
  const float4 pbi = *reinterpret_cast<const float4*>(p.be + (chok ? chb : 0));
  const f32x4 bias4 = (f32x4){pbi.x, pbi.y, pbi.z, pbi.w};
  for (int u = t; u < (K * K + 1) * C::NC4; u += 256) {
    const int tp = u / C::NC4, cc = c0 + 4 * (u - tp * C::NC4);
    const float4 w = *reinterpret_cast<const float4*>((tp < K * K ? p.wd + tp * p.E : p.bd) +
                                                      (cc < p.E ? cc : 0));
    wsh[tp][u - tp * C::NC4] = cc < p.E ? w : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x), (short)0, (int)(uint32_t)((int64_t)p.B * p.x_bs * 4), 0x00020000);
  const int cq = ((t >> 4) & 3) * 4;
  const int spx0 = (t >> 6) * 16 + (t & 15);
  // expanded rows are computed from input row e0 = hb0 - PAD on, R per step
  const int e0 = hb0 - C::PAD;
  const int nsteps = (hb1 - hb0 + 2 * C::PAD + R - 1) / R;
  const int nitem = nsteps * p.Kc;
  float4 pf[C::NPF];
  auto load_stage = [&](int it) {
    const int s = it / p.Kc, kc = it - s * p.Kc;
    const int cofs = 16 * kc + cq;
    const uint32_t base = (uint32_t)(b * p.x_bs + cofs);
    const bool cok = cofs < p.Cin;
#pragma unroll
    for (int u = 0; u < C::NPF; ++u) {
      const int px = u * 64 + spx0;
      const int r = px / C::NPX, c = px - r * C::NPX;
      const int ih = e0 + s * R + r, iw = iw0 + c;
      const bool ok = cok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const uint32_t off = ok ? (base + (uint32_t)((ih * p.W + iw) * p.x_ps)) * 4u : 0xFFFFFFF0u;
      pf[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  int c4, sl;
  dw_lane<C::NC4>(lane, c4, sl);
  const int chl = 4 * c4;
  const bool chv = c0 + chl < p.E;
  float* yb = p.y + (int64_t)b * p.y_bs + c0 + chl;
  float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
  f32x4 acc[C::BPW];
  load_stage(0);
  for (int it = 0; it < nitem; ++it) {
    const int s = it / p.Kc, kc = it - s * p.Kc;
    if (kc == 0) {
#pragma unroll
      for (int u = 0; u < C::BPW; ++u) acc[u] = bias4;
    }
    f32x4 a = wpk[(kc * p.Ntiles + ntc) * 64 + lane];
#pragma unroll
    for (int u = 0; u < C::NPF; ++u)
      *reinterpret_cast<float4*>(xs + ((cq / 4) * C::SPX + u * 64 + spx0) * 4) = pf[u];
    if (!ntv) a = (f32x4){0.f, 0.f, 0.f, 0.f};
    asm volatile("" : "+v"(a));
    lds_barrier();
    if (it + 1 < nitem) load_stage(it + 1);
    if (ntv) {
#pragma unroll
      for (int u = 0; u < C::BPW; ++u) {
        const int pb = (wave + 4 * u) / C::NT;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(xs + (g * C::SPX + pb * 16 + j) * 4);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bv.x, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bv.y, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bv.z, acc[u], 0, 0, 0);
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bv.w, acc[u], 0, 0, 0);
      }
    }
    if (kc + 1 < p.Kc) {
      lds_barrier();
      continue;
    }
    // step s complete: activated rows e0 + s R .. + R - 1 into the ring (zero
    // outside the image: the depthwise conv zero-pads the activated map)
#pragma unroll
    for (int u = 0; u < C::BPW; ++u) {
      const int pb = (wave + 4 * u) / C::NT;
      const int px = pb * 16 + j;
      const int r = px / C::NPX, c = px - r * C::NPX;
      const int ih = e0 + s * R + r, iw = iw0 + c;
      const bool ok = chok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const int slot = (s * R + r) % C::NR;
      float4 o;
      o.x = ok ? xd_act<ACT>(acc[u][0]) : 0.f;
      o.y = ok ? xd_act<ACT>(acc[u][1]) : 0.f;
      o.z = ok ? xd_act<ACT>(acc[u][2]) : 0.f;
      o.w = ok ? xd_act<ACT>(acc[u][3]) : 0.f;
      *reinterpret_cast<float4*>(er + (slot * C::NPX + c) * C::EP + 16 * ntw + 4 * g) = o;
    }
    lds_barrier();  // LDS only: keeps the next stage's loads in flight
    // depthwise: output rows oh = hb0 + s R - 2 PAD + orow, those inside the band
    if (chv) {
      const float4 bias2 = wsh[K * K][c4];
#pragma unroll 1
      for (int pass = 0; pass * 256 < C::ITEMS; ++pass) {
        const int item = (pass * 4 + wave) * (64 / C::NC4) + sl;
        if (item >= R * C::NSTRIP) break;
        const int orow = item / C::NSTRIP, st = item - orow * C::NSTRIP;
        const int oh = hb0 + s * R - 2 * C::PAD + orow;
        const int owb = ow0 + st * C::PW;
        if (oh < hb0 || oh >= hb1 || owb >= p.OW) continue;
        float4 a2[C::PW];
#pragma unroll
        for (int o = 0; o < C::PW; ++o) a2[o] = bias2;
#pragma unroll 1
        for (int kh = 0; kh < K; ++kh) {
          const int slot = (oh - e0 - C::PAD + kh) % C::NR;
          const float* rowp = er + (slot * C::NPX + st * C::PW) * C::EP + chl;
          float4 row[C::SPAN];
#pragma unroll
          for (int c = 0; c < C::SPAN; ++c)
            row[c] = *reinterpret_cast<const float4*>(rowp + c * C::EP);
          float4 wk[K];
#pragma unroll
          for (int kw = 0; kw < K; ++kw) wk[kw] = wsh[kh * K + kw][c4];
#pragma unroll
          for (int o = 0; o < C::PW; ++o)
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
              const float4 xv = row[o + kw], wv = wk[kw];
              a2[o] = fma4pk(xv, wv, a2[o]);
            }
        }
#pragma unroll
        for (int o = 0; o < C::PW; ++o) {
          if (owb + o >= p.OW) break;
          float4 v;
          v.x = xd_act<ACT>(a2[o].x);
          v.y = xd_act<ACT>(a2[o].y);
          v.z = xd_act<ACT>(a2[o].z);
          v.w = xd_act<ACT>(a2[o].w);
          *reinterpret_cast<float4*>(yb + ((int64_t)oh * p.OW + owb + o) * p.y_ps) = v;
          psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
        }
      }
    }
    // the next step's first stage rewrites xs only after this barrier; the
    // ring rows this step read are rewritten after the next step's barriers
    lds_barrier();
  }
  if (p.part) {
    __syncthreads();
    red[t] = psum;
    __syncthreads();
    if (t < C::NC4 && c0 + 4 * t < p.E) {
      // threads holding channel quad t (dw_lane), summed in thread order
      float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int u = 0; u < 256; ++u) {
        int cu, su;
        dw_lane<C::NC4>(u & 63, cu, su);
        if (cu != t) continue;
        const float4 v = red[u];
        sm.x += v.x; sm.y += v.y; sm.z += v.z; sm.w += v.w;
      }
      *reinterpret_cast<float4*>(p.part + ((int64_t)b * (int)dv.tiles_img.d + t_in) * p.E + c0 +
                                 4 * t) = sm;
    }
  }
}

// ---------------------------------------------------------------------------
// Wave-specialised persistent form (JABD_EXPDW_WS=1; off by default, see
// xw_enabled).  Phase-skip builds of expdw1_kernel (XD_SKIP) showed its
// expand-MFMA and depthwise phases are additive in wall time (skipping both
// saves the sum of skipping each): the resident workgroups run their phases
// in step and never overlap matrix work with vector work.  Here one
// workgroup per CU (XW_NE expand waves + 4 depthwise waves) walks its items
// (item = blockIdx.x + n * gridDim.x, same XCD-aware decode) as a two-role
// pipeline:
//  * expand waves: wave w owns pixel blocks w, w + XW_NE, ... of the staged
//    tile for every 16-channel n-tile; its B operands (pixel j, channel quad
//    g of a 16-channel stage) are loaded straight into registers through the
//    buffer descriptor (no LDS staging, no barrier per stage) from a D-deep
//    ring of stages that runs across item boundaries; the activated tile is
//    written to expanded buffer (item & 1);
//  * depthwise waves: the depthwise phase, ECA partials and the fused
//    skip branch of the previous item from the other buffer.
// Step n: expand item n while the depthwise waves finish item n - 1; one
// LDS-only barrier per step.  Each output element is computed by exactly the
// operation sequence of expdw1_kernel (accumulators start at the bias, the
// same k order of MFMAs, the same depthwise lane map, tap order and ECA
// reduction), so the two kernels agree bit for bit.
// ---------------------------------------------------------------------------
// expand waves per workgroup (the depthwise waves are always 4)
#ifndef XW_NE
#define XW_NE 4
#endif
template <int K, int S, int TH, int TW, int EC, bool SKIP>
struct XwCfg {
  using C = XdCfg<K, S, TH, TW, EC>;
  static constexpr int NE = XW_NE, NT = 64 * (NE + 4);
  static constexpr int NBW = (C::NPB + NE - 1) / NE;  // pixel blocks per expand wave
  static constexpr int SKC = SKIP ? 160 : 4;
  // dynamic LDS: expanded buffers, depthwise taps, ECA partials, skip taps
  static constexpr int OFF_W = 2 * C::LDS_E * 4;
  static constexpr int OFF_R = OFF_W + 2 * (K * K + 1) * C::NC4 * 16;
  static constexpr int OFF_S = OFF_R + 2 * 4 * C::NC4 * 16;
  static constexpr int BYTES = OFF_S + 10 * (SKC / 4) * 16;
  static_assert(BYTES <= 160 * 1024, "LDS");
};

template <int NBW, int NNT>
struct XwSlot {
  float4 b[NBW];
  f32x4 a[NNT];
  float4 bias[NNT];
  float4 taps;  // depthwise tap / bias float4 (thread t < NWD) of the item's chunk
};

template <int NBW, int NNT>
__device__ __forceinline__ void xw_touch(XwSlot<NBW, NNT>& sl) {
#pragma unroll
  for (int u = 0; u < NBW; ++u)
    asm volatile("" : "+v"(sl.b[u].x), "+v"(sl.b[u].y), "+v"(sl.b[u].z), "+v"(sl.b[u].w));
#pragma unroll
  for (int nt = 0; nt < NNT; ++nt) {
    asm volatile("" : "+v"(sl.a[nt]));
    asm volatile("" : "+v"(sl.bias[nt].x), "+v"(sl.bias[nt].y), "+v"(sl.bias[nt].z),
                 "+v"(sl.bias[nt].w));
  }
  asm volatile("" : "+v"(sl.taps.x), "+v"(sl.taps.y), "+v"(sl.taps.z), "+v"(sl.taps.w));
}

// One stage's MFMAs of an expand wave: blocks u < NBU, n-tiles nt < NTU, k
// order x, y, z, w per accumulator (as expdw1_kernel), independent
// accumulators interleaved.
template <int NBU, int NTU, int NBW, int NNT>
__device__ __forceinline__ void xw_mfma(f32x4 (&acc)[NBW][NNT], const XwSlot<NBW, NNT>& sl) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int u = 0; u < NBU; ++u)
#pragma unroll
      for (int nt = 0; nt < NTU; ++nt) {
        const float av = e == 0 ? sl.a[nt].x : e == 1 ? sl.a[nt].y : e == 2 ? sl.a[nt].z : sl.a[nt].w;
        const float bv = e == 0 ? sl.b[u].x : e == 1 ? sl.b[u].y : e == 2 ? sl.b[u].z : sl.b[u].w;
        acc[u][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[u][nt], 0, 0, 0);
      }
}

template <int K, int S, int TH, int TW, int EC, int ACT, bool SKIP, int D>
__global__ __launch_bounds__(64 * (XW_NE + 4)) void expdw_ws_kernel(const jabd_expdw_args p, const XdDivs dv,
                                                      int nitems) {
  using C = XdCfg<K, S, TH, TW, EC>;
  using W = XwCfg<K, S, TH, TW, EC, SKIP>;
  constexpr int NBW = W::NBW, NNT = C::NNT, NC4 = C::NC4, NE = W::NE;
  constexpr int NWD = (K * K + 1) * NC4;
  static_assert(NWD <= 64 * NE, "taps: one float4 per expand thread");
  extern __shared__ __attribute__((aligned(16))) unsigned char xw_smem[];
  float* ebuf = reinterpret_cast<float*>(xw_smem);                            // [2][LDS_E]
  float4* wsh = reinterpret_cast<float4*>(xw_smem + W::OFF_W);                // [2][K*K+1][NC4]
  float4* red = reinterpret_cast<float4*>(xw_smem + W::OFF_R);                // [2][4][NC4]
  float4* sws = reinterpret_cast<float4*>(xw_smem + W::OFF_S);                // [10][SKC/4]
  const int G = gridDim.x;
  const int nmine = (nitems - (int)blockIdx.x + G - 1) / G;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  if (SKIP) {
    for (int i = t; i < 10 * (p.Cin >> 2); i += W::NT) {
      const int q = i / (p.Cin >> 2), c4 = i - q * (p.Cin >> 2);
      sws[q * (W::SKC / 4) + c4] =
          *reinterpret_cast<const float4*>((q < 9 ? p.sw + q * p.Cin : p.sb) + 4 * c4);
    }
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x), (short)0, (int)(uint32_t)((int64_t)p.B * p.x_bs * 4), 0x00020000);
  auto decode = [&](int n, XdItem& it) -> bool {
    it = XdItem{0, 0, 0, 0, 0, 0, 0};
    return n < nmine && xd_item<K, S, TH, TW, EC>(p, (int)blockIdx.x + n * G, dv, nitems, it);
  };

  if (wave < NE) {
    // ------------------------------------------------------------- expand
    const int j = lane & 15, g = lane >> 4;
    const f32x4* wpk = reinterpret_cast<const f32x4*>(p.we);
    const int U = (nmine * p.Kc + D - 1) / D * D;  // stages, padded to the ring depth
    int ls = 0, lkc = 0;                            // load cursor (item seq, stage)
    XdItem li;
    bool lv = decode(0, li);
    // per-item load state of the load cursor's item: byte offsets of each
    // block's (pixel, channel 4g) at stage 0 (0xFFFFFFF0: out of the image /
    // tile, reads zeros), weight / bias / tap indices; a stage then only adds
    // its 64-byte channel offset (the address arithmetic stays out of the
    // per-stage instruction stream)
    uint32_t boff[NBW];
    int aoff[NNT], boffb[NNT];
    const float* tptr = p.bd;
    auto prep = [&]() {
#pragma unroll
      for (int u = 0; u < NBW; ++u) {
        const int pb = wave + NE * u;
        const int px = pb * 16 + j;
        const int r = px / C::IW, c = px - r * C::IW;
        const int ih = li.ih0 + r, iw = li.iw0 + c;
        const bool ok = lv && px < C::IPX && (unsigned)ih < (unsigned)p.H &&
                        (unsigned)iw < (unsigned)p.W && !(XD_SKIP & 128);
        boff[u] = ok ? (uint32_t)(li.b * p.x_bs + (ih * p.W + iw) * p.x_ps + 4 * g) * 4u
                     : 0xFFFFF000u;  // stays out of range (host: x < 0xFFFFF000 bytes) + 64 Kc
      }
#pragma unroll
      for (int nt = 0; nt < NNT; ++nt) {
        const int ntg = li.c0 / 16 + nt;
        aoff[nt] = (lv && ntg < p.Ntiles ? ntg : 0) * 64 + lane;
        const int chb = li.c0 + 16 * nt + 4 * g;
        boffb[nt] = chb < p.E ? chb : 0;
      }
      const int dd = t < NWD ? t : 0;
      const int tp = dd / NC4, cc = li.c0 + 4 * (dd - tp * NC4);
      tptr = (tp < K * K ? p.wd + tp * p.E : p.bd) + (cc < p.E ? cc : 0);
    };
    prep();
    auto issue = [&](XwSlot<NBW, NNT>& sl) {
      // channels past Cin read zeros: the offset is raised out of range by a
      // max (no select / branch per load)
      const uint32_t lim = 16 * lkc + 4 * g < p.Cin ? 0u : 0xFFFFF000u;
#pragma unroll
      for (int u = 0; u < NBW; ++u) {
        const uint32_t off = max(boff[u] + 64u * (uint32_t)lkc, lim);
        sl.b[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      }
#pragma unroll
      for (int nt = 0; nt < NNT; ++nt) {
        sl.a[nt] = wpk[aoff[nt] + lkc * p.Ntiles * 64];
        sl.bias[nt] = *reinterpret_cast<const float4*>(p.be + boffb[nt]);
      }
      sl.taps = *reinterpret_cast<const float4*>(tptr);
      if (++lkc == p.Kc) {
        lkc = 0;
        ++ls;
        lv = decode(ls, li);
        prep();
      }
    };
    int cs = 0, ckc = 0;  // consume cursor
    XdItem ci;
    bool cv = decode(0, ci);
    f32x4 acc[NBW][NNT];
    float4 taps = make_float4(0.f, 0.f, 0.f, 0.f);
    auto stage = [&](XwSlot<NBW, NNT>& sl) {
      // retire this slot's loads on every path here: a load left pending on
      // a path that skips its consumer (an unused n-tile, an invalid item)
      // makes the compiler wait before the slot's registers are reused,
      // draining the other slots' loads too (one stage of latency cover)
      xw_touch(sl);
      if (ckc == 0) {
        taps = sl.taps;
#pragma unroll
        for (int u = 0; u < NBW; ++u)
#pragma unroll
          for (int nt = 0; nt < NNT; ++nt)
            acc[u][nt] = (f32x4){sl.bias[nt].x, sl.bias[nt].y, sl.bias[nt].z, sl.bias[nt].w};
      }
      // every wave runs the full NBW x NNT block of MFMAs: blocks past the
      // tile read zeros, n-tiles past E and invalid items compute values
      // the epilogue never stores (a uniform branch per variant made the
      // compiler shuffle accumulators between variants)
      if (!(XD_SKIP & 32)) xw_mfma<NBW, NNT>(acc, sl);
      issue(sl);  // this slot's registers now take the stage D ahead
      if (ckc == p.Kc - 1 && cs < nmine) {
        if (cv && !(XD_SKIP & 256)) {
          float* eb = ebuf + (cs & 1) * C::LDS_E;
#pragma unroll
          for (int u = 0; u < NBW; ++u) {
            const int pb = wave + NE * u;
            if (pb >= C::NPB) continue;
            const int px = pb * 16 + j;
            const int r = px / C::IW, c = px - r * C::IW;
            const int ih = ci.ih0 + r, iw = ci.iw0 + c;
            const bool pok = px < C::IPX && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
#pragma unroll
            for (int nt = 0; nt < NNT; ++nt) {
              const bool ok = pok && ci.c0 + 16 * nt + 4 * g < p.E;
              float4 o;
              o.x = ok ? xd_act<ACT>(acc[u][nt][0]) : 0.f;
              o.y = ok ? xd_act<ACT>(acc[u][nt][1]) : 0.f;
              o.z = ok ? xd_act<ACT>(acc[u][nt][2]) : 0.f;
              o.w = ok ? xd_act<ACT>(acc[u][nt][3]) : 0.f;
              *reinterpret_cast<float4*>(eb + px * C::EP + 16 * nt + 4 * g) = o;
            }
          }
          if (t < NWD) {
            const int tp = t / NC4, cc = ci.c0 + 4 * (t - tp * NC4);
            const bool ok = cc < p.E;
            wsh[(cs & 1) * NWD + t] =
                make_float4(ok ? taps.x : 0.f, ok ? taps.y : 0.f, ok ? taps.z : 0.f, ok ? taps.w : 0.f);
          }
        }
        if (!(XD_SKIP & 512)) lds_barrier();  // end of step cs: buffers (cs & 1) hold item cs
      }
      if (++ckc == p.Kc) {
        ckc = 0;
        ++cs;
        cv = decode(cs, ci);
      }
    };
    XwSlot<NBW, NNT> sl[D];
#pragma unroll
    for (int d = 0; d < D; ++d) issue(sl[d]);
    for (int u = 0; u < U; u += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) stage(sl[d]);
    }
    if (!(XD_SKIP & 512)) lds_barrier();  // the depthwise waves' last step
    return;
  }
  if (XD_SKIP & 512) return;

  // ------------------------------------------------------------- depthwise
  const int dt = t - 64 * NE, dwv = wave - NE;
  auto finalize = [&](int n) {  // ECA partial of item n from red[n & 1]
    XdItem it;
    if (dwv != 0 || !decode(n, it) || !p.part) return;
    if (lane < NC4 && it.c0 + 4 * lane < p.E) {
      const float4* rb = red + (n & 1) * 4 * NC4;
      float4 v[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) v[w] = rb[w * NC4 + lane];
#pragma unroll
      for (int h = 2; h >= 1; h >>= 1)
#pragma unroll
        for (int w = 0; w < h; ++w) {
          v[w].x += v[w + h].x;
          v[w].y += v[w + h].y;
          v[w].z += v[w + h].z;
          v[w].w += v[w + h].w;
        }
      *reinterpret_cast<float4*>(p.part + ((int64_t)it.b * (int)dv.tiles_img.d + it.t_in) * p.E +
                                 it.c0 + 4 * lane) = v[0];
    }
  };
  int c4, sl;
  dw_lane<NC4>(lane, c4, sl);
  const int chl = 4 * c4;
  constexpr int SPW = 64 / NC4;
  lds_barrier();  // the expand waves' step 0 (item 0)
  for (int n = 0; n < nmine; ++n) {
    XdItem it;
    const bool valid = decode(n, it);
    if (valid && SKIP && it.c0 == 0) {
      // skip branch dw3x3/s2 + bias on x: output (orow, ocol), channel quad sq
      const int nq = p.Cin >> 2;
      for (int i = dt; i < 64 * nq; i += 256) {
        const int sq = i >> 6, op = i & 63, orow = op / TW, ocol = op - orow * TW;
        const int oh = it.oh0 + orow, ow = it.ow0 + ocol;
        if (orow >= TH || oh >= p.OH || ow >= p.OW) continue;
        float4 v = sws[9 * (W::SKC / 4) + sq];
        const uint32_t base = (uint32_t)(it.b * p.x_bs + 4 * sq);
#pragma unroll 1
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int ih = 2 * oh + kh - 1, iw = 2 * ow + kw - 1;
            const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            const uint32_t off = ok ? (base + (uint32_t)((ih * p.W + iw) * p.x_ps)) * 4u : 0xFFFFFFF0u;
            const float4 xv =
                __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            const float4 wv = sws[(kh * 3 + kw) * (W::SKC / 4) + sq];
            v = fma4pk(xv, wv, v);
          }
        *reinterpret_cast<float4*>(p.sy + (int64_t)it.b * p.sy_bs +
                                   ((int64_t)oh * p.OW + ow) * p.sy_ps + 4 * sq) = v;
      }
    }
    float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid && it.c0 + chl < p.E && !(XD_SKIP & 64)) {
      const float* eb = ebuf + (n & 1) * C::LDS_E;
      const float4* wb = wsh + (n & 1) * (K * K + 1) * NC4;
      const float4 bias2 = wb[K * K * NC4 + c4];
      float* yb = p.y + (int64_t)it.b * p.y_bs + it.c0 + chl;
#pragma unroll 1
      for (int pass = 0; pass * 256 < C::ITEMS; ++pass) {
        const int strip = (pass * 4 + dwv) * SPW + sl;
        if (strip >= TH * C::NSTRIP) break;
        const int orow = strip / C::NSTRIP, st = strip - orow * C::NSTRIP;
        const int oh = it.oh0 + orow, owb = it.ow0 + st * C::PW;
        if (oh >= p.OH || owb >= p.OW) continue;
        float4 a2[C::PW];
#pragma unroll
        for (int o = 0; o < C::PW; ++o) a2[o] = bias2;
#pragma unroll 1
        for (int kh = 0; kh < K; ++kh) {
          const float* rowp = eb + ((orow * S + kh) * C::IW + st * C::PW * S) * C::EP + chl;
          float4 row[C::SPAN];
#pragma unroll
          for (int c = 0; c < C::SPAN; ++c)
            row[c] = *reinterpret_cast<const float4*>(rowp + c * C::EP);
          float4 wk[K];
#pragma unroll
          for (int kw = 0; kw < K; ++kw) wk[kw] = wb[(kh * K + kw) * NC4 + c4];
#pragma unroll
          for (int o = 0; o < C::PW; ++o)
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
              const float4 xv = row[o * S + kw], wv = wk[kw];
              a2[o] = fma4pk(xv, wv, a2[o]);
            }
        }
#pragma unroll
        for (int o = 0; o < C::PW; ++o) {
          if (owb + o >= p.OW) break;
          float4 v;
          v.x = xd_act<ACT>(a2[o].x);
          v.y = xd_act<ACT>(a2[o].y);
          v.z = xd_act<ACT>(a2[o].z);
          v.w = xd_act<ACT>(a2[o].w);
          *reinterpret_cast<float4*>(yb + ((int64_t)oh * p.OW + owb + o) * p.y_ps) = v;
          psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
        }
      }
    }
    if (p.part) {
      constexpr int NX = NC4 == 8 ? 3 : 4;
      constexpr int X8[3] = {12, 20, 32}, X4[4] = {4, 8, 16, 32};
#pragma unroll
      for (int r = 0; r < NX; ++r) {
        const int off = NC4 == 8 ? X8[r] : X4[r];
        psum.x += __shfl_xor(psum.x, off);
        psum.y += __shfl_xor(psum.y, off);
        psum.z += __shfl_xor(psum.z, off);
        psum.w += __shfl_xor(psum.w, off);
      }
      if (lane < NC4) red[(n & 1) * 4 * NC4 + dwv * NC4 + lane] = psum;
      if (n >= 1) finalize(n - 1);
    }
    lds_barrier();
  }
  if (p.part && nmine >= 1) finalize(nmine - 1);
}

// expand-wave load ring depth (stages in flight) of expdw_ws_kernel
#ifndef XW_D
#define XW_D 2
#endif

// 3x3 stride 1: 14 x 16 outputs (16 x 18 = 288 input pixels, 18 MFMA blocks
// with no padding; the 32-channel expanded tile is 37 KB, 4 workgroups per
// CU where 16 x 16 (41.6 KB) allows 3); 5x5 stride 1: 16 x 16; stride 2: 8 x 8
XdTile xd_tile(int k, int s) {
  if (s == 1) return k == 3 ? XdTile{14, 16} : XdTile{16, 16};
  return XdTile{8, 8};
}

// skip-branch LDS taps: the smallest staged channel count >= Cin
int xd_skc(int cin) { return cin <= 40 ? 40 : cin <= 112 ? 112 : 160; }

}  // namespace jabd

using namespace jabd;

// JABD_EXPDW_KP=2|3: input register ring depth (A/B).  Default 1: deeper
// rings measured 0-7% slower (b3/b4/b11/b12 in tools/convbench.py --set xd),
// the VGPRs they take cost occupancy and the stage latency is not the bound.
static int xd_kp() {
  static int kp = -1;
  if (kp < 0) {
    const char* e = getenv("JABD_EXPDW_KP");
    kp = e && (e[0] == '2' || e[0] == '3') ? e[0] - '0' : 1;
  }
  return kp;
}

// Waves per workgroup.  The expanded tile's LDS caps resident workgroups
// at 2-3 per CU, so 8-wave workgroups double the resident waves on the same
// tile (half the accumulators and prefetch registers per wave).
// JABD_EXPDW_NW=4|8 forces one form for A/B.
static int xd_nw(const jabd_expdw_args& a, int EC) {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("JABD_EXPDW_NW");
    env = e && e[0] == '8' ? 8 : (e && e[0] == '4' ? 4 : 0);
  }
  (void)a;
  (void)EC;
  if (env) return env;
  return 4;
}

// Strip form (stride 1), JABD_EXPDW_STRIP=1 for A/B; off by default: it
// measured slower than the 16x16 tile kernel on every stride-1 layer (b1
// 295 vs 271 us, b3 405 vs 347, b12 525 vs 347, b15 346 vs 204;
// tools/convbench.py --set xd): a row step carries less MFMA work per input
// stage and per barrier than a tile, and the NB = 3 / EC = 32 form holds
// 55 KB of LDS (2 workgroups per CU).  See DESIGN.md section 4.
static bool xs_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("JABD_EXPDW_STRIP");
    on = e && e[0] == '1' ? 1 : 0;
  }
  return on == 1;
}

// Wave-specialised persistent kernel (expdw_ws_kernel): off by default —
// bit-identical to expdw1_kernel but measured 13% slower over the twelve
// C2 layer shapes (3.50 vs 3.10 ms in tools/convbench.py --set xd; parity on
// the K >= 112 layers, 17-33% slower on the one- and two-stage layers, see
// DESIGN.md section 4).  JABD_EXPDW_WS=1 or jabd_expand_dw_select(2) selects it.
static int xw_form = 0;  // jabd_expand_dw_select
static bool xw_enabled() {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("JABD_EXPDW_WS");
    env = e && e[0] == '1' ? 1 : 0;
  }
  return xw_form ? xw_form == 2 : env == 1;
}
// persistent per-chunk form (expdw2.hip): off by default — it halves the
// VALU instructions per item (SQ counters: 294 vs 586 per wave on the 8x8
// stride-2 tile) yet runs 5-65% slower per layer: the one-item workgroups'
// turnover hides latency that a persistent workgroup waits out (DESIGN.md
// section 4).  JABD_EXPDW2=1 or jabd_expand_dw_select(3) selects it.
static bool x2_enabled() {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("JABD_EXPDW2");
    env = e && e[0] == '1' ? 1 : 0;
  }
  return xw_form ? xw_form == 3 : env == 1;
}

template <int K, int S, int TH, int TW, int EC, int ACT, bool SKIP>
static int xw_launch(const jabd_expdw_args& a, const XdDivs& dv, int64_t nitems, hipStream_t st) {
  constexpr int D = XW_D;
  auto kern = expdw_ws_kernel<K, S, TH, TW, EC, ACT, SKIP, D>;
  constexpr int bytes = XwCfg<K, S, TH, TW, EC, SKIP>::BYTES;
  static int occ = -1, ncu = 0;
  if (occ < 0) {
    int dev = 0;
    JABD_HIP(hipGetDevice(&dev));
    JABD_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    JABD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    int o = 0;
    JABD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, XwCfg<K, S, TH, TW, EC, SKIP>::NT,
                                                          bytes));
    occ = o < 1 ? 1 : o;
  }
  // expand-wave input offsets use 0xFFFFF000 + 64 Kc as "out of range"
  JABD_REQUIRE((int64_t)a.B * a.x_bs * 4 <= 0xFFFFF000ll - 1024,
               "expand_dw: input must be < 4 GiB - 5 KiB (split the batch)");
  const int64_t cap = (int64_t)ncu * occ;
  const int grid = (int)(nitems < cap ? nitems : cap);
  kern<<<grid, XwCfg<K, S, TH, TW, EC, SKIP>::NT, bytes, st>>>(a, dv, (int)nitems);
  return check_launch("expand_dw_ws");
}

struct XsPlan {
  int nb, nstrip, hb, nband;
};

// strip width 16 NB input columns: the NB in {2, 3} with the fewest computed
// columns (the smaller on ties); bands of 64 rows on maps >= 256 rows, else 32
static XsPlan xs_plan(int OH, int OW, int k) {
  XsPlan pl;
  int best = 0;
  for (int nb = 2; nb <= 3; ++nb) {
    const int ows = 16 * nb - 2 * (k / 2);
    const int ns = (int)cdiv(OW, ows);
    if (!best || ns * 16 * nb < best) {
      best = ns * 16 * nb;
      pl.nb = nb;
      pl.nstrip = ns;
    }
  }
  pl.hb = OH >= 256 ? 64 : 32;
  pl.nband = (int)cdiv(OH, pl.hb);
  return pl;
}

#if XD_TRACE
extern "C" int jabd_xd_trace_set(void* buf) {
  unsigned long long* p = static_cast<unsigned long long*>(buf);
  JABD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(xd_trace_buf), &p, sizeof(p)));
  return JABD_OK;
}
#endif

extern "C" int jabd_expand_dw_select(int32_t form) {
  const int prev = xw_form;
  xw_form = form >= 1 && form <= 4 ? form : 0;
  return prev;
}

extern "C" int64_t jabd_expand_dw_nblk(int32_t OH, int32_t OW, int32_t k, int32_t stride) {
  if (OH <= 0 || OW <= 0 || (stride != 1 && stride != 2)) return -1;
  if (stride == 1 && xs_enabled()) {
    const XsPlan pl = xs_plan(OH, OW, k);
    return (int64_t)pl.nband * pl.nstrip;
  }
  const XdTile tl = xd_tile(k, stride);
  return cdiv(OH, tl.th) * cdiv(OW, tl.tw);
}

extern "C" int jabd_expand_dw_nhwc_f32(const jabd_expdw_args* args, jabd_stream_t stream) {
  JABD_REQUIRE(args, "expand_dw: null args");
  const jabd_expdw_args& a = *args;
  JABD_REQUIRE(a.x && a.we && a.be && a.wd && a.bd && a.y, "expand_dw: null pointer");
  JABD_REQUIRE(a.Cin % 4 == 0 && a.x_ps % 4 == 0 && a.E % 4 == 0 && a.y_ps % 4 == 0 &&
                   a.y_ps >= a.E && a.x_ps >= a.Cin,
               "expand_dw: channel counts / strides must be multiples of 4");
  JABD_REQUIRE(a.Kc == (a.Cin + 15) / 16 && a.Ntiles * 16 >= a.E, "expand_dw: packing mismatch");
  JABD_REQUIRE((a.k == 3 || a.k == 5) && (a.stride == 1 || a.stride == 2) &&
                   a.OH == (a.H + 2 * (a.k / 2) - a.k) / a.stride + 1 &&
                   a.OW == (a.W + 2 * (a.k / 2) - a.k) / a.stride + 1,
               "expand_dw: unsupported geometry");
  JABD_REQUIRE(a.act == ACT_NONE || a.act == ACT_RELU || a.act == ACT_HSWISH,
               "expand_dw: act %d", a.act);
  JABD_REQUIRE(!a.sy || (a.stride == 2 && a.sw && a.sb && a.sy_ps % 4 == 0 && a.sy_ps >= a.Cin &&
                         a.Cin <= 160),
               "expand_dw: the fused skip branch needs stride 2, Cin <= 160, weights, bias and "
               "sy_ps %% 4 == 0");
  if (a.stride == 1 && xs_enabled()) {
    const XsPlan pl = xs_plan(a.OH, a.OW, a.k);
    const int tiles_img = pl.nband * pl.nstrip;
    JABD_REQUIRE(!a.part || a.nblk == tiles_img, "expand_dw: nblk %d != %d", a.nblk, tiles_img);
    const int EC = a.E <= 16 ? 16 : 32;
    const int nch = (int)cdiv(a.E, EC);
    const int64_t nitems = cdiv((int64_t)a.B * tiles_img, 8) * 8 * nch;
    JABD_REQUIRE(nitems < ((int64_t)1 << 31) && (int64_t)a.H * a.W * a.x_ps < ((int64_t)1 << 31) &&
                     (int64_t)a.B * a.x_bs * 4 < ((int64_t)1 << 32) - 16,
                 "expand_dw: problem too large for 32-bit indexing / buffer offsets (split the batch)");
    const XdDivs dv{make_fastdiv((uint32_t)nch), make_fastdiv((uint32_t)tiles_img),
                    make_fastdiv((uint32_t)pl.nstrip)};
    hipStream_t st = as_stream(stream);
#define XS_LAUNCH(K_, EC_, NB_, ACT_)                                                       \
  expdw_strip_kernel<K_, EC_, NB_, 4, ACT_><<<(unsigned)nitems, 256, 0, st>>>(a, dv, (int)nitems, \
                                                                             pl.nstrip, pl.hb)
#define XS_ACTS(K_, EC_, NB_)                              \
  if (a.k == K_ && EC == EC_ && pl.nb == NB_) {            \
    if (a.act == ACT_RELU)                                 \
      XS_LAUNCH(K_, EC_, NB_, ACT_RELU);                   \
    else if (a.act == ACT_HSWISH)                          \
      XS_LAUNCH(K_, EC_, NB_, ACT_HSWISH);                 \
    else                                                   \
      XS_LAUNCH(K_, EC_, NB_, ACT_NONE);                   \
    return check_launch("expand_dw_strip");                \
  }
    XS_ACTS(3, 16, 2) XS_ACTS(3, 16, 3) XS_ACTS(3, 32, 2) XS_ACTS(3, 32, 3)
    XS_ACTS(5, 16, 2) XS_ACTS(5, 16, 3) XS_ACTS(5, 32, 2) XS_ACTS(5, 32, 3)
#undef XS_ACTS
#undef XS_LAUNCH
    set_error("expand_dw: no strip kernel for k=%d", a.k);
    return JABD_EINVAL;
  }
  const XdTile tl = xd_tile(a.k, a.stride);
  const int tiles_w = (int)cdiv(a.OW, tl.tw);
  const int tiles_img = (int)cdiv(a.OH, tl.th) * tiles_w;
  JABD_REQUIRE(!a.part || a.nblk == tiles_img, "expand_dw: nblk %d != %d", a.nblk, tiles_img);
  static int ec16 = -1;
  if (ec16 < 0) {
    const char* e = getenv("JABD_EXPDW_EC16");
    ec16 = e && e[0] == '1' ? 1 : 0;
  }
  // 16-channel chunks for small E, and for the 5x5 stride-2 tile (19x19 input
  // pixels: the 32-channel tile's LDS allows only 2 resident workgroups)
  const int EC = (a.E <= 16 || ec16 || (a.k == 5 && a.stride == 2 && a.Cin <= 32)) ? 16 : 32;
  const int nch = (int)cdiv(a.E, EC);
  const int64_t ntiles = (int64_t)a.B * tiles_img;
  const int64_t nitems = cdiv(ntiles, 8) * 8 * nch;
  JABD_REQUIRE(nitems < ((int64_t)1 << 31) && (int64_t)a.H * a.W * a.x_ps < ((int64_t)1 << 31),
               "expand_dw: problem too large for 32-bit item / pixel indexing");
  // the input is read through a buffer descriptor with 32-bit byte offsets:
  // a larger x would be truncated to zeros, so refuse it (the caller splits
  // the batch, engine.py)
  JABD_REQUIRE((int64_t)a.B * a.x_bs * 4 < ((int64_t)1 << 32),
               "expand_dw: input must be < 4 GiB (split the batch)");
  const int nw = xd_nw(a, EC);
  const int skc = xd_skc(a.Cin);
  hipStream_t st = as_stream(stream);
  const XdDivs dv{make_fastdiv((uint32_t)nch), make_fastdiv((uint32_t)tiles_img),
                  make_fastdiv((uint32_t)tiles_w)};
  JABD_REQUIRE((int64_t)a.B * a.x_bs * 4 < ((int64_t)1 << 32) - 16,
               "expand_dw: input must be < 4 GiB (buffer-descriptor offsets)");
  if (a.pw) {  // the previous block's project fused in front (one form)
    JABD_REQUIRE(a.pb && a.pg && a.pres && a.pg_bs >= a.Cin &&
                     (a.pact == ACT_NONE || a.pact == ACT_RELU || a.pact == ACT_HSWISH),
                 "expand_dw: bad fused-project arguments");
    JABD_REQUIRE(a.k == 3 && a.stride == 2 && EC == 32 && a.sy && a.Cin == 16 && a.Kc == 1 &&
                     a.x_ps == 16 && skc == 40 && nw == 4,
                 "expand_dw: the fused previous project takes the 3x3/s2 Cin-16 skip form only");
    // E <= 64: all expanded channels in one 8-wave workgroup (the project and
    // the input tiles once per tile instead of once per 32-channel chunk);
    // JABD_EXPDW_PRE_EC=32 keeps 32-channel chunks (A/B)
    static int pre_ec = -1;
    if (pre_ec < 0) {
      const char* e = getenv("JABD_EXPDW_PRE_EC");
      pre_ec = e && e[0] == '3' ? 32 : 64;
    }
    if (pre_ec == 64 && a.E <= 64) {
      const XdDivs dv1{make_fastdiv(1u), dv.tiles_img, dv.tiles_w};
      const int64_t n1 = cdiv(ntiles, 8) * 8;
#define XP_LAUNCH(ACT_)                                                                        \
  expdw1_kernel<3, 2, 8, 8, 64, ACT_, 1, true, 8, 40, 1, true><<<(unsigned)n1, 512, 0, st>>>( \
      a, dv1, (int)n1)
      if (a.act == ACT_RELU)
        XP_LAUNCH(ACT_RELU);
      else if (a.act == ACT_HSWISH)
        XP_LAUNCH(ACT_HSWISH);
      else
        XP_LAUNCH(ACT_NONE);
#undef XP_LAUNCH
      return check_launch("expand_dw (fused project, one chunk)");
    }
#define XP_LAUNCH(ACT_)                                                                       \
  expdw1_kernel<3, 2, 8, 8, 32, ACT_, 1, true, 4, 40, 1, true><<<(unsigned)nitems, 256, 0, st>>>( \
      a, dv, (int)nitems)
    if (a.act == ACT_RELU)
      XP_LAUNCH(ACT_RELU);
    else if (a.act == ACT_HSWISH)
      XP_LAUNCH(ACT_HSWISH);
    else
      XP_LAUNCH(ACT_NONE);
#undef XP_LAUNCH
    return check_launch("expand_dw (fused project)");
  }
  if (xw_form == 0 || xw_form == 4) {   // the chunk-pipelined form: opt-in (expdw3.hip)
    const int e = expdw3_dispatch(a, dv, tiles_img, xw_form == 4, st);
    if (e != JABD_EINVAL) return e;   // else: not covered, the forms below
  }
  if (x2_enabled() && !xw_enabled()) {
    const int e = expdw2_dispatch(a, dv, nitems, EC, nch, st);
    if (e != JABD_EINVAL) return e;   // else: no persistent instantiation, expdw1 below
  }
  if (xw_enabled()) {
#define XW_ACT(K_, S_, TH_, TW_, EC_, SK_)                                         \
  {                                                                              \
    if (a.act == ACT_RELU) return xw_launch<K_, S_, TH_, TW_, EC_, ACT_RELU, SK_>(a, dv, nitems, st);     \
    if (a.act == ACT_HSWISH) return xw_launch<K_, S_, TH_, TW_, EC_, ACT_HSWISH, SK_>(a, dv, nitems, st); \
    return xw_launch<K_, S_, TH_, TW_, EC_, ACT_NONE, SK_>(a, dv, nitems, st);                           \
  }
#define XW_CASE(K_, S_, TH_, TW_, EC_)                          \
  if (a.k == K_ && a.stride == S_ && EC == EC_) {               \
    if (S_ == 2 && a.sy) XW_ACT(K_, S_, TH_, TW_, EC_, true)    \
    XW_ACT(K_, S_, TH_, TW_, EC_, false)                        \
  }
    XW_CASE(3, 1, 14, 16, 16) XW_CASE(3, 1, 14, 16, 32)
    XW_CASE(5, 1, 16, 16, 16) XW_CASE(5, 1, 16, 16, 32)
    XW_CASE(3, 2, 8, 8, 16) XW_CASE(3, 2, 8, 8, 32)
    XW_CASE(5, 2, 8, 8, 16) XW_CASE(5, 2, 8, 8, 32)
#undef XW_CASE
#undef XW_ACT
  }
#define XD_LAUNCH(K_, S_, TH_, TW_, EC_, ACT_)                                                \
  do {                                                                                        \
    if (S_ == 2 && a.sy && nw == 8)                                                           \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, true, 8><<<(unsigned)nitems, 512, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (S_ == 2 && a.sy && skc == 40 && a.Kc == 2)                                       \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, true, 4, 40, 2><<<(unsigned)nitems, 256, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (S_ == 2 && a.sy && skc == 40)                                                    \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, true, 4, 40><<<(unsigned)nitems, 256, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (S_ == 2 && a.sy && skc == 112)                                                   \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, true, 4, 112><<<(unsigned)nitems, 256, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (S_ == 2 && a.sy)                                                                 \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, true><<<(unsigned)nitems, 256, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (nw == 8)                                                                         \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, false, 8><<<(unsigned)nitems, 512, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (a.Kc == 1)                                                                       \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1, false, 4, 160, 1><<<(unsigned)nitems, 256, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (a.Kc == 2)                                                                       \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 2, false, 4, 160, 2><<<(unsigned)nitems, 256, 0, st>>>( \
          a, dv, (int)nitems);                                                                \
    else if (xd_kp() == 1)                                                                    \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 1><<<(unsigned)nitems, 256, 0, st>>>(       \
          a, dv, (int)nitems);                                                                \
    else if (xd_kp() == 2)                                                                    \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 2><<<(unsigned)nitems, 256, 0, st>>>(       \
          a, dv, (int)nitems);                                                                \
    else                                                                                      \
      expdw1_kernel<K_, S_, TH_, TW_, EC_, ACT_, 3><<<(unsigned)nitems, 256, 0, st>>>(       \
          a, dv, (int)nitems);                                                                \
  } while (0)
#define XD_CASE(K_, S_, TH_, TW_, EC_)                                    \
  if (a.k == K_ && a.stride == S_ && EC == EC_) {                         \
    if (a.act == ACT_RELU)                                                \
      XD_LAUNCH(K_, S_, TH_, TW_, EC_, ACT_RELU);                         \
    else if (a.act == ACT_HSWISH)                                         \
      XD_LAUNCH(K_, S_, TH_, TW_, EC_, ACT_HSWISH);                       \
    else                                                                  \
      XD_LAUNCH(K_, S_, TH_, TW_, EC_, ACT_NONE);                         \
    return check_launch("expand_dw");                                     \
  }
  XD_CASE(3, 1, 14, 16, 16) XD_CASE(3, 1, 14, 16, 32)
  XD_CASE(5, 1, 16, 16, 16) XD_CASE(5, 1, 16, 16, 32)
  XD_CASE(3, 2, 8, 8, 16) XD_CASE(3, 2, 8, 8, 32)
  XD_CASE(5, 2, 8, 8, 16) XD_CASE(5, 2, 8, 8, 32)
#undef XD_CASE
#undef XD_LAUNCH
  set_error("expand_dw: no kernel for k=%d stride=%d", a.k, a.stride);
  return JABD_EINVAL;
}
