// A1 fused MobileNetV3 block front half (nets/mobilenetV3.py:141-142),
// persistent form, bit-identical to expdw.hip's one-item-per-workgroup
// expdw1_kernel (the default; this one is selected by JABD_EXPDW2=1 or
// jabd_expand_dw_select(3), see expdw.hip x2_enabled for why it is off).
#include "expdw_shared.h"

namespace jabd {

// ---------------------------------------------------------------------------
// Persistent form (A/B; expdw1_kernel is the default): expdw1's phases and
// arithmetic (bit-identical results), restructured for instruction count.
// SQ counters of expdw1 showed the kernel is VALU-issue-bound, not MFMA- or
// memory-bound: ~550 VALU per wave per 8x8 stride-2 item against 38 MFMAs
// (58% VALU busy, 32% MFMA busy), most of them per-item setup — item
// decode, stage-load addresses with 32x32-bit multiplies and bounds,
// bias / tap loads and their index math, canonicalising ReLU maxima.  Here:
//  * a workgroup walks items blockIdx.x + k G with G a multiple of 8 nch, so
//    its channel chunk and XCD never change: expand bias, depthwise taps
//    (LDS) and bias, the skip-branch taps and (Kc <= 2) the expand weights
//    are loaded once per workgroup;
//  * every per-thread address (stage slots relative to the tile origin, LDS
//    stage / MFMA / epilogue / depthwise offsets, output offsets relative to
//    the tile origin) is computed once; an interior item only moves two
//    scalar bases (a buffer descriptor at the input tile origin, the output
//    tile origin); border items take the per-pixel-bounds path;
//  * every barrier is LDS-only (no drain of outstanding loads and stores);
//  * ReLU is one v_maximum (NaN-propagating, as torch.relu), the ECA lane
//    reduction uses swizzles instead of bpermute address math.
// ---------------------------------------------------------------------------
template <int ACT>
__device__ __forceinline__ float xd2_act(float v) {
  if (ACT == ACT_RELU) return relu_f(v);
  if (ACT == ACT_HSWISH) return hswish_f(v);
  return v;
}

// psum lanes holding the same channel quad (dw_lane) summed in expdw1's order
template <int NC4>
__device__ __forceinline__ float xd2_lane_sum(float v) {
  if (NC4 == 8) {
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (12 << 10) | 0x1f));
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (20 << 10) | 0x1f));
  } else {
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (4 << 10) | 0x1f));
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (8 << 10) | 0x1f));
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (16 << 10) | 0x1f));
  }
  return v + __shfl_xor(v, 32);
}

struct Xd2Item {
  int b, t_in, oh0, ow0, ih0, iw0;
  bool interior, out_full;
};

template <int K, int S, int TH, int TW, int EC>
__device__ __forceinline__ bool xd2_item(const jabd_expdw_args& p, int i, const XdDivs& dv,
                                         Xd2Item& it) {
  using C = XdCfg<K, S, TH, TW, EC>;
  const int xcd = i & 7, q = i >> 3;
  const int qn = fdiv(q, dv.nch);
  const int tile = qn * 8 + xcd;
  if (tile >= p.B * (int)dv.tiles_img.d) return false;
  it.b = fdiv(tile, dv.tiles_img);
  it.t_in = tile - it.b * (int)dv.tiles_img.d;
  const int ty = fdiv(it.t_in, dv.tiles_w), tx = it.t_in - ty * (int)dv.tiles_w.d;
  it.oh0 = ty * TH;
  it.ow0 = tx * TW;
  it.ih0 = it.oh0 * S - C::PAD;
  it.iw0 = it.ow0 * S - C::PAD;
  it.interior = it.ih0 >= 0 && it.iw0 >= 0 && it.ih0 + C::IH <= p.H && it.iw0 + C::IW <= p.W;
  it.out_full = it.oh0 + TH <= p.OH && it.ow0 + TW <= p.OW;
  return true;
}

// workgroups per CU the LDS allows (capped at 4: 128 VGPRs per lane)
template <int K, int S, int TH, int TW, int EC, bool SKIP, int SKC>
struct Xd2Occ {
  using C = XdCfg<K, S, TH, TW, EC>;
  static constexpr int BYTES = C::LDS * 4 + K * K * C::NC4 * 16 + (SKIP ? 10 * SKC / 4 * 16 : 16);
  static constexpr int LDSOCC = 163840 / BYTES;
  static constexpr int value = LDSOCC < 1 ? 1 : (LDSOCC > 4 ? 4 : LDSOCC);
};

template <int K, int S, int TH, int TW, int EC, int ACT, bool SKIP, int SKC, int KCR>
__global__ __launch_bounds__(256, (Xd2Occ<K, S, TH, TW, EC, SKIP, SKC>::value)) void expdw2_kernel(
    const jabd_expdw_args p, const XdDivs dv, int nitems, int G) {
  using C = XdCfg<K, S, TH, TW, EC>;
  constexpr int NW = 4, T = 256;
  constexpr int NPF = (C::IPAD * 4 + T - 1) / T;
  constexpr int BPW = (C::NBLK + NW - 1) / NW;
  constexpr int NWD = K * K * C::NC4;
  constexpr int SPW = 64 / C::NC4;                     // depthwise strips per wave per pass
  constexpr int NPASS = (TH * C::NSTRIP + NW * SPW - 1) / (NW * SPW);
  static_assert(NW % C::NNT == 0, "waves split evenly over the 16-channel tiles");
  __shared__ __attribute__((aligned(16))) float lds[C::LDS];
  __shared__ float4 wsh[K * K][C::NC4];
  __shared__ float4 sws[SKIP ? 10 : 1][SKIP ? SKC / 4 : 1];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, j = lane & 15, g = lane >> 4;
  const int qb = blockIdx.x >> 3;
  const int chunk = qb - fdiv(qb, dv.nch) * (int)dv.nch.d;   // fixed: G % (8 nch) == 0
  const int c0 = chunk * EC;
  const bool skip = SKIP && c0 == 0;
  // ---- per-workgroup constants
  const int ntw = wave % C::NNT;
  const int nt = c0 / 16 + ntw;
  const bool ntv = nt < p.Ntiles;
  const int ntc = ntv ? nt : 0;
  const f32x4* wpk = reinterpret_cast<const f32x4*>(p.we);
  const int chb = c0 + 16 * ntw + 4 * g;
  const bool chok = chb < p.E;
  const float4 pbi = *reinterpret_cast<const float4*>(p.be + (chok ? chb : 0));
  const f32x4 bias4 = (f32x4){pbi.x, pbi.y, pbi.z, pbi.w};
  f32x4 areg[KCR > 0 ? KCR : 1];
#pragma unroll
  for (int kc = 0; kc < KCR; ++kc) {
    areg[kc] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (ntv && kc < p.Kc) areg[kc] = wpk[(kc * p.Ntiles + ntc) * 64 + lane];
  }
  if (t < NWD) {
    const int tp = t / C::NC4, cc = c0 + 4 * (t - tp * C::NC4);
    const float4 w = *reinterpret_cast<const float4*>(p.wd + tp * p.E + (cc < p.E ? cc : 0));
    wsh[tp][t - tp * C::NC4] = cc < p.E ? w : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (skip) {
    for (int i = t; i < 10 * (p.Cin >> 2); i += T) {
      const int q = i / (p.Cin >> 2), c4 = i - q * (p.Cin >> 2);
      sws[q][c4] = *reinterpret_cast<const float4*>((q < 9 ? p.sw + q * p.Cin : p.sb) + 4 * c4);
    }
  }
  int c4, sl;
  dw_lane<C::NC4>(lane, c4, sl);
  const int chl = 4 * c4;
  const bool chv = c0 + chl < p.E;
  const float4 bias2 = *reinterpret_cast<const float4*>(p.bd + (chv ? c0 + chl : 0));
  // stage slot u of this thread: pixel u*64 + spx0 of the tile, channel quad cq/4
  const int cq = ((t >> 4) & 3) * 4;
  const int spx0 = (t >> 6) * 16 + (t & 15);
  // interior items: byte offset of each slot from the input tile origin
  // (0xFFFFF000: pad pixel or channel past Cin -> out of range, reads zeros)
  uint32_t rel[NPF];
#pragma unroll
  for (int u = 0; u < NPF; ++u) {
    const int px = u * 64 + spx0;
    const int r = px / C::IW, c = px - r * C::IW;
    rel[u] = px < C::IPX ? (__umul24(__umul24(r, p.W) + c, p.x_ps) + cq) * 4u : 0xFFFFF000u;
  }
  const uint32_t x_bytes = (uint32_t)((int64_t)p.B * p.x_bs * 4);
  float4 pf[NPF];
  auto load_stage = [&](const Xd2Item& it, int kc) {
    const int cofs = 16 * kc + cq;
    const bool cok = cofs < p.Cin;
    if (it.interior) {
      const int64_t tb = ((int64_t)it.b * p.x_bs + ((int64_t)it.ih0 * p.W + it.iw0) * p.x_ps) * 4;
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char*>(reinterpret_cast<const char*>(p.x) + tb), (short)0,
          (int)(x_bytes - (uint32_t)tb), 0x00020000);
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const uint32_t off = cok ? rel[u] + 64u * kc : 0xFFFFF000u;
        pf[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      }
    } else {
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(p.x), (short)0, (int)x_bytes, 0x00020000);
      const uint32_t base = (uint32_t)(it.b * p.x_bs + cofs);
      // border items are rare: an opaque pixel base keeps the compiler from
      // hoisting (and holding) this path's per-slot coordinates
      int sp = spx0;
      asm volatile("" : "+v"(sp));
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int px = u * 64 + sp;
        const int r = px / C::IW, c = px - r * C::IW;
        const int ih = it.ih0 + r, iw = it.iw0 + c;
        const bool ok = px < C::IPX && cok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        const uint32_t off = ok ? (base + (uint32_t)((ih * p.W + iw) * p.x_ps)) * 4u : 0xFFFFF000u;
        pf[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      }
    }
  };
  Xd2Item it;
  int i = blockIdx.x;
  while (i < nitems && !xd2_item<K, S, TH, TW, EC>(p, i, dv, it)) i += G;
  if (i >= nitems) return;
  load_stage(it, 0);
  lds_barrier();   // wsh / sws written
  float* part_c = p.part ? p.part + c0 : nullptr;
  for (;;) {
    // next valid item of this workgroup (its first stage is prefetched)
    Xd2Item nx;
    int ni = i + G;
    while (ni < nitems && !xd2_item<K, S, TH, TW, EC>(p, ni, dv, nx)) ni += G;
    const bool has_next = ni < nitems;
    f32x4 acc[BPW];
#pragma unroll
    for (int u = 0; u < BPW; ++u) acc[u] = bias4;
    for (int kc = 0; kc < p.Kc; ++kc) {
      f32x4 a;
      if (KCR > 0) {
        a = areg[0];
#pragma unroll
        for (int r = 1; r < KCR; ++r)
          if (kc == r) a = areg[r];
      } else {
        a = wpk[(kc * p.Ntiles + ntc) * 64 + lane];
        if (!ntv) a = (f32x4){0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+v"(a));
      }
#pragma unroll
      for (int u = 0; u < NPF; ++u)
        if (u * 64 + spx0 < C::IPAD)
          *reinterpret_cast<float4*>(lds + (cq / 4 * C::IPAD + u * 64 + spx0) * 4) = pf[u];
      lds_barrier();
      if (kc + 1 < p.Kc) load_stage(it, kc + 1);
      const int sc = 16 * kc + 4 * (t >> 6);
      if (skip && sc < p.Cin) {
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
      if (ntv) {
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
    // expanded tile: act, zero outside the image / on padded channels
    const int q = 4 * ntw + g;
    if (it.interior && c0 + EC <= p.E) {
#pragma unroll
      for (int u = 0; u < BPW; ++u) {
        const int blk = wave + NW * u;
        if (blk < C::NBLK) {
          const int pb = blk / C::NNT;
          const int px = pb * 16 + j;
          float4 o;
          o.x = xd2_act<ACT>(acc[u][0]);
          o.y = xd2_act<ACT>(acc[u][1]);
          o.z = xd2_act<ACT>(acc[u][2]);
          o.w = xd2_act<ACT>(acc[u][3]);
          if (pb * 16 + 16 <= C::IPX || px < C::IPX)
            *reinterpret_cast<float4*>(lds + (q * C::QP + px) * 4) = o;
        }
      }
    } else {
      int jj = j;   // opaque: not hoisted out of the item loop (rare path)
      asm volatile("" : "+v"(jj));
#pragma unroll
      for (int u = 0; u < BPW; ++u) {
        const int blk = wave + NW * u;
        if (blk < C::NBLK) {
          const int pb = blk / C::NNT;
          const int px = pb * 16 + jj;
          const int r = px / C::IW, c = px - r * C::IW;
          const int ih = it.ih0 + r, iw = it.iw0 + c;
          const bool ok = chok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
          float4 o;
          o.x = ok ? xd2_act<ACT>(acc[u][0]) : 0.f;
          o.y = ok ? xd2_act<ACT>(acc[u][1]) : 0.f;
          o.z = ok ? xd2_act<ACT>(acc[u][2]) : 0.f;
          o.w = ok ? xd2_act<ACT>(acc[u][3]) : 0.f;
          if (px < C::IPX) *reinterpret_cast<float4*>(lds + (q * C::QP + px) * 4) = o;
        }
      }
    }
    lds_barrier();
    // depthwise phase
    float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
    if (chv) {
      float* yb = p.y + (int64_t)it.b * p.y_bs + ((int64_t)it.oh0 * p.OW + it.ow0) * p.y_ps;
      const int rlim = p.OH - it.oh0, clim = p.OW - it.ow0;
#pragma unroll 1
      for (int ps = 0; ps < NPASS; ++ps) {
        // this pass's strip: output row orow, columns dcol .. dcol + PW - 1
        const int strip = (ps * NW + wave) * SPW + sl;
        const int orow = strip / C::NSTRIP, dcol = (strip - orow * C::NSTRIP) * C::PW;
        if (strip >= TH * C::NSTRIP || orow >= rlim || dcol >= clim) continue;
        const int dwl = c4 * C::QP + orow * S * C::IW + dcol * S;
        const int dwo = (__umul24(orow, p.OW) + dcol) * p.y_ps + c0 + chl;
        float4 a2[C::PW];
#pragma unroll
        for (int o = 0; o < C::PW; ++o) a2[o] = bias2;
#pragma unroll 1
        for (int kh = 0; kh < K; ++kh) {
          const float* rowp = lds + (dwl + kh * C::IW) * 4;
          float4 row[C::SPAN];
#pragma unroll
          for (int c = 0; c < C::SPAN; ++c) row[c] = *reinterpret_cast<const float4*>(rowp + c * 4);
          float4 wk[K];
#pragma unroll
          for (int kw = 0; kw < K; ++kw) wk[kw] = wsh[kh * K + kw][c4];
#pragma unroll
          for (int o = 0; o < C::PW; ++o)
#pragma unroll
            for (int kw = 0; kw < K; ++kw) a2[o] = fma4pk(row[o * S + kw], wk[kw], a2[o]);
        }
#pragma unroll
        for (int o = 0; o < C::PW; ++o) {
          if (!it.out_full && dcol + o >= clim) break;
          float4 v;
          v.x = xd2_act<ACT>(a2[o].x);
          v.y = xd2_act<ACT>(a2[o].y);
          v.z = xd2_act<ACT>(a2[o].z);
          v.w = xd2_act<ACT>(a2[o].w);
          *reinterpret_cast<float4*>(yb + dwo + o * p.y_ps) = v;
          psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
        }
      }
    }
    if (part_c) {
      psum.x = xd2_lane_sum<C::NC4>(psum.x);
      psum.y = xd2_lane_sum<C::NC4>(psum.y);
      psum.z = xd2_lane_sum<C::NC4>(psum.z);
      psum.w = xd2_lane_sum<C::NC4>(psum.w);
      float4* red = reinterpret_cast<float4*>(lds);
      lds_barrier();   // every depthwise read of the tile is done
      if (lane < C::NC4) red[wave * C::NC4 + lane] = psum;
      lds_barrier();
      if (t < C::NC4 && c0 + 4 * t < p.E) {
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
        *reinterpret_cast<float4*>(part_c + ((int64_t)it.b * (int)dv.tiles_img.d + it.t_in) * p.E +
                                   4 * t) = v[0];
      }
    }
    // the next item's first stage: issued after this item's output stores, so
    // waiting for it does not also wait for them (one in-order VMEM counter)
    if (has_next) load_stage(nx, 0);
    lds_barrier();   // the next item's stage overwrites the tile / reduction buffer
    if (!has_next) break;
    i = ni;
    it = nx;
  }
}


template <int K, int S, int TH, int TW, int EC, int ACT, bool SKIP, int SKC, int KCR>
static int xd2_launch(const jabd_expdw_args& a, const XdDivs& dv, int64_t nitems, int nch,
                      hipStream_t st) {
  auto kern = expdw2_kernel<K, S, TH, TW, EC, ACT, SKIP, SKC, KCR>;
  static int occ = -1, ncu = 0;
  if (occ < 0) {
    int dev = 0, o = 0;
    JABD_HIP(hipGetDevice(&dev));
    JABD_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    JABD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, 256, 0));
    occ = o < 1 ? 1 : o;
  }
  // G: a multiple of 8 nch (fixed channel chunk and XCD per workgroup), at
  // most the resident workgroups, the items spread evenly over it
  const int64_t unit = 8ll * nch;
  int64_t gmax = (int64_t)ncu * occ / unit * unit;
  if (gmax < unit) gmax = unit;
  const int64_t per = cdiv(nitems, gmax);
  int64_t G = cdiv(cdiv(nitems, per), unit) * unit;
  if (G > nitems) G = nitems;
  kern<<<(unsigned)G, 256, 0, st>>>(a, dv, (int)nitems, (int)G);
  return check_launch("expand_dw2");
}

int expdw2_dispatch(const jabd_expdw_args& a, const XdDivs& dv, int64_t nitems, int EC, int nch,
                    hipStream_t st) {
  JABD_REQUIRE((int64_t)a.B * a.x_bs * 4 <= 0xFFFFF000ll - 4096,
               "expand_dw: input must be < 4 GiB - 8 KiB (split the batch)");
  const bool sk = a.sy != nullptr;
  const int skc = xd_skc(a.Cin);
#define XD2_GO(K_, S_, TH_, TW_, EC_, ACT_)                                                     \
  do {                                                                                          \
    if (S_ == 2 && sk && skc == 40)                                                             \
      return xd2_launch<K_, S_, TH_, TW_, EC_, ACT_, true, 40, 0>(a, dv, nitems, nch, st);      \
    if (S_ == 2 && sk && skc == 112)                                                            \
      return xd2_launch<K_, S_, TH_, TW_, EC_, ACT_, true, 112, 0>(a, dv, nitems, nch, st);     \
    if (sk) break;                                                                              \
    return xd2_launch<K_, S_, TH_, TW_, EC_, ACT_, false, 16, 0>(a, dv, nitems, nch, st);       \
  } while (0)
#define XD2_CASE(K_, S_, TH_, TW_, EC_)                             \
  if (a.k == K_ && a.stride == S_ && EC == EC_) {                   \
    if (a.act == ACT_RELU) XD2_GO(K_, S_, TH_, TW_, EC_, ACT_RELU);     \
    else if (a.act == ACT_HSWISH) XD2_GO(K_, S_, TH_, TW_, EC_, ACT_HSWISH); \
    else XD2_GO(K_, S_, TH_, TW_, EC_, ACT_NONE);                   \
  }
  XD2_CASE(3, 1, 14, 16, 16) XD2_CASE(3, 1, 14, 16, 32)
  XD2_CASE(5, 1, 16, 16, 16) XD2_CASE(5, 1, 16, 16, 32)
  XD2_CASE(3, 2, 8, 8, 16) XD2_CASE(3, 2, 8, 8, 32)
  XD2_CASE(5, 2, 8, 8, 16) XD2_CASE(5, 2, 8, 8, 32)
#undef XD2_CASE
#undef XD2_GO
  return JABD_EINVAL;
}

}  // namespace jabd
