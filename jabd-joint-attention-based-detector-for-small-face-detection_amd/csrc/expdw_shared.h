// Shared device code of the fused expand + depthwise kernels (expdw.hip:
// expdw1 / strip / wave-specialised forms and the dispatcher; expdw2.hip:
// the persistent default form).
#pragma once
#include <stdlib.h>

#include "common.h"
#include "conv_args.h"

namespace jabd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Phase-skip mask for timing experiments only (tools/xd_variant.sh builds
// libraries with -DXD_SKIP=n; results are wrong): 1 expand MFMAs, 2 expanded-
// tile LDS writes, 4 depthwise phase, 8 ECA reduce, 16 input loads;
// expdw_ws_kernel: 32 expand-wave MFMAs, 64 depthwise-wave depthwise phase,
// 128 expand-wave input loads (out-of-range offsets: zeros, no traffic), 256
// expand-wave epilogue (activation + expanded-tile writes).
#ifndef XD_SKIP
#define XD_SKIP 0
#endif

// Phase trace for timing experiments only (tools/xd_variant.sh builds with
// -DXD_TRACE=1; jabd_xd_trace_set(buf) arms it): wave 0 of every workgroup
// stamps s_memtime (shader clock) at the phase boundaries and s_memrealtime
// (100 MHz, device-global) at entry and exit into buf[blockIdx.x][8].
#ifndef XD_TRACE
#define XD_TRACE 0
#endif
#if XD_TRACE
__device__ unsigned long long* xd_trace_buf;
#define XD_T(i)                                                                          \
  do {                                                                                   \
    if (xd_trace_buf && threadIdx.x == 0)                                                \
      xd_trace_buf[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();        \
  } while (0)
#define XD_RT(i)                                                                         \
  do {                                                                                   \
    if (xd_trace_buf && threadIdx.x == 0)                                                \
      xd_trace_buf[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
#else
#define XD_T(i) do { } while (0)
#define XD_RT(i) do { } while (0)
#endif

// Activation fixed at compile time (no per-element branch).  Hardswish
// multiplies by 1/6 instead of dividing (<= 1 ulp from x*relu6(x+3)/6; an
// IEEE divide is ~10 VALU instructions per element here).
template <int ACT>
__device__ __forceinline__ float xd_act(float v) {
  // one v_maximum_f32 (NaN-propagating, as torch.relu); fmaxf compiled to a
  // canonicalising v_max plus the v_max (2 VALU per element)
  if (ACT == ACT_RELU) return relu_f(v);
  if (ACT == ACT_HSWISH) return hswish_f(v);
  return v;
}

// xd_act on a float4 with the packed fp32 ALU where it applies: Hardswish as
// two v_pk_fma + four v_med3 + two v_pk_mul instead of 12 scalar VALU
// (the same IEEE operations per element as hswish_f: bit-identical).
template <int ACT>
__device__ __forceinline__ float4 xd_act4(float4 v) {
  if (ACT == ACT_HSWISH) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 k = {1.f / 6.f, 1.f / 6.f}, h = {0.5f, 0.5f};
    const f2 a = {v.x, v.y}, b = {v.z, v.w};
    f2 ta = __builtin_elementwise_fma(a, k, h), tb = __builtin_elementwise_fma(b, k, h);
    ta.x = __builtin_amdgcn_fmed3f(ta.x, 0.f, 1.f);
    ta.y = __builtin_amdgcn_fmed3f(ta.y, 0.f, 1.f);
    tb.x = __builtin_amdgcn_fmed3f(tb.x, 0.f, 1.f);
    tb.y = __builtin_amdgcn_fmed3f(tb.y, 0.f, 1.f);
    const f2 ra = a * ta, rb = b * tb;
    return make_float4(ra.x, ra.y, rb.x, rb.y);
  }
  return make_float4(xd_act<ACT>(v.x), xd_act<ACT>(v.y), xd_act<ACT>(v.z), xd_act<ACT>(v.w));
}

template <int K, int S, int TH, int TW, int EC>
struct XdCfg {
  static constexpr int PAD = K / 2;
  static constexpr int IH = (TH - 1) * S + K, IW = (TW - 1) * S + K;
  static constexpr int IPX = IH * IW;
  static constexpr int IPAD = (IPX + 15) / 16 * 16;
  static constexpr int XP = 16;      // staged input: 4 quad planes of IPAD float4
  static constexpr int EP = EC + 4;  // expanded-tile pitch (pixel-major form, expdw_ws_kernel)
  static constexpr int NPB = IPAD / 16, NNT = EC / 16, NBLK = NPB * NNT;
  static constexpr int LDS_X = IPAD * XP, LDS_E = IPAD * EP;
  // expdw1_kernel's expanded tile: channel-quad-major planes Eq[q][QP] of
  // float4, QP = IPX rounded up to odd (conflict-free without padding the
  // channels, see the LDS-layout note below); pad pixels are not stored
  static constexpr int QP = IPX | 1;
  static constexpr int LDS_EQ = (EC / 4) * QP * 4;
  static constexpr int LDS = LDS_X > LDS_EQ ? LDS_X : LDS_EQ;
  static constexpr int LDS_PM = LDS_X > LDS_E ? LDS_X : LDS_E;
  static constexpr int PW = S == 1 ? 4 : 2, NSTRIP = TW / PW, NC4 = EC / 4;
  static constexpr int ITEMS = TH * NSTRIP * NC4;
  static constexpr int SPAN = (PW - 1) * S + K;
  static_assert(TW % PW == 0 && 256 % NC4 == 0, "tile shape");
  static_assert(LDS * 4 <= 160 * 1024 && LDS_PM * 4 <= 160 * 1024, "LDS");
  static_assert((K * K + 1) * NC4 <= 256, "dw taps: one float4 per thread");
  static_assert(NC4 == 4 || NC4 == 8 || NC4 == 16, "dw_lane: 16-, 32- or 64-channel chunks");
};

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is also a
// workgroup-scope fence on global memory, so the compiler drains every
// outstanding global load (s_waitcnt vmcnt(0)) before it — which would
// retire an in-flight register prefetch at the first barrier after it is
// issued.  The LDS ordering this kernel needs is just lgkmcnt(0) + s_barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct XdItem {
  int b, t_in, oh0, ow0, ih0, iw0, c0;
};

// n / d for 0 <= n < 2^31 by multiply-high and shift (host-built divisor):
// the per-item decode would otherwise run three ~40-instruction integer
// divisions on the scalar unit.
// (FastDiv / make_fastdiv / fdiv: common.h)
struct XdDivs {
  FastDiv nch, tiles_img, tiles_w;
};

template <int K, int S, int TH, int TW, int EC>
__device__ __forceinline__ bool xd_item(const jabd_expdw_args& p, int i, const XdDivs& dv,
                                        int nitems, XdItem& it) {
  using C = XdCfg<K, S, TH, TW, EC>;
  if (i >= nitems) return false;
  const int xcd = i & 7;
  const int q = i >> 3;
  const int qn = fdiv(q, dv.nch);
  const int chunk = q - qn * (int)dv.nch.d;
  const int tile = qn * 8 + xcd;
  if (tile >= p.B * (int)dv.tiles_img.d) return false;
  it.b = fdiv(tile, dv.tiles_img);
  it.t_in = tile - it.b * (int)dv.tiles_img.d;
  const int ty = fdiv(it.t_in, dv.tiles_w), tx = it.t_in - ty * (int)dv.tiles_w.d;
  it.oh0 = ty * TH;
  it.ow0 = tx * TW;
  it.ih0 = it.oh0 * S - C::PAD;
  it.iw0 = it.ow0 * S - C::PAD;
  it.c0 = chunk * EC;
  return true;
}

// ---------------------------------------------------------------------------
// One workgroup per work item (tile x EC-chunk), no state carried across
// items (a persistent cross-item-prefetch form measured 5-30% slower on every
// layer: SGPR spills, loop-carried operand copies).  The item is decoded
// once; loads go through a buffer descriptor whose range check zeroes
// out-of-image pixels (no branch per load); the expanded tile is built with
// selects.  Latency hiding comes from the resident workgroups.
//
// LDS layouts (bank rules: MI355X_MICROARCH.md §LDS), all conflict-free:
//  * staged input, channel-quad-major Xs[q][px][4] (q = 4 channels of the
//    16-channel stage): an MFMA B read (pixel j, quad g per lane) hits slot
//    px mod 16 in every ds_read_b128 lane group, and the stage stores (8
//    contiguous lanes = 8 consecutive pixels of one quad) hit 8 distinct slots;
//  * expanded tile, channel-quad-major Eq[q][QP] float4 with QP odd: the
//    epilogue's ds_write_b128 8-lane groups are 8 consecutive pixels of one
//    quad (32 consecutive dwords); the depthwise reads assign lanes to
//    (strip, channel quad) so that each ds_read_b128 16-lane group reads 4
//    strips 4 pixels apart x 4 quads, banks 4 (q QP + px) mod 64 — distinct
//    because QP is odd.  No per-pixel channel padding (the pixel-major
//    [px][EC + 4] form of expdw_ws_kernel takes 12.5% more LDS), which is
//    what lets one more workgroup per CU fit on most layers (occupancy is
//    LDS-bound, and the kernel's time is the latency chain of its phases,
//    hidden only by the other resident workgroups).
// ---------------------------------------------------------------------------
// Depthwise-phase lane assignment.  The four ds_read_b128 lane groups are the
// lane quads q = (l >> 2) & 7 of even popcount {0,3,5,6} and odd popcount
// {1,2,4,7}, in each 32-lane half.  EC = 32 (8 channel quads): the parity
// picks channel quads 0-3 / 4-7 and q >> 1 the strip; EC = 16: the group
// picks the strip row.  Returns (channel quad, strip within the wave's slice).
template <int NC4>
__device__ __forceinline__ void dw_lane(int l, int& c4, int& sl) {
  // EC = 64 (16 channel quads): quad l & 15, strip l >> 4; a 16-lane read
  // group is one strip's 16 quads, banks 4 (q QP + px) mod 64 = 4q + const
  // (QP odd): distinct
  if (NC4 == 16) {
    c4 = l & 15;
    sl = l >> 4;
    return;
  }
  const int h = l >> 5, q = (l >> 2) & 7, par = __builtin_popcount(q) & 1, k = q >> 1;
  if (NC4 == 8) {
    c4 = (l & 3) + 4 * par;
    sl = 4 * h + k;
  } else {
    c4 = l & 3;
    sl = 4 * (2 * h + par) + k;
  }
}

struct XdTile {
  int th, tw;
};
XdTile xd_tile(int k, int s);
int xd_skc(int cin);
// expdw2.hip: launch the persistent form for this geometry (JABD_EINVAL when
// no instantiation covers it; the caller then uses expdw1_kernel)
int expdw2_dispatch(const jabd_expdw_args& a, const XdDivs& dv, int64_t nitems, int EC, int nch,
                    hipStream_t st);
// expdw3.hip: the chunk-pipelined persistent form for input-narrow layers
// (JABD_EINVAL when it does not cover the geometry; the caller falls back)
int expdw3_dispatch(const jabd_expdw_args& a, const XdDivs& dv, int tiles_img, bool forced,
                    hipStream_t st);

}  // namespace jabd
