// A1 fused MobileNetV3 block front half (eval), chunk-pipelined persistent
// form for the early, input-narrow layers (Cin <= 80, E <= 256: blocks 1-10
// of JABD-MNv3, nets/mobilenetV3.py:141-142): expand 1x1 + folded BN + act ->
// depthwise k x k + folded BN + act -> ECA pool partials (+ the stride-2
// block's dw3x3/s2 skip branch), the same contract as expdw1_kernel.
//
// Why another form.  expdw1_kernel runs one (tile, 16/32-channel chunk) per
// workgroup: every chunk re-stages the whole input tile, re-reads its weights
// and pays the item decode, and its phases (load -> MFMA -> LDS -> depthwise)
// run in step with the other resident workgroups, so the matrix and vector
// pipes never work at the same time (phase-skip builds).  Here:
//  * one workgroup per CU walks its tiles; expand weights, expand bias,
//    depthwise taps and bias go to LDS once per workgroup;
//  * a tile's input is loaded once for all its chunks: LDS-DMA (buffer_load
//    ... lds, no VGPRs held) copies it into a pixel-major LDS image in whole
//    1 KiB pieces (the tile's rows are contiguous in NHWC, so every piece is
//    a coalesced read); each wave then reads its MFMA B operands (lane =
//    pixel j of a 16-pixel block, channel quad g of a 16-channel stage) into
//    registers once for all chunks, and the NEXT tile's DMA is issued into
//    the freed image while this tile's chunks run (a whole tile of latency
//    cover);
//  * step i issues the expand MFMAs of chunk i and then runs the depthwise
//    phase of chunk i - 1 (VALU + LDS) while those MFMAs execute, then writes
//    chunk i's activated tile to the other LDS buffer: one LDS barrier per
//    step, the two pipes busy together inside every wave.
// The depthwise phase, ECA partials (part[b][tile][E], a fixed-order sum: per
// wave by shuffles, then over waves) and skip branch keep expdw1_kernel's
// tiles (xd_tile), so jabd_expand_dw_nblk and the partials' consumers are
// unchanged.  Each output is one fixed sequence of fp32 operations
// (accumulators start at the bias, k order of the packed weights, taps kh
// then kw): deterministic and independent of the batch it runs in.
#include "expdw_shared.h"

namespace jabd {

template <int K, int S, int TH, int TW, int CQ, int NW>
struct X3Cfg {
  using C = XdCfg<K, S, TH, TW, 16>;
  static constexpr int NS = (CQ + 3) / 4;  // 16-channel MFMA K stages
  static constexpr int PAD = K / 2, IH = C::IH, IW = C::IW, IPX = C::IPX, IPAD = C::IPAD;
  // pixel-major input image [IPX][CQ] float4, padded to whole 1 KiB DMA pieces
  static constexpr int XF = IPX * CQ, NDMA = (XF + 63) / 64, XPAD = NDMA * 64;
  static constexpr int NPB = C::NPB, QP = C::QP;
  static constexpr int T = 64 * NW;
  static constexpr int BPW = (NPB + NW - 1) / NW;  // 16-pixel MFMA blocks per wave
  // depthwise unit = (output row, strip of PW columns, channel quad)
  static constexpr int PW = S == 2 ? 1 : 2;
  static constexpr int NSTRIP = TW / PW;
  static constexpr int STRIPS = TH * NSTRIP;
  static constexpr int SPAN = (PW - 1) * S + K;
  static_assert(TW % PW == 0, "strip width");
};

// LDS carve (float4 units), shared by the host's size query and the kernel
struct X3Lds {
  int w, be, taps, bd, e, red, xs, sw, total;
};
__host__ __device__ inline X3Lds x3_lds(int K, int NS, int CQ, int NW, int nt, int QP, int XPAD, bool skip) {
  X3Lds l;
  l.w = 0;
  l.be = l.w + nt * NS * 64;
  l.taps = l.be + nt * 4;
  l.bd = l.taps + K * K * nt * 4;
  l.e = l.bd + nt * 4;
  l.red = l.e + 2 * 4 * QP;
  l.xs = l.red + 2 * NW * 4;
  l.sw = l.xs + XPAD;
  l.total = l.sw + (skip ? 10 * CQ : 0);
  return l;
}

// float4 store issued from inline asm (`s_nop 1` inside the string: the data
// registers must not be rewritten before the store has read them).  Inside
// the tile loop every store goes this way: with compiler-visible stores and
// no compiler-visible loads in the chunk loop, hipcc's wait-count pass
// flushes vmcnt in the loop preheader ("stores only" heuristic), which would
// drain the next tile's LDS-DMA right after it is issued.
__device__ __forceinline__ void x3_st4(float* ptr, float4 v) {
  const f32x4 d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(ptr), "v"(d) : "memory");
}

// LDS read through an address-space-3 pointer: where hipcc cannot infer the
// address space of a generic pointer it reads with flat loads, which also
// count on vmcnt (and then wait for the LDS-DMA and stores in flight)
__device__ __forceinline__ float4 x3_lds4(const float4* p) {
  const f32x4 v = *(const __attribute__((address_space(3))) f32x4*)p;
  return make_float4(v[0], v[1], v[2], v[3]);
}

struct X3Tile {
  int b, t_in, oh0, ow0, ih0, iw0;
  bool interior;
};

template <int K, int S, int TH, int TW, int CQ, int ACT, int NW>
__global__ __launch_bounds__(64 * NW, 1) void expdw3_kernel(const jabd_expdw_args p,
                                                          const XdDivs dv, int ntiles) {
  using C = X3Cfg<K, S, TH, TW, CQ, NW>;
  constexpr int BPW = C::BPW, NPB = C::NPB, IW = C::IW, QP = C::QP, NS = C::NS;
  extern __shared__ float4 x3_smem[];
  const int nt = p.Ntiles;  // expanded-channel chunks of 16
  const bool skip = p.sy != nullptr;
  // timing experiments only (tools/convbench.py XD_DBG; results wrong): 1 no
  // tile-start DMA wait, 2 no depthwise phase, 4 no MFMAs, 8 no DMA, 16 no
  // epilogue, 32 no per-step barrier
  const int dbg = p.reserved0;
  const X3Lds L = x3_lds(K, NS, CQ, NW, nt, QP, C::XPAD, skip);
  float4* Wl = x3_smem + L.w;     // [nt][NS][64] expand A fragments
  float4* Bl = x3_smem + L.be;    // [nt*4] expand bias quads
  float4* Tl = x3_smem + L.taps;  // [K*K][nt*4] depthwise taps
  float4* Dl = x3_smem + L.bd;    // [nt*4] depthwise bias quads
  float4* Eb = x3_smem + L.e;     // [2][4][QP] activated expanded chunk tiles
  float4* Rd = x3_smem + L.red;   // [2][NW][4] ECA per-wave quad sums
  float4* Xs = x3_smem + L.xs;    // [XPAD] input tile, pixel-major [IPX][CQ]
  float4* Sw = x3_smem + L.sw;    // [10][CQ] skip taps + bias
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, j = lane & 15, g = lane >> 4;
  const int Epad4 = nt * 4;
  {  // one-time staging of every small operand
    const float4* wsrc = reinterpret_cast<const float4*>(p.we);  // packed [Kc][Ntiles][64]
    for (int i = t; i < nt * NS * 64; i += C::T) {
      const int l = i & 63, q = i >> 6, c = q / NS, s = q - c * NS;
      Wl[i] = wsrc[((int64_t)s * nt + c) * 64 + l];
    }
    for (int i = t; i < Epad4; i += C::T) {
      const bool ok = 4 * i < p.E;
      Bl[i] = ok ? *reinterpret_cast<const float4*>(p.be + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
      Dl[i] = ok ? *reinterpret_cast<const float4*>(p.bd + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int i = t; i < K * K * Epad4; i += C::T) {
      const int tp = i / Epad4, q = i - tp * Epad4;
      Tl[i] = 4 * q < p.E ? *reinterpret_cast<const float4*>(p.wd + tp * p.E + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (skip)
      for (int i = t; i < 10 * CQ; i += C::T) {
        const int q = i / CQ, c4 = i - q * CQ;
        Sw[i] = *reinterpret_cast<const float4*>((q < 9 ? p.sw + q * p.Cin : p.sb) + 4 * c4);
      }
  }

  const int G = gridDim.x;
  const int nmine = ((int)blockIdx.x < ntiles) ? (ntiles - (int)blockIdx.x + G - 1) / G : 0;
  const int N = nmine * nt;  // (tile, chunk) steps of this workgroup
  auto decode = [&](int n) -> X3Tile {
    X3Tile d;
    const int tile = (int)blockIdx.x + n * G;
    d.b = fdiv(tile, dv.tiles_img);
    d.t_in = tile - d.b * (int)dv.tiles_img.d;
    const int ty = fdiv(d.t_in, dv.tiles_w), tx = d.t_in - ty * (int)dv.tiles_w.d;
    d.oh0 = ty * TH;
    d.ow0 = tx * TW;
    d.ih0 = d.oh0 * S - C::PAD;
    d.iw0 = d.ow0 * S - C::PAD;
    d.interior = d.ih0 >= 0 && d.iw0 >= 0 && d.ih0 + C::IH <= p.H && d.iw0 + C::IW <= p.W;
    return d;
  };
  // input tile -> Xs by LDS-DMA (buffer_load_dwordx4 ... lds) through a
  // buffer descriptor: an out-of-range offset 0xFFFFFFF0 (host: x < 4 GiB -
  // 16) lands zeros (pixels outside the image, the pad past IPX * CQ).  Piece
  // k (1 KiB: flat float4 64k..64k+63 of the [IPX][CQ] image) is issued by
  // wave k % NW.  Issued from inline asm so that hipcc's wait-count pass does
  // not see it: with the builtin, hipcc treats every later LDS read as a
  // possible reader of the DMA and drains it (vmcnt(0)) before the chunk
  // loop.  Completion is this kernel's own `s_waitcnt vmcnt(0)` + barrier at
  // the next tile start (an asm VMEM op can only make hipcc's own counted
  // waits conservative, never short).
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const uint64_t xb = reinterpret_cast<uint64_t>(p.x);
  const i32x4 xr = {(int)(uint32_t)xb, (int)(uint32_t)(xb >> 32),
                    (int)(uint32_t)((int64_t)p.B * p.x_bs * 4), 0x00020000};
  const uint32_t xs_lds = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) float4*)Xs);
  auto dma = [&](const X3Tile& d) {
    if (dbg & 8) return;
#pragma unroll
    for (int k0 = 0; k0 < C::NDMA; k0 += NW) {
      const int k = k0 + wave;
      if (k < C::NDMA) {
        const int f = 64 * k + lane;
        const int px = f / CQ, q = f - px * CQ;
        const int r = px / IW, c = px - r * IW;
        const int ih = d.ih0 + r, iw = d.iw0 + c;
        const bool ok = f < C::XF &&
                        (d.interior || ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W));
        const uint32_t off =
            ok ? (uint32_t)(d.b * p.x_bs + (ih * p.W + iw) * p.x_ps + 4 * q) * 4u : 0xFFFFFFF0u;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(xs_lds + 1024u * k);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %3\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(off), "s"(xr), "s"(dst)
            : "memory");
      }
    }
  };

  // depthwise lane map (EC = 16): channel quad c4, strip sl of the wave's 16
  int c4, sl;
  dw_lane<4>(lane, c4, sl);

  float4 bc[BPW][NS];
  f32x4 acc[BPW];
  X3Tile td{}, tf{};  // tiles of the depthwise item and of the finalized item
  int cd = 0, cf = 0;  // their chunks
  // one pipeline step: expand MFMAs of item i = (tile te, chunk ce) when
  // has_e, the depthwise phase of item i - 1, the ECA partials of item i - 2,
  // the skip branch of item i - 1's tile (first chunk), then item i's
  // activated tile into LDS buffer i & 1 and one LDS barrier
  auto step = [&](int i, bool has_e, int ce, const X3Tile& te) __attribute__((always_inline)) {
    // ---- expand MFMAs of chunk ce (accumulators start at the bias)
    if (has_e && !(dbg & 4)) {
      const float4 bi = Bl[ce * 4 + g];
#pragma unroll
      for (int u = 0; u < BPW; ++u) acc[u] = (f32x4){bi.x, bi.y, bi.z, bi.w};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const float4 a4 = Wl[(ce * NS + s) * 64 + lane];
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
          if (wave + NW * u < NPB) {
            const float4 bv = bc[u][s];
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, bv.x, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, bv.y, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, bv.z, acc[u], 0, 0, 0);
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, bv.w, acc[u], 0, 0, 0);
          }
        }
      }
    }
    // ---- depthwise phase of the previous step's chunk (overlaps the MFMAs)
    if (i >= 1 && !(dbg & 2)) {
      const float4* eb = Eb + ((i - 1) & 1) * 4 * QP + c4 * QP;
      const int ch = 16 * cd + 4 * c4;
      float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ch < p.E) {
        const float4 bias2 = Dl[cd * 4 + c4];
        float* yb = p.y + (int64_t)td.b * p.y_bs + ch;
#pragma unroll 1
        for (int pass = 0; pass * 16 * NW < C::STRIPS; ++pass) {
          const int strip = (pass * NW + wave) * 16 + sl;
          if (strip >= C::STRIPS) break;
          const int orow = strip / C::NSTRIP, st = strip - orow * C::NSTRIP;
          const int oh = td.oh0 + orow, owb = td.ow0 + st * C::PW;
          if (oh >= p.OH || owb >= p.OW) continue;
          float4 a2[C::PW];
#pragma unroll
          for (int o = 0; o < C::PW; ++o) a2[o] = bias2;
#pragma unroll 1
          for (int kh = 0; kh < K; ++kh) {
            const float4* rowp = eb + (orow * S + kh) * IW + st * C::PW * S;
            float4 row[C::SPAN];
#pragma unroll
            for (int c = 0; c < C::SPAN; ++c) row[c] = rowp[c];
            const float4* tp = Tl + (kh * K) * Epad4 + cd * 4 + c4;
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
              const float4 wv = tp[kw * Epad4];
#pragma unroll
              for (int o = 0; o < C::PW; ++o) a2[o] = fma4pk(row[o * S + kw], wv, a2[o]);
            }
          }
#pragma unroll
          for (int o = 0; o < C::PW; ++o) {
            if (owb + o >= p.OW) break;
            const float4 v = xd_act4<ACT>(a2[o]);
            x3_st4(yb + ((int64_t)oh * p.OW + owb + o) * p.y_ps, v);
            psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
          }
        }
      }
      if (p.part) {
        // lanes of one channel quad: xor 4, 8, 16, 32 (dw_lane<4>), fixed order
#pragma unroll
        for (int off = 4; off <= 32; off <<= 1) {
          psum.x += __shfl_xor(psum.x, off);
          psum.y += __shfl_xor(psum.y, off);
          psum.z += __shfl_xor(psum.z, off);
          psum.w += __shfl_xor(psum.w, off);
        }
        if (lane < 4) Rd[((i - 1) & 1) * NW * 4 + wave * 4 + lane] = psum;
      }
    }
    // ---- ECA partials of step i - 2 (its per-wave sums passed a barrier)
    if (p.part && i >= 2 && t < 4 && 16 * cf + 4 * t < p.E) {
      const float4* rb = Rd + (i & 1) * NW * 4;  // (i - 2) & 1
      float4 v[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) v[w] = rb[w * 4 + t];
#pragma unroll
      for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
        for (int w = 0; w < h; ++w) {
          v[w].x += v[w + h].x; v[w].y += v[w + h].y; v[w].z += v[w + h].z; v[w].w += v[w + h].w;
        }
      x3_st4(p.part + ((int64_t)tf.b * (int)dv.tiles_img.d + tf.t_in) * p.E + 16 * cf + 4 * t, v[0]);
    }
    // ---- activated expanded chunk into LDS buffer i & 1 (zero outside the image)
    if (has_e && !(dbg & 16)) {
      float4* eb = Eb + (i & 1) * 4 * QP + g * QP;
#pragma unroll
      for (int u = 0; u < BPW; ++u) {
        const int pb = wave + NW * u;
        if (pb >= NPB) continue;
        const int px = pb * 16 + j;
        float4 o = xd_act4<ACT>(make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]));
        if (!te.interior) {
          const int r = px / IW, c = px - r * IW;
          const int ih = te.ih0 + r, iw = te.iw0 + c;
          const bool in = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
          o.x = in ? o.x : 0.f; o.y = in ? o.y : 0.f; o.z = in ? o.z : 0.f; o.w = in ? o.w : 0.f;
        }
        if (px < C::IPX) eb[px] = o;
      }
    }
    if (!(dbg & 32)) lds_barrier();
    tf = td;
    cf = cd;
    if (has_e) {
      td = te;
      cd = ce;
    }
  };


  // tiles in order: Xs holds tile n (its DMA was issued during tile n - 1);
  // the waves take their B operands and the skip branch from it, and after
  // one barrier the DMA of tile n + 1 overwrites it while tile n's chunks run
  X3Tile tn{};
  if (nmine > 0) {
    tn = decode(0);
    dma(tn);
  }
  int i = 0;
#pragma unroll 1
  for (int ne = 0; ne <= nmine; ++ne) {
    // ne == nmine: only the pipeline's last step (depthwise of the last item)
    const bool tile = ne < nmine;
    const X3Tile te = tn;
    if (tile) {
    if (!(dbg & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces
    lds_barrier();                                     // everyone's
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
      const int pb = wave + NW * u;
      const int px = pb * 16 + j;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bool ok = pb < NPB && px < C::IPX && 4 * s + g < CQ;
        bc[u][s] = ok ? x3_lds4(Xs + px * CQ + 4 * s + g) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (S == 2 && skip) {  // the block's dw3x3/s2 skip branch on the same input tile
      for (int u = t; u < TH * TW * CQ; u += C::T) {
        const int sq = u / (TH * TW), op = u - sq * (TH * TW);
        const int orow = op / TW, ocol = op - orow * TW;
        const int oh = te.oh0 + orow, ow = te.ow0 + ocol;
        if (oh >= p.OH || ow >= p.OW) continue;
        float4 v = x3_lds4(Sw + 9 * CQ + sq);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int px = (2 * orow + kh + C::PAD - 1) * IW + 2 * ocol + kw + C::PAD - 1;
            v = fma4pk(x3_lds4(Xs + px * CQ + sq), x3_lds4(Sw + (kh * 3 + kw) * CQ + sq), v);
          }
        x3_st4(p.sy + (int64_t)te.b * p.sy_bs + ((int64_t)oh * p.OW + ow) * p.sy_ps + 4 * sq, v);
      }
    }
    lds_barrier();  // Xs free
    if (ne + 1 < nmine) {
      tn = decode(ne + 1);
      dma(tn);
    }
    }
    const int nc = tile ? nt : (N > 0 ? 1 : 0);
#pragma unroll 1
    for (int ce = 0; ce < nc; ++ce, ++i) step(i, tile, ce, te);
  }
  // ECA partials of the last step
  if (p.part && N >= 1 && t < 4 && 16 * cf + 4 * t < p.E) {
    const float4* rb = Rd + ((N - 1) & 1) * NW * 4;
    float4 v[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) v[w] = rb[w * 4 + t];
#pragma unroll
    for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
      for (int w = 0; w < h; ++w) {
        v[w].x += v[w + h].x; v[w].y += v[w + h].y; v[w].z += v[w + h].z; v[w].w += v[w + h].w;
      }
    *reinterpret_cast<float4*>(p.part + ((int64_t)tf.b * (int)dv.tiles_img.d + tf.t_in) * p.E +
                               16 * cf + 4 * t) = v[0];
  }
}

template <int K, int S, int TH, int TW, int CQ, int ACT, int NW>
static int x3_launch(const jabd_expdw_args& a, const XdDivs& dv, int ntiles, hipStream_t st) {
  using C = X3Cfg<K, S, TH, TW, CQ, NW>;
  auto kern = expdw3_kernel<K, S, TH, TW, CQ, ACT, NW>;
  const X3Lds L = x3_lds(K, C::NS, CQ, NW, a.Ntiles, C::QP, C::XPAD, a.sy != nullptr);
  const int bytes = L.total * 16;
  if (bytes > 160 * 1024) return JABD_EINVAL;
  static int ncu = 0;
  static bool attr = false;
  if (!ncu) {
    int dev = 0;
    JABD_HIP(hipGetDevice(&dev));
    JABD_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (!attr) {
    JABD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024));
    attr = true;
  }
  const int grid = ntiles < ncu ? ntiles : ncu;
  kern<<<grid, C::T, bytes, st>>>(a, dv, ntiles);
  return check_launch("expand_dw3");
}

// Off by default (JABD_EXPDW3=1 or jabd_expand_dw_select(4) selects it): it
// measured 1.2-1.9x SLOWER than expdw1_kernel on every covered layer
// (tools/convbench.py --set xd).  Phase-skip builds
// (tools/xd3_dbg.sh) show its expand-MFMA and depthwise phases add up even
// inside one wave, and tools/micro/mfma_valu_overlap.hip shows why: on gfx950
// the fp32 MFMA and fp32 VALU work of a SIMD do not execute concurrently
// (same wave or different waves: the time is the sum), so issuing the next
// chunk's MFMAs ahead of the depthwise VALU buys nothing, and one barrier-
// synchronised workgroup per CU exposes every step's latency chain.
static bool x3_enabled(bool forced) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("JABD_EXPDW3");
    on = e && e[0] == '1' ? 1 : 0;
  }
  return forced || on == 1;
}

int expdw3_dispatch(const jabd_expdw_args& a, const XdDivs& dv, int tiles_img, bool forced,
                    hipStream_t st) {
  if (!x3_enabled(forced) || a.Ntiles > 16 || a.Cin > 80 || a.x_ps != a.Cin) return JABD_EINVAL;
  const int64_t nt64 = (int64_t)a.B * tiles_img;
  if (nt64 >= ((int64_t)1 << 31)) return JABD_EINVAL;
  const int ntiles = (int)nt64;
  const int cq = a.Cin / 4;
#define X3_ACT(K_, S_, TH_, TW_, CQ_)                                                     \
  if (a.k == K_ && a.stride == S_ && cq == CQ_) {                                         \
    if (a.act == ACT_RELU) return x3_launch<K_, S_, TH_, TW_, CQ_, ACT_RELU, 8>(a, dv, ntiles, st);     \
    if (a.act == ACT_HSWISH) return x3_launch<K_, S_, TH_, TW_, CQ_, ACT_HSWISH, 8>(a, dv, ntiles, st); \
    return x3_launch<K_, S_, TH_, TW_, CQ_, ACT_NONE, 8>(a, dv, ntiles, st);                            \
  }
  // JABD-MNv3 blocks 1-7 (Cin, k, stride): (16,3,1) (16,3,2) (24,3,1) (24,5,2)
  // (40,5,1) x2 (40,3,2)
  X3_ACT(3, 1, 14, 16, 4) X3_ACT(3, 1, 14, 16, 6)
  X3_ACT(5, 1, 16, 16, 10)
  X3_ACT(3, 2, 8, 8, 4) X3_ACT(3, 2, 8, 8, 10)
  X3_ACT(5, 2, 8, 8, 6)
#undef X3_ACT
  return JABD_EINVAL;
}

}  // namespace jabd
