// A1/A4 short-K, narrow-N 1x1 convolutions as a streaming GEMM: the
// MobileNetV3 project convs at 512^2..128^2 (K 16-120, Cout 16-40), the FPN
// laterals (K 40-80, Cout 40) and the training-forward twins of those layers
// (nets/mobilenetV3.py:146-150 conv3 + bn3 + skip, nets/retinaface_r.py FPN
// output1..3).
//
// These layers are HBM-bound (2 K N / 4 (K + N) = 6-20 FLOP/B, left of the
// 19.7 FLOP/B ridge), and the tile kernel (conv1x1_kernel) holds one or two
// 16-channel K stages in flight per wave: ~1-2 KiB per wave, too little to
// cover HBM latency at the occupancy it gets, and every wave re-reads the
// whole packed weight matrix through L1 for its 16 pixels.  Here:
//  * a persistent workgroup copies the packed weights (Kc x Ntiles KiB) and
//    the per-image ECA gates once into LDS; the four waves then walk 16-pixel
//    blocks (block = wave id + k * waves in the grid, so neighbouring waves
//    stream neighbouring pixels);
//  * every K stage of the NEXT block is issued while the current block runs
//    its MFMAs: stage kc's register is refilled as soon as it has been
//    consumed, so a wave keeps the whole K extent (Kc KiB) of loads in
//    flight and the in-order vmcnt needs no per-stage drain;
//  * B fragments come from LDS (ds_read_b128, one per 4 MFMAs), the ECA gate
//    is applied to A on consumption, bias + residual + activation in
//    registers, NHWC float4 stores straight from the accumulators (four lane
//    groups cover 64 contiguous bytes of a pixel row).
// Operand mapping and packing are those of conv.hip (Wp[kc][nt][lane] =
// float4{W[16kc+4g+e][16nt+j]}); Ntiles == TN (one workgroup covers every
// output channel, so A is read from HBM exactly once).
#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "conv_args.h"

namespace jabd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float cs_act(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return relu_f(v);
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: return hswish_f(v);
    case ACT_HSIGMOID: return hsigmoid_f(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// KC >= p.Kc stages are compiled; stages past p.Kc issue a load of the last
// real stage (an L1 hit, keeps the load sequence unpredicated) and skip their
// MFMAs (wave-uniform branch).
// Workgroup: 4 waves; 8 when the weights exceed 24 KiB (Kc x Ntiles > 24: the
// Cout = 80 layers), so the one workgroup that fits a CU's LDS still gives
// each SIMD two waves.
template <int TN, int KC>
struct CsCfg {
  static constexpr int NW = KC * TN > 24 ? 8 : 4;
};

// ST: also the BatchNorm statistics of the output for the training forward
// (MNv3 Block_eca conv1 -> bn1; no gate, residual or second source): per
// workgroup the shifted sums sum(y - sh), sum((y - sh)^2) over its blocks,
// reduced in a fixed order to stp[blockIdx.x][0|1][Cout] (bn_stats_part's
// format) around sh = the output at pixel 0, which every workgroup computes
// with the same MFMA sequence as the real pixel 0 (workgroup 0 stores it to
// shift[] for bn_stats_final).  Saves bn1's statistics pass over the
// expanded tensor.
template <int TN, int KC, int X2, bool AS, bool ST = false>
__global__ __launch_bounds__((CsCfg<TN, KC>::NW * 64)) void conv1x1_stream_kernel(
    const ConvArgs p, int nblk, int ohw, float* __restrict__ stp, float* __restrict__ shift) {
  constexpr int NW = CsCfg<TN, KC>::NW, NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  f32x4* wl = reinterpret_cast<f32x4*>(smem);
  float4* gl = reinterpret_cast<float4*>(smem + p.Kc * TN * 64 * 4);
  const int t = threadIdx.x, lane = t & 63, g = lane >> 4, j = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  {
    const f32x4* ws = reinterpret_cast<const f32x4*>(p.w);
    const int nw = p.Kc * TN * 64;
    for (int i = t; i < nw; i += NT) wl[i] = ws[i];
    if (AS) {
      const int c4n = p.Cin >> 2;
      for (int i = t; i < p.B * c4n; i += NT) {
        const int b = i / c4n, c = i - b * c4n;
        gl[i] = *reinterpret_cast<const float4*>(p.ascale + (int64_t)b * p.ascale_bs + 4 * c);
      }
    }
  }
  __syncthreads();
  const int nwv = gridDim.x * NW;
  int blk = blockIdx.x * NW + wave;
  // ST: the shift (pixel 0's output, channels 16u + 4g .. +3 in every lane)
  float4 sh[ST ? TN : 1], ss[ST ? TN : 1], sq[ST ? TN : 1];
  if (ST) {
    f32x4 a0[TN];
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int n0 = 16 * u + 4 * g;
      const float4 bb = p.bias && n0 < p.Cout ? *reinterpret_cast<const float4*>(p.bias + n0)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
      a0[u] = (f32x4){bb.x, bb.y, bb.z, bb.w};
    }
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      if (kc >= p.Kc) break;
      const int kq = kc * 16 + 4 * g;
      const float4 a = kq < p.Cin ? *reinterpret_cast<const float4*>(p.x + p.x_c0 + kq)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const f32x4 w = wl[(kc * TN + u) * 64 + lane];
        a0[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, a.x, a0[u], 0, 0, 0);
        a0[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, a.y, a0[u], 0, 0, 0);
        a0[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, a.z, a0[u], 0, 0, 0);
        a0[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, a.w, a0[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      sh[u] = make_float4(cs_act(a0[u][0], p.act, p.slope), cs_act(a0[u][1], p.act, p.slope),
                          cs_act(a0[u][2], p.act, p.slope), cs_act(a0[u][3], p.act, p.slope));
      ss[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      sq[u] = ss[u];
      const int n0 = 16 * u + 4 * g;
      if (blockIdx.x == 0 && wave == 0 && j == 0 && n0 < p.Cout)
        *reinterpret_cast<float4*>(shift + n0) = sh[u];
    }
  }
  if (!ST && blk >= nblk) return;  // no barrier below (ST: the reduction has one)
  const int M = (int)p.M, Cin = p.Cin, Ktot = p.Cin + (X2 ? p.Cin2 : 0);
  const int c4n = Cin >> 2;
  const float* xg = p.x + p.x_c0;

  // one float4 of A: pixel of lane j in block bk, channels 16kc + 4g .. +3
  auto issue = [&](int bk, int kc) -> float4 {
    int m = bk * 16 + j;
    m = m < M ? m : M - 1;
    const int kq = (kc < p.Kc ? kc : p.Kc - 1) * 16 + 4 * g;
    const float* src;
    if (X2 && kq >= Cin) {
      const int k2 = kq - Cin < p.Cin2 ? kq - Cin : 0;
      src = p.x2 + m * p.x2_ps + k2;
    } else {
      src = xg + m * p.x_ps + (kq < Cin ? kq : 0);
    }
    return *reinterpret_cast<const float4*>(src);
  };

  float4 bias[TN];
#pragma unroll
  for (int u = 0; u < TN; ++u) {
    const int n0 = 16 * u + 4 * g;
    bias[u] = p.bias && n0 < p.Cout ? *reinterpret_cast<const float4*>(p.bias + n0)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 A[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) A[kc] = issue(blk < nblk ? blk : 0, kc);

  for (; blk < nblk;) {
    const int nxt = blk + nwv;
    const int bnx = nxt < nblk ? nxt : blk;  // last block: harmless re-read
    const int m = blk * 16 + j;
    // residual loads are issued unconditionally (a null residual reads the
    // first weight float4, an L2 hit) so the vmcnt of the A stages behind
    // them stays exact
    float4 R[TN];
    {
      const int mr = m < M ? m : M - 1;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const int n0 = 16 * u + 4 * g;
        const float* rs = p.res ? p.res + mr * p.res_ps + p.res_c0 + (n0 < p.Cout ? n0 : 0)
                                : reinterpret_cast<const float*>(p.w);
        R[u] = *reinterpret_cast<const float4*>(rs);
      }
    }
    const int gb = AS ? (blk * 16) / ohw : 0;  // block-uniform (host: ohw % 16 == 0)
    f32x4 acc[TN];
#pragma unroll
    for (int u = 0; u < TN; ++u) acc[u] = (f32x4){bias[u].x, bias[u].y, bias[u].z, bias[u].w};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      float4 a = A[kc];
      const int kq = kc * 16 + 4 * g;
      if (kc * 16 + 16 > Ktot && kq >= Ktot) a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (AS) {  // unpredicated LDS read; skip-source channels keep scale 1
        const bool gk = kq < Cin;
        const float4 s = gl[gb * c4n + (gk ? kq >> 2 : 0)];
        a.x *= gk ? s.x : 1.f; a.y *= gk ? s.y : 1.f;
        a.z *= gk ? s.z : 1.f; a.w *= gk ? s.w : 1.f;
      }
      if (kc < p.Kc) {
#pragma unroll
        for (int u = 0; u < TN; ++u) {
          const f32x4 w = wl[(kc * TN + u) * 64 + lane];
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, a.x, acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, a.y, acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, a.z, acc[u], 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, a.w, acc[u], 0, 0, 0);
        }
      }
      // refill after the MFMAs have read the stage: the load can take the
      // stage's own registers (no loop-carried copy, which would wait vmcnt(0))
      A[kc] = issue(bnx, kc);
    }
    // acc[u][r] = Y[pixel m][16u + 4g + r]
    if (m < M) {
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const int n0 = 16 * u + 4 * g;
        if (n0 < p.Cout) {
          float4 v = make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
          if (p.res) {
            v.x += R[u].x; v.y += R[u].y; v.z += R[u].z; v.w += R[u].w;
          }
          v.x = cs_act(v.x, p.act, p.slope);
          v.y = cs_act(v.y, p.act, p.slope);
          v.z = cs_act(v.z, p.act, p.slope);
          v.w = cs_act(v.w, p.act, p.slope);
          *reinterpret_cast<float4*>(p.y + m * p.y_ps + p.y_c0 + n0) = v;
          if (ST) {
            const float4 d = make_float4(v.x - sh[u].x, v.y - sh[u].y, v.z - sh[u].z, v.w - sh[u].w);
            ss[u].x += d.x; ss[u].y += d.y; ss[u].z += d.z; ss[u].w += d.w;
            sq[u].x = fmaf(d.x, d.x, sq[u].x); sq[u].y = fmaf(d.y, d.y, sq[u].y);
            sq[u].z = fmaf(d.z, d.z, sq[u].z); sq[u].w = fmaf(d.w, d.w, sq[u].w);
          }
        }
      }
    }
    if (nxt >= nblk) break;
    blk = nxt;
  }
  if (ST) {
    // lanes j of a channel quad g: xor-tree over j (fixed order), then the
    // waves in order through LDS (the weights are dead by now)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        ss[u].x += __shfl_xor(ss[u].x, off); ss[u].y += __shfl_xor(ss[u].y, off);
        ss[u].z += __shfl_xor(ss[u].z, off); ss[u].w += __shfl_xor(ss[u].w, off);
        sq[u].x += __shfl_xor(sq[u].x, off); sq[u].y += __shfl_xor(sq[u].y, off);
        sq[u].z += __shfl_xor(sq[u].z, off); sq[u].w += __shfl_xor(sq[u].w, off);
      }
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(smem);  // [NW][2][TN * 4]
    if (j == 0) {
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        red[(wave * 2 + 0) * TN * 4 + 4 * u + g] = ss[u];
        red[(wave * 2 + 1) * TN * 4 + 4 * u + g] = sq[u];
      }
    }
    __syncthreads();
    if (t < 2 * TN * 4) {
      const int which = t / (TN * 4), q = t - which * (TN * 4);  // q = 4u + g: channels 4q..
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int w = 0; w < NW; ++w) {
        const float4 a = red[(w * 2 + which) * TN * 4 + q];
        v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      }
      if (4 * q < p.Cout)
        *reinterpret_cast<float4*>(stp + ((int64_t)blockIdx.x * 2 + which) * p.Cout + 4 * q) = v;
    }
  }
}

// JABD_CONV_STREAM=0 disables the streaming kernel (A/B).
static bool conv_stream_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JABD_CONV_STREAM");
    v = e && e[0] == '0' ? 0 : 1;
  }
  return v == 1;
}

static int stream_kc(int kc) {
  static const int ks[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 13, 16, 18};
  for (int k : ks)
    if (kc <= k) return k;
  return -1;
}

template <typename Kern>
static int stream_grid(Kern kern, int threads, size_t lds, int64_t nwg) {
  int dev = 0, ncu = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, threads, lds) != hipSuccess ||
      occ < 1)
    return -1;
  const int64_t cap = (int64_t)ncu * occ;
  return (int)(nwg < cap ? nwg : cap);
}

// Called from jabd_conv2d_nhwc_f32 for the fast-1x1 layouts (contiguous NHWC
// rows, v4 epilogue, x2 at the same resolution).  Returns -1 when the shape is
// not one this kernel serves.
// ss != nullptr: the statistics form (ST; no gate, no second source, no
// residual).  ss->query: only report the grid (= partial rows) in ss->nblk;
// otherwise launch and require ss->nblk to match it.
int conv1x1_stream_dispatch(const ConvArgs& a, hipStream_t st, StreamStats* ss) {
  if (!conv_stream_on()) return -1;
  if (ss && (a.x2 || a.ascale || a.res || stream_kc(a.Kc) > 4)) return -1;
  const int TN = a.Ntiles, KC = stream_kc(a.Kc);
  if (TN < 1 || TN > 5 || KC < 0) return -1;
  if (a.x2 && a.x2_stride != 1) return -1;
  const int64_t ohw = (int64_t)a.OH * a.OW;
  if (a.ascale && (ohw % 16 || a.ascale_bs % 4)) return -1;
  const size_t lds = (size_t)a.Kc * TN * 1024 + (a.ascale ? (size_t)a.B * a.Cin * 4 : 0);
  if (lds > (a.Kc * TN > 24 ? 150 : 40) * 1024) return -1;
  const int64_t nblk = cdiv(a.M, 16);
  if (nblk >= ((int64_t)1 << 27)) return -1;
  // the kernel forms pixel offsets m * ps in 32-bit ints (the caller's fast1x1
  // condition already bounds (M + 64) * (max ps + 16) < 2^31; kept here so the
  // kernel never relies on a caller's check)
  const int64_t maxps = std::max<int64_t>(std::max<int64_t>(a.x_ps, a.y_ps),
                                          std::max<int64_t>(a.res ? a.res_ps : 0,
                                                            a.x2 ? a.x2_ps : 0));
  if ((a.M + 16) * (maxps + 16) >= ((int64_t)1 << 31)) return -1;
  const int x2 = a.x2 ? 1 : 0;
  const bool as = a.ascale != nullptr;
#define CS_LAUNCH(TN_, KC_, X2_, AS_)                                                       \
  do {                                                                                      \
    auto kern = conv1x1_stream_kernel<TN_, KC_, X2_, AS_>;                                  \
    constexpr int nw_ = CsCfg<TN_, KC_>::NW;                                                \
    if ((a.Kc * TN > 24) != (nw_ == 8)) return -1;                                          \
    const int grid = stream_grid(kern, nw_ * 64, lds, cdiv(nblk, nw_));                     \
    if (grid < 1) return -1;                                                                \
    kern<<<grid, nw_ * 64, lds, st>>>(a, (int)nblk, (int)ohw, nullptr, nullptr);            \
    return check_launch("conv1x1_stream");                                                  \
  } while (0)
#define CS_LAUNCH_ST(TN_, KC_)                                                              \
  do {                                                                                      \
    auto kern = conv1x1_stream_kernel<TN_, KC_, 0, false, true>;                            \
    constexpr int nw_ = CsCfg<TN_, KC_>::NW;                                                \
    if ((a.Kc * TN > 24) != (nw_ == 8)) return -1;                                          \
    const int grid = stream_grid(kern, nw_ * 64, lds, cdiv(nblk, nw_));                     \
    if (grid < 1) return -1;                                                                \
    if (ss->query) {                                                                        \
      ss->nblk = grid;                                                                      \
      return 0;                                                                             \
    }                                                                                       \
    JABD_REQUIRE(ss->nblk == grid && ss->part && ss->shift,                                 \
                 "conv1x1_bn_stats: %lld partial rows given, kernel grid %d",               \
                 (long long)ss->nblk, grid);                                                \
    kern<<<grid, nw_ * 64, lds, st>>>(a, (int)nblk, (int)ohw, ss->part, ss->shift);         \
    return check_launch("conv1x1_stream_stats");                                            \
  } while (0)
#define CS_FLAGS_ST(TN_, KC_) \
  if (ss && TN == TN_ && KC == KC_) CS_LAUNCH_ST(TN_, KC_);
  CS_FLAGS_ST(1, 1) CS_FLAGS_ST(2, 1) CS_FLAGS_ST(3, 1) CS_FLAGS_ST(4, 1) CS_FLAGS_ST(5, 1)
  CS_FLAGS_ST(1, 2) CS_FLAGS_ST(2, 2) CS_FLAGS_ST(3, 2) CS_FLAGS_ST(4, 2) CS_FLAGS_ST(5, 2)
  CS_FLAGS_ST(1, 3) CS_FLAGS_ST(2, 3) CS_FLAGS_ST(3, 3) CS_FLAGS_ST(4, 3) CS_FLAGS_ST(5, 3)
  CS_FLAGS_ST(1, 4) CS_FLAGS_ST(2, 4) CS_FLAGS_ST(3, 4) CS_FLAGS_ST(4, 4) CS_FLAGS_ST(5, 4)
  if (ss) return -1;
#undef CS_FLAGS_ST
#undef CS_LAUNCH_ST
#define CS_FLAGS(TN_, KC_)                      \
  if (TN == TN_ && KC == KC_) {                 \
    if (x2 == 0 && !as) CS_LAUNCH(TN_, KC_, 0, false); \
    if (x2 == 0 && as) CS_LAUNCH(TN_, KC_, 0, true);   \
    if (x2 == 1 && !as) CS_LAUNCH(TN_, KC_, 1, false); \
    CS_LAUNCH(TN_, KC_, 1, true);               \
  }
#define CS_KC(TN_) \
  CS_FLAGS(TN_, 1) CS_FLAGS(TN_, 2) CS_FLAGS(TN_, 3) CS_FLAGS(TN_, 4) CS_FLAGS(TN_, 5) \
  CS_FLAGS(TN_, 6) CS_FLAGS(TN_, 8)
  CS_KC(1) CS_KC(2) CS_KC(3) CS_KC(4) CS_KC(5)
  CS_FLAGS(2, 10) CS_FLAGS(3, 10) CS_FLAGS(3, 12)
  CS_FLAGS(5, 10) CS_FLAGS(5, 12) CS_FLAGS(5, 13) CS_FLAGS(5, 16) CS_FLAGS(5, 18)
#undef CS_KC
#undef CS_FLAGS
#undef CS_LAUNCH
  return -1;
}

}  // namespace jabd
