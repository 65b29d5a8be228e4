// A1 depthwise k x k convolution (NHWC, fp32 VALU) with folded BN, activation
// and the ECA average-pool partial sums fused into the epilogue.
//
// Thread = 4 channels (one float4) x a strip of PW output pixels along W.
// Each thread keeps its k*k float4 taps in registers across all strips it
// computes, and loads each input row segment of a strip once (sliding
// window), so input re-reads come from L1 instead of HBM.  The ECA partial
// sums of the activated output are reduced per workgroup in fixed order and
// written to part[b][blk][c] (deterministic; no atomics).
#include "common.h"
#include "conv_args.h"

namespace jabd {

__device__ __forceinline__ float dw_act(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return relu_f(v);
    case ACT_LEAKY: return v > 0.f ? v : v * slope;
    case ACT_HSWISH: return hswish_f(v);
    default: return v;
  }
}

constexpr int kDwThreads = 256;
constexpr int kPW = 4;

__device__ __forceinline__ float4 f4fma(float4 a, float4 w, float4 c) { return fma4pk(a, w, c); }

// ST: also the BatchNorm statistics of the output for the training forward
// (MNv3 Block_eca bn2 follows the depthwise conv): per workgroup the shifted
// sums sum(y - sh), sum((y - sh)^2) of its outputs, rows added in a fixed
// order, to stp[blk][0|1][C] (blk = blockIdx.y * gridDim.x + blockIdx.x) in
// bn_stats_part's format; sh = the output at pixel (0, 0) of image 0, which
// every workgroup recomputes with the main loop's tap order (workgroup (0, 0)
// writes it to shift[] for bn_stats_final).  Saves bn2's statistics pass.
// IT: the input is act(bn(x)) of the stored pre-BN tensor x, applied on load
// (MNv3 Block_eca bn1 + act feeding conv2) as act(fma((x - mean) * invstd,
// gamma, beta)) — bn_act_fwd's and the BN backward's operation order
// (common.h dw_bn_in, shared with the weight gradient in train.hip) — in-bounds
// taps only (padding stays zero), so the activated expansion is never written.
struct DwBnIn {
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  int act;
  float slope;
};

template <int K, int S, bool ST, bool IT = false>
__global__ __launch_bounds__(kDwThreads) void dw_kernel(const DwArgs p, int strips_per_blk,
                                                       float* __restrict__ stp,
                                                       float* __restrict__ shift,
                                                       const DwBnIn bi) {
  constexpr int SPAN = (kPW - 1) * S + K;
  const int CG = p.C >> 2;
  const int SP = kDwThreads / CG;  // strips in flight per pass
  const int tid = threadIdx.x;
  const int cg = tid % CG, sp = tid / CG;
  const bool active = sp < SP;
  const int b = blockIdx.y;
  const int OWs = (p.OW + kPW - 1) / kPW;
  const int64_t nstrip = (int64_t)p.OH * OWs;
  const int64_t s0 = (int64_t)blockIdx.x * strips_per_blk;
  const float* xb = p.x + (int64_t)b * p.x_bs + 4 * cg;
  float* yb = p.y + (int64_t)b * p.y_bs + 4 * cg;

  float4 wr[K * K];
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
  if (active) {
#pragma unroll
    for (int t = 0; t < K * K; ++t) wr[t] = reinterpret_cast<const float4*>(p.w + t * p.C)[cg];
    if (p.bias) bias = reinterpret_cast<const float4*>(p.bias)[cg];
  }
  DwBnCoef bc{};
  if (IT && active) bc = dw_bn_coef(bi.mean, bi.invstd, bi.gamma, bi.beta, cg);
  auto ldx = [&](const float* ptr) -> float4 {
    const float4 v = *reinterpret_cast<const float4*>(ptr);
    return IT ? dw_bn_in(v, bc, bi.act, bi.slope) : v;
  };
  float4 psum = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sh = make_float4(0.f, 0.f, 0.f, 0.f), ss = sh, sq = sh;
  if (ST && active) {
    float4 a0 = bias;
    const float* x0 = p.x + 4 * cg;  // image 0
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ih = -p.pad + kh;
      if (ih < 0 || ih >= p.H) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int iw = -p.pad + kw;
        const float4 r = (iw >= 0 && iw < p.W) ? ldx(x0 + ((int64_t)ih * p.W + iw) * p.x_ps)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
        a0 = f4fma(r, wr[kh * K + kw], a0);
      }
    }
    sh.x = dw_act(a0.x, p.act, p.slope);
    sh.y = dw_act(a0.y, p.act, p.slope);
    sh.z = dw_act(a0.z, p.act, p.slope);
    sh.w = dw_act(a0.w, p.act, p.slope);
    if (blockIdx.x == 0 && blockIdx.y == 0 && sp == 0) reinterpret_cast<float4*>(shift)[cg] = sh;
  }

  for (int it = 0; active && it * SP < strips_per_blk; ++it) {
    const int64_t s = s0 + it * SP + sp;
    if (s >= nstrip || it * SP + sp >= strips_per_blk) break;
    const int oh = (int)(s / OWs);
    const int ow0 = (int)(s - (int64_t)oh * OWs) * kPW;
    float4 acc[kPW];
#pragma unroll
    for (int o = 0; o < kPW; ++o) acc[o] = bias;
    const int iw0 = ow0 * S - p.pad;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - p.pad + kh;
      if (ih < 0 || ih >= p.H) continue;
      float4 row[SPAN];
      const float* xr = xb + (int64_t)ih * p.W * p.x_ps;
#pragma unroll
      for (int c = 0; c < SPAN; ++c) {
        const int iw = iw0 + c;
        row[c] = (iw >= 0 && iw < p.W) ? ldx(xr + (int64_t)iw * p.x_ps)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int o = 0; o < kPW; ++o)
#pragma unroll
        for (int kw = 0; kw < K; ++kw) acc[o] = f4fma(row[o * S + kw], wr[kh * K + kw], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < kPW; ++o) {
      if (ow0 + o >= p.OW) break;
      float4 v;
      v.x = dw_act(acc[o].x, p.act, p.slope);
      v.y = dw_act(acc[o].y, p.act, p.slope);
      v.z = dw_act(acc[o].z, p.act, p.slope);
      v.w = dw_act(acc[o].w, p.act, p.slope);
      *reinterpret_cast<float4*>(yb + ((int64_t)oh * p.OW + ow0 + o) * p.y_ps) = v;
      psum.x += v.x; psum.y += v.y; psum.z += v.z; psum.w += v.w;
      if (ST) {
        const float4 d = make_float4(v.x - sh.x, v.y - sh.y, v.z - sh.z, v.w - sh.w);
        ss.x += d.x; ss.y += d.y; ss.z += d.z; ss.w += d.w;
        sq.x = fmaf(d.x, d.x, sq.x); sq.y = fmaf(d.y, d.y, sq.y);
        sq.z = fmaf(d.z, d.z, sq.z); sq.w = fmaf(d.w, d.w, sq.w);
      }
    }
  }

  if (ST) {
    __shared__ float4 rs[kDwThreads], rq[kDwThreads];
    rs[tid] = ss;
    rq[tid] = sq;
    __syncthreads();
    if (tid < CG) {
      float4 S_ = make_float4(0.f, 0.f, 0.f, 0.f), Q_ = S_;
      for (int q = 0; q < SP; ++q) {
        const float4 a = rs[q * CG + tid], b = rq[q * CG + tid];
        S_.x += a.x; S_.y += a.y; S_.z += a.z; S_.w += a.w;
        Q_.x += b.x; Q_.y += b.y; Q_.z += b.z; Q_.w += b.w;
      }
      const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
      reinterpret_cast<float4*>(stp + blk * 2 * p.C)[tid] = S_;
      reinterpret_cast<float4*>(stp + blk * 2 * p.C + p.C)[tid] = Q_;
    }
  }

  if (p.part) {
    __shared__ float4 red[kDwThreads];
    red[tid] = psum;
    __syncthreads();
    if (tid < CG) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int q = 0; q < SP; ++q) {
        float4 v = red[q * CG + tid];
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
      reinterpret_cast<float4*>(p.part + ((int64_t)b * p.nblk + blockIdx.x) * p.C)[tid] = t;
    }
  }
}

// The 3x3 training forward with BatchNorm statistics as a row walker: a
// thread owns PW output columns x 4 channels and a chunk of R output rows,
// and keeps the input rows it still needs in registers (stride 1: a ring of
// three rows rotated by unrolling; stride 2: the row shared by consecutive
// outputs), so every input row is loaded once per chunk (+2 / +1 halo rows)
// instead of once per output row it feeds.  Each output is accumulated in
// dw_kernel's tap order (rows outside the image skipped, in-row padding as
// zeros): the outputs are dw_kernel's bit for bit.  Workgroup blockIdx.x =
// band * nchunks + chunk (blocks past nbands * nchunks write zero partials,
// so the statistics rows keep jabd_dwconv_stats_nblk's count).
template <int S, int PW, bool IT>
__global__ __launch_bounds__(kDwThreads) void dw_rows_kernel(const DwArgs p, int nbands,
                                                            int nchunks, int R,
                                                            float* __restrict__ stp,
                                                            float* __restrict__ shift,
                                                            const DwBnIn bi) {
  constexpr int K = 3;
  constexpr int SPAN = (PW - 1) * S + K;
  const int CG = p.C >> 2;
  const int SP = kDwThreads / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG, sp = tid / CG;
  const int b = blockIdx.y;
  const int band = blockIdx.x / nchunks, chunk = blockIdx.x % nchunks;
  const int OWs = (p.OW + PW - 1) / PW;
  const int strip = band * SP + sp;
  const bool active = sp < SP && band < nbands && strip < OWs;
  const float* xb = p.x + (int64_t)b * p.x_bs + 4 * cg;
  float* yb = p.y + (int64_t)b * p.y_bs + 4 * cg;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 wr[K * K];
  float4 bias = z;
  if (sp < SP) {
#pragma unroll
    for (int t = 0; t < K * K; ++t) wr[t] = reinterpret_cast<const float4*>(p.w + t * p.C)[cg];
    if (p.bias) bias = reinterpret_cast<const float4*>(p.bias)[cg];
  }
  DwBnCoef bc{};
  if (IT && sp < SP) bc = dw_bn_coef(bi.mean, bi.invstd, bi.gamma, bi.beta, cg);
  auto ldx = [&](const float* ptr) -> float4 {
    const float4 v = *reinterpret_cast<const float4*>(ptr);
    return IT ? dw_bn_in(v, bc, bi.act, bi.slope) : v;
  };
  float4 sh = z, ss = z, sq = z;
  if (sp < SP) {  // the shift: output (0, 0) of image 0, dw_kernel's expression
    float4 a0 = bias;
    const float* x0 = p.x + 4 * cg;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ih = -p.pad + kh;
      if (ih < 0 || ih >= p.H) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int iw = -p.pad + kw;
        const float4 r = (iw >= 0 && iw < p.W) ? ldx(x0 + ((int64_t)ih * p.W + iw) * p.x_ps) : z;
        a0 = f4fma(r, wr[kh * K + kw], a0);
      }
    }
    sh.x = dw_act(a0.x, p.act, p.slope);
    sh.y = dw_act(a0.y, p.act, p.slope);
    sh.z = dw_act(a0.z, p.act, p.slope);
    sh.w = dw_act(a0.w, p.act, p.slope);
    if (blockIdx.x == 0 && blockIdx.y == 0 && sp == 0) reinterpret_cast<float4*>(shift)[cg] = sh;
  }
  const int oh0 = chunk * R, oh1 = min(p.OH, oh0 + R);
  const int ow0 = strip * PW, iw0 = ow0 * S - p.pad;
  auto load_row = [&](int ih, float4 (&r)[SPAN]) {
    const bool rv = ih >= 0 && ih < p.H;
    const float* xr = xb + (int64_t)(rv ? ih : 0) * p.W * p.x_ps;
#pragma unroll
    for (int c = 0; c < SPAN; ++c) {
      const int iw = iw0 + c;
      r[c] = (rv && iw >= 0 && iw < p.W) ? ldx(xr + (int64_t)iw * p.x_ps) : z;
    }
  };
  // output row oh from input rows ih0, ih0 + 1, ih0 + 2 (held in r0, r1, r2)
  auto emit = [&](int oh, int ih0, const float4 (&r0)[SPAN], const float4 (&r1)[SPAN],
                  const float4 (&r2)[SPAN]) {
    float4 acc[PW];
#pragma unroll
    for (int o = 0; o < PW; ++o) acc[o] = bias;
    auto tap_row = [&](int kh, const float4 (&r)[SPAN]) {
      if (ih0 + kh < 0 || ih0 + kh >= p.H) return;
#pragma unroll
      for (int o = 0; o < PW; ++o)
#pragma unroll
        for (int kw = 0; kw < K; ++kw) acc[o] = f4fma(r[o * S + kw], wr[kh * K + kw], acc[o]);
    };
    tap_row(0, r0);
    tap_row(1, r1);
    tap_row(2, r2);
#pragma unroll
    for (int o = 0; o < PW; ++o) {
      if (ow0 + o >= p.OW) break;
      float4 v;
      v.x = dw_act(acc[o].x, p.act, p.slope);
      v.y = dw_act(acc[o].y, p.act, p.slope);
      v.z = dw_act(acc[o].z, p.act, p.slope);
      v.w = dw_act(acc[o].w, p.act, p.slope);
      *reinterpret_cast<float4*>(yb + ((int64_t)oh * p.OW + ow0 + o) * p.y_ps) = v;
      const float4 d = make_float4(v.x - sh.x, v.y - sh.y, v.z - sh.z, v.w - sh.w);
      ss.x += d.x; ss.y += d.y; ss.z += d.z; ss.w += d.w;
      sq.x = fmaf(d.x, d.x, sq.x); sq.y = fmaf(d.y, d.y, sq.y);
      sq.z = fmaf(d.z, d.z, sq.z); sq.w = fmaf(d.w, d.w, sq.w);
    }
  };
  if (active && oh0 < oh1) {
    if constexpr (S == 1) {
      float4 rA[SPAN], rB[SPAN], rC[SPAN];
      load_row(oh0 - p.pad, rA);
      load_row(oh0 - p.pad + 1, rB);
      for (int oh = oh0; oh < oh1; oh += 3) {
        const int ih = oh - p.pad;
        load_row(ih + 2, rC);
        emit(oh, ih, rA, rB, rC);
        if (oh + 1 >= oh1) break;
        load_row(ih + 3, rA);
        emit(oh + 1, ih + 1, rB, rC, rA);
        if (oh + 2 >= oh1) break;
        load_row(ih + 4, rB);
        emit(oh + 2, ih + 2, rC, rA, rB);
      }
    } else {
      float4 rP[SPAN], rA[SPAN], rB[SPAN];
      load_row(2 * oh0 - p.pad, rP);
      for (int oh = oh0; oh < oh1; oh += 2) {
        const int ih = 2 * oh - p.pad;
        load_row(ih + 1, rA);
        load_row(ih + 2, rB);
        emit(oh, ih, rP, rA, rB);
        if (oh + 1 >= oh1) break;
        load_row(ih + 3, rA);
        load_row(ih + 4, rP);
        emit(oh + 1, ih + 2, rB, rA, rP);
      }
    }
  }
  __shared__ float4 rs[kDwThreads], rq[kDwThreads];
  rs[tid] = ss;
  rq[tid] = sq;
  __syncthreads();
  if (tid < CG) {
    float4 S_ = z, Q_ = z;
    for (int q = 0; q < SP; ++q) {
      const float4 a = rs[q * CG + tid], c = rq[q * CG + tid];
      S_.x += a.x; S_.y += a.y; S_.z += a.z; S_.w += a.w;
      Q_.x += c.x; Q_.y += c.y; Q_.z += c.z; Q_.w += c.w;
    }
    const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    reinterpret_cast<float4*>(stp + blk * 2 * p.C)[tid] = S_;
    reinterpret_cast<float4*>(stp + blk * 2 * p.C + p.C)[tid] = Q_;
  }
}

static int64_t dw_strips_per_blk(int64_t B, int64_t OH, int64_t OW, int64_t C) {
  const int64_t SP = kDwThreads / (C / 4);
  const int64_t nstrip = OH * ((OW + kPW - 1) / kPW);
  // aim for >= ~2048 workgroups over the batch, at least one pass per block
  int64_t per = cdiv(nstrip * B, 2048);
  per = cdiv(per, SP) * SP;
  if (per < SP) per = SP;
  return per;
}

}  // namespace jabd

using namespace jabd;

extern "C" int64_t jabd_dw_nblk(int64_t B, int64_t OH, int64_t OW, int64_t C) {
  if (B <= 0 || OH <= 0 || OW <= 0 || C <= 0 || C % 4 || C / 4 > kDwThreads) return -1;
  const int64_t nstrip = OH * ((OW + kPW - 1) / kPW);
  return cdiv(nstrip, dw_strips_per_blk(B, OH, OW, C));
}

extern "C" int jabd_dwconv_nhwc_f32(const jabd_dw_args* args, jabd_stream_t stream) {
  JABD_REQUIRE(args, "dw: null args");
  const DwArgs& a = *args;
  JABD_REQUIRE(a.x && a.w && a.y, "dw: null pointer");
  JABD_REQUIRE(a.C % 4 == 0 && a.C / 4 <= kDwThreads, "dw: C=%d must be a multiple of 4, <= 1024",
               a.C);
  JABD_REQUIRE(a.x_ps % 4 == 0 && a.y_ps % 4 == 0, "dw: pixel strides must be multiples of 4");
  JABD_REQUIRE(a.OH == (a.H + 2 * a.pad - a.k) / a.stride + 1 &&
                   a.OW == (a.W + 2 * a.pad - a.k) / a.stride + 1,
               "dw: output size mismatch");
  const int64_t per = dw_strips_per_blk(a.B, a.OH, a.OW, a.C);
  const int64_t nblk = jabd_dw_nblk(a.B, a.OH, a.OW, a.C);
  JABD_REQUIRE(!a.part || a.nblk == nblk, "dw: nblk %d != %lld", a.nblk, (long long)nblk);
  dim3 grid((unsigned)nblk, (unsigned)a.B);
  hipStream_t st = as_stream(stream);
#define DW_CASE(K, S)                                                                       \
  if (a.k == K && a.stride == S) {                                                         \
    dw_kernel<K, S, false><<<grid, kDwThreads, 0, st>>>(a, (int)per, nullptr, nullptr, {}); \
    return check_launch("dwconv");                                                         \
  }
  DW_CASE(3, 1)
  DW_CASE(3, 2)
  DW_CASE(5, 1)
  DW_CASE(5, 2)
#undef DW_CASE
  set_error("dw: unsupported k=%d stride=%d", a.k, a.stride);
  return JABD_EINVAL;
}

extern "C" int64_t jabd_dwconv_stats_nblk(int64_t B, int64_t OH, int64_t OW, int64_t C) {
  const int64_t n = jabd_dw_nblk(B, OH, OW, C);
  return n < 0 ? n : n * B;
}

static int dwconv_stats(const jabd_dw_args* args, float* stats_part, float* shift,
                        const DwBnIn* bi, jabd_stream_t stream) {
  JABD_REQUIRE(args && stats_part && shift, "dw_stats: null args");
  JABD_REQUIRE(!bi || (bi->mean && bi->invstd && bi->gamma && bi->beta), "dw_stats: null BN input");
  const DwArgs& a = *args;
  JABD_REQUIRE(a.x && a.w && a.y && !a.part, "dw_stats: null pointer / ECA partials not supported");
  JABD_REQUIRE(a.C % 4 == 0 && a.C / 4 <= kDwThreads && a.x_ps % 4 == 0 && a.y_ps % 4 == 0,
               "dw_stats: channel layout");
  JABD_REQUIRE(a.OH == (a.H + 2 * a.pad - a.k) / a.stride + 1 &&
                   a.OW == (a.W + 2 * a.pad - a.k) / a.stride + 1,
               "dw_stats: output size mismatch");
  const int64_t per = dw_strips_per_blk(a.B, a.OH, a.OW, a.C);
  const int64_t nblk = jabd_dw_nblk(a.B, a.OH, a.OW, a.C);
  dim3 grid((unsigned)nblk, (unsigned)a.B);
  hipStream_t st = as_stream(stream);
  // 3x3: the row walker, within the same partial-block count
  // (JABD_DW_ROWS=0: dw_kernel)
  static const bool rows_on = [] {
    const char* e = getenv("JABD_DW_ROWS");
    return !(e && e[0] == '0');
  }();
#define DWR_CASE(S, PW)                                                                      \
  if (rows_on && a.k == 3 && a.stride == S && a.pad == 1) {                                 \
    const int SP = kDwThreads / (a.C / 4);                                                   \
    const int nbands = (int)cdiv((int64_t)cdiv(a.OW, PW), SP);                               \
    if (nbands <= nblk) {                                                                    \
      const int want = (int)std::max<int64_t>(1, std::min<int64_t>(a.OH, nblk / nbands));    \
      const int R = (int)cdiv(a.OH, want);                                                   \
      const int nch = (int)cdiv(a.OH, R);                                                    \
      if (bi)                                                                                \
        dw_rows_kernel<S, PW, true><<<grid, kDwThreads, 0, st>>>(a, nbands, nch, R, stats_part, \
                                                                  shift, *bi);               \
      else                                                                                   \
        dw_rows_kernel<S, PW, false><<<grid, kDwThreads, 0, st>>>(a, nbands, nch, R,           \
                                                                   stats_part, shift, {});   \
      return check_launch("dwconv_stats_rows");                                              \
    }                                                                                        \
  }
  DWR_CASE(1, 4)
  DWR_CASE(2, 2)
#undef DWR_CASE
#define DWS_CASE(K, S)                                                                      \
  if (a.k == K && a.stride == S) {                                                         \
    if (bi)                                                                                \
      dw_kernel<K, S, true, true><<<grid, kDwThreads, 0, st>>>(a, (int)per, stats_part, shift, \
                                                               *bi);                       \
    else                                                                                   \
      dw_kernel<K, S, true><<<grid, kDwThreads, 0, st>>>(a, (int)per, stats_part, shift, {}); \
    return check_launch("dwconv_stats");                                                   \
  }
  DWS_CASE(3, 1)
  DWS_CASE(3, 2)
  DWS_CASE(5, 1)
  DWS_CASE(5, 2)
#undef DWS_CASE
  set_error("dw_stats: unsupported k=%d stride=%d", a.k, a.stride);
  return JABD_EINVAL;
}

extern "C" int jabd_dwconv_stats_f32(const jabd_dw_args* args, float* stats_part, float* shift,
                                     jabd_stream_t stream) {
  return dwconv_stats(args, stats_part, shift, nullptr, stream);
}

extern "C" int jabd_dwconv_bnin_stats_f32(const jabd_dw_args* args, const float* mean,
                                          const float* invstd, const float* gamma,
                                          const float* beta, int32_t act, float slope,
                                          float* stats_part, float* shift, jabd_stream_t stream) {
  JABD_REQUIRE(act == ACT_NONE || act == ACT_RELU || act == ACT_LEAKY || act == ACT_HSWISH,
               "dw_bnin: act %d not supported", act);
  const DwBnIn bi{mean, invstd, gamma, beta, act, slope};
  return dwconv_stats(args, stats_part, shift, &bi, stream);
}
