// A5 ResNet-50 stem: conv 7x7 / stride 2 / pad 3, 3 -> 64 channels, read
// straight from the NCHW network input (nets/resnet_pytorch_r.py:174-178,
// conv1 + bn1 + relu; eval folds bn1 into the weights and bias).
//
// The generic implicit GEMM gathers this layer's A operand element by element
// (3 channels: no float4 per tap) with two integer divisions per element, and
// ran at 25 % of the fp32 MFMA peak (forward) / 21 % (weight gradient).  Both
// kernels here stage a zero-padded input window per tile in LDS with coalesced
// row loads and read every MFMA operand from it at a per-lane base plus a
// compile-time offset:
//
// forward   Y[px][n] = sum_k W[n][k] X[px][k].  Workgroup tile = 4 output rows
//           (one per wave) x 64 columns; the k index of MFMA step s for lane
//           group g is (ci, kh, kw = g + 4 kwh), so the A read of step s is
//           window[base(lane) + ci*plane + kh*WC + 4 kwh + 32 t] (t = 16-pixel
//           subtile) — 42 steps (147 taps + 21 zero-weight kw = 7 slots).  The
//           weights sit in LDS as one float4 (4 output-channel tiles) per
//           (step, lane).  Persistent workgroups; the next tile's window is in
//           registers while this one computes.
// wgrad     dW[k][n] = sum_px X[px][k] dY[px][n], k = tap * 3 + ci (the packed
//           / wgrad_reduce2 order).  Task = 64 output pixels of one row; wave
//           u owns output channels 16u..16u+15 and all ten 16-row k tiles; the
//           MFMA reduction index is the pixel (4 per step).  dY is staged in LDS
//           with a 80-float pitch (the 4 pixel rows of one read land on
//           disjoint bank quarters).  Per-workgroup partials [wg][147][64] are
//           combined by wgrad_reduce2_kernel (train.hip) in a fixed order.
#include <algorithm>

#include "common.h"
#include "conv_args.h"

namespace jabd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace s7 {
constexpr int KH = 7, KW = 7, S = 2, CIN = 3, COUT = 64;
constexpr int K = KH * KW * CIN;       // 147
constexpr int KWH = 2;                 // kw = g + 4 * kwh (kw == 7: zero weight)
constexpr int NS = CIN * KH * KWH;     // 42 MFMA k-steps
constexpr int TR = 4, TC = 64;         // forward tile: 4 rows x 64 columns
constexpr int WR = (TR - 1) * S + KH;  // 13 window rows
constexpr int WC = 136;                // >= (TC - 1) * S + 4 * KWH = 134
constexpr int WPL = WR * WC;
constexpr int WS = CIN * WPL;          // 5304 floats
constexpr int NPF = (WS + 255) / 256;  // window prefetch registers per thread
// weight gradient
constexpr int GWR = KH;                // one output row: 7 window rows
constexpr int GWPL = GWR * WC;
constexpr int GWS = CIN * GWPL;        // 2856 floats
constexpr int GNPF = (GWS + 255) / 256;
constexpr int NKT = (K + 15) / 16;     // 10 k tiles
constexpr int DYP = 80;                // dY LDS pitch (floats)
constexpr int GMAX = 1024;             // persistent weight-gradient workgroups
}  // namespace s7

bool stem7_ok(const ConvArgs& a) {
  using namespace s7;
  return a.nchw_in && !a.tconv && !a.x2 && !a.y2 && !a.ascale && !a.res && a.Cin == CIN &&
         a.KH == KH && a.KW == KW && a.stride == S && a.Cout == COUT && a.H > 0 && a.W > 0;
}

template <int ACT>
__global__ __launch_bounds__(256, 2) void stem7_fwd_kernel(const ConvArgs p, int tiles_w,
                                                          int tiles_h, int ntiles) {
  using namespace s7;
  __shared__ f32x4 wl[NS * 64];
  __shared__ float win[WS];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int j = lane & 15, g = lane >> 4;
  // packed weights Wp[kc][nt][g'*16 + j'] = float4{W[k = 16kc + 4g' + e][n = 16nt + j']}
  const f32x4* wp = reinterpret_cast<const f32x4*>(p.w);
  for (int idx = t; idx < NS * 64; idx += 256) {
    const int s = idx >> 6, l = idx & 63, lj = l & 15, lg = l >> 4;
    const int ci = s / (KH * KWH), rem = s - ci * (KH * KWH);
    const int kh = rem / KWH, kwh = rem - kh * KWH;
    const int kw = lg + 4 * kwh;
    f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (kw < KW) {
      const int k = (kh * KW + kw) * CIN + ci;
      const int kc = k >> 4, kg = (k >> 2) & 3, ke = k & 3;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = wp[((int64_t)kc * p.Ntiles + u) * 64 + kg * 16 + lj][ke];
    }
    wl[idx] = v;
  }
  const int per_img = tiles_w * tiles_h;
  float pf[NPF];
  auto fetch = [&](int tile) {
    const int b = tile / per_img, r = tile - b * per_img;
    const int th = r / tiles_w, tw = r - th * tiles_w;
    const int iy0 = th * TR * S - p.pad, ix0 = tw * TC * S - p.pad;
    const float* xb = p.x + (int64_t)b * p.x_bs;
#pragma unroll
    for (int q = 0; q < NPF; ++q) {
      const int e = q * 256 + t;
      const int ci = e / WPL, r2 = e - ci * WPL;
      const int rr = r2 / WC, cc = r2 - rr * WC;
      const int iy = iy0 + rr, ix = ix0 + cc;
      float v = 0.f;
      if (e < WS && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
        v = xb[((int64_t)ci * p.H + iy) * p.W + ix];
      pf[q] = v;
    }
  };
  int tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  const float* wb = win + wave * S * WC + j * S + g;
  for (; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's window reads are done (and wl is filled)
#pragma unroll
    for (int q = 0; q < NPF; ++q) {
      const int e = q * 256 + t;
      if (e < WS) win[e] = pf[q];
    }
    __syncthreads();
    const int b = tile / per_img, r = tile - b * per_img;
    const int th = r / tiles_w, tw = r - th * tiles_w;
    if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);
    f32x4 acc[4][4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[tt][u] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int ci = s / (KH * KWH), rem = s - ci * (KH * KWH);
      const int kh = rem / KWH, kwh = rem - kh * KWH;
      const int off = ci * WPL + kh * WC + 4 * kwh;
      const f32x4 w4 = wl[s * 64 + lane];
      float a[4];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) a[tt] = wb[off + 16 * S * tt];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
          acc[tt][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[u], a[tt], acc[tt][u], 0, 0, 0);
    }
    // acc[tt][u][rr] = Y[row th*4 + wave, col tw*64 + 16tt + j][channel 16u + 4g + rr]
    const int oh = th * TR + wave;
    if (oh < p.OH) {
      float* yr = p.y + (int64_t)b * p.y_bs + (int64_t)oh * p.OW * p.y_ps + p.y_c0 + 4 * g;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int ow = tw * TC + 16 * tt + j;
        if (ow >= p.OW) continue;
        float* yp = yr + (int64_t)ow * p.y_ps;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          f32x4 v = acc[tt][u];
          if (p.bias) {
            const float4 bb = *reinterpret_cast<const float4*>(p.bias + 16 * u + 4 * g);
            v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
          }
          if (ACT == ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = relu_f(v[e]);
          }
          *reinterpret_cast<f32x4*>(yp + 16 * u) = v;
        }
      }
    }
  }
}

int stem7_fwd_launch(const ConvArgs& a, hipStream_t st) {
  using namespace s7;
  JABD_REQUIRE(stem7_ok(a) && (a.flags & 1) && a.Ntiles >= 4, "stem7: unsupported layer");
  JABD_REQUIRE(a.act == ACT_NONE || a.act == ACT_RELU, "stem7: act %d", a.act);
  const int tiles_w = (int)cdiv(a.OW, TC), tiles_h = (int)cdiv(a.OH, TR);
  const int64_t nt = (int64_t)a.B * tiles_w * tiles_h;
  JABD_REQUIRE(nt < (int64_t)0x7fffffff, "stem7: too many tiles");
  const unsigned grid = (unsigned)std::min<int64_t>(nt, 2 * 256);
  if (a.act == ACT_RELU)
    stem7_fwd_kernel<ACT_RELU><<<grid, 256, 0, st>>>(a, tiles_w, tiles_h, (int)nt);
  else
    stem7_fwd_kernel<ACT_NONE><<<grid, 256, 0, st>>>(a, tiles_w, tiles_h, (int)nt);
  return check_launch("stem7_fwd");
}

__global__ __launch_bounds__(256) void stem7_wgrad_kernel(const ConvArgs p, int64_t ntask,
                                                         float* __restrict__ part) {
  using namespace s7;
  __shared__ float win[GWS];
  __shared__ float dys[TC * DYP];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int i = lane & 15, g = lane >> 4;
  // A row offsets: k = 16 kt + i = tap * 3 + ci (rows >= 147 read slot 0; their
  // accumulator rows are never stored and no other row depends on them)
  int aoff[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int k = 16 * kt + i;
    const int tap = k / CIN, ci = k - tap * CIN;
    const int kh = tap / KW, kw = tap - kh * KW;
    aoff[kt] = k < K ? ci * GWPL + kh * WC + kw + g * S : 0;
  }
  const int nseg = (p.OW + TC - 1) / TC;
  float pw[GNPF];
  f32x4 pd[4];
  auto fetch = [&](int64_t task) {
    const int seg = (int)(task % nseg);
    const int64_t row = task / nseg;
    const int oy = (int)(row % p.OH), b = (int)(row / p.OH);
    const int ox0 = seg * TC;
    const int iy0 = oy * S - p.pad, ix0 = ox0 * S - p.pad;
    const float* xb = p.x + (int64_t)b * p.x_bs;
#pragma unroll
    for (int q = 0; q < GNPF; ++q) {
      const int e = q * 256 + t;
      const int ci = e / GWPL, r2 = e - ci * GWPL;
      const int rr = r2 / WC, cc = r2 - rr * WC;
      const int iy = iy0 + rr, ix = ix0 + cc;
      float v = 0.f;
      if (e < GWS && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
        v = xb[((int64_t)ci * p.H + iy) * p.W + ix];
      pw[q] = v;
    }
    const float* dyr = p.y + (int64_t)b * p.y_bs + (int64_t)oy * p.OW * p.y_ps + p.y_c0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = q * 256 + t, px = e >> 4, c4 = (e & 15) * 4;
      f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (ox0 + px < p.OW) v = *reinterpret_cast<const f32x4*>(dyr + (int64_t)(ox0 + px) * p.y_ps + c4);
      pd[q] = v;
    }
  };
  f32x4 acc[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) acc[kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int64_t task = blockIdx.x;
  if (task < ntask) fetch(task);
  for (; task < ntask; task += gridDim.x) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < GNPF; ++q) {
      const int e = q * 256 + t;
      if (e < GWS) win[e] = pw[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = q * 256 + t, px = e >> 4, c4 = (e & 15) * 4;
      *reinterpret_cast<f32x4*>(dys + px * DYP + c4) = pd[q];
    }
    __syncthreads();
    if (task + gridDim.x < ntask) fetch(task + gridDim.x);
    const float* db = dys + g * DYP + 16 * wave + i;
#pragma unroll
    for (int q = 0; q < TC / 4; ++q) {
      const float d = db[4 * q * DYP];
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const float a = win[aoff[kt] + 4 * S * q];
        acc[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, d, acc[kt], 0, 0, 0);
      }
    }
  }
  // acc[kt][r] = dW[k = 16 kt + 4g + r][n = 16 wave + i]
  float* pc = part + (int64_t)blockIdx.x * K * COUT + 16 * wave + i;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = 16 * kt + 4 * g + r;
      if (k < K) pc[(int64_t)k * COUT] = acc[kt][r];
    }
}

int64_t stem7_wgrad_groups(const ConvArgs& a) {
  const int64_t ntask = (int64_t)a.B * a.OH * cdiv(a.OW, s7::TC);
  return std::min<int64_t>(ntask, s7::GMAX);
}

int stem7_wgrad_launch(const ConvArgs& a, float* part, hipStream_t st) {
  using namespace s7;
  JABD_REQUIRE(stem7_ok(a) && a.y_ps % 4 == 0 && a.y_c0 % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.y) & 15) == 0 && a.y_bs % 4 == 0,
               "stem7_wgrad: unsupported layer");
  const int64_t ntask = (int64_t)a.B * a.OH * cdiv(a.OW, TC);
  const int64_t g = stem7_wgrad_groups(a);
  stem7_wgrad_kernel<<<(unsigned)g, 256, 0, st>>>(a, ntask, part);
  return check_launch("stem7_wgrad");
}

}  // namespace jabd
