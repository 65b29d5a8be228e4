// Small device-side glue of the training graph, so a training step launches
// no PyTorch (ATen) kernels for its bookkeeping:
//  * windowed copies, many tensors per launch: the zero-padding of the SSH
//    10-channel branches' weights / BN parameters / running statistics to 12
//    channels (nets/layers.py:37-68 channel widths) and the crop back of
//    their gradients and running statistics;
//  * the tap-major transpose of depthwise weights (nets/mobilenetV3.py:105);
//  * the final fixed-order reduction of per-block channel sums (conv bias
//    gradients);
//  * the sum of the gradients of a tensor that feeds several consumers
//    (the autograd engine would add them pairwise with ATen kernels);
//  * the heads' three 1x1 weights of a level packed into one matrix (and the
//    gradient unpacked), with zero columns at the padded SSH channels.
#include "common.h"

namespace jabd {

struct WindowSet {
  jabd_window_copy d[JABD_WINDOW_MAX];
};

// dst[i0][i1][i2] over the destination dims = src[i0][i1][i2] where inside the
// source dims, else fill.  blockIdx.y = descriptor.
__global__ void window_copy_kernel(const WindowSet ws) {
  const jabd_window_copy& w = ws.d[blockIdx.y];
  const int64_t n = (int64_t)w.d0 * w.d1 * w.d2;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i2 = e % w.d2, r = e / w.d2;
    const int64_t i1 = r % w.d1, i0 = r / w.d1;
    float v = w.fill;
    if (i0 < w.s0 && i1 < w.s1 && i2 + w.off2 < w.s2)
      v = w.scale * w.src[(i0 * w.s1 + i1) * w.s2 + i2 + w.off2];
    w.dst[e] = v;
  }
}

__global__ void transpose_kernel(const float* __restrict__ src, int rows, int cols,
                                 float* __restrict__ dst) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e % rows, r = e / rows;  // dst[r][c] = src[c][r], dst is [cols][rows]
    dst[e] = src[c * cols + r];
  }
}

// out[c] = sum over rows r of part[r][c] in a fixed order: a workgroup owns
// CB channels; its RG = 1024 / CB row groups each sum rows g, g + RG, ... in
// order, then the RG partials are added pairwise in a fixed tree (the
// decomposition depends only on (rows, C), so the result is deterministic).
// One thread per channel walking all rows serially took ~290 us per call at
// 2048 rows (15 calls per MNv3 training step).
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part, int64_t rows,
                                                      int C, int CB, float* __restrict__ out) {
  __shared__ float red[1024];
  const int RG = 1024 / CB;
  const int t = threadIdx.x, cl = t % CB, g = t / CB;
  const int c = blockIdx.x * CB + cl;
  float s = 0.f;
  if (g < RG && c < C) {
    const float* p = part + c;
    int64_t r = g;
    for (; r + 3 * RG < rows; r += 4 * RG) {
      const float v0 = p[r * C], v1 = p[(r + RG) * C], v2 = p[(r + 2 * RG) * C],
                  v3 = p[(r + 3 * RG) * C];
      s += v0; s += v1; s += v2; s += v3;
    }
    for (; r < rows; r += RG) s += p[r * C];
  }
  red[t] = s;
  __syncthreads();
  for (int h = 1; h < RG; h <<= 1) {  // pairwise: group g += group g + h
    if (g % (2 * h) == 0 && g + h < RG) red[t] += red[t + h * CB];
    __syncthreads();
  }
  if (g == 0 && c < C) out[c] = red[t];
}

struct SumSet {
  const float* in[JABD_SUM_MAX];
};

// out = in[0] + in[1] + ... (left to right, as autograd's pairwise adds)
__global__ void sum_multi_kernel(const SumSet ss, int n_in, int64_t n, float* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    float v = ss.in[0][e];
    for (int i = 1; i < n_in; ++i) v += ss.in[i][e];
    out[e] = v;
  }
}

__global__ void weighted_sum3_kernel(const float* a, const float* b, const float* c, float wa,
                                     float* out) {
  // rounded like the three separate torch ops (no fma contraction)
  if (threadIdx.x == 0) out[0] = __fadd_rn(__fadd_rn(__fmul_rn(wa, a[0]), b[0]), c[0]);
}

// out[(t * cin + ci) * cout + co] = w[(co * cin + ci) * taps + t]
__global__ void conv_w2d_kernel(const float* __restrict__ w, int cout, int cin, int taps,
                                float* __restrict__ out) {
  const int n = cout * cin * taps;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int co = e % cout, r = e / cout;
    const int ci = r % cin, t = r / cin;
    out[e] = w[(co * cin + ci) * taps + t];
  }
}

// Heads weights of one pyramid level: rows 0-7 BboxHead, 8-11 ClassHead,
// 12-31 LandmarkHead (nets/retinaface_r.py:19-58, 1x1 convs over C feature
// channels) as one [32][Cf] matrix whose column for feature channel j is
// map(j) = j < half + q ? j : j + qp - q (the SSH output stored with its two
// q-channel branches padded to qp; q == qp: identity).  dir 0 packs (zero
// columns at the pad channels, bias [32]); dir 1 unpacks a [32][Cf] weight
// gradient into the three [rows][C] gradients.
__global__ void heads_wpack_kernel(float* __restrict__ wb, float* __restrict__ wc,
                                   float* __restrict__ wl, const float* __restrict__ bb,
                                   const float* __restrict__ bc, const float* __restrict__ bl,
                                   int C, int half, int q, int qp, float* __restrict__ wt, int Cf,
                                   float* __restrict__ bias, int dir) {
  const int n = 32 * Cf;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int r = e / Cf, col = e - r * Cf;
    // feature channel of this column, or -1 at a pad column
    int j = col;
    if (col >= half + q) j = col < half + qp ? -1 : col - (qp - q);
    if (j >= C) j = -1;
    float* src = r < 8 ? wb + r * C : (r < 12 ? wc + (r - 8) * C : wl + (r - 12) * C);
    if (dir == 0) {
      wt[e] = j >= 0 ? src[j] : 0.f;
    } else if (j >= 0) {
      src[j] = wt[e];
    }
  }
  if (dir == 0 && blockIdx.x == 0 && threadIdx.x < 32) {
    const int r = threadIdx.x;
    bias[r] = r < 8 ? bb[r] : (r < 12 ? bc[r - 8] : bl[r - 12]);
  }
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_sum_multi_f32(int32_t n_in, const float* const* in, int64_t n, float* out,
                                  jabd_stream_t stream) {
  JABD_REQUIRE(n_in >= 1 && n_in <= JABD_SUM_MAX && in && out && n >= 0,
               "sum_multi: n_in = %d (1..%d)", n_in, JABD_SUM_MAX);
  if (n == 0) return JABD_OK;
  SumSet ss;
  for (int i = 0; i < n_in; ++i) {
    JABD_REQUIRE(in[i], "sum_multi: null input %d", i);
    ss.in[i] = in[i];
  }
  const unsigned gx = (unsigned)(cdiv(n, 256) < 2048 ? cdiv(n, 256) : 2048);
  sum_multi_kernel<<<gx, 256, 0, as_stream(stream)>>>(ss, n_in, n, out);
  return check_launch("sum_multi");
}

extern "C" int jabd_weighted_sum3_f32(const float* a, const float* b, const float* c, float wa,
                                      float* out, jabd_stream_t stream) {
  JABD_REQUIRE(a && b && c && out, "weighted_sum3: null pointer");
  weighted_sum3_kernel<<<1, 64, 0, as_stream(stream)>>>(a, b, c, wa, out);
  return check_launch("weighted_sum3");
}

extern "C" int jabd_conv_w2d_f32(const float* w, int32_t cout, int32_t cin, int32_t taps,
                                 float* out, jabd_stream_t stream) {
  JABD_REQUIRE(w && out && cout > 0 && cin > 0 && taps > 0 &&
                   (int64_t)cout * cin * taps < ((int64_t)1 << 31),
               "conv_w2d: bad arguments");
  const int n = cout * cin * taps;
  conv_w2d_kernel<<<(unsigned)cdiv(n, 256), 256, 0, as_stream(stream)>>>(w, cout, cin, taps, out);
  return check_launch("conv_w2d");
}

extern "C" int jabd_heads_wpack_f32(float* wb, float* wc, float* wl, const float* bb,
                                    const float* bc, const float* bl, int32_t C, int32_t half,
                                    int32_t q, int32_t qp, float* wt, int32_t Cf, float* bias,
                                    int32_t dir, jabd_stream_t stream) {
  JABD_REQUIRE(wb && wc && wl && wt && C > 0 && Cf >= C && q >= 0 && qp >= q && half >= 0 &&
                   (dir == 1 || (bb && bc && bl && bias)) && (dir == 0 || dir == 1) &&
                   (q == qp ? Cf == C : Cf == half + 2 * qp && C == half + 2 * q),
               "heads_wpack: bad arguments (C %d Cf %d half %d q %d qp %d dir %d)", C, Cf, half,
               q, qp, dir);
  const int n = 32 * Cf;
  heads_wpack_kernel<<<(unsigned)cdiv(n, 256), 256, 0, as_stream(stream)>>>(
      wb, wc, wl, bb, bc, bl, C, half, q, qp, wt, Cf, bias, dir);
  return check_launch("heads_wpack");
}

extern "C" int jabd_window_copy_multi_f32(int32_t n, const jabd_window_copy* descs,
                                          jabd_stream_t stream) {
  JABD_REQUIRE(n >= 0 && n <= JABD_WINDOW_MAX && (n == 0 || descs),
               "window_copy: n = %d (0..%d)", n, JABD_WINDOW_MAX);
  if (n == 0) return JABD_OK;
  WindowSet ws;
  int64_t most = 1;
  for (int i = 0; i < n; ++i) {
    const jabd_window_copy& w = descs[i];
    JABD_REQUIRE(w.dst && w.d0 >= 0 && w.d1 >= 0 && w.d2 >= 0 && w.s0 >= 0 && w.s1 >= 0 &&
                     w.s2 >= 0 && w.off2 >= 0 && (w.src || (int64_t)w.s0 * w.s1 * w.s2 == 0),
                 "window_copy: bad descriptor %d", i);
    ws.d[i] = w;
    const int64_t m = (int64_t)w.d0 * w.d1 * w.d2;
    if (m > most) most = m;
  }
  const unsigned gx = (unsigned)(cdiv(most, 256) < 1024 ? cdiv(most, 256) : 1024);
  window_copy_kernel<<<dim3(gx, n), 256, 0, as_stream(stream)>>>(ws);
  return check_launch("window_copy");
}

extern "C" int jabd_transpose_f32(const float* src, int32_t rows, int32_t cols, float* dst,
                                  jabd_stream_t stream) {
  JABD_REQUIRE(src && dst && rows > 0 && cols > 0, "transpose: bad arguments");
  const int64_t n = (int64_t)rows * cols;
  const unsigned gx = (unsigned)(cdiv(n, 256) < 1024 ? cdiv(n, 256) : 1024);
  transpose_kernel<<<gx, 256, 0, as_stream(stream)>>>(src, rows, cols, dst);
  return check_launch("transpose");
}

extern "C" int jabd_colsum_f32(const float* part, int64_t rows, int32_t C, float* out,
                               jabd_stream_t stream) {
  JABD_REQUIRE(part && out && rows > 0 && C > 0, "colsum: bad arguments");
  const int CB = C < 64 ? C : 64;
  colsum_kernel<<<(unsigned)cdiv(C, CB), 1024, 0, as_stream(stream)>>>(part, rows, C, CB, out);
  return check_launch("colsum");
}
