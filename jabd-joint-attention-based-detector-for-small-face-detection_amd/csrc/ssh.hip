// A4 SSH tail + heads, eval (nets/layers.py:37-68, nets/retinaface_r.py:
// 17-57,335-343), one launch per pyramid level for the 40-channel SSH of the
// MobileNetV3 detectors (out_channel 40: branches 20 / 10 / 10).
//
// The level's first GEMM (the input-reading conv3X3 and conv5X5_1, fused
// along N) writes relu(conv3X3) [B,h,w,20] and t = leaky(conv5X5_1)
// [B,h,w,12] (10 channels + 2 zero pad).  This kernel does everything after
// it on one output tile per workgroup:
//   u   = leaky(conv7X7_2(t))            on the tile + 1-pixel halo (LDS)
//   c52 = conv5X5_2(t), c73 = conv7x7_3(u) on the tile
//   f   = relu(cat[conv3X3, c52, c73])   (40 channels, registers)
//   the three 1x1 heads on f (+ the eval softmax of each anchor's 2 logits),
//   stored straight into loc / conf / landm [B, A, k] at the level's anchor
//   offset (the reference's permute(0,2,3,1).view + cat order).
// It replaces three launches per level (the 10-channel 3x3 GEMMs, which ran
// at 4-14 % of their roofline, and heads_kernel) and the 40-channel feature
// tensor's write and re-read.  Arithmetic: one thread per pixel, fp32 FMAs
// with the (BN-folded) weights as wave-uniform scalar operands, taps in
// (kh, kw, channel) order, then the bias-initialised head sums in channel
// order — one fixed operation sequence per output (deterministic, batch-
// invariant).
#include "common.h"

namespace jabd {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kSshTH = 8, kSshTW = 32;           // output tile (16 MFMA pixel blocks)
constexpr int kSshQ = 10, kSshQP = 12;           // branch width, padded (3 float4)
constexpr int kSshR1H = kSshTH + 2, kSshR1W = kSshTW + 2;  // conv7X7_2 region
constexpr int kSshR0H = kSshTH + 4, kSshR0W = kSshTW + 4;  // t region
constexpr int kSshR1PX = kSshR1H * kSshR1W;                // 340
constexpr int kSshR1BLK = (kSshR1PX + 15) / 16;            // 22
// packed weights, float4 units, MFMA A fragments (lane = 16 g + j; e = the
// component = the MFMA of a 4-MFMA k group, channel 4g + e of a 16-channel
// k chunk):
//   conv c (0 conv5X5_2, 1 conv7X7_2, 2 conv7x7_3), tap p: [c][p][lane] =
//     W_c[n = j][p][ch = 4g + e]  (0 for n >= 10 or ch >= 10)
//   conv biases [c][g] = b_c[4g .. 4g + 3]  (acc init of lane (px j, g))
//   heads, k chunk kc, n tile nt: [kc][nt][lane] = Wh[16 nt + j][ch(kc, 4g + e)]
//     with ch(0, k) = k (conv3X3 0-15), ch(1, k) = 16 + k for k < 4 (conv3X3
//     16-19), ch(2, k) = 20 + k, ch(3, k) = 30 + k for k < 10 (the branches)
//   heads biases [nt][g] = bh[16 nt + 4g .. + 3]
constexpr int kSshOffCB = 3 * 9 * 64;           // conv biases
constexpr int kSshOffH = kSshOffCB + 3 * 4;     // heads A fragments
constexpr int kSshOffHB = kSshOffH + 4 * 2 * 64;
constexpr int kSshWF4 = kSshOffHB + 2 * 4;      // float4 total

__device__ __forceinline__ f32x4_t ssh_mfma4(const float4& a, const float4& b, f32x4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

// acc = bias + one 3x3 10->10 conv of a 16-pixel block: B fragment of tap p
// for lane (j, g) = region[(idx_j + tapoff(p)) * 3 + g] (g < 3; g = 3 reads 0)
template <int RW>
__device__ __forceinline__ f32x4_t ssh_conv_blk(const float4* __restrict__ reg, int idx, int g,
                                                const float4 (&A)[9], f32x4_t acc) {
  float4 bv[9];
#pragma unroll
  for (int p = 0; p < 9; ++p)
    bv[p] = g < 3 ? reg[(idx + (p / 3) * RW + p % 3) * 3 + g] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int p = 0; p < 9; ++p) acc = ssh_mfma4(A[p], bv[p], acc);
  return acc;
}

__global__ __launch_bounds__(256) void ssh_tail_heads_kernel(
    const float* __restrict__ c33, int64_t c33_bs, int c33_ps, const float* __restrict__ t,
    int64_t t_bs, int H, int W, int tiles_w, const float4* __restrict__ wb, float leaky,
    int64_t A, int64_t a_off, int softmax, float* __restrict__ loc, float* __restrict__ conf,
    float* __restrict__ landm) {
  __shared__ float4 r0[kSshR0H * kSshR0W * 3];  // t, zero outside the image
  __shared__ float4 r1[kSshR1PX * 3];           // leaky(conv7X7_2(t)), zero outside
  const int b = blockIdx.y;
  const int ty = blockIdx.x / tiles_w, tx = blockIdx.x - ty * tiles_w;
  const int oy0 = ty * kSshTH, ox0 = tx * kSshTW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 15, g = lane >> 4;
  const float4* tb = reinterpret_cast<const float4*>(t + (int64_t)b * t_bs);
  // t region: rows oy0 - 2 .. oy0 + TH + 1, columns ox0 - 2 .. ox0 + TW + 1
  for (int i = tid; i < kSshR0H * kSshR0W * 3; i += 256) {
    const int px = i / 3, q = i - px * 3;
    const int ry = px / kSshR0W, rx = px - ry * kSshR0W;
    const int y = oy0 - 2 + ry, x = ox0 - 2 + rx;
    r0[i] = ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
                ? tb[((int64_t)y * W + x) * 3 + q]
                : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 Aw[9];
#pragma unroll
  for (int p = 0; p < 9; ++p) Aw[p] = wb[(1 * 9 + p) * 64 + lane];  // conv7X7_2
  const float4 b72 = wb[kSshOffCB + 1 * 4 + g];
  __syncthreads();
  // conv7X7_2 + leaky on the tile and its 1-pixel halo (22 blocks over 4 waves)
  for (int pb = wave; pb < kSshR1BLK; pb += 4) {
    const int px = pb * 16 + j;
    const int pq = px < kSshR1PX ? px : 0;
    const int ry = pq / kSshR1W, rx = pq - ry * kSshR1W;
    f32x4_t acc = (f32x4_t){b72.x, b72.y, b72.z, b72.w};
    acc = ssh_conv_blk<kSshR0W>(r0, ry * kSshR0W + rx, g, Aw, acc);
    const int y = oy0 - 1 + ry, x = ox0 - 1 + rx;
    const bool in = px < kSshR1PX && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    float4 o;
    o.x = in ? (acc[0] > 0.f ? acc[0] : acc[0] * leaky) : 0.f;
    o.y = in ? (acc[1] > 0.f ? acc[1] : acc[1] * leaky) : 0.f;
    o.z = in ? (acc[2] > 0.f ? acc[2] : acc[2] * leaky) : 0.f;
    o.w = in ? (acc[3] > 0.f ? acc[3] : acc[3] * leaky) : 0.f;
    if (px < kSshR1PX && g < 3) r1[px * 3 + g] = o;
  }
  __syncthreads();
  // per output block (4 per wave): conv5X5_2, conv7x7_3, conv3X3 (global),
  // then the heads on relu(cat); all operands in the MFMA fragment layout
  const float4 b52 = wb[kSshOffCB + 0 * 4 + g], b73 = wb[kSshOffCB + 2 * 4 + g];
  float4 A52[9], A73[9];
#pragma unroll
  for (int p = 0; p < 9; ++p) {
    A52[p] = wb[(0 * 9 + p) * 64 + lane];
    A73[p] = wb[(2 * 9 + p) * 64 + lane];
  }
#pragma unroll 1
  for (int pb = wave; pb < kSshTH * kSshTW / 16; pb += 4) {
    const int p = pb * 16 + j;
    const int ly = p / kSshTW, lx = p - ly * kSshTW;
    const int y = oy0 + ly, x = ox0 + lx;
    const bool pv = y < H && x < W;
    f32x4_t a52 = (f32x4_t){b52.x, b52.y, b52.z, b52.w};
    a52 = ssh_conv_blk<kSshR0W>(r0, (ly + 1) * kSshR0W + lx + 1, g, A52, a52);
    f32x4_t a73 = (f32x4_t){b73.x, b73.y, b73.z, b73.w};
    a73 = ssh_conv_blk<kSshR1W>(r1, ly * kSshR1W + lx, g, A73, a73);
    const float4* cp = reinterpret_cast<const float4*>(
        c33 + (int64_t)b * c33_bs + ((int64_t)(pv ? y : 0) * W + (pv ? x : 0)) * c33_ps);
    const float4 k0 = cp[g];                                                   // ch 4g..4g+3
    const float4 k1 = g == 0 ? cp[4] : make_float4(0.f, 0.f, 0.f, 0.f);      // ch 16..19
    const float4 k2 = make_float4(relu_f(a52[0]), relu_f(a52[1]), relu_f(a52[2]), relu_f(a52[3]));
    const float4 k3 = make_float4(relu_f(a73[0]), relu_f(a73[1]), relu_f(a73[2]), relu_f(a73[3]));
    float4 o[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const float4 hb = wb[kSshOffHB + nt * 4 + g];
      f32x4_t h = (f32x4_t){hb.x, hb.y, hb.z, hb.w};
      h = ssh_mfma4(wb[kSshOffH + (0 * 2 + nt) * 64 + lane], k0, h);
      h = ssh_mfma4(wb[kSshOffH + (1 * 2 + nt) * 64 + lane], k1, h);
      h = ssh_mfma4(wb[kSshOffH + (2 * 2 + nt) * 64 + lane], k2, h);
      h = ssh_mfma4(wb[kSshOffH + (3 * 2 + nt) * 64 + lane], k3, h);
      o[nt] = make_float4(h[0], h[1], h[2], h[3]);
    }
    // lane (j, g) holds head outputs 4g..4g+3 (o[0]) and 16 + 4g..+3 (o[1]):
    // g 0-1 loc, g 2 conf (softmax per anchor pair), g 3 + o[1] landm
    if (softmax && g == 2) {  // F.softmax over each anchor's 2 logits (as heads_kernel)
      float m = fmaxf(o[0].x, o[0].y), e0 = expf(o[0].x - m), e1 = expf(o[0].y - m), s = e0 + e1;
      o[0].x = e0 / s; o[0].y = e1 / s;
      m = fmaxf(o[0].z, o[0].w); e0 = expf(o[0].z - m); e1 = expf(o[0].w - m); s = e0 + e1;
      o[0].z = e0 / s; o[0].w = e1 / s;
    }
    if (pv) {
      const int64_t row = (int64_t)b * A + a_off + ((int64_t)y * W + x) * 2;  // anchor 0 row
      if (g < 2)
        reinterpret_cast<float4*>(loc + row * 4)[g] = o[0];
      else if (g == 2)
        *reinterpret_cast<float4*>(conf + row * 2) = o[0];
      else
        *reinterpret_cast<float4*>(landm + row * 10) = o[0];
      reinterpret_cast<float4*>(landm + row * 10 + 4)[g] = o[1];
    }
  }
}

}  // namespace jabd

extern "C" int64_t jabd_ssh_tail_weight_floats(void) { return 4 * (int64_t)jabd::kSshWF4; }

extern "C" int jabd_ssh_tail_heads_f32(const float* c33, int64_t c33_bs, int32_t c33_ps,
                                       const float* t, int64_t t_bs, int32_t B, int32_t H,
                                       int32_t W, const float* wb, float leaky, int64_t A,
                                       int64_t a_off, int32_t softmax, float* loc, float* conf,
                                       float* landm, jabd_stream_t stream) {
  using namespace jabd;
  JABD_REQUIRE(c33 && t && wb && loc && conf && landm && B > 0 && H > 0 && W > 0,
               "ssh_tail_heads: bad args");
  JABD_REQUIRE(c33_ps >= 20 && c33_ps % 4 == 0 && t_bs >= (int64_t)H * W * kSshQP &&
                   c33_bs >= (int64_t)H * W * c33_ps,
               "ssh_tail_heads: strides (c33 >= 20 channels, t = 12 channels per pixel)");
  JABD_REQUIRE(a_off % 2 == 0 && A % 2 == 0 && a_off + 2 * (int64_t)H * W <= A,
               "ssh_tail_heads: anchor range");
  const int tiles_w = (int)cdiv(W, kSshTW);
  const int64_t tiles = cdiv(H, kSshTH) * (int64_t)tiles_w;
  JABD_REQUIRE(tiles < (1ll << 31) && B <= 65535, "ssh_tail_heads: grid too large");
  dim3 g((unsigned)tiles, (unsigned)B);
  ssh_tail_heads_kernel<<<g, 256, 0, as_stream(stream)>>>(c33, c33_bs, c33_ps, t, t_bs, H, W,
                                                           tiles_w, reinterpret_cast<const float4*>(wb), leaky, A, a_off, softmax,
                                                           loc, conf, landm);
  return check_launch("ssh_tail_heads");
}
