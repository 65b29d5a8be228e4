// Attention core of the general-width NLM — the BECA variant's NLM(40) with
// ch = 40 and PSP sizes (1, 3, 6, 8), S = 110 (train_mobilenetV3_ecagai.py:
// 182-234); the ch = 4 NLM of the other models has its own fused kernels
// (head.hip, nlm_train.hip).
//
//   ctx[p] = softmax_s(q[p] . K[s]) . V          (:216-226, scale 1 ** -.5 = 1)
//
// q [B, P, CH] (the f_query 1x1 conv of the up-sampled map, NHWC), K/V
// [B, S, CH] (f_key / f_value of the PSP-pooled map: pooling is linear with
// unit-sum bins, so psp(conv(x)) = conv(psp(x)) and the projections run on
// the S pooled rows).  One thread per pixel; the image's K and V sit in LDS
// and every lane reads the same row (broadcast), so the loop is VALU bound
// (2*CH FMAs + one exp per (pixel, s)).  The forward is a single-pass online
// softmax (running max m, denominator l, rescaled accumulator) and saves
// lse = m + log(l) per pixel; it never materialises the [P, S] map.
//
// Backward, per pixel (P_s = exp(q.K_s - lse), dP_s = dctx.V_s):
//   D     = sum_s P_s dP_s = dctx . ctx          (ctx = the forward output)
//   dS_s  = P_s (dP_s - D)
//   dq    = sum_s dS_s K_s
// and P / dS are written S-major ([B, S, P], coalesced over pixels) for the
// two per-image reductions dK = dS . q and dV = P . dctx.
#include <math.h>

#include <algorithm>

#include "common.h"

namespace jabd {

template <int CH>
__device__ __forceinline__ void load_row(const float* __restrict__ src, float (&v)[CH]) {
#pragma unroll
  for (int c = 0; c < CH; c += 4) {
    const float4 t = *reinterpret_cast<const float4*>(src + c);
    v[c] = t.x;
    v[c + 1] = t.y;
    v[c + 2] = t.z;
    v[c + 3] = t.w;
  }
}

template <int CH>
__device__ __forceinline__ void store_row(float* __restrict__ dst, const float (&v)[CH], float s) {
#pragma unroll
  for (int c = 0; c < CH; c += 4)
    *reinterpret_cast<float4*>(dst + c) = make_float4(v[c] * s, v[c + 1] * s, v[c + 2] * s,
                                                      v[c + 3] * s);
}

// K then V of image b into LDS (S*CH floats each).
template <int CH>
__device__ __forceinline__ void stage_kv(const float* __restrict__ kp, const float* __restrict__ vp,
                                         int b, int S, float* sK, float* sV) {
  const int n4 = S * CH / 4;
  const float4* k4 = reinterpret_cast<const float4*>(kp + (int64_t)b * S * CH);
  const float4* v4 = reinterpret_cast<const float4*>(vp + (int64_t)b * S * CH);
  for (int i = threadIdx.x; i < n4; i += blockDim.x) {
    reinterpret_cast<float4*>(sK)[i] = k4[i];
    reinterpret_cast<float4*>(sV)[i] = v4[i];
  }
  __syncthreads();
}

template <int CH>
__device__ __forceinline__ float dot_lds(const float (&a)[CH], const float* row) {
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int c = 0; c < CH; c += 4) {
    const float4 k = *reinterpret_cast<const float4*>(row + c);
    s0 = fmaf(a[c], k.x, s0);
    s1 = fmaf(a[c + 1], k.y, s1);
    s0 = fmaf(a[c + 2], k.z, s0);
    s1 = fmaf(a[c + 3], k.w, s1);
  }
  return s0 + s1;
}

template <int CH>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ q,
                                                       const float* __restrict__ kp,
                                                       const float* __restrict__ vp, int P, int S,
                                                       float* __restrict__ ctx,
                                                       float* __restrict__ lse) {
  extern __shared__ float4 attn_sm[];
  float* sK = reinterpret_cast<float*>(attn_sm);
  float* sV = sK + S * CH;
  const int b = blockIdx.y;
  stage_kv<CH>(kp, vp, b, S, sK, sV);
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int64_t row = (int64_t)b * P + p;
  float qv[CH], acc[CH];
  load_row<CH>(q + row * CH, qv);
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int s = 0; s < S; ++s) {
    const float sc = dot_lds<CH>(qv, sK + s * CH);
    if (sc > m) {  // new running max: rescale (exp(-inf) = 0 on the first row)
      const float corr = __expf(m - sc);
      l *= corr;
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] *= corr;
      m = sc;
    }
    const float e = __expf(sc - m);
    l += e;
    const float* vr = sV + s * CH;
#pragma unroll
    for (int c = 0; c < CH; c += 4) {
      const float4 v = *reinterpret_cast<const float4*>(vr + c);
      acc[c] = fmaf(e, v.x, acc[c]);
      acc[c + 1] = fmaf(e, v.y, acc[c + 1]);
      acc[c + 2] = fmaf(e, v.z, acc[c + 2]);
      acc[c + 3] = fmaf(e, v.w, acc[c + 3]);
    }
  }
  store_row<CH>(ctx + row * CH, acc, 1.f / l);
  if (lse) lse[row] = m + __logf(l);
}

template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_kernel(
    const float* __restrict__ q, const float* __restrict__ kp, const float* __restrict__ vp,
    const float* __restrict__ ctx, const float* __restrict__ lse, const float* __restrict__ dctx,
    int P, int S, float* __restrict__ dq, float* __restrict__ pm, float* __restrict__ dsm) {
  extern __shared__ float4 attn_sm[];
  float* sK = reinterpret_cast<float*>(attn_sm);
  float* sV = sK + S * CH;
  const int b = blockIdx.y;
  stage_kv<CH>(kp, vp, b, S, sK, sV);
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int64_t row = (int64_t)b * P + p;
  float qv[CH], g[CH], acc[CH];
  load_row<CH>(q + row * CH, qv);
  load_row<CH>(dctx + row * CH, g);
  load_row<CH>(ctx + row * CH, acc);
  float D = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    D = fmaf(g[c], acc[c], D);
    acc[c] = 0.f;
  }
  const float L = lse[row];
  float* pr = pm + (int64_t)b * S * P + p;
  float* dr = dsm + (int64_t)b * S * P + p;
  for (int s = 0; s < S; ++s) {
    const float* kr = sK + s * CH;
    const float e = __expf(dot_lds<CH>(qv, kr) - L);
    const float ds = e * (dot_lds<CH>(g, sV + s * CH) - D);
#pragma unroll
    for (int c = 0; c < CH; c += 4) {
      const float4 k = *reinterpret_cast<const float4*>(kr + c);
      acc[c] = fmaf(ds, k.x, acc[c]);
      acc[c + 1] = fmaf(ds, k.y, acc[c + 1]);
      acc[c + 2] = fmaf(ds, k.z, acc[c + 2]);
      acc[c + 3] = fmaf(ds, k.w, acc[c + 3]);
    }
    pr[(int64_t)s * P] = e;
    dr[(int64_t)s * P] = ds;
  }
  store_row<CH>(dq + row * CH, acc, 1.f);
}

// y = a + b (+ c): the NLM's residual (context += x) and the FPN's lateral add
// (train_mobilenetV3_ecagai.py:233, 271).
__global__ __launch_bounds__(256) void add3_kernel(const float4* __restrict__ a,
                                                   const float4* __restrict__ b,
                                                   const float4* __restrict__ c, int64_t n4,
                                                   float4* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    const float4 w = b[i];
    v.x += w.x;
    v.y += w.y;
    v.z += w.z;
    v.w += w.w;
    if (c) {
      const float4 u = c[i];
      v.x += u.x;
      v.y += u.y;
      v.z += u.z;
      v.w += u.w;
    }
    y[i] = v;
  }
}

}  // namespace jabd

using namespace jabd;

#define JABD_ATTN_WIDTHS(X) \
  X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

static int attn_check(const char* what, int B, int P, int S, int ch) {
  JABD_REQUIRE(B > 0 && P > 0 && S > 0, "%s: bad shape B=%d P=%d S=%d", what, B, P, S);
  JABD_REQUIRE(ch % 4 == 0 && ch >= 8 && ch <= 64, "%s: ch=%d (multiples of 4 in 8..64)", what,
               ch);
  JABD_REQUIRE((size_t)S * ch * 8 <= 160 * 1024, "%s: K/V of S=%d x ch=%d exceed LDS", what, S,
               ch);
  return JABD_OK;
}

extern "C" int jabd_nlm_attn_fwd_f32(const float* q, const float* kp, const float* vp, int32_t B,
                                     int32_t P, int32_t S, int32_t ch, float* ctx, float* lse,
                                     jabd_stream_t stream) {
  JABD_REQUIRE(q && kp && vp && ctx, "nlm_attn_fwd: null pointer");
  if (int e = attn_check("nlm_attn_fwd", B, P, S, ch)) return e;
  const dim3 g((unsigned)cdiv(P, 256), (unsigned)B);
  const size_t sm = (size_t)S * ch * 8;
  hipStream_t st = as_stream(stream);
  switch (ch) {
#define X(C)                                                                     \
  case C:                                                                        \
    if (sm > 65536)                                                              \
      (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<C>,                 \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm); \
    attn_fwd_kernel<C><<<g, 256, sm, st>>>(q, kp, vp, P, S, ctx, lse); \
    break;
    JABD_ATTN_WIDTHS(X)
#undef X
  }
  return check_launch("nlm_attn_fwd");
}

extern "C" int jabd_nlm_attn_bwd_f32(const float* q, const float* kp, const float* vp,
                                     const float* ctx, const float* lse, const float* dctx,
                                     int32_t B, int32_t P, int32_t S, int32_t ch, float* dq,
                                     float* pmat, float* dsmat, jabd_stream_t stream) {
  JABD_REQUIRE(q && kp && vp && ctx && lse && dctx && dq && pmat && dsmat,
               "nlm_attn_bwd: null pointer");
  if (int e = attn_check("nlm_attn_bwd", B, P, S, ch)) return e;
  const dim3 g((unsigned)cdiv(P, 256), (unsigned)B);
  const size_t sm = (size_t)S * ch * 8;
  hipStream_t st = as_stream(stream);
  switch (ch) {
#define X(C)                                                                                 \
  case C:                                                                                    \
    if (sm > 65536)                                                                          \
      (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<C>,                             \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);        \
    attn_bwd_kernel<C><<<g, 256, sm, st>>>(q, kp, vp, ctx, lse, dctx, P, S, dq, pmat, dsmat); \
    break;
    JABD_ATTN_WIDTHS(X)
#undef X
  }
  return check_launch("nlm_attn_bwd");
}

// dK = dS . q and dV = P . dctx per image: out[b][s][c] = sum_p A[b][s][p] X[b][p][c]
// (A = dsmat / pmat [B, S, P], X = q / dctx [B, P, ch]) on the 16x16x4 fp32
// MFMA: a workgroup takes 16 rows s x all ch columns x one chunk of kDkvChunk
// pixels (its 4 waves a quarter each, summed in LDS), writes the chunk's
// partial sums, and dkv_sum_kernel adds the chunks in order (deterministic).
// Four consecutive pixels per lane and MFMA group: A as one float4 load when
// P % 4 == 0 (rows 16-byte aligned), else four scalar loads.
constexpr int kDkvChunk = 2048;
typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int NT>  // 16-column tiles covering ch
__global__ __launch_bounds__(256) void dkv_part_kernel(const float* __restrict__ dsm,
                                                       const float* __restrict__ pm,
                                                       const float* __restrict__ q,
                                                       const float* __restrict__ dctx, int P,
                                                       int S, int ch, int nchunk,
                                                       float* __restrict__ part) {
  __shared__ float red[4][16][NT * 16];
  const int which = blockIdx.z;  // 0: dK (dsm, q), 1: dV (pm, dctx)
  const float* A = which ? pm : dsm;
  const float* X = which ? dctx : q;
  const int b = blockIdx.y / nchunk, chunk = blockIdx.y - b * nchunk;
  const int s0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i = lane & 15, k = lane >> 4;
  const int srow = s0 + i < S ? s0 + i : S - 1;
  const float* Ab = A + ((int64_t)b * S + srow) * P;
  const float* Xb = X + (int64_t)b * P * ch;
  const bool vec = (P & 3) == 0;  // rows 16-byte aligned
  const int p_beg = chunk * kDkvChunk + wave * (kDkvChunk / 4);
  const int p_end = min(P, p_beg + kDkvChunk / 4);
  f32x4v acc[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) acc[u] = (f32x4v){0.f, 0.f, 0.f, 0.f};
  for (int p = p_beg; p < p_end; p += 16) {
    const int pa = p + 4 * k;  // this lane's four pixels pa .. pa + 3
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec && pa + 3 < p_end) a = *reinterpret_cast<const float4*>(Ab + pa);
    else {
      if (pa < p_end) a.x = Ab[pa];
      if (pa + 1 < p_end) a.y = Ab[pa + 1];
      if (pa + 2 < p_end) a.z = Ab[pa + 2];
      if (pa + 3 < p_end) a.w = Ab[pa + 3];
    }
    const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int c = 16 * u + i;
      float xv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        xv[t] = (c < ch && pa + t < p_end) ? Xb[(int64_t)(pa + t) * ch + c] : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], xv[t], acc[u], 0, 0, 0);
    }
  }
  // acc[u][r] = out[s0 + 4k + r][16u + i]
#pragma unroll
  for (int u = 0; u < NT; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][4 * k + r][16 * u + i] = acc[u][r];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * NT * 16; e += 256) {
    const int r = e / (NT * 16), c = e - r * (NT * 16);
    const float v = ((red[0][r][c] + red[1][r][c]) + red[2][r][c]) + red[3][r][c];
    if (s0 + r < S && c < ch)
      part[(((int64_t)which * gridDim.y + blockIdx.y) * S + s0 + r) * ch + c] = v;
  }
}

// out[which][b][s][c] = sum over the image's chunks, in order
__global__ void dkv_sum_kernel(const float* __restrict__ part, int B, int S, int ch, int nchunk,
                               float* __restrict__ dk, float* __restrict__ dv) {
  const int64_t n = (int64_t)B * S * ch;
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int which = blockIdx.y;
  if (e >= n) return;
  const int64_t b = e / ((int64_t)S * ch), r = e - b * S * ch;
  const float* src = part + ((int64_t)which * B * nchunk + b * nchunk) * S * ch + r;
  float v = 0.f;
  for (int c = 0; c < nchunk; ++c) v += src[(int64_t)c * S * ch];
  (which ? dv : dk)[e] = v;
}

extern "C" int64_t jabd_nlm_attn_dkv_ws_floats(int32_t B, int32_t P, int32_t S, int32_t ch) {
  if (B <= 0 || P <= 0 || S <= 0 || ch <= 0) return 0;
  return 2 * (int64_t)B * cdiv(P, kDkvChunk) * S * ch;
}

extern "C" int jabd_nlm_attn_dkv_f32(const float* dsmat, const float* pmat, const float* q,
                                     const float* dctx, int32_t B, int32_t P, int32_t S,
                                     int32_t ch, float* ws, int64_t ws_floats, float* dk,
                                     float* dv, jabd_stream_t stream) {
  JABD_REQUIRE(dsmat && pmat && q && dctx && ws && dk && dv, "nlm_attn_dkv: null pointer");
  JABD_REQUIRE(B > 0 && P > 0 && S > 0 && ch > 0 && ch <= 64,
               "nlm_attn_dkv: bad shape B=%d P=%d S=%d ch=%d (ch <= 64)", B, P, S, ch);
  JABD_REQUIRE(ws_floats >= jabd_nlm_attn_dkv_ws_floats(B, P, S, ch),
               "nlm_attn_dkv: workspace too small");
  hipStream_t st = as_stream(stream);
  const int nchunk = (int)cdiv(P, kDkvChunk);
  const dim3 g((unsigned)cdiv(S, 16), (unsigned)(B * nchunk), 2);
  const int nt = (ch + 15) / 16;
  if (nt == 1) dkv_part_kernel<1><<<g, 256, 0, st>>>(dsmat, pmat, q, dctx, P, S, ch, nchunk, ws);
  else if (nt == 2) dkv_part_kernel<2><<<g, 256, 0, st>>>(dsmat, pmat, q, dctx, P, S, ch, nchunk, ws);
  else if (nt == 3) dkv_part_kernel<3><<<g, 256, 0, st>>>(dsmat, pmat, q, dctx, P, S, ch, nchunk, ws);
  else dkv_part_kernel<4><<<g, 256, 0, st>>>(dsmat, pmat, q, dctx, P, S, ch, nchunk, ws);
  if (int e = check_launch("nlm_attn_dkv_part")) return e;
  const int64_t n = (int64_t)B * S * ch;
  dkv_sum_kernel<<<dim3((unsigned)cdiv(n, 256), 2), 256, 0, st>>>(ws, B, S, ch, nchunk, dk, dv);
  return check_launch("nlm_attn_dkv_sum");
}

extern "C" int jabd_add3_f32(const float* a, const float* b, const float* c, int64_t n, float* y,
                             jabd_stream_t stream) {
  JABD_REQUIRE(a && b && y && n >= 0 && n % 4 == 0, "add3: bad args (n %% 4 == 0 required)");
  JABD_REQUIRE(((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)y) % 16 == 0,
               "add3: pointers must be 16-byte aligned");
  if (n == 0) return JABD_OK;
  const int64_t n4 = n / 4;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n4, 256), 8192);
  add3_kernel<<<grid, 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
      reinterpret_cast<const float4*>(c), n4, reinterpret_cast<float4*>(y));
  return check_launch("add3");
}
