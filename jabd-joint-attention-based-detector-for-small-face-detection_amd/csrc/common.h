// Shared helpers for libjabd: status/error plumbing and launch checks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/jabd.h"

namespace jabd {

// Thread-local last-error text (DataParallel threads / DDP ranks call
// concurrently; each sees only its own message).
void set_error(const char* fmt, ...);

inline hipStream_t as_stream(jabd_stream_t s) {
  return reinterpret_cast<hipStream_t>(s);
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return JABD_EHIP;
  }
  return JABD_OK;
}

// nn.Hardsigmoid / nn.Hardswish (relu6(x + 3) / 6 and x * that) as
// clamp(x/6 + 1/2, 0, 1): one fma + one med3 (+ one mul) instead of add, max,
// min, mul (, mul).  Within 2 ulp of the reference formula.
__device__ __forceinline__ float hsigmoid_f(float v) {
  return __builtin_amdgcn_fmed3f(fmaf(v, 1.f / 6.f, 0.5f), 0.f, 1.f);
}
__device__ __forceinline__ float hswish_f(float v) { return v * hsigmoid_f(v); }
// ReLU with torch.relu's NaN rule (NaN stays NaN): one v_maximum_f32.  Every
// kernel's ReLU goes through this, so fused and unfused forms of a layer agree
// on NaN inputs too (fmaxf and `v > 0 ? v : 0` both map NaN to 0).
__device__ __forceinline__ float relu_f(float v) { return __builtin_elementwise_maximum(v, 0.f); }

// c + a * b per component as two packed v_pk_fma_f32 (one IEEE fma per
// element, the same result as four fmaf; the compiler emits scalar v_fma_f32
// for the float4 form, half the VALU rate).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 fma4pk(float4 a, float4 b, float4 c) {
  const f32x2_t r0 =
      __builtin_elementwise_fma((f32x2_t){a.x, a.y}, (f32x2_t){b.x, b.y}, (f32x2_t){c.x, c.y});
  const f32x2_t r1 =
      __builtin_elementwise_fma((f32x2_t){a.z, a.w}, (f32x2_t){b.z, b.w}, (f32x2_t){c.z, c.w});
  return make_float4(r0.x, r0.y, r1.x, r1.y);
}

// BatchNorm + activation applied on load by the BN-input depthwise kernels
// (dwconv.hip forward, train.hip weight gradient; both use this, so they see
// the same values): act(z), z = fma((x - mean) * invstd, gamma, beta) — the
// exact fp32 operation order of train.hip's bn_act_fwd and of the mask the
// BN backward kernels (bn_bwd_*, dw_dgrad_bn) derive, so the forward's
// activation region and the backward's mask agree element for element (a
// folded x * a + c rounds differently next to a kink).  Packed: one
// v_pk_add, one v_pk_mul and one v_pk_fma per two elements.
struct DwBnCoef {
  float4 nmu, is, g, b;  // -mean, invstd, gamma, beta
};

__device__ __forceinline__ DwBnCoef dw_bn_coef(const float* mean, const float* invstd,
                                               const float* gamma, const float* beta, int cg) {
  const float4 mu = reinterpret_cast<const float4*>(mean)[cg];
  DwBnCoef k;
  k.nmu = make_float4(-mu.x, -mu.y, -mu.z, -mu.w);
  k.is = reinterpret_cast<const float4*>(invstd)[cg];
  k.g = reinterpret_cast<const float4*>(gamma)[cg];
  k.b = reinterpret_cast<const float4*>(beta)[cg];
  return k;
}

__device__ __forceinline__ float4 dw_bn_z(float4 v, const DwBnCoef& k) {
  // x + (-mean) is x - mean exactly (IEEE); products and fma per element
  const f32x2_t h0 = ((f32x2_t){v.x, v.y} + (f32x2_t){k.nmu.x, k.nmu.y}) * (f32x2_t){k.is.x, k.is.y};
  const f32x2_t h1 = ((f32x2_t){v.z, v.w} + (f32x2_t){k.nmu.z, k.nmu.w}) * (f32x2_t){k.is.z, k.is.w};
  const f32x2_t z0 = __builtin_elementwise_fma(h0, (f32x2_t){k.g.x, k.g.y}, (f32x2_t){k.b.x, k.b.y});
  const f32x2_t z1 = __builtin_elementwise_fma(h1, (f32x2_t){k.g.z, k.g.w}, (f32x2_t){k.b.z, k.b.w});
  return make_float4(z0.x, z0.y, z1.x, z1.y);
}

// act: 1 relu, 2 leaky, 3 hswish (JABD_ACT_*), else identity
__device__ __forceinline__ float4 dw_bn_in(float4 v, const DwBnCoef& k, int act, float slope) {
  float4 z = dw_bn_z(v, k);
  if (act == 1) {
    z.x = relu_f(z.x); z.y = relu_f(z.y); z.z = relu_f(z.z); z.w = relu_f(z.w);
  } else if (act == 2) {
    z.x = z.x > 0.f ? z.x : z.x * slope; z.y = z.y > 0.f ? z.y : z.y * slope;
    z.z = z.z > 0.f ? z.z : z.z * slope; z.w = z.w > 0.f ? z.w : z.w * slope;
  } else if (act == 3) {
    z.x = hswish_f(z.x); z.y = hswish_f(z.y); z.z = hswish_f(z.z); z.w = hswish_f(z.w);
  }
  return z;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace.
struct Carve {
  char* base;
  size_t cap;
  size_t used = 0;
  Carve(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    size_t off = align_up(used);
    used = off + align_up(count * sizeof(T));
    return reinterpret_cast<T*>(base + off);
  }
  bool ok() const { return used <= cap; }
};

// Several (pointer, bytes, 32-bit word) fills in one launch (fill.hip); bytes
// and pointers 4-byte granular; ranges with bytes <= 0 are skipped.
struct FillRange {
  void* ptr;
  int64_t bytes;
  uint32_t value;
};
constexpr int kFillMax = 12;
struct FillArgs {
  FillRange r[kFillMax];
};
int fill_ranges(const FillRange* r, int n, hipStream_t st);

// Size-only twin of Carve, used by the *_workspace_size queries so the
// query and the carve can never disagree.
struct Sizer {
  size_t used = 0;
  template <typename T>
  T* take(size_t count) {
    used = align_up(used) + align_up(count * sizeof(T));
    return nullptr;
  }
};

// n / d for 0 <= n < 2^31 by multiply-high and shift with a host-built
// divisor (a runtime-divisor integer division is ~15-40 instructions)
struct FastDiv {
  uint32_t m, l, d;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((((uint64_t)1 << l) - d) << 32) / d + 1;
  return FastDiv{(uint32_t)m, l, d};
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((uint32_t)n, f.m) + (uint32_t)n) >> f.l);
}

}  // namespace jabd

#define JABD_REQUIRE(cond, ...)      \
  do {                               \
    if (!(cond)) {                   \
      ::jabd::set_error(__VA_ARGS__); \
      return JABD_EINVAL;            \
    }                                \
  } while (0)

#define JABD_HIP(call)                                                   \
  do {                                                                   \
    hipError_t e_ = (call);                                              \
    if (e_ != hipSuccess) {                                              \
      ::jabd::set_error("%s: %s", #call, hipGetErrorString(e_));        \
      return JABD_EHIP;                                                  \
    }                                                                    \
  } while (0)
