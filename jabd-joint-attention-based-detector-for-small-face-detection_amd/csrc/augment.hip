// GPU data augmentation — utils/dataloader.py:71-149 (DataGenerator.get_random_data)
// plus the __getitem__ tail (:62-64: preprocess_input, HWC -> CHW), for one image
// whose random draws (nw, nh, dx, dy, flip, hue, sat, val) the host has made in
// the reference's np.random order.  Two launches:
//   1. horizontal pass of PIL's Image.resize(BICUBIC) (Pillow Resample.c restated:
//      bicubic a = -0.5, support 2 * max(scale, 1), double coefficients normalised
//      per output pixel then rounded to 22-bit fixed point, uint8 intermediate
//      with clip8) into a [ih, nw, 3] u8 workspace;
//   2. per canvas pixel: the vertical pass, paste at (dx, dy) on grey 128, the
//      left-right flip, cv2 RGB2HSV (float), the hue/sat/val jitter and clamps of
//      :107-115, cv2 HSV2RGB (float) * 255, minus (104, 117, 123), NCHW store.
// Compiled with -ffp-contract=off: every fp op rounds as the restated code's.
#include <float.h>
#include <math.h>

#include "common.h"

namespace jabd {

constexpr int kPrecBits = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ double bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

struct Taps {
  int xmin, n;
  double center, ss, ww;
};

// precompute_coeffs for output index o (in0 = 0, in1 = in).
__device__ __forceinline__ Taps taps_for(int o, int in, int out) {
  const double scale = (double)in / out;
  const double fscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * fscale;
  Taps t;
  t.center = (o + 0.5) * scale;
  t.ss = 1.0 / fscale;
  int xmin = (int)(t.center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(t.center + support + 0.5);
  if (xmax > in) xmax = in;
  t.xmin = xmin;
  t.n = xmax - xmin;
  double ww = 0.0;
  for (int x = 0; x < t.n; ++x) ww += bicubic((x + xmin - t.center + 0.5) * t.ss);
  t.ww = ww;
  return t;
}

__device__ __forceinline__ int tap_fixed(const Taps& t, int x) {
  double k = bicubic((x + t.xmin - t.center + 0.5) * t.ss);
  if (t.ww != 0.0) k /= t.ww;
  return k < 0 ? (int)(-0.5 + k * (1 << kPrecBits)) : (int)(0.5 + k * (1 << kPrecBits));
}

__device__ __forceinline__ uint8_t clip8(int ss) {
  int v = ss >> kPrecBits;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__global__ __launch_bounds__(256) void resample_h_kernel(const uint8_t* __restrict__ src, int ih,
                                                         int iw, int nw,
                                                         uint8_t* __restrict__ tmp) {
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (xx >= nw) return;
  const Taps t = taps_for(xx, iw, nw);
  const uint8_t* row = src + (int64_t)y * iw * 3;
  int s0 = 1 << (kPrecBits - 1), s1 = s0, s2 = s0;
  for (int x = 0; x < t.n; ++x) {
    const int k = tap_fixed(t, x);
    const uint8_t* p = row + (int64_t)(x + t.xmin) * 3;
    s0 += p[0] * k;
    s1 += p[1] * k;
    s2 += p[2] * k;
  }
  uint8_t* o = tmp + ((int64_t)y * nw + xx) * 3;
  o[0] = clip8(s0);
  o[1] = clip8(s1);
  o[2] = clip8(s2);
}

__global__ __launch_bounds__(256) void augment_kernel(const uint8_t* __restrict__ tmp, int ih,
                                                      int nw, int nh, int h, int w, int dx,
                                                      int dy, int flip, float hue360, float sat,
                                                      float val, float* __restrict__ dst) {
  const int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pix >= (int64_t)h * w) return;
  const int y = (int)(pix / w), x = (int)(pix - (int64_t)y * w);
  const int cx = flip ? w - 1 - x : x;  // FLIP_LEFT_RIGHT of the pasted canvas
  const int rx = cx - dx, ry = y - dy;
  float rgb[3] = {128.f, 128.f, 128.f};
  if (rx >= 0 && rx < nw && ry >= 0 && ry < nh) {
    const Taps t = taps_for(ry, ih, nh);
    int s0 = 1 << (kPrecBits - 1), s1 = s0, s2 = s0;
    for (int k = 0; k < t.n; ++k) {
      const int c = tap_fixed(t, k);
      const uint8_t* p = tmp + ((int64_t)(k + t.xmin) * nw + rx) * 3;
      s0 += p[0] * c;
      s1 += p[1] * c;
      s2 += p[2] * c;
    }
    rgb[0] = (float)clip8(s0);
    rgb[1] = (float)clip8(s1);
    rgb[2] = (float)clip8(s2);
  }
  // np.array(image, np.float32) / 255, cv2 RGB2HSV (float, hrange 360)
  const float r = rgb[0] / 255.f, g = rgb[1] / 255.f, b = rgb[2] / 255.f;
  float v = r, vmin = r;
  if (v < g) v = g;
  if (v < b) v = b;
  if (vmin > g) vmin = g;
  if (vmin > b) vmin = b;
  float diff = v - vmin;
  float s = diff / (float)(fabsf(v) + FLT_EPSILON);
  diff = (float)(60. / (diff + FLT_EPSILON));
  float hh;
  if (v == r)
    hh = (g - b) * diff;
  else if (v == g)
    hh = (b - r) * diff + 120.f;
  else
    hh = (r - g) * diff + 240.f;
  if (hh < 0) hh += 360.f;
  // :107-115 (the wrap is at 1, as written in the reference)
  hh += hue360;
  if (hh > 1.f) hh -= 1.f;
  if (hh < 0.f) hh += 1.f;
  s *= sat;
  v *= val;
  if (hh > 360.f) hh = 360.f;
  if (s > 1.f) s = 1.f;
  if (v > 1.f) v = 1.f;
  if (hh < 0.f) hh = 0.f;
  if (s < 0.f) s = 0.f;
  if (v < 0.f) v = 0.f;
  // cv2 HSV2RGB (float)
  float ro, go, bo;
  if (s == 0.f) {
    ro = go = bo = v;
  } else {
    const int sector_data[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1},
                                   {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
    hh *= 6.f / 360.f;
    if (hh < 0) {
      do hh += 6; while (hh < 0);
    } else if (hh >= 6) {
      do hh -= 6; while (hh >= 6);
    }
    int sector = (int)floorf(hh);
    hh -= sector;
    if ((unsigned)sector >= 6u) { sector = 0; hh = 0.f; }
    float tab[4];
    tab[0] = v;
    tab[1] = v * (1.f - s);
    tab[2] = v * (1.f - s * hh);
    tab[3] = v * (1.f - s * (1.f - hh));
    bo = tab[sector_data[sector][0]];
    go = tab[sector_data[sector][1]];
    ro = tab[sector_data[sector][2]];
  }
  const int64_t plane = (int64_t)h * w;
  dst[pix] = ro * 255.f - 104.f;
  dst[plane + pix] = go * 255.f - 117.f;
  dst[2 * plane + pix] = bo * 255.f - 123.f;
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_augment_workspace_size(int ih, int nw, size_t* bytes) {
  JABD_REQUIRE(bytes && ih >= 0 && nw >= 0, "augment_workspace_size: bad args");
  *bytes = (size_t)ih * nw * 3;
  return JABD_OK;
}

extern "C" int jabd_augment_u8(const uint8_t* src, int ih, int iw, int nw, int nh, int h, int w,
                               int dx, int dy, int flip, double hue, float sat, float val,
                               float* dst, void* ws, size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(ih > 0 && iw > 0 && nw > 0 && nh > 0 && h > 0 && w > 0, "augment: bad size");
  JABD_REQUIRE(src && dst && ws, "augment: null pointer");
  JABD_REQUIRE(ws_bytes >= (size_t)ih * nw * 3, "augment: workspace too small");
  hipStream_t st = as_stream(stream);
  uint8_t* tmp = static_cast<uint8_t*>(ws);
  dim3 g1((unsigned)cdiv(nw, 256), (unsigned)ih);
  resample_h_kernel<<<g1, 256, 0, st>>>(src, ih, iw, nw, tmp);
  if (int e = check_launch("augment_resample_h")) return e;
  // hue*360 in double (Python), then NEP-50 cast to the float32 array's dtype
  const float hue360 = (float)(hue * 360.0);
  augment_kernel<<<(unsigned)cdiv((int64_t)h * w, 256), 256, 0, st>>>(
      tmp, ih, nw, nh, h, w, dx, dy, flip, hue360, sat, val, dst);
  return check_launch("augment");
}
