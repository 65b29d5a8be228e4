// Kernel-side view of the C-ABI argument structs.
#pragma once
#include "../../include/jabd.h"

namespace jabd {
typedef jabd_conv_args ConvArgs;
typedef jabd_dw_args DwArgs;
enum {
  ACT_NONE = JABD_ACT_NONE,
  ACT_RELU = JABD_ACT_RELU,
  ACT_LEAKY = JABD_ACT_LEAKY,
  ACT_HSWISH = JABD_ACT_HSWISH,
  ACT_HSIGMOID = JABD_ACT_HSIGMOID,
  ACT_SIGMOID = JABD_ACT_SIGMOID,
};
// The 32x32 GEMM's BatchNorm-backward epilogue (jabd_conv_bn_bwd_sums_f32):
// the GEMM output is the dy of a BatchNorm (+ act) whose pre-BN input x and
// parameters these are; rows: per-32-pixel-tile sums of dz and dz * xhat.
// mask set (jabd_conv_bn_bwd_sums_res_f32): the BatchNorm's act is a ReLU
// after a residual add, taken from its saved output: dz = (y + res) *
// [mask > 0] is what the GEMM writes (gamma / beta / act unused).
struct BnEpi {
  const float* x;
  const float *mean, *invstd, *gamma, *beta;
  float* rows;
  int x_ps, act;
  float slope;
  const float* mask;
  int mask_ps;
};
// conv1x1_stream_dispatch's statistics form (jabd_conv1x1_bn_stats_*)
struct StreamStats {
  float* part;
  float* shift;
  int64_t nblk;
  bool query;
};
}  // namespace jabd
