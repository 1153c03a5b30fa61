// predictor.h — internal interfaces of the style-predictor kernels (predictor.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace rst {

enum PredAct { ACT_NONE = 0, ACT_RELU = 1, ACT_HSWISH = 2, ACT_HSIGMOID = 3 };

// Rescaling(2,-1) + Conv2D(16, 3, s2, same, no bias) + folded BN + act. w [3][3][3][16].
hipError_t stem_launch(const float* x, const float* w, const float* ba, const float* bb, float* y, int B, int H,
                       int W, int Ho, int Wo, int pad_t, int pad_l, int act, hipStream_t st);
// DUMMY extractor conv: Conv2D(1, 9, s5, same) + bias. w [9][9][C]; part (B, dummy_conv_parts) sums.
int dummy_conv_parts(int HWo);
hipError_t dummy_conv_launch(const float* x, const float* w, const float* bias, float* y, float* part, int B, int H,
                             int W, int C, int Ho, int Wo, int pad_t, int pad_l, hipStream_t st);
// 1x1 conv, w [cin][cout]; se (B, cin) input-channel scale or null; res (B, HW, cout) or null;
// part (B, pw_parts(HW), cout) per-tile channel sums of the output, or null.
int pw_chunk(int cout, int HW);
int pw_parts(int HW);
hipError_t pw_launch(const float* x, const float* se, const float* w, const float* ba, const float* bb,
                     const float* res, float* y, float* part, int B, int HW, int cin, int cout, int act,
                     hipStream_t st);
// depthwise kxk conv, w [k][k][C]; part (B, n_wg, C) channel partial sums or null.
void dw_geometry(int C, int HWo, int* block, int* slots, int* ppw, int* n_wg);
hipError_t dw_launch(const float* x, const float* w, const float* ba, const float* bb, float* y, float* part, int B,
                     int H, int W, int C, int Ho, int Wo, int k, int stride, int pad_t, int pad_l, int act,
                     hipStream_t st);
// squeeze-excitation: part (B, n_part, C) -> se (B, C); optional saved g (B, C), pre-ReLU s1 (B, R),
// pre-hard_sigmoid s2 (B, C) for the backward.
hipError_t se_launch(const float* part, int n_part, int hw, int B, int C, int R, const float* w1, const float* b1,
                     const float* w2, const float* b2, float* se, float* g_out, float* s1_out, float* s2_out,
                     hipStream_t st);
// GAP (from part, (B, n_part, C) sums over hw pixels) -> Conv2D(NS, 1) -> hidden (B, NS) -> Conv2D(P, 1) -> out.
hipError_t head_launch(const float* part, int n_part, int hw, int B, int C, int NS, int P, const float* w1,
                       const float* b1, const float* w2, const float* b2, float* hidden, float* out, int out_stride,
                       float* g_out, hipStream_t st);

}  // namespace rst
