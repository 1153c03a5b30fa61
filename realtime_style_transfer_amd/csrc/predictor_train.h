// predictor_train.h — training-mode kernel interfaces of the style predictor (predictor_train.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace rst {

// training-mode BatchNormalization forward of a raw conv output z (B, HW, C):
// stats -> finalize (ab, mr, moving statistics in place) -> y = act(a z + b) [+ res], y_part optional
// per-(image, tile) channel sums of y ([b][tile][C], tiles as dw_geometry).
hipError_t bn_forward_launch(const float* z, int B, int HW, int C, float* gamma_beta_mm_mv, float eps, float momentum,
                             float4* part, float2* ab, float2* mr, const float* res, float* y, int act,
                             float* y_part, hipStream_t st);

struct BnBwdArgs {
    const float* z;         // raw conv output (B, HW, C)
    const float* dy;        // gradient w.r.t. the unit output (B, HW, C), or null
    const float* mul;       // dy multiplier per (b, c) (SE scale), or null
    const float* bcast;     // broadcast gradient per (b, c) added to dy*mul, or null
    const float2* ab;       // forward (a, b) per channel
    const float2* mr;       // forward (mean, rstd) per channel
    float2* consts;         // scratch (C): (S1/N, S2/N)
    float4* part;           // scratch: per-(image, tile) {S1, S2}
    float* dz;              // out: gradient w.r.t. z
    float* dgamma;          // out: d gamma at [0, C), d beta at [C, 2C)
    int B, HW, C, act;
    int ppw, slots, n_tiles;  // set by bn_backward_launch
};
hipError_t bn_backward_launch(BnBwdArgs a, hipStream_t st);

// Every 1x1 kernel's transpose ([cin][cout] -> [cout][cin], the input-gradient conv's weights) in one launch: job j
// reads rows x cols at w + src[j] and writes the transpose at wt + dst[j]; end[j] = cumulative element count.
struct TransposeJobs {
    static constexpr int MAX = 32;
    int n = 0;
    long long src[MAX], dst[MAX], end[MAX];
    int rows[MAX], cols[MAX];
};
hipError_t transpose_batch_launch(const float* w, const TransposeJobs& jobs, float* wt, hipStream_t st);

int pw_wgrad_splits(int B, int HW, int cin, int cout, int* pps);
hipError_t pw_wgrad_launch(const float* x, const float* se, const float* dz, int B, int HW, int cin, int cout,
                           float* slab, float* dW, hipStream_t st);
hipError_t transpose_launch(const float* w, int rows, int cols, float* wt, hipStream_t st);
hipError_t dw_dgrad_launch(const float* dz, const float* w, float* dx, int B, int H, int W, int C, int Ho, int Wo,
                           int k, int stride, int pad_t, int pad_l, hipStream_t st);
int dw_wgrad_splits(int B, int HWo, int C, int* pps, int* block, int* slots);
hipError_t dw_wgrad_launch(const float* x, const float* dz, int B, int H, int W, int C, int Ho, int Wo, int k,
                           int stride, int pad_t, int pad_l, float* slab, float* dW, hipStream_t st);
int stem_wgrad_splits(int B, int HWo, int* pps);
hipError_t stem_wgrad_launch(const float* x, const float* dz, int B, int H, int W, int Ho, int Wo, int pad_t,
                             int pad_l, float* slab, float* dW, hipStream_t st);
hipError_t dummy_wgrad_launch(const float* x, const float* dg, int B, int H, int W, int C, int Ho, int Wo, int pad_t,
                              int pad_l, float* dW, float* db, hipStream_t st);
hipError_t se_dscale_launch(const float* dxin, const float* u, int B, int HW, int C, float* part, int* n_part,
                            hipStream_t st);
hipError_t se_bwd_launch(const float* part, int n_part, int B, int C, int R, int hw, const float* w1, const float* w2,
                         const float* s1, const float* s2, float* ds1, float* ds2, float* dgb, hipStream_t st);
hipError_t rowdot_launch(const float* in, int B, int K, const float* Wm, int N, float scale, float* out,
                         hipStream_t st);
hipError_t outer_launch(const float* a, int M, const float* d, int N, int B, int relu_a, float* dW, float* db,
                        hipStream_t st);

}  // namespace rst
