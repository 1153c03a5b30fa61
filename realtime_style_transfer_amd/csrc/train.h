// train.h — backward / optimizer kernel interfaces (train.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>

namespace rst {

// Norm (CIN or training-mode BatchNorm) backward, see train.hip.
struct NormBwdArgs {
    const float* g;          // gradient w.r.t. the post-activation output [B][hw][C]
    const float* z;          // stored conv output (pre-norm) [B][hw][C]
    const float2* ab;        // forward affine (a, b) per (b, c)
    const float2* mr;        // forward (mean, rstd) per (b, c)
    float2* part;            // [B][C][n_tiles] {S1, S2}
    float2* consts;          // [B][C] {S1/N, S2/N}
    float* dscale;           // scale / gamma gradient (or null)
    float* dbias;            // bias / beta gradient (or null)
    int dstride;             // image stride of dscale/dbias (CIN: style-param vector length)
    float* dz;               // output: gradient w.r.t. the conv output (pre conv-ReLU) [B][hw][C]
    int batch, hw, C, tile, n_tiles;
    int post;                // 0 relu, 1 none, 2 sigmoid
    int conv_relu;           // conv carries a built-in ReLU (mask dz by z > 0)
    int merge_images;        // BatchNorm: statistics over the whole batch
    float* dconv_bias;       // conv bias gradient = sum of dz over images and pixels (or null)
};
hipError_t norm_bwd_launch(const NormBwdArgs& a, hipStream_t st);

hipError_t add_launch(const float* x1, const float* x2, float* y, size_t n, hipStream_t st);

// Weight gradient of a conv (transposed == 0) or transposed conv (transposed == 1).
struct WgradArgs {
    const float* X;          // conv input (post-prologue) [B][XH][XW][C1]   (convT: its input)
    const float* D;          // gradient w.r.t. the conv output [B][DH][DW][C2] (convT: its output)
    float* slab;             // workspace, wgrad_slab_bytes()
    float* dW;               // canonical Keras layout
    int batch, XH, XW, C1, DH, DW, C2;
    int Qh, Qw;              // GEMM pixel grid: conv -> output dims, convT -> input dims
    int kh, kw, stride, pad_t, pad_l;
    int transposed;
    int nsplit;
    long span;               // set by wgrad_launch
    int x6;                  // 1: residual-conv shape on the split-bf16 x6 kernel (fp32-level products)
};
int wgrad_choose_splits(const WgradArgs& a);
size_t wgrad_slab_bytes(const WgradArgs& a);
hipError_t wgrad_launch(WgradArgs a, hipStream_t st);

// x_bf16: the pooled forward activations x are stored as bf16 bits (the plain-bf16 VGG16); g_bf16: gy and gx too,
// with acc (f32, separate from gx) added before gx's one rounding instead of accumulate
hipError_t maxpool2_bwd_launch(const float* x, const float* gy, float* gx, int B, int H, int W, int C, int accumulate,
                               hipStream_t st, bool x_bf16 = false, bool g_bf16 = false, const float* acc = nullptr);
// in_bf16: a and b hold bf16 bits; g_bf16: g is written as bf16 bits (needs in_bf16, no accumulate)
hipError_t scaled_diff_launch(const float* a, const float* b, float scale, float* g, size_t n, int accumulate,
                              hipStream_t st, bool in_bf16 = false, bool g_bf16 = false);
hipError_t tv_bwd_launch(const float* x, float factor, float* g, int B, int H, int W, int C, hipStream_t st);
hipError_t tap3_sum_launch(const float* p, float* out, int B, int H, int W, hipStream_t st);
hipError_t gram_bwd_weights_bf16_launch(const float* gp, const float* gs, const int* map, int n16, int C, float scale,
                                        unsigned short* packed, int B, hipStream_t st);
hipError_t gram_bwd_weights_launch(const float* gp, const float* gs, const int* map, int n_packed, int C, float scale,
                                   float* packed, int B, hipStream_t st);
hipError_t preprocess_bwd_launch(const float* gpre, float* gx, size_t pixels, int accumulate, hipStream_t st);
hipError_t rmsprop_launch(float* w, float* ms, const float* g, size_t n, float lr, float rho, float eps, hipStream_t st);
hipError_t gather_launch(const float* src, const int* map, float* dst, size_t n, hipStream_t st);
// batched gathers dst_j[i] = src[map_j[i]] (0 where map_j[i] < 0), one launch; gather_batch_launch resets jobs.n
constexpr int GATHER_MAX_JOBS = 48;
struct GatherJobs {
    const int* map[GATHER_MAX_JOBS];
    float* dst[GATHER_MAX_JOBS];
    size_t count[GATHER_MAX_JOBS];
    int first[GATHER_MAX_JOBS + 1];
    int n;
};
hipError_t gather_batch_launch(const float* src, GatherJobs& jobs, hipStream_t st);
hipError_t scatter_div_launch(const float* src, const int* index, float* dst, size_t n, float divisor, hipStream_t st);
// Diagnostic (RST_LDS_POISON): fill the whole LDS of every CU with the bit pattern `bits`, so that the next kernel on
// the stream finds that pattern wherever it reads LDS it did not write first
hipError_t lds_poison_launch(unsigned bits, hipStream_t st);

}  // namespace rst
