// predictor.hip — kernels of the style predictor (create_style_prediction_model,
// realtime_style_transfer/models/stylePrediction.py:25-75): the MobileNetV3Small feature extractor
// (Keras 2.9 keras/applications/mobilenet_v3.py, restated in oracle/predictor_ref.py), the DUMMY
// extractor, global average pooling and the two 1x1 heads.
//
// Roofline: the whole predictor is ~0.5 GFLOP per 480x960 style image against ~40 MB of
// activations; every layer has arithmetic intensity far below the fp32 ridge (or too little work
// to fill 256 CUs), so it is bounded by HBM/L2 traffic and launch latency, not by MFMA. The
// kernels are therefore VALU kernels built for traffic and occupancy:
//   * 1x1 convs: one lane per output pixel, CO output channels per lane; the weight row of
//     each input channel is wave-uniform (scalar loads, SGPR operands of v_fma), the SE channel
//     scale of the producing block is applied while the input is read, BN (folded to a, b),
//     activation and the residual add run in the epilogue.
//   * depthwise convs: one lane per (pixel, 4 channels) with float4 loads along channels (NHWC
//     rows are contiguous, so a wave reads whole cache lines); BN + activation fused; the SE
//     squeeze (global average pool) is produced as per-workgroup channel partial sums in a fixed
//     order (deterministic, no atomics) and finished by the SE kernel.
//   * SE excitation: one workgroup per image (FC -> ReLU -> FC -> hard_sigmoid), tiny.
//   * stem (Rescaling(2,-1) + 3x3 s2 conv + BN + hard_swish) and the DUMMY 9x9 s5 conv: one lane
//     per output pixel, wave-uniform weights.
#include <hip/hip_runtime.h>

#include "predictor.h"

namespace rst {

__device__ __forceinline__ float hsig(float x) { return fminf(fmaxf(x + 3.f, 0.f), 6.f) * (1.f / 6.f); }

__device__ __forceinline__ float act_apply(float x, int act) {
    if (act == ACT_RELU) return fmaxf(x, 0.f);
    if (act == ACT_HSWISH) return x * hsig(x);
    return x;
}

// ---------------------------------------------------------------------------------------- stem
// x (B,H,W,3) in [0,1] -> Rescaling(2,-1) (only in-bounds pixels: the zero padding of the SAME conv
// is in the rescaled space) -> Conv2D(16, 3, s2, same, no bias) -> BN -> hard_swish.
__global__ __launch_bounds__(64) void stem_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                  const float* __restrict__ ba, const float* __restrict__ bb,
                                                  float* __restrict__ y, int H, int W, int Ho, int Wo, int pad_t,
                                                  int pad_l, int stride, float in_scale, float in_shift,
                                                  int act) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= Ho * Wo) return;
    const int oy = p / Wo, ox = p - oy * Wo;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    const float* xb = x + (size_t)b * H * W * 3;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
        const int iy = oy * stride - pad_t + ky;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int ix = ox * stride - pad_l + kx;
            float v0 = 0.f, v1 = 0.f, v2 = 0.f;
            if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
                const float* px = xb + ((size_t)iy * W + ix) * 3;
                v0 = px[0] * in_scale + in_shift;
                v1 = px[1] * in_scale + in_shift;
                v2 = px[2] * in_scale + in_shift;
            }
            const float* wt = w + (ky * 3 + kx) * 3 * 16;
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = fmaf(v0, wt[j], acc[j]);
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = fmaf(v1, wt[16 + j], acc[j]);
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = fmaf(v2, wt[32 + j], acc[j]);
        }
    }
    float4* out = reinterpret_cast<float4*>(y + ((size_t)b * Ho * Wo + p) * 16);
#pragma unroll
    for (int j = 0; j < 16; j += 4)
        out[j / 4] = make_float4(act_apply(fmaf(acc[j], ba[j], bb[j]), act),
                                 act_apply(fmaf(acc[j + 1], ba[j + 1], bb[j + 1]), act),
                                 act_apply(fmaf(acc[j + 2], ba[j + 2], bb[j + 2]), act),
                                 act_apply(fmaf(acc[j + 3], ba[j + 3], bb[j + 3]), act));
}

// DUMMY extractor: Conv2D(1, 9, strides=5, padding='same') with bias, no activation
// (stylePrediction.py:31-32). One lane per output pixel.
__global__ __launch_bounds__(64) void dummy_conv_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        int H, int W, int C, int Ho, int Wo, int pad_t, int pad_l) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= Ho * Wo) return;
    const int oy = p / Wo, ox = p - oy * Wo;
    const float* xb = x + (size_t)b * H * W * C;
    float acc = 0.f;
    for (int ky = 0; ky < 9; ++ky) {
        const int iy = oy * 5 - pad_t + ky;
        if (iy < 0 || iy >= H) continue;
        for (int kx = 0; kx < 9; ++kx) {
            const int ix = ox * 5 - pad_l + kx;
            if (ix < 0 || ix >= W) continue;
            const float* px = xb + ((size_t)iy * W + ix) * C;
            const float* wt = w + (ky * 9 + kx) * C;
            for (int c = 0; c < C; ++c) acc = fmaf(px[c], wt[c], acc);
        }
    }
    y[(size_t)b * Ho * Wo + p] = acc + bias[0];
}

// ------------------------------------------------------------------------------- 1x1 conv
// y[b][p][co] = act(a[co] * sum_ci x[b][p][ci] * se[b][ci] * w[ci][co] + b[co]) (+ res[b][p][co])
template <int CO>
__global__ __launch_bounds__(64) void pw_kernel(const float* __restrict__ x, const float* __restrict__ se,
                                                const float* __restrict__ w, const float* __restrict__ ba,
                                                const float* __restrict__ bb, const float* __restrict__ res,
                                                float* __restrict__ y, int HW, int cin, int cout, int act) {
    const int b = blockIdx.z;
    const int co0 = blockIdx.y * CO;
    const int p = blockIdx.x * 64 + threadIdx.x;
    const bool valid = p < HW;
    const float* xp = x + ((size_t)b * HW + (valid ? p : 0)) * cin;
    const float* sb = se != nullptr ? se + (size_t)b * cin : nullptr;
    float acc[CO];
#pragma unroll
    for (int j = 0; j < CO; ++j) acc[j] = 0.f;
    for (int ci = 0; ci < cin; ci += 4) {
        float4 v = *reinterpret_cast<const float4*>(xp + ci);
        if (sb != nullptr) {
            v.x *= sb[ci];
            v.y *= sb[ci + 1];
            v.z *= sb[ci + 2];
            v.w *= sb[ci + 3];
        }
        const float* wr = w + (size_t)ci * cout + co0;
#pragma unroll
        for (int j = 0; j < CO; ++j) acc[j] = fmaf(v.x, wr[j], acc[j]);
#pragma unroll
        for (int j = 0; j < CO; ++j) acc[j] = fmaf(v.y, wr[cout + j], acc[j]);
#pragma unroll
        for (int j = 0; j < CO; ++j) acc[j] = fmaf(v.z, wr[2 * cout + j], acc[j]);
#pragma unroll
        for (int j = 0; j < CO; ++j) acc[j] = fmaf(v.w, wr[3 * cout + j], acc[j]);
    }
    if (!valid) return;
    const size_t o = ((size_t)b * HW + p) * cout + co0;
#pragma unroll
    for (int j = 0; j < CO; j += 4) {
        float4 r = make_float4(act_apply(fmaf(acc[j], ba[co0 + j], bb[co0 + j]), act),
                               act_apply(fmaf(acc[j + 1], ba[co0 + j + 1], bb[co0 + j + 1]), act),
                               act_apply(fmaf(acc[j + 2], ba[co0 + j + 2], bb[co0 + j + 2]), act),
                               act_apply(fmaf(acc[j + 3], ba[co0 + j + 3], bb[co0 + j + 3]), act));
        if (res != nullptr) {
            const float4 q = *reinterpret_cast<const float4*>(res + o + j);
            r.x += q.x; r.y += q.y; r.z += q.z; r.w += q.w;
        }
        *reinterpret_cast<float4*>(y + o + j) = r;
    }
}

// ----------------------------------------------------------------------------- depthwise conv
// Block = cg * slots threads (cg = C/4 channel quads, slots pixel slots); workgroup blockIdx.x owns
// pixels [blockIdx.x * ppw, +ppw) of image blockIdx.y. part (optional): per-workgroup channel sums
// of the activated output, [b][wg][C], summed over slots in a fixed order.
template <int K, int S>
__global__ __launch_bounds__(256) void dw_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                 const float* __restrict__ ba, const float* __restrict__ bb,
                                                 float* __restrict__ y, float* __restrict__ part, int H, int W,
                                                 int C, int Ho, int Wo, int pad_t, int pad_l, int ppw, int slots,
                                                 int act) {
    __shared__ float4 red[256];
    const int cg = C >> 2;
    const int t = threadIdx.x;
    const int q = t % cg, slot = t / cg;
    const int b = blockIdx.y;
    const int HWo = Ho * Wo;
    const int p0 = blockIdx.x * ppw;
    const int p1 = min(p0 + ppw, HWo);
    const float4* xb = reinterpret_cast<const float4*>(x + (size_t)b * H * W * C);
    const float4* wq = reinterpret_cast<const float4*>(w);
    const float4 a4 = reinterpret_cast<const float4*>(ba)[q];
    const float4 b4 = reinterpret_cast<const float4*>(bb)[q];
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = p0 + slot; p < p1; p += slots) {
        const int oy = p / Wo, ox = p - oy * Wo;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int iy = oy * S - pad_t + ky;
            if (iy < 0 || iy >= H) continue;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int ix = ox * S - pad_l + kx;
                if (ix < 0 || ix >= W) continue;
                const float4 v = xb[((size_t)iy * W + ix) * cg + q];
                const float4 k = wq[(ky * K + kx) * cg + q];
                acc.x = fmaf(v.x, k.x, acc.x);
                acc.y = fmaf(v.y, k.y, acc.y);
                acc.z = fmaf(v.z, k.z, acc.z);
                acc.w = fmaf(v.w, k.w, acc.w);
            }
        }
        float4 r = make_float4(act_apply(fmaf(acc.x, a4.x, b4.x), act), act_apply(fmaf(acc.y, a4.y, b4.y), act),
                               act_apply(fmaf(acc.z, a4.z, b4.z), act), act_apply(fmaf(acc.w, a4.w, b4.w), act));
        reinterpret_cast<float4*>(y)[((size_t)b * HWo + p) * cg + q] = r;
        s.x += r.x; s.y += r.y; s.z += r.z; s.w += r.w;
    }
    if (part == nullptr) return;
    red[t] = s;
    __syncthreads();
    if (slot == 0) {
        for (int k = 1; k < slots; ++k) {
            const float4 o = red[k * cg + q];
            s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
        }
        reinterpret_cast<float4*>(part)[((size_t)b * gridDim.x + blockIdx.x) * cg + q] = s;
    }
}

// ------------------------------------------------------------------------ squeeze-excitation
// One workgroup per image: g = (sum of the n_part partials) / hw; h = relu(g W1 + b1);
// se = hard_sigmoid(h W2 + b2).
__global__ __launch_bounds__(256) void se_kernel(const float* __restrict__ part, int n_part, float inv_hw, int C,
                                                 int R, const float* __restrict__ w1, const float* __restrict__ b1,
                                                 const float* __restrict__ w2, const float* __restrict__ b2,
                                                 float* __restrict__ se) {
    __shared__ float g[1024];
    __shared__ float h[256];
    const int b = blockIdx.x, t = threadIdx.x;
    for (int c = t; c < C; c += 256) {
        float s = 0.f;
        for (int k = 0; k < n_part; ++k) s += part[((size_t)b * n_part + k) * C + c];
        g[c] = s * inv_hw;
    }
    __syncthreads();
    for (int r = t; r < R; r += 256) {
        float s = b1[r];
        for (int c = 0; c < C; ++c) s = fmaf(g[c], w1[(size_t)c * R + r], s);
        h[r] = fmaxf(s, 0.f);
    }
    __syncthreads();
    for (int c = t; c < C; c += 256) {
        float s = b2[c];
        for (int r = 0; r < R; ++r) s = fmaf(h[r], w2[(size_t)r * C + c], s);
        se[(size_t)b * C + c] = hsig(s);
    }
}

// ------------------------------------------------------------------------------ head
// Global average pool: block = ct channels x (256/ct) pixel rows, grid (ceil(C/ct), B).
__global__ __launch_bounds__(256) void gap_kernel(const float* __restrict__ x, int HW, int C, int ct,
                                                  float* __restrict__ g) {
    __shared__ float red[256];
    const int t = threadIdx.x;
    const int rows = 256 / ct;
    const int cl = t % ct, r = t / ct;
    const int c = blockIdx.x * ct + cl;
    const int b = blockIdx.y;
    float s = 0.f;
    if (c < C && r < rows)
        for (int p = r; p < HW; p += rows) s += x[((size_t)b * HW + p) * C + c];
    red[t] = s;
    __syncthreads();
    if (r == 0 && c < C) {
        for (int k = 1; k < rows; ++k) s += red[k * ct + cl];
        g[(size_t)b * C + c] = s / (float)HW;
    }
}

// StylePredictor (C -> NS, bias) then StyleNormPredictor (NS -> P, bias), no activation in between
// (stylePrediction.py:60-71). grid (ceil(P/256), B); every workgroup recomputes the NS-wide hidden
// vector (C*NS MACs, L2-resident weights) so no extra launch is needed.
__global__ __launch_bounds__(256) void head_kernel(const float* __restrict__ g, int C, int NS, int P,
                                                   const float* __restrict__ w1, const float* __restrict__ b1,
                                                   const float* __restrict__ w2, const float* __restrict__ b2,
                                                   float* __restrict__ out, int out_stride) {
    __shared__ float gs[1024];
    __shared__ float hs[512];
    const int b = blockIdx.y, t = threadIdx.x;
    for (int c = t; c < C; c += 256) gs[c] = g[(size_t)b * C + c];
    __syncthreads();
    for (int k = t; k < NS; k += 256) {
        float s = b1[k];
        for (int c = 0; c < C; ++c) s = fmaf(gs[c], w1[(size_t)c * NS + k], s);
        hs[k] = s;
    }
    __syncthreads();
    const int j = blockIdx.x * 256 + t;
    if (j >= P) return;
    float s = b2[j];
    for (int k = 0; k < NS; ++k) s = fmaf(hs[k], w2[(size_t)k * P + j], s);
    out[(size_t)b * out_stride + j] = s;
}

// ------------------------------------------------------------------------------ launchers
hipError_t stem_launch(const float* x, const float* w, const float* ba, const float* bb, float* y, int B, int H,
                       int W, int Ho, int Wo, int pad_t, int pad_l, hipStream_t st) {
    dim3 grid((Ho * Wo + 63) / 64, B);
    stem_kernel<<<grid, 64, 0, st>>>(x, w, ba, bb, y, H, W, Ho, Wo, pad_t, pad_l, 2, 2.f, -1.f, ACT_HSWISH);
    return hipGetLastError();
}

hipError_t dummy_conv_launch(const float* x, const float* w, const float* bias, float* y, int B, int H, int W, int C,
                             int Ho, int Wo, int pad_t, int pad_l, hipStream_t st) {
    dim3 grid((Ho * Wo + 63) / 64, B);
    dummy_conv_kernel<<<grid, 64, 0, st>>>(x, w, bias, y, H, W, C, Ho, Wo, pad_t, pad_l);
    return hipGetLastError();
}

int pw_chunk(int cout) {
    for (int co : {48, 40, 32, 24, 16, 8})
        if (cout % co == 0) return co;
    return 0;
}

hipError_t pw_launch(const float* x, const float* se, const float* w, const float* ba, const float* bb,
                     const float* res, float* y, int B, int HW, int cin, int cout, int act, hipStream_t st) {
    const int co = pw_chunk(cout);
    if (co == 0 || (cin & 3) != 0) return hipErrorInvalidValue;
    dim3 grid((HW + 63) / 64, cout / co, B);
#define PW_CASE(N) \
    case N: pw_kernel<N><<<grid, 64, 0, st>>>(x, se, w, ba, bb, res, y, HW, cin, cout, act); break;
    switch (co) {
        PW_CASE(48) PW_CASE(40) PW_CASE(32) PW_CASE(24) PW_CASE(16) PW_CASE(8)
        default: return hipErrorInvalidValue;
    }
#undef PW_CASE
    return hipGetLastError();
}

void dw_geometry(int C, int HWo, int* block, int* slots, int* ppw, int* n_wg) {
    const int cg = C / 4;
    *slots = cg >= 256 ? 1 : 256 / cg;
    *block = cg * *slots;
    int it = HWo / (*slots * 512);
    it = it < 1 ? 1 : (it > 8 ? 8 : it);
    *ppw = *slots * it;
    *n_wg = (HWo + *ppw - 1) / *ppw;
}

hipError_t dw_launch(const float* x, const float* w, const float* ba, const float* bb, float* y, float* part, int B,
                     int H, int W, int C, int Ho, int Wo, int k, int stride, int pad_t, int pad_l, int act,
                     hipStream_t st) {
    if ((C & 3) != 0 || C / 4 > 256) return hipErrorInvalidValue;
    int block, slots, ppw, n_wg;
    dw_geometry(C, Ho * Wo, &block, &slots, &ppw, &n_wg);
    dim3 grid(n_wg, B);
    if (k == 3 && stride == 1)
        dw_kernel<3, 1><<<grid, block, 0, st>>>(x, w, ba, bb, y, part, H, W, C, Ho, Wo, pad_t, pad_l, ppw, slots, act);
    else if (k == 3 && stride == 2)
        dw_kernel<3, 2><<<grid, block, 0, st>>>(x, w, ba, bb, y, part, H, W, C, Ho, Wo, pad_t, pad_l, ppw, slots, act);
    else if (k == 5 && stride == 1)
        dw_kernel<5, 1><<<grid, block, 0, st>>>(x, w, ba, bb, y, part, H, W, C, Ho, Wo, pad_t, pad_l, ppw, slots, act);
    else if (k == 5 && stride == 2)
        dw_kernel<5, 2><<<grid, block, 0, st>>>(x, w, ba, bb, y, part, H, W, C, Ho, Wo, pad_t, pad_l, ppw, slots, act);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t se_launch(const float* part, int n_part, int hw, int B, int C, int R, const float* w1, const float* b1,
                     const float* w2, const float* b2, float* se, hipStream_t st) {
    if (C > 1024 || R > 256) return hipErrorInvalidValue;
    se_kernel<<<B, 256, 0, st>>>(part, n_part, 1.f / (float)hw, C, R, w1, b1, w2, b2, se);
    return hipGetLastError();
}

hipError_t gap_launch(const float* x, int B, int HW, int C, float* g, hipStream_t st) {
    const int ct = C >= 64 ? 64 : C;
    dim3 grid((C + ct - 1) / ct, B);
    gap_kernel<<<grid, 256, 0, st>>>(x, HW, C, ct, g);
    return hipGetLastError();
}

hipError_t head_launch(const float* g, int B, int C, int NS, int P, const float* w1, const float* b1, const float* w2,
                       const float* b2, float* out, int out_stride, hipStream_t st) {
    if (C > 1024 || NS > 512) return hipErrorInvalidValue;
    dim3 grid((P + 255) / 256, B);
    head_kernel<<<grid, 256, 0, st>>>(g, C, NS, P, w1, b1, w2, b2, out, out_stride);
    return hipGetLastError();
}

}  // namespace rst
