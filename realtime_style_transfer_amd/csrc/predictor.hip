// predictor.hip — kernels of the style predictor (create_style_prediction_model,
// realtime_style_transfer/models/stylePrediction.py:25-75): the MobileNetV3Small feature extractor
// (Keras 2.9 keras/applications/mobilenet_v3.py, restated in oracle/predictor_ref.py), the DUMMY
// extractor, global average pooling and the two 1x1 heads.
//
// Roofline: the whole predictor is ~0.5 GFLOP and ~107 MB of algorithmic fp32 traffic per
// 480x960 style image, spread over ~45 layers whose arithmetic intensity is far below the fp32
// ridge and most of which are too small to fill 256 CUs (the late layers have 450 pixels). It is
// bounded by memory latency and launch count, not by MFMA or HBM bandwidth, so the kernels are
// VALU kernels designed for SHORT CRITICAL PATHS: every thread's chain of dependent global-memory
// round trips is kept to a handful (each costs ~0.5 us), with many loads in flight per thread.
//   * 1x1 convs: 64 pixels x (waves x CO) output channels per workgroup; the K dimension is
//     staged through LDS in 32-channel chunks loaded cooperatively (all loads in flight at once,
//     next chunk prefetched into registers during the FMAs of this one); weights are read as
//     wave-uniform LDS broadcasts. The SE channel scale of the producing block is applied while
//     staging; BN (folded to a, b), activation and the residual add run in the epilogue, plus,
//     for the last layer, per-tile channel sums feeding global average pooling.
//   * depthwise convs: one lane per (pixel, 4 channels), float4 loads along NHWC channels; BN +
//     activation fused; at most 64 workgroups per image, each writing its channel sums of the
//     activated output (SE squeeze) in a fixed order — deterministic, no atomics.
//   * SE excitation / pooling heads: one 1024-thread workgroup per image; each fully-connected
//     layer splits its reduction into <= 32 slices per output and merges them in a fixed order.
//   * stem (Rescaling(2,-1) + 3x3 s2 conv + BN + hard_swish): LDS-staged input patch per
//     8x32-pixel tile, wave-uniform weights.
#include <hip/hip_runtime.h>

#include "predictor.h"

namespace rst {

__device__ __forceinline__ float hsig(float x) { return fminf(fmaxf(x + 3.f, 0.f), 6.f) * (1.f / 6.f); }

__device__ __forceinline__ float act_apply(float x, int act) {
    if (act == ACT_RELU) return fmaxf(x, 0.f);
    if (act == ACT_HSWISH) return x * hsig(x);
    if (act == ACT_HSIGMOID) return hsig(x);
    return x;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---------------------------------------------------------------------------------------- stem
// x (B,H,W,3) in [0,1] -> Rescaling(2,-1) (in-bounds pixels only: the SAME conv's zero padding is
// in the rescaled space) -> Conv2D(16, 3, s2, same, no bias) -> BN -> hard_swish.
// Workgroup: 8 x 32 output pixels, one per thread, 16 output channels per thread.
constexpr int STEM_TH = 8, STEM_TW = 32, STEM_PH = 2 * STEM_TH + 1, STEM_PW = 2 * STEM_TW + 1;

__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ ba, const float* __restrict__ bb,
                                                   float* __restrict__ y, int H, int W, int Ho, int Wo, int pad_t,
                                                   int pad_l, int act) {
    __shared__ float patch[STEM_PH * STEM_PW * 3];
    const int b = blockIdx.z, t = threadIdx.x;
    const int oy0 = blockIdx.y * STEM_TH, ox0 = blockIdx.x * STEM_TW;
    const int iy0 = oy0 * 2 - pad_t, ix0 = ox0 * 2 - pad_l;
    const float* xb = x + (size_t)b * H * W * 3;
    constexpr int NP = STEM_PH * STEM_PW * 3, NI = (NP + 255) / 256;
    float pv[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {            // branch-free: all loads in flight
        const int e = min(t + i * 256, NP - 1);
        const int r = e / (STEM_PW * 3), rem = e - r * (STEM_PW * 3);
        const int iy = min(max(iy0 + r, 0), H - 1), ix = min(max(ix0 + rem / 3, 0), W - 1);
        pv[i] = xb[((size_t)iy * W + ix) * 3 + rem % 3];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int e = t + i * 256;
        if (e < NP) {
            const int r = e / (STEM_PW * 3), rem = e - r * (STEM_PW * 3);
            const int iy = iy0 + r, ix = ix0 + rem / 3;
            patch[e] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? pv[i] * 2.f - 1.f : 0.f;
        }
    }
    __syncthreads();
    const int ty = t / STEM_TW, tx = t - ty * STEM_TW;
    const int oy = oy0 + ty, ox = ox0 + tx;
    if (oy >= Ho || ox >= Wo) return;
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int ci = 0; ci < 3; ++ci) {
                const float v = patch[((2 * ty + ky) * STEM_PW + 2 * tx + kx) * 3 + ci];
                const float* wt = w + ((ky * 3 + kx) * 3 + ci) * 16;
#pragma unroll
                for (int j = 0; j < 16; ++j) acc[j] = fmaf(v, wt[j], acc[j]);
            }
    float4* out = reinterpret_cast<float4*>(y + (((size_t)b * Ho + oy) * Wo + ox) * 16);
#pragma unroll
    for (int j = 0; j < 16; j += 4)
        out[j / 4] = make_float4(act_apply(fmaf(acc[j], ba[j], bb[j]), act),
                                 act_apply(fmaf(acc[j + 1], ba[j + 1], bb[j + 1]), act),
                                 act_apply(fmaf(acc[j + 2], ba[j + 2], bb[j + 2]), act),
                                 act_apply(fmaf(acc[j + 3], ba[j + 3], bb[j + 3]), act));
}

// DUMMY extractor: Conv2D(1, 9, strides=5, padding='same') with bias, no activation
// (stylePrediction.py:31-32). One lane per output pixel; part[b][wave] = per-wave output sums.
__global__ __launch_bounds__(64) void dummy_conv_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        float* __restrict__ part, int H, int W, int C, int Ho,
                                                        int Wo, int pad_t, int pad_l) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * 64 + threadIdx.x;
    float out = 0.f;
    if (p < Ho * Wo) {
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
        out = acc + bias[0];
        y[(size_t)b * Ho * Wo + p] = out;
    }
    const float s = wave_sum(out);
    if (threadIdx.x == 0) part[(size_t)b * gridDim.x + blockIdx.x] = s;
}

// ------------------------------------------------------------------------------- 1x1 conv
// y[b][p][co] = act(a[co] * sum_ci x[b][p][ci] * se[b][ci] * w[ci][co] + b[co]) (+ res[b][p][co]).
// grid (ceil(HW/64), cout/CO, B), block 256: the workgroup computes CO output channels of 64 pixels
// (one pixel per lane); its 4 waves split every 32-channel K chunk four ways and their partial sums
// are merged through LDS in a fixed order at the end (deterministic). The late layers have few
// pixels (450) and long K (576): the K split and a small CO keep enough waves in flight.
// part (optional): per-(tile, channel) sums of y over the tile's pixels, [b][tile][cout].
constexpr int PW_KC = 32;

template <int CO>
__global__ __launch_bounds__(256) void pw_kernel(const float* __restrict__ x, const float* __restrict__ se,
                                                 const float* __restrict__ w, const float* __restrict__ ba,
                                                 const float* __restrict__ bb, const float* __restrict__ res,
                                                 float* __restrict__ y, float* __restrict__ part, int HW, int cin,
                                                 int cout, int act) {
    constexpr int WN = (PW_KC * CO / 4 + 255) / 256;   // weight float4 per thread per chunk (<= 2)
    static_assert(WN <= 2, "pw_kernel: CO <= 64");
    __shared__ float xs[64 * (PW_KC + 1)];
    __shared__ float4 wl[256 * WN];
    __shared__ float red[3 * CO * 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int b = blockIdx.z, p0 = blockIdx.x * 64, co0 = blockIdx.y * CO;
    constexpr int co4 = CO / 4;
    const float* xb = x + (size_t)b * HW * cin;
    const float* sb = se != nullptr ? se + (size_t)b * cin : nullptr;

    // Branch-free prefetch of a chunk (clamped addresses; masked when staged) into named registers,
    // so every load of the chunk is in flight at once and overlaps the previous chunk's FMAs.
    float4 x0, x1, s0, s1, w0, w1;
    auto xload = [&](int k0, int i, float4& xv, float4& sv) {
        const int kc4 = min(PW_KC, cin - k0) / 4;
        const int e = min(t + i * 256, 64 * kc4 - 1);
        const int px = e / kc4, c4 = e - px * kc4;
        const int pc = min(p0 + px, HW - 1);
        xv = *reinterpret_cast<const float4*>(xb + (size_t)pc * cin + k0 + 4 * c4);
        sv = *reinterpret_cast<const float4*>((sb != nullptr ? sb : xb) + k0 + 4 * c4);
    };
    auto wload = [&](int k0, int i) -> float4 {
        const int kc = min(PW_KC, cin - k0);
        const int e = min(t + i * 256, kc * co4 - 1);
        const int row = e / co4, c4 = e - row * co4;
        return *reinterpret_cast<const float4*>(w + (size_t)(k0 + row) * cout + co0 + 4 * c4);
    };
    auto xstage = [&](int k0, int i, float4 v, float4 sc) {
        const int kc4 = min(PW_KC, cin - k0) / 4;
        const int e = t + i * 256;
        if (e < 64 * kc4) {
            const int px = e / kc4, c4 = e - px * kc4;
            if (sb == nullptr) sc = make_float4(1.f, 1.f, 1.f, 1.f);
            v.x *= sc.x; v.y *= sc.y; v.z *= sc.z; v.w *= sc.w;
            if (p0 + px >= HW) v = make_float4(0.f, 0.f, 0.f, 0.f);
            float* d = xs + px * (PW_KC + 1) + 4 * c4;
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
    };

    float acc[CO];
#pragma unroll
    for (int j = 0; j < CO; ++j) acc[j] = 0.f;
    xload(0, 0, x0, s0);
    xload(0, 1, x1, s1);
    w0 = wload(0, 0);
    if (WN > 1) w1 = wload(0, 1);
    for (int k0 = 0; k0 < cin; k0 += PW_KC) {
        const int kc = min(PW_KC, cin - k0);
        xstage(k0, 0, x0, s0);
        xstage(k0, 1, x1, s1);
        wl[t] = w0;                         // rows >= kc are never read
        if (WN > 1) wl[t + 256] = w1;
        __syncthreads();
        if (k0 + PW_KC < cin) {             // next chunk in flight during this chunk's FMAs
            xload(k0 + PW_KC, 0, x0, s0);
            xload(k0 + PW_KC, 1, x1, s1);
            w0 = wload(k0 + PW_KC, 0);
            if (WN > 1) w1 = wload(k0 + PW_KC, 1);
        }
        const int q = kc / 4;               // this wave's K slice of the chunk
        const float* xrow = xs + lane * (PW_KC + 1) + wv * q;
        const float4* wrow = wl + wv * q * co4;
        for (int ci = 0; ci < q; ++ci) {
            const float xv = xrow[ci];
#pragma unroll
            for (int j = 0; j < co4; ++j) {
                const float4 wq = wrow[ci * co4 + j];
                acc[4 * j] = fmaf(xv, wq.x, acc[4 * j]);
                acc[4 * j + 1] = fmaf(xv, wq.y, acc[4 * j + 1]);
                acc[4 * j + 2] = fmaf(xv, wq.z, acc[4 * j + 2]);
                acc[4 * j + 3] = fmaf(xv, wq.w, acc[4 * j + 3]);
            }
        }
        __syncthreads();
    }
    // merge the four K slices: waves 1..3 -> LDS, wave 0 adds them in order
    if (wv > 0) {
#pragma unroll
        for (int j = 0; j < CO; ++j) red[((wv - 1) * CO + j) * 64 + lane] = acc[j];
    }
    __syncthreads();
    if (wv > 0) return;
#pragma unroll
    for (int j = 0; j < CO; ++j)
        acc[j] = ((acc[j] + red[j * 64 + lane]) + red[(CO + j) * 64 + lane]) + red[(2 * CO + j) * 64 + lane];
    const int p = p0 + lane;
    const bool valid = p < HW;
    const size_t o = ((size_t)b * HW + (valid ? p : 0)) * cout + co0;
#pragma unroll
    for (int j = 0; j < CO; j += 4) {
        float4 r = make_float4(act_apply(fmaf(acc[j], ba[co0 + j], bb[co0 + j]), act),
                               act_apply(fmaf(acc[j + 1], ba[co0 + j + 1], bb[co0 + j + 1]), act),
                               act_apply(fmaf(acc[j + 2], ba[co0 + j + 2], bb[co0 + j + 2]), act),
                               act_apply(fmaf(acc[j + 3], ba[co0 + j + 3], bb[co0 + j + 3]), act));
        if (valid) {
            if (res != nullptr) {
                const float4 qv = *reinterpret_cast<const float4*>(res + o + j);
                r.x += qv.x; r.y += qv.y; r.z += qv.z; r.w += qv.w;
            }
            *reinterpret_cast<float4*>(y + o + j) = r;
        } else {
            r = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        acc[j] = r.x; acc[j + 1] = r.y; acc[j + 2] = r.z; acc[j + 3] = r.w;
    }
    if (part != nullptr) {
        float* pp = part + ((size_t)b * gridDim.x + blockIdx.x) * cout + co0;
#pragma unroll
        for (int j = 0; j < CO; ++j) {
            const float sj = wave_sum(acc[j]);
            if (lane == 0) pp[j] = sj;
        }
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
        // branch-free taps: every load is issued (clamped in-bounds address) and masked afterwards,
        // so all K*K loads of a pixel are in flight together
        float4 v[K * K];
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int iy = oy * S - pad_t + ky;
            const int cy = min(max(iy, 0), H - 1);
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int ix = ox * S - pad_l + kx;
                const int cx = min(max(ix, 0), W - 1);
                v[ky * K + kx] = xb[((size_t)cy * W + cx) * cg + q];
            }
        }
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int iy = oy * S - pad_t + ky;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int ix = ox * S - pad_l + kx;
                const float m = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? 1.f : 0.f;
                const float4 k = wq[(ky * K + kx) * cg + q];
                const float4 x4 = v[ky * K + kx];
                acc.x = fmaf(x4.x * m, k.x, acc.x);
                acc.y = fmaf(x4.y * m, k.y, acc.y);
                acc.z = fmaf(x4.z * m, k.z, acc.z);
                acc.w = fmaf(x4.w * m, k.w, acc.w);
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

// ------------------------------------------------------------------- 1024-thread FC helpers
constexpr int FC_THREADS = 1024;

// g[c] = (sum over the n_part rows of part[k][c]) * scale, c < C <= 1024. Threads (channel quad, slice):
// the rows are split into Q <= 32 slices (4 float4 loads in flight per thread) merged in a fixed
// order. part is the image's [n_part][C] block. g: LDS, red: LDS scratch (>= 1024 floats).
__device__ void squeeze(const float* __restrict__ part, int n_part, int C, float scale, float* g, float* red) {
    const int t = threadIdx.x;
    if ((C & 3) == 0) {
        const int CQ = C / 4;
        const int Q = max(1, min(32, FC_THREADS / CQ));
        const int cq = t % CQ, qq = t / CQ;
        float4* red4 = reinterpret_cast<float4*>(red);    // Q * CQ <= 1024 float4: red must hold 4096 floats
        if (qq < Q) {
            float4 s[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) s[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4* p4 = reinterpret_cast<const float4*>(part) + cq;
            int k = qq;
            for (; k + 3 * Q < n_part; k += 4 * Q) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = p4[(size_t)(k + u * Q) * CQ];
#pragma unroll
                for (int u = 0; u < 4; ++u) { s[u].x += v[u].x; s[u].y += v[u].y; s[u].z += v[u].z; s[u].w += v[u].w; }
            }
            for (; k < n_part; k += Q) {
                const float4 v = p4[(size_t)k * CQ];
                s[0].x += v.x; s[0].y += v.y; s[0].z += v.z; s[0].w += v.w;
            }
            red4[qq * CQ + cq] = make_float4((s[0].x + s[1].x) + (s[2].x + s[3].x), (s[0].y + s[1].y) + (s[2].y + s[3].y),
                                             (s[0].z + s[1].z) + (s[2].z + s[3].z), (s[0].w + s[1].w) + (s[2].w + s[3].w));
        }
        __syncthreads();
        for (int c = t; c < C; c += FC_THREADS) {
            float sum = 0.f;
            for (int q2 = 0; q2 < Q; ++q2) sum += red[(q2 * CQ) * 4 + c];
            g[c] = sum * scale;
        }
        __syncthreads();
        return;
    }
    const int Q = max(1, min(32, FC_THREADS / C));
    const int c = t % C, qq = t / C;
    if (qq < Q && c < C) {
        float s = 0.f;
        for (int k = qq; k < n_part; k += Q) s += part[(size_t)k * C + c];
        red[qq * C + c] = s;
    }
    __syncthreads();
    for (int cc = t; cc < C; cc += FC_THREADS) {
        float s = 0.f;
        for (int q2 = 0; q2 < Q; ++q2) s += red[q2 * C + cc];
        g[cc] = s * scale;
    }
    __syncthreads();
}

// out[j] = act(bias[j] + sum_k in[k] * W[k][j]) for j < N <= 1024; in: LDS (K values); each output's
// K-reduction is split into Q <= 32 slices (threads (j, q)) merged in a fixed order.
__device__ void fc_layer(const float* in, int K, const float* __restrict__ Wt, const float* __restrict__ bias, int N,
                         int act, float* out, float* red) {
    const int t = threadIdx.x;
    const int Q = max(1, min(32, FC_THREADS / N));
    const int j = t % N, qq = t / N;
    if (qq < Q) {
        const int k0 = (K * qq) / Q, k1 = (K * (qq + 1)) / Q;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int k = k0;
        for (; k + 8 <= k1; k += 8)
#pragma unroll
            for (int u = 0; u < 8; ++u) s[u] = fmaf(in[k + u], Wt[(size_t)(k + u) * N + j], s[u]);
        for (; k < k1; ++k) s[0] = fmaf(in[k], Wt[(size_t)k * N + j], s[0]);
        red[qq * N + j] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    }
    __syncthreads();
    if (t < N) {
        float s = bias[t];
        for (int q2 = 0; q2 < Q; ++q2) s += red[q2 * N + t];
        out[t] = act_apply(s, act);
    }
    __syncthreads();
}

// ------------------------------------------------------------------------ squeeze-excitation
// One workgroup per image: g = (sum of the n_part partials) / hw; h = relu(g W1 + b1);
// se = hard_sigmoid(h W2 + b2).
__global__ __launch_bounds__(FC_THREADS) void se_kernel(const float* __restrict__ part, int n_part, float inv_hw,
                                                        int C, int R, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, float* __restrict__ se,
                                                        float* __restrict__ g_out, float* __restrict__ s1_out,
                                                        float* __restrict__ s2_out) {
    __shared__ float g[1024];
    __shared__ float h[1024];
    __shared__ float s_out[1024];
    __shared__ float red[4 * FC_THREADS];
    const int b = blockIdx.x, t = threadIdx.x;
    squeeze(part + (size_t)b * n_part * C, n_part, C, inv_hw, g, red);
    fc_layer(g, C, w1, b1, R, ACT_NONE, h, red);          // pre-ReLU s1
    for (int r = t; r < R; r += FC_THREADS) {
        if (s1_out != nullptr) s1_out[(size_t)b * R + r] = h[r];
        h[r] = fmaxf(h[r], 0.f);
    }
    __syncthreads();
    fc_layer(h, R, w2, b2, C, ACT_NONE, s_out, red);      // pre-hard_sigmoid s2
    for (int c = t; c < C; c += FC_THREADS) {
        se[(size_t)b * C + c] = hsig(s_out[c]);
        if (s2_out != nullptr) s2_out[(size_t)b * C + c] = s_out[c];
        if (g_out != nullptr) g_out[(size_t)b * C + c] = g[c];
    }
}

// ------------------------------------------------------------------------------ head
// GlobalAveragePooling2D (from the last layer's per-tile channel sums) + StylePredictor
// Conv2D(NS, 1) (stylePrediction.py:55-64): one workgroup per image -> hidden[b][NS].
__global__ __launch_bounds__(FC_THREADS) void head1_kernel(const float* __restrict__ part, int n_part, float inv_hw,
                                                           int C, int NS, const float* __restrict__ w1,
                                                           const float* __restrict__ b1,
                                                           float* __restrict__ hidden, float* __restrict__ g_out) {
    __shared__ float g[1024];
    __shared__ float h[1024];
    __shared__ float red[4 * FC_THREADS];
    const int b = blockIdx.x;
    squeeze(part + (size_t)b * n_part * C, n_part, C, inv_hw, g, red);
    fc_layer(g, C, w1, b1, NS, ACT_NONE, h, red);
    for (int k = threadIdx.x; k < NS; k += FC_THREADS) hidden[(size_t)b * NS + k] = h[k];
    if (g_out != nullptr)
        for (int c = threadIdx.x; c < C; c += FC_THREADS) g_out[(size_t)b * C + c] = g[c];
}

// StyleNormPredictor Conv2D(P, 1) (stylePrediction.py:67-71), no activation: one output per
// thread, grid (ceil(P/256), B).
__global__ __launch_bounds__(256) void head2_kernel(const float* __restrict__ hidden, int NS, int P,
                                                    const float* __restrict__ w2, const float* __restrict__ b2,
                                                    float* __restrict__ out, int out_stride) {
    __shared__ float hs[1024];
    const int b = blockIdx.y, t = threadIdx.x;
    for (int k = t; k < NS; k += 256) hs[k] = hidden[(size_t)b * NS + k];
    __syncthreads();
    const int j = blockIdx.x * 256 + t;
    if (j >= P) return;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 8 <= NS; k += 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] = fmaf(hs[k + u], w2[(size_t)(k + u) * P + j], s[u]);
    for (; k < NS; ++k) s[0] = fmaf(hs[k], w2[(size_t)k * P + j], s[0]);
    out[(size_t)b * out_stride + j] = b2[j] + (((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7])));
}

// ------------------------------------------------------------------------------ launchers
hipError_t stem_launch(const float* x, const float* w, const float* ba, const float* bb, float* y, int B, int H,
                       int W, int Ho, int Wo, int pad_t, int pad_l, int act, hipStream_t st) {
    dim3 grid((Wo + STEM_TW - 1) / STEM_TW, (Ho + STEM_TH - 1) / STEM_TH, B);
    stem_kernel<<<grid, 256, 0, st>>>(x, w, ba, bb, y, H, W, Ho, Wo, pad_t, pad_l, act);
    return hipGetLastError();
}

int dummy_conv_parts(int HWo) { return (HWo + 63) / 64; }

hipError_t dummy_conv_launch(const float* x, const float* w, const float* bias, float* y, float* part, int B, int H,
                             int W, int C, int Ho, int Wo, int pad_t, int pad_l, hipStream_t st) {
    dim3 grid(dummy_conv_parts(Ho * Wo), B);
    dummy_conv_kernel<<<grid, 64, 0, st>>>(x, w, bias, y, part, H, W, C, Ho, Wo, pad_t, pad_l);
    return hipGetLastError();
}

// Output channels per workgroup: the largest of {48, 40, 32, 24, 16, 8} dividing cout that still gives
// >= 512 workgroups per image, else the smallest divisor (more, smaller workgroups for the late layers).
int pw_chunk(int cout, int HW) {
    const int tiles = (HW + 63) / 64;
    int best = 0;
    for (int co : {48, 40, 32, 24, 16, 8}) {
        if (cout % co != 0) continue;
        best = co;
        if (tiles * (cout / co) >= 512) return co;
    }
    return best;
}

int pw_parts(int HW) { return (HW + 63) / 64; }

hipError_t pw_launch(const float* x, const float* se, const float* w, const float* ba, const float* bb,
                     const float* res, float* y, float* part, int B, int HW, int cin, int cout, int act,
                     hipStream_t st) {
    const int co = pw_chunk(cout, HW);
    if (co == 0 || (cin & 7) != 0) return hipErrorInvalidValue;
    dim3 grid(pw_parts(HW), cout / co, B);
#define PW_CASE(N) \
    case N: pw_kernel<N><<<grid, 256, 0, st>>>(x, se, w, ba, bb, res, y, part, HW, cin, cout, act); break;
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
    // <= 256 workgroups per image: 1-2 pixels per thread, <= 256 SE-squeeze partial rows
    int n = (HWo + *slots - 1) / *slots;
    n = n < 256 ? n : 256;
    int per = (HWo + n - 1) / n;
    per = (per + *slots - 1) / *slots * *slots;
    *ppw = per;
    *n_wg = (HWo + per - 1) / per;
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
                     const float* w2, const float* b2, float* se, float* g_out, float* s1_out, float* s2_out,
                     hipStream_t st) {
    if (C > 1024 || R > 1024) return hipErrorInvalidValue;
    se_kernel<<<B, FC_THREADS, 0, st>>>(part, n_part, 1.f / (float)hw, C, R, w1, b1, w2, b2, se, g_out, s1_out,
                                        s2_out);
    return hipGetLastError();
}

hipError_t head_launch(const float* part, int n_part, int hw, int B, int C, int NS, int P, const float* w1,
                       const float* b1, const float* w2, const float* b2, float* hidden, float* out, int out_stride,
                       float* g_out, hipStream_t st) {
    if (C > 1024 || NS > 1024) return hipErrorInvalidValue;
    head1_kernel<<<B, FC_THREADS, 0, st>>>(part, n_part, 1.f / (float)hw, C, NS, w1, b1, hidden, g_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    dim3 grid((P + 255) / 256, B);
    head2_kernel<<<grid, 256, 0, st>>>(hidden, NS, P, w2, b2, out, out_stride);
    return hipGetLastError();
}

}  // namespace rst
