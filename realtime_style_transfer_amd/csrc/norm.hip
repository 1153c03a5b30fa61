// norm.hip — conditional-instance-norm statistics and element-wise apply kernels.
//
// ConditionalInstanceNormalization.call (realtime_style_transfer/models/styleTransfer.py:57-71):
//   mean, var = tf.nn.moments(x, axes=[1,2])        (biased variance, per (b, c))
//   x = x * rsqrt(var + eps) + (-mean * rsqrt(var + eps));  x = bias + x * scale
// The producing conv writes per-tile {sum, M2, n} (two-pass inside the tile). finalize merges
// them in one f64 pass (sum of M2_t + s_t^2/n_t, minus S^2/N: Chan's merge rearranged) —
// deterministic (no atomics, fixed order) and immune to the f32 E[x^2]-E[x]^2 cancellation that
// ReLU'd, positive-weight residual convs (mean/std ~ 20) would suffer — and folds scale/bias/rsqrt into one affine (a, b) per
// (b, c) that the consumer applies in its prologue: y = a*x + b.
#include <hip/hip_runtime.h>
#include "kernels.h"

namespace rst {

constexpr int FIN_THREADS = 512;

// Sum over the 64 lanes of a wave, every lane ends with the same value, fixed order (deterministic):
// DPP butterflies inside each 16-lane row (quad xor 1, xor 2, half-row mirror, row mirror) on each
// 32-bit half, then the four row sums read out of lanes 0/16/32/48. VALU only: the ds_bpermute chain of
// __shfl_xor (6 dependent LDS round trips per value) was most of a residual finalize's 3.6 us.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xFFFFFFFFll), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float lane_read(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double lane_read(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);   // row_half_mirror
    v += dpp_f<0x140>(v);   // row_mirror
    return (lane_read(v, 0) + lane_read(v, 16)) + (lane_read(v, 32) + lane_read(v, 48));
}

template <int NT, typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
    v = wave_sum(v);
    if constexpr (NT == 64) {
        return v;
    } else {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (lane == 0) scratch[wave] = v;
        __syncthreads();
        T t = scratch[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) t += scratch[w];   // fixed order: deterministic
        return t;
    }
}

// One pass over the partials of channel c: S = sum s_t, N = sum n_t, Q = sum (M2_t + s_t^2 / n_t), all
// in f64; then M2 = Q - S^2/N. Equal to Chan's pairwise merge sum M2_t + n_t (mean_t - mean)^2; the
// cancellation in Q - S^2/N costs log2(mean^2/var) bits of f64's 53 (mean/std ~ 20 here: ~9 bits),
// far below f32 resolution. The (image, phase, tile) index space is walked as ONE flat range with
// FIN_UNROLL unconditional loads per thread (index clamped, value masked) issued before any is
// consumed — a guarded load per item made hipcc wait on each load before the next. Shapes at B=1:
// residual CINs 128 x 225 partials (one wave per channel), expand_0 32 x 3600 and expand_1 16 x 14400
// (512 threads), expand_last 3 x 450. tools/fin_probe: a launch costs ~1.5-1.9 us empty and ~3.8 us
// for the residual shape; expand_1 (11 us) is bound by the f64 statistics arithmetic on its 16 CUs.
// The style affine is fetched before the loop so its latency overlaps the partial reads.
// Summation order is fixed (accumulator j = k mod 4, then a fixed-order block sum): deterministic.
constexpr int FIN_UNROLL = 8;

// One channel's finalize by NT threads (tid < NT): the merged statistics -> the affine (a, b) the consumer
// applies, written by thread 0 (also returned in aa / bb on thread 0). Shared by finalize_kernel and the fused
// output kernel below, so both produce the same bits.
template <int NT, int U = FIN_UNROLL>
__device__ __forceinline__ void finalize_channel(const FinalizeArgs& a, int c, int b, int tid, double (*scratch)[NT / 64],
                                                 float& aa_out, float& bb_out) {
    const int b0 = a.merge_images ? 0 : b, nb = a.merge_images ? a.batch : 1;
    float scale = 1.f, bias = 0.f, scale1 = 0.f, bias1 = 0.f;
    if (tid == 0) {   // issued before the partial loads: independent of them
        if (a.style != nullptr) {
            const float* sp = a.style + (size_t)b * a.style_stride + a.style_offset;
            scale = sp[c];
            bias = sp[a.C + c];
            if (a.ab1 != nullptr) {
                scale1 = sp[a.style1_offset + c];
                bias1 = sp[a.style1_offset + a.C + c];
            }
        } else if (a.scale != nullptr) {
            scale = a.scale[b * a.affine_bstride + c];
            bias = a.bias[b * a.affine_bstride + c];
        }
    }
    // s_t^2 / n_t uses v_rcp_f64 plus one Newton step (error ~1 ulp of f64, 2^-52 relative: far below
    // the f32 result) instead of the IEEE f64 division sequence (~11 f64 instructions, the bulk of
    // this kernel's time: the statistics arithmetic, not the reads, set expand_1's 12 us);
    // n accumulates in f32 (tile counts are small integers: exact below 2^24 per accumulator).
    double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
    float n[4] = {0.f, 0.f, 0.f, 0.f};
    auto add = [&](const float4& v, int j) __attribute__((always_inline)) {
        if (v.z > 0.f) {
            const double sv = (double)v.x, nv = (double)v.z;
            double r = __builtin_amdgcn_rcp(nv);
            r = fma(fma(-nv, r, 1.0), r, r);
            s[j] += sv;
            n[j] += v.z;
            q[j] += (double)v.y + sv * sv * r;
        }
    };
    const int per_img = a.phases * a.n_part, total = nb * per_img;
    auto item = [&](int i) __attribute__((always_inline)) -> const float4* {
        const int bi = i / per_img, r = i - bi * per_img;
        const int ph = r / a.n_part, t = r - ph * a.n_part;
        return a.part + ((size_t)(b0 + bi) * a.ntot + ph * a.C + c) * a.n_part + t;
    };
    const int hi = total;
    for (int base = tid; base < hi; base += U * NT) {
        // unconditional loads (index clamped into range, the value masked afterwards): a guarded load
        // per k made hipcc wait for each load before issuing the next (one load in flight per lane)
        float4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = *item(min(base + k * NT, hi - 1));
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (base + k * NT < hi) add(v[k], k & 3);
    }
    double S = block_sum<NT>((s[0] + s[1]) + (s[2] + s[3]), scratch[0]);
    double N = block_sum<NT>(((double)n[0] + (double)n[1]) + ((double)n[2] + (double)n[3]), scratch[1]);
    double Q = block_sum<NT>((q[0] + q[1]) + (q[2] + q[3]), scratch[2]);
    if (tid == 0) {
        const double mean = N > 0.0 ? S / N : 0.0;
        const double m2 = N > 0.0 ? fmax(Q - S * mean, 0.0) : 0.0;
        const double var = N > 0.0 ? m2 / N : 0.0;
        const float rstd = (float)(1.0 / sqrt(var + (double)a.eps));
        const float aa = scale * rstd;
        aa_out = aa;
        bb_out = bias - (float)mean * aa;
        a.ab[b * a.C + c] = make_float2(aa, bb_out);
        if (a.ab1 != nullptr) {   // second style (styleTransfer.py:36-44 blends the affine per pixel)
            const float a1 = scale1 * rstd;
            a.ab1[b * a.C + c] = make_float2(a1, bias1 - (float)mean * a1);
        }
        if (a.mr != nullptr) a.mr[b * a.C + c] = make_float2((float)mean, rstd);
        if (a.moving_mean != nullptr && b == 0) {
            const double unbiased = N > 1.0 ? m2 / (N - 1.0) : var;
            a.moving_mean[c] = (float)(a.momentum * a.moving_mean[c] + (1.0 - a.momentum) * mean);
            a.moving_var[c] = (float)(a.momentum * a.moving_var[c] + (1.0 - a.momentum) * unbiased);
        }
    }
}

template <int NT, int U = FIN_UNROLL>
__global__ __launch_bounds__(NT) void finalize_kernel(FinalizeArgs a) {
    __shared__ double scratch[3][NT / 64];
    float aa, bb;
    finalize_channel<NT, U>(a, blockIdx.x, blockIdx.y, threadIdx.x, scratch, aa, bb);
}

// The network output (styleTransfer.py:269-276, 329): sigmoid(CIN(x)) of the last layer's 3 channels, with that
// CIN's finalize fused in front (num_styles = 1): the last layer added its statistics into fixed-point accumulators
// (kernels.h CinAcc), so every workgroup (g, b) forms image b's three affines itself (cin_affine_table), then applies
// affine + sigmoid to its slice of the image as float4s (hw * 3 is a multiple of 4 here). Workgroup (0, b) also
// stores the affine (rst_copy_activation reads it). No finalize kernel and no separate activation pass.
__global__ __launch_bounds__(256) void fin_sigmoid3_kernel(CinSrc s, const float* __restrict__ x,
                                                           float* __restrict__ y, int n4_img) {
    __shared__ float2 aff[3];
    const int b = blockIdx.y;
    const float4* __restrict__ xi = reinterpret_cast<const float4*>(x) + (size_t)b * n4_img;
    float4* __restrict__ yo = reinterpret_cast<float4*>(y) + (size_t)b * n4_img;
    // the thread's first two float4 are loaded before the affine merge: their latency overlaps the accumulator loads'
    // instead of following them (the merge's loads and these are independent)
    const int i0 = blockIdx.x * 256 + threadIdx.x, i1 = i0 + gridDim.x * 256;
    const float4 pre0 = xi[min(i0, n4_img - 1)], pre1 = xi[min(i1, n4_img - 1)];
    cin_affine_table<256>(s, b, 1, aff, nullptr, blockIdx.x == 0 && s.ab_out != nullptr ? s.ab_out + b * 3 : nullptr,
                          nullptr);
    __syncthreads();
    const float a0 = aff[0].x, b0 = aff[0].y, a1 = aff[1].x, b1 = aff[1].y, a2 = aff[2].x, b2 = aff[2].y;
    auto sig = [](float v) __attribute__((always_inline)) { return 1.f / (1.f + __expf(-v)); };
    for (int i = i0; i < n4_img; i += gridDim.x * 256) {
        const float4 v = i == i0 ? pre0 : (i == i1 ? pre1 : xi[i]);
        // element 4i + k has channel (4i + k) % 3: the float4 starts at channel (i % 3) ... (4i % 3 = i % 3)
        const int c0 = i % 3;
        const float aA = c0 == 0 ? a0 : (c0 == 1 ? a1 : a2), bA = c0 == 0 ? b0 : (c0 == 1 ? b1 : b2);
        const float aB = c0 == 0 ? a1 : (c0 == 1 ? a2 : a0), bB = c0 == 0 ? b1 : (c0 == 1 ? b2 : b0);
        const float aC = c0 == 0 ? a2 : (c0 == 1 ? a0 : a1), bC = c0 == 0 ? b2 : (c0 == 1 ? b0 : b1);
        yo[i] = make_float4(sig(fmaf(aA, v.x, bA)), sig(fmaf(aB, v.y, bB)), sig(fmaf(aC, v.z, bC)), sig(fmaf(aA, v.w, bA)));
    }
}

hipError_t fin_sigmoid3_launch(const CinSrc& s, const float* x, float* y, long hw, int batch, hipStream_t st) {
    if (s.acc == nullptr || s.C != 3 || s.batch != batch || s.nslot < 1 || s.nslot > CIN_ACC_MAX_SLOTS ||
        s.style == nullptr || (hw * 3) % 4 != 0 || hw * 3 / 4 >= (1L << 31))
        return hipErrorInvalidValue;
    const int n4 = (int)(hw * 3 / 4);
    // ~2 float4 per thread, about 700 workgroups at 480 x 960: every workgroup's affine merge runs in parallel
    // and the loads of a thread are independent (8 per thread in 169 workgroups: 7.5 us, latency-bound)
    int g = (n4 + 256 * 2 - 1) / (256 * 2);
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(fin_sigmoid3_kernel, dim3(g, batch), dim3(256), 0, st, s, x, y, n4);
    return hipGetLastError();
}

hipError_t finalize_launch(const FinalizeArgs& a, hipStream_t st) {
    const long per_channel = (long)a.n_part * a.phases * (a.merge_images ? a.batch : 1);
    if (per_channel <= FIN_UNROLL * 64)
        hipLaunchKernelGGL(finalize_kernel<64>, dim3(a.C, a.batch), dim3(64), 0, st, a);
    else   // expand_1 (16 x 14400 at B=1) is f64-arithmetic-bound on its 16 CUs (tools/fin_probe: the
           // same reads alone take 4 us of its 11); a 1024-thread variant measured no faster, and a
           // split over 15 workgroups per channel with a last-arriver merge no faster either (the
           // agent-scope release each writer needs costs an L2 write-back)
        hipLaunchKernelGGL(finalize_kernel<FIN_THREADS>, dim3(a.C, a.batch), dim3(FIN_THREADS), 0, st, a);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void affine_act_kernel(const float* __restrict__ x, const float2* __restrict__ ab,
                                                         const float* __restrict__ res, float* __restrict__ y,
                                                         long total, long hwc, int C, int act) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
        const int b = (int)(i / hwc);
        const int c = (int)(i % C);
        const float2 p = ab[b * C + c];
        float v = fmaf(p.x, x[i], p.y);
        if (res != nullptr) v += res[i];
        if (act == 1) v = fmaxf(v, 0.f);
        else if (act == 2) v = 1.f / (1.f + __expf(-v));
        y[i] = v;
    }
}

hipError_t affine_act_launch(const float* x, const float2* ab, const float* res, float* y, int batch, long hw, int C,
                             int act, hipStream_t st) {
    const long total = (long)batch * hw * C;
    long blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(affine_act_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, ab, res, y, total, hw * C, C, act);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void affine_act_blend_kernel(const float* __restrict__ x,
                                                               const float2* __restrict__ ab,
                                                               const float2* __restrict__ ab1,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ res, float* __restrict__ y,
                                                               long total, long hwc, int C, int act) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
        const int b = (int)(i / hwc);
        const int c = (int)(i % C);
        const float2 p0 = ab[b * C + c], p1 = ab1[b * C + c];
        const float xv = x[i];
        const float y0 = fmaf(p0.x, xv, p0.y), y1 = fmaf(p1.x, xv, p1.y);
        float v = style_blend(w[i / C], y0, y1);
        if (res != nullptr) v += res[i];
        if (act == 1) v = fmaxf(v, 0.f);
        else if (act == 2) v = 1.f / (1.f + __expf(-v));
        y[i] = v;
    }
}

hipError_t affine_act_blend_launch(const float* x, const float2* ab, const float2* ab1, const float* w,
                                   const float* res, float* y, int batch, long hw, int C, int act, hipStream_t st) {
    const long total = (long)batch * hw * C;
    long blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(affine_act_blend_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, ab, ab1, w, res, y,
                       total, hw * C, C, act);
    return hipGetLastError();
}

// Per-pixel style parameters of a two-style model: out[b][p][c] = blend(w1[b][p], params[b][0][c],
// params[b][1][c]) — the affine the conv prologues apply, exposed for the _apply_style_weights KAT.
__global__ __launch_bounds__(256) void style_param_map_kernel(const float* __restrict__ w1,
                                                              const float* __restrict__ params,
                                                              float* __restrict__ out, long total, long hw, int n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
        const int c = (int)(i % n);
        const long p = i / n;
        const int b = (int)(p / hw);
        const float* pb = params + (size_t)b * 2 * n;
        out[i] = style_blend(w1[p], pb[c], pb[n + c]);
    }
}

hipError_t style_param_map_launch(const float* w1, const float* params, float* out, int batch, long hw, int n,
                                  hipStream_t st) {
    const long total = (long)batch * hw * n;
    long blocks = (total + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(style_param_map_kernel, dim3((unsigned)blocks), dim3(256), 0, st, w1, params, out, total, hw, n);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void avgpool2_1ch_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                           int B, int H, int W) {
    const int Ho = H / 2, Wo = W / 2;
    const long total = (long)B * Ho * Wo;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256L) {
        const int ox = (int)(i % Wo);
        const int oy = (int)((i / Wo) % Ho);
        const int b = (int)(i / ((long)Wo * Ho));
        const float* p = x + ((size_t)b * H + 2 * oy) * W + 2 * ox;
        y[i] = ((p[0] + p[1]) + (p[W] + p[W + 1])) * 0.25f;
    }
}

hipError_t avgpool2_1ch_launch(const float* x, float* y, int batch, int H, int W, hipStream_t st) {
    const long total = (long)batch * (H / 2) * (W / 2);
    long blocks = (total + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(avgpool2_1ch_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, y, batch, H, W);
    return hipGetLastError();
}

// Per-tile {sum, M2, n} of x [B][hw][C] over tiles of `tile` pixels; part [B][C][n_tiles].
__global__ __launch_bounds__(256) void tile_stats_kernel(const float* __restrict__ x, float4* __restrict__ part,
                                                         long hw, int C, int tile, int n_tiles) {
    const int t = blockIdx.x, b = blockIdx.y;
    const long p0 = (long)t * tile;
    const long p1 = (p0 + tile < hw) ? p0 + tile : hw;
    for (int c = threadIdx.x; c < C; c += 256) {
        float s = 0.f;
        for (long p = p0; p < p1; ++p) s += x[((size_t)b * hw + p) * C + c];
        const float cnt = (float)(p1 - p0);
        const float mean = s / cnt;
        float m2 = 0.f;
        for (long p = p0; p < p1; ++p) {
            const float d = x[((size_t)b * hw + p) * C + c] - mean;
            m2 = fmaf(d, d, m2);
        }
        part[((size_t)b * C + c) * n_tiles + t] = make_float4(s, m2, cnt, 0.f);
    }
}

hipError_t tile_stats_launch(const float* x, float4* part, int batch, long hw, int C, int tile, hipStream_t st) {
    const int n_tiles = (int)((hw + tile - 1) / tile);
    hipLaunchKernelGGL(tile_stats_kernel, dim3(n_tiles, batch), dim3(256), 0, st, x, part, hw, C, tile, n_tiles);
    return hipGetLastError();
}

}  // namespace rst
