// predictor_train.hip — training-mode kernels of the style predictor (train_network.py fits the
// MobileNetV3Small predictor jointly with the transfer network: stylePrediction.py:25-75 with
// training=True, BatchNormalization eps 1e-3 / momentum 0.999 (keras mobilenet_v3), RMSprop).
//
// Forward (training mode): the inference conv kernels run "raw" (a = 1, b = 0, no activation) and
// BatchNormalization uses the batch statistics, so every conv unit is conv -> stats -> finalize ->
// apply:
//   bn_stats      per-(image, tile) {sum, M2 about the tile mean} of the raw conv output
//   bn_finalize   per channel: Chan merge in f64 over all tiles of all images -> mean, biased var,
//                 (a, b) = (gamma rstd, beta - mean a), moving statistics (momentum 0.999,
//                 Bessel-corrected variance) updated in place in the canonical weights
//   bn_apply      y = act(a z + b) [+ shortcut], with per-(image, tile) channel sums of y for the SE
//                 squeeze / global average pool
// Backward (gradient of sum(style_params * d_style_params)):
//   bn_bwd        dn = act'(n) dy with dy = dy_full * mul[b][c] + bcast[b][c]; S1 = sum dn,
//                 S2 = sum dn xhat (per tile, then f64 per channel: d gamma = S2, d beta = S1);
//                 dz = a (dn - S1/N - xhat S2/N)
//   1x1 conv      wgrad: split-K over pixels (LDS-staged 32-pixel chunks, 16 x 64 output tile per
//                 workgroup) into slabs, then a fixed-order slab sum; dgrad: the forward 1x1 kernel on
//                 the transposed weights (its residual input accumulates the shortcut gradient)
//   depthwise     dgrad: one lane per (input pixel, 4 channels), every tap that hits it; wgrad:
//                 K*K float4 accumulators per lane over a pixel split, slab + fixed-order sum
//   stem          wgrad only (the image needs no gradient): 27 x 16 GEMM over pixels
//   SE / heads    per-image 1024-thread kernels (sliced dot products) + batch-summed outer products
// All reductions have a fixed order (no atomics): repeated steps are bitwise identical.
#include <hip/hip_runtime.h>

#include "predictor.h"
#include "predictor_train.h"

namespace rst {

__device__ __forceinline__ float hsig_t(float x) { return fminf(fmaxf(x + 3.f, 0.f), 6.f) * (1.f / 6.f); }

__device__ __forceinline__ float act_f(float x, int act) {
    if (act == ACT_RELU) return fmaxf(x, 0.f);
    if (act == ACT_HSWISH) return x * hsig_t(x);
    return x;
}

// d act(n) / dn as TF differentiates it: ReLU' = [n > 0]; hard_swish = n * relu6(n + 3) / 6 ->
// relu6(n+3)/6 + n [0 < n+3 < 6] / 6.
__device__ __forceinline__ float act_d(float n, int act) {
    if (act == ACT_RELU) return n > 0.f ? 1.f : 0.f;
    if (act == ACT_HSWISH) {
        const float u = n + 3.f;
        const float r6 = fminf(fmaxf(u, 0.f), 6.f) * (1.f / 6.f);
        return r6 + ((u > 0.f && u < 6.f) ? n * (1.f / 6.f) : 0.f);
    }
    return 1.f;
}

__device__ __forceinline__ float4 f4(float v) { return make_float4(v, v, v, v); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 mul4(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }

// ------------------------------------------------------------------------------------ BN forward
// Tiling shared by the per-image element kernels: block = cg quads x slots, workgroup blockIdx.x
// of image blockIdx.y covers pixels [blockIdx.x * ppw, +ppw) (dw_geometry).
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ z, int HW, int C, int ppw, int slots,
                                                       float4* __restrict__ part) {
    __shared__ float4 red[256];
    const int cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg, b = blockIdx.y;
    const int p0 = blockIdx.x * ppw, p1 = min(p0 + ppw, HW);
    const float4* zb = reinterpret_cast<const float4*>(z + (size_t)b * HW * C);
    float4 s = f4(0.f);
    for (int p = p0 + slot; p < p1; p += slots) s = add4(s, zb[(size_t)p * cg + q]);
    red[t] = s;
    __syncthreads();
    s = red[q];                                                      // every thread: the tile sum
    for (int k = 1; k < slots; ++k) s = add4(s, red[k * cg + q]);
    const float n = (float)max(p1 - p0, 0);
    const float4 mean = n > 0.f ? make_float4(s.x / n, s.y / n, s.z / n, s.w / n) : f4(0.f);
    float4 m2 = f4(0.f);
    for (int p = p0 + slot; p < p1; p += slots) {
        const float4 v = zb[(size_t)p * cg + q];
        const float4 d = make_float4(v.x - mean.x, v.y - mean.y, v.z - mean.z, v.w - mean.w);
        m2 = add4(m2, mul4(d, d));
    }
    __syncthreads();
    red[t] = m2;
    __syncthreads();
    if (slot == 0) {
        for (int k = 1; k < slots; ++k) m2 = add4(m2, red[k * cg + q]);
        // layout [b][tile][C] x {sum, m2}: part[((b * n_t + tile) * C + c) * 2 + {0,1}] as float4 pairs
        float4* o = part + ((size_t)b * gridDim.x + blockIdx.x) * (size_t)cg * 2;
        o[2 * q] = s;
        o[2 * q + 1] = m2;
    }
}

// Sum over the 64 lanes of a wave in f64, the same value in every lane, fixed order (deterministic): DPP
// butterflies inside each 16-lane row (quad xor 1, xor 2, half-row mirror, row mirror) on both 32-bit
// halves, then the four row sums read from lanes 0/16/32/48 (as norm.hip's wave_sum; the ds_bpermute chain
// of a double __shfl_xor butterfly was most of these small finalize kernels).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xFFFFFFFFll), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    return (lane_d(v, 0) + lane_d(v, 16)) + (lane_d(v, 32) + lane_d(v, 48));
}

// One workgroup (256 threads) per channel quad: Chan merge over all tiles of all images. Every partial float4
// carries the quad's four channels, so each is read once for all four (the one-channel-per-workgroup form read
// every 16-B partial four times, one lane per scattered line: 17.6 us per call on the training step's BN layers).
// Per channel: f64 sums in a fixed order (lane-strided loop, DPP wave sums, the four wave sums added in order).
__device__ __forceinline__ double block4_sum_d(double v, double* red, int t) {
    v = wave_sum_d(v);
    __syncthreads();
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float4* __restrict__ part, int n_tiles, int B, int HW,
                                                          int C, int ppw, float* __restrict__ gamma_beta_mm_mv,
                                                          float eps, float momentum, float2* __restrict__ ab,
                                                          float2* __restrict__ mr) {
    __shared__ double red[4];
    const int q = blockIdx.x, t = threadIdx.x, cg = C >> 2;
    const int total = B * n_tiles;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = t; i < total; i += 256) {
        const float4 v = part[(size_t)i * cg * 2 + 2 * q];
        s[0] += (double)v.x;
        s[1] += (double)v.y;
        s[2] += (double)v.z;
        s[3] += (double)v.w;
    }
    const double N = (double)B * HW;
    double mean[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) mean[l] = block4_sum_d(s[l], red, t) / N;
    double m2[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = t; i < total; i += 256) {
        const int tile = i % n_tiles;
        const double n = (double)max(min(ppw, HW - tile * ppw), 0);
        if (n <= 0.0) continue;
        const float4 sv = part[(size_t)i * cg * 2 + 2 * q];
        const float4 mv = part[(size_t)i * cg * 2 + 2 * q + 1];
        const double ts[4] = {(double)sv.x, (double)sv.y, (double)sv.z, (double)sv.w};
        const double tm[4] = {(double)mv.x, (double)mv.y, (double)mv.z, (double)mv.w};
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const double d = ts[l] / n - mean[l];
            m2[l] += tm[l] + n * d * d;
        }
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) m2[l] = block4_sum_d(m2[l], red, t);
    if (t < 4) {
        const int c = 4 * q + t;
        const double mn = t == 0 ? mean[0] : t == 1 ? mean[1] : t == 2 ? mean[2] : mean[3];
        const double mm = t == 0 ? m2[0] : t == 1 ? m2[1] : t == 2 ? m2[2] : m2[3];
        const double var = mm / N;
        const double rstd = 1.0 / sqrt(var + (double)eps);
        float* gb = gamma_beta_mm_mv;
        const double a = (double)gb[c] * rstd;
        ab[c] = make_float2((float)a, (float)((double)gb[C + c] - mn * a));
        mr[c] = make_float2((float)mn, (float)rstd);
        const double unbiased = N > 1.0 ? mm / (N - 1.0) : var;
        gb[2 * C + c] = (float)((double)gb[2 * C + c] * momentum + mn * (1.0 - momentum));
        gb[3 * C + c] = (float)((double)gb[3 * C + c] * momentum + unbiased * (1.0 - momentum));
    }
}

// y = act(a z + b) [+ res]; part (optional): per-(image, tile) channel sums of y, [b][tile][C]
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ z, const float2* __restrict__ ab,
                                                       const float* __restrict__ res, float* __restrict__ y, int HW,
                                                       int C, int ppw, int slots, int act, float* __restrict__ part) {
    __shared__ float4 red[256];
    const int cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg, b = blockIdx.y;
    const int p0 = blockIdx.x * ppw, p1 = min(p0 + ppw, HW);
    const size_t base = (size_t)b * HW * cg;
    const float4* z4 = reinterpret_cast<const float4*>(z) + base;
    const float4* r4 = res != nullptr ? reinterpret_cast<const float4*>(res) + base : nullptr;
    float4* y4 = reinterpret_cast<float4*>(y) + base;
    const float2 a0 = ab[4 * q], a1 = ab[4 * q + 1], a2 = ab[4 * q + 2], a3 = ab[4 * q + 3];
    float4 s = f4(0.f);
    for (int p = p0 + slot; p < p1; p += slots) {
        const float4 v = z4[(size_t)p * cg + q];
        float4 o = make_float4(act_f(fmaf(a0.x, v.x, a0.y), act), act_f(fmaf(a1.x, v.y, a1.y), act),
                               act_f(fmaf(a2.x, v.z, a2.y), act), act_f(fmaf(a3.x, v.w, a3.y), act));
        if (r4 != nullptr) o = add4(o, r4[(size_t)p * cg + q]);
        y4[(size_t)p * cg + q] = o;
        s = add4(s, o);
    }
    if (part == nullptr) return;
    red[t] = s;
    __syncthreads();
    if (slot == 0) {
        for (int k = 1; k < slots; ++k) s = add4(s, red[k * cg + q]);
        reinterpret_cast<float4*>(part)[((size_t)b * gridDim.x + blockIdx.x) * cg + q] = s;
    }
}

// ----------------------------------------------------------------------------------- BN backward
// dn = act'(a z + b) * (dy[b][p][c] * mul[b][c] + bcast[b][c]); per tile {S1 = sum dn, S2 = sum dn xhat}
__device__ __forceinline__ float4 bn_dn(const float4 z, const float4 dyv, const float4 mulv, const float4 bc,
                                         const float2* ab, int q, int act) {
    float4 d = add4(mul4(dyv, mulv), bc);
    const float2 a0 = ab[4 * q], a1 = ab[4 * q + 1], a2 = ab[4 * q + 2], a3 = ab[4 * q + 3];
    d.x *= act_d(fmaf(a0.x, z.x, a0.y), act);
    d.y *= act_d(fmaf(a1.x, z.y, a1.y), act);
    d.z *= act_d(fmaf(a2.x, z.z, a2.y), act);
    d.w *= act_d(fmaf(a3.x, z.w, a3.y), act);
    return d;
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnBwdArgs a) {
    __shared__ float4 red[256];
    const int C = a.C, cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg, b = blockIdx.y;
    const int p0 = blockIdx.x * a.ppw, p1 = min(p0 + a.ppw, a.HW);
    const size_t base = (size_t)b * a.HW * cg;
    const float4* z4 = reinterpret_cast<const float4*>(a.z) + base;
    const float4* d4 = a.dy != nullptr ? reinterpret_cast<const float4*>(a.dy) + base : nullptr;
    const float4 mulv = a.mul != nullptr ? reinterpret_cast<const float4*>(a.mul)[(size_t)b * cg + q] : f4(1.f);
    const float4 bc = a.bcast != nullptr ? reinterpret_cast<const float4*>(a.bcast)[(size_t)b * cg + q] : f4(0.f);
    const float2 m0 = a.mr[4 * q], m1 = a.mr[4 * q + 1], m2 = a.mr[4 * q + 2], m3 = a.mr[4 * q + 3];
    float4 s1 = f4(0.f), s2 = f4(0.f);
    for (int p = p0 + slot; p < p1; p += a.slots) {
        const float4 z = z4[(size_t)p * cg + q];
        const float4 dn = bn_dn(z, d4 != nullptr ? d4[(size_t)p * cg + q] : f4(0.f), mulv, bc, a.ab, q, a.act);
        s1 = add4(s1, dn);
        s2.x = fmaf(dn.x, (z.x - m0.x) * m0.y, s2.x);
        s2.y = fmaf(dn.y, (z.y - m1.x) * m1.y, s2.y);
        s2.z = fmaf(dn.z, (z.z - m2.x) * m2.y, s2.z);
        s2.w = fmaf(dn.w, (z.w - m3.x) * m3.y, s2.w);
    }
    red[t] = s1;
    __syncthreads();
    if (slot == 0)
        for (int k = 1; k < a.slots; ++k) s1 = add4(s1, red[k * cg + q]);
    __syncthreads();
    red[t] = s2;
    __syncthreads();
    if (slot == 0) {
        for (int k = 1; k < a.slots; ++k) s2 = add4(s2, red[k * cg + q]);
        float4* o = a.part + ((size_t)b * gridDim.x + blockIdx.x) * (size_t)cg * 2;
        o[2 * q] = s1;
        o[2 * q + 1] = s2;
    }
}

__global__ __launch_bounds__(64) void bn_bwd_finalize_kernel(BnBwdArgs a) {
    const int c = blockIdx.x, t = threadIdx.x, cg = a.C >> 2, q = c >> 2, l = c & 3;
    const int total = a.B * a.n_tiles;
    double s1 = 0.0, s2 = 0.0;
    for (int i = t; i < total; i += 64) {
        const float4 v1 = a.part[(size_t)i * cg * 2 + 2 * q];
        const float4 v2 = a.part[(size_t)i * cg * 2 + 2 * q + 1];
        s1 += (double)(l == 0 ? v1.x : l == 1 ? v1.y : l == 2 ? v1.z : v1.w);
        s2 += (double)(l == 0 ? v2.x : l == 1 ? v2.y : l == 2 ? v2.z : v2.w);
    }
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    if (t == 0) {
        const double N = (double)a.B * a.HW;
        a.consts[c] = make_float2((float)(s1 / N), (float)(s2 / N));
        a.dgamma[c] = (float)s2;
        a.dgamma[a.C + c] = (float)s1;   // beta
    }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdArgs a) {
    const int C = a.C, cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg, b = blockIdx.y;
    const int p0 = blockIdx.x * a.ppw, p1 = min(p0 + a.ppw, a.HW);
    const size_t base = (size_t)b * a.HW * cg;
    const float4* z4 = reinterpret_cast<const float4*>(a.z) + base;
    const float4* d4 = a.dy != nullptr ? reinterpret_cast<const float4*>(a.dy) + base : nullptr;
    float4* o4 = reinterpret_cast<float4*>(a.dz) + base;
    const float4 mulv = a.mul != nullptr ? reinterpret_cast<const float4*>(a.mul)[(size_t)b * cg + q] : f4(1.f);
    const float4 bc = a.bcast != nullptr ? reinterpret_cast<const float4*>(a.bcast)[(size_t)b * cg + q] : f4(0.f);
    const float2 m[4] = {a.mr[4 * q], a.mr[4 * q + 1], a.mr[4 * q + 2], a.mr[4 * q + 3]};
    const float2 k[4] = {a.consts[4 * q], a.consts[4 * q + 1], a.consts[4 * q + 2], a.consts[4 * q + 3]};
    const float2 ab[4] = {a.ab[4 * q], a.ab[4 * q + 1], a.ab[4 * q + 2], a.ab[4 * q + 3]};
    for (int p = p0 + slot; p < p1; p += a.slots) {
        const float4 z = z4[(size_t)p * cg + q];
        const float4 dn = bn_dn(z, d4 != nullptr ? d4[(size_t)p * cg + q] : f4(0.f), mulv, bc, a.ab, q, a.act);
        float4 r;
        r.x = ab[0].x * (dn.x - k[0].x - (z.x - m[0].x) * m[0].y * k[0].y);
        r.y = ab[1].x * (dn.y - k[1].x - (z.y - m[1].x) * m[1].y * k[1].y);
        r.z = ab[2].x * (dn.z - k[2].x - (z.z - m[2].x) * m[2].y * k[2].y);
        r.w = ab[3].x * (dn.w - k[3].x - (z.w - m[3].x) * m[3].y * k[3].y);
        o4[(size_t)p * cg + q] = r;
    }
}

// ---------------------------------------------------------------------------------- 1x1 wgrad
// slab[s][ci][co] = sum over pixel split s of (x[p][ci] * se[b][ci]) * dz[p][co]; p runs over B*HW.
// grid (ceil(cin/16), ceil(cout/64), S); block 256: thread (ci = t/16, co4 = t%16) -> 4 outputs.
constexpr int WG_PC = 32;

__global__ __launch_bounds__(256) void pw_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ se,
                                                       const float* __restrict__ dz, int B, int HW, int cin, int cout,
                                                       int pps, float* __restrict__ slab) {
    __shared__ float xs[WG_PC][16];
    __shared__ float4 ds[WG_PC][16];
    const int t = threadIdx.x, ci_l = t >> 4, co4 = t & 15;
    const int ci0 = blockIdx.x * 16, co0 = blockIdx.y * 64;
    const long N = (long)B * HW;
    const long q0 = (long)blockIdx.z * pps, q1 = min(N, q0 + pps);
    float4 acc = f4(0.f);
    for (long c0 = q0; c0 < q1; c0 += WG_PC) {
        // stage x [32][16] (2 values per thread) and dz [32][64] (2 float4 per thread), branch-free
        float xv[2];
        float4 dv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = t + i * 256;                  // 512 = 32 px x 16 ci
            const int px = e >> 4, cl = e & 15;
            const long p = min(c0 + px, q1 - 1);
            const int ci = min(ci0 + cl, cin - 1);
            const int b = (int)(p / HW);
            float v = x[(size_t)p * cin + ci];
            if (se != nullptr) v *= se[(size_t)b * cin + ci];
            xv[i] = (c0 + px < q1 && ci0 + cl < cin) ? v : 0.f;
            const int px2 = e >> 4, c4 = e & 15;         // 512 float4 = 32 px x 16 co4
            const long p2 = min(c0 + px2, q1 - 1);
            const int co = min(co0 + 4 * c4, cout - 4);
            const float4 d = *reinterpret_cast<const float4*>(dz + (size_t)p2 * cout + co);
            dv[i] = (c0 + px2 < q1 && co0 + 4 * c4 < cout) ? d : f4(0.f);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = t + i * 256;
            xs[e >> 4][e & 15] = xv[i];
            ds[e >> 4][e & 15] = dv[i];
        }
        __syncthreads();
#pragma unroll 8
        for (int px = 0; px < WG_PC; ++px) {
            const float a = xs[px][ci_l];
            const float4 d = ds[px][co4];
            acc.x = fmaf(a, d.x, acc.x);
            acc.y = fmaf(a, d.y, acc.y);
            acc.z = fmaf(a, d.z, acc.z);
            acc.w = fmaf(a, d.w, acc.w);
        }
        __syncthreads();
    }
    const int ci = ci0 + ci_l, co = co0 + 4 * co4;
    if (ci < cin && co < cout)
        *reinterpret_cast<float4*>(slab + ((size_t)blockIdx.z * cin + ci) * cout + co) = acc;
}

// out[i] = sum_s slab[s][i], fixed order: a workgroup owns 64 consecutive outputs; its four waves sum
// contiguous quarters of the split range (8 loads in flight per lane) and wave 0 adds the quarters in
// order (one lane per output walking all S splits serially was latency-bound: 34 us for S = 512)
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int S, size_t n,
                                                       float* __restrict__ out) {
    __shared__ float part[3][64];
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const size_t i = (size_t)blockIdx.x * 64 + lane;
    float s = 0.f;
    if (i < n) {
        const int k0 = (S * q) / 4, k1 = (S * (q + 1)) / 4;
#pragma unroll 8
        for (int k = k0; k < k1; ++k) s += slab[(size_t)k * n + i];
    }
    if (q > 0) part[q - 1][lane] = s;
    __syncthreads();
    if (q == 0 && i < n) out[i] = ((s + part[0][lane]) + part[1][lane]) + part[2][lane];
}

// w [rows][cols] -> wt [cols][rows]
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ w, int rows, int cols,
                                                        float* __restrict__ wt) {
    const size_t n = (size_t)rows * cols;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int r = (int)(i / cols), c = (int)(i % cols);
        wt[(size_t)c * rows + r] = w[i];
    }
}

__global__ __launch_bounds__(256) void transpose_batch_kernel(const float* __restrict__ w, TransposeJobs jobs,
                                                              float* __restrict__ wt) {
    const long long total = jobs.end[jobs.n - 1];
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        int j = 0;
        while (i >= jobs.end[j]) ++j;
        const long long e = i - (j ? jobs.end[j - 1] : 0);
        const int cols = jobs.cols[j], r = (int)(e / cols), c = (int)(e - (long long)r * cols);
        wt[jobs.dst[j] + (long long)c * jobs.rows[j] + r] = w[jobs.src[j] + e];
    }
}

// -------------------------------------------------------------------------------- depthwise bwd
// dx[b][iy][ix][c] = sum over taps (ky, kx) with oy = (iy + pad_t - ky) / S integral and in range of
// w[ky][kx][c] dz[b][oy][ox][c]. One lane per (input pixel, channel quad), dw-style tiling over input
// pixels.
template <int K, int S>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const float* __restrict__ dz, const float* __restrict__ w,
                                                       float* __restrict__ dx, int H, int W, int C, int Ho, int Wo,
                                                       int pad_t, int pad_l, int ppw, int slots) {
    const int cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg, b = blockIdx.y;
    const int HWi = H * W;
    const int p0 = blockIdx.x * ppw, p1 = min(p0 + ppw, HWi);
    const float4* d4 = reinterpret_cast<const float4*>(dz + (size_t)b * Ho * Wo * C);
    const float4* w4 = reinterpret_cast<const float4*>(w);
    float4* o4 = reinterpret_cast<float4*>(dx + (size_t)b * HWi * C);
    for (int p = p0 + slot; p < p1; p += slots) {
        const int iy = p / W, ix = p - iy * W;
        float4 v[K * K];
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int ny = iy + pad_t - ky, nx = ix + pad_l - kx;
                const int oy = min(max(ny / S, 0), Ho - 1), ox = min(max(nx / S, 0), Wo - 1);
                v[ky * K + kx] = d4[((size_t)oy * Wo + ox) * cg + q];
            }
        float4 acc = f4(0.f);
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int ny = iy + pad_t - ky, nx = ix + pad_l - kx;
                const bool ok = ny >= 0 && nx >= 0 && (ny % S) == 0 && (nx % S) == 0 && ny / S < Ho && nx / S < Wo;
                const float m = ok ? 1.f : 0.f;
                const float4 k = w4[(ky * K + kx) * cg + q];
                const float4 d = v[ky * K + kx];
                acc.x = fmaf(d.x * m, k.x, acc.x);
                acc.y = fmaf(d.y * m, k.y, acc.y);
                acc.z = fmaf(d.z * m, k.z, acc.z);
                acc.w = fmaf(d.w * m, k.w, acc.w);
            }
        o4[(size_t)p * cg + q] = acc;
    }
}

// slab[s][tap][C]: per pixel split s (over B*Ho*Wo output pixels) the sums of x(shifted) * dz
template <int K, int S>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                       int B, int H, int W, int C, int Ho, int Wo, int pad_t, int pad_l,
                                                       int pps, int slots, float* __restrict__ slab) {
    __shared__ float4 red[256];
    const int cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg;
    const long N = (long)B * Ho * Wo;
    const long q0 = (long)blockIdx.x * pps, q1 = min(N, q0 + pps);
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* d4 = reinterpret_cast<const float4*>(dz);
    float4 acc[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) acc[i] = f4(0.f);
    for (long p = q0 + slot; p < q1; p += slots) {
        const int b = (int)(p / (Ho * Wo));
        const int r = (int)(p - (long)b * Ho * Wo);
        const int oy = r / Wo, ox = r - oy * Wo;
        const float4 d = d4[(size_t)p * cg + q];
        float4 v[K * K];
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int iy = min(max(oy * S - pad_t + ky, 0), H - 1), ix = min(max(ox * S - pad_l + kx, 0), W - 1);
                v[ky * K + kx] = x4[(((size_t)b * H + iy) * W + ix) * cg + q];
            }
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int iy = oy * S - pad_t + ky, ix = ox * S - pad_l + kx;
                const float m = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? 1.f : 0.f;
                const float4 xv = v[ky * K + kx];
                float4& a = acc[ky * K + kx];
                a.x = fmaf(xv.x * m, d.x, a.x);
                a.y = fmaf(xv.y * m, d.y, a.y);
                a.z = fmaf(xv.z * m, d.z, a.z);
                a.w = fmaf(xv.w * m, d.w, a.w);
            }
    }
    float4* o = reinterpret_cast<float4*>(slab) + (size_t)blockIdx.x * K * K * cg;
#pragma unroll
    for (int i = 0; i < K * K; ++i) {
        __syncthreads();
        red[t] = acc[i];
        __syncthreads();
        if (slot == 0) {
            float4 s = acc[i];
            for (int k = 1; k < slots; ++k) s = add4(s, red[k * cg + q]);
            o[(size_t)i * cg + q] = s;
        }
    }
}

// ------------------------------------------------------------------------------------ stem wgrad
// slab[s][m][co], m = (ky*3 + kx)*3 + ci: sum over the split's output pixels of xr[m] * dz[co], where
// xr = 2x - 1 inside the image and 0 in the SAME padding. block 128: thread (m < 27, co4 < 4).
constexpr int STEM_WPC = 64;

__global__ __launch_bounds__(128) void stem_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                         int B, int H, int W, int Ho, int Wo, int pad_t, int pad_l,
                                                         int pps, float* __restrict__ slab) {
    __shared__ float xs[STEM_WPC][28];
    __shared__ float4 ds[STEM_WPC][4];
    const int t = threadIdx.x, m = t >> 2, co4 = t & 3;
    const long N = (long)B * Ho * Wo;
    const long q0 = (long)blockIdx.x * pps, q1 = min(N, q0 + pps);
    float4 acc = f4(0.f);
    for (long c0 = q0; c0 < q1; c0 += STEM_WPC) {
        constexpr int NX = (STEM_WPC * 27 + 127) / 128;
        float xv[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int e = min(t + i * 128, STEM_WPC * 27 - 1);
            const int px = e / 27, mm = e - px * 27;
            const long p = min(c0 + px, q1 - 1);
            const int b = (int)(p / (Ho * Wo));
            const int r = (int)(p - (long)b * Ho * Wo);
            const int oy = r / Wo, ox = r - oy * Wo;
            const int tap = mm / 3, ci = mm - tap * 3;
            const int iy = oy * 2 - pad_t + tap / 3, ix = ox * 2 - pad_l + tap % 3;
            const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
            const float v = x[(((size_t)b * H + cy) * W + cx) * 3 + ci];
            xv[i] = (iy >= 0 && iy < H && ix >= 0 && ix < W && c0 + px < q1) ? 2.f * v - 1.f : 0.f;
        }
        float4 dv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = t + i * 128;                   // 256 float4 = 64 px x 4 co4
            const long p = min(c0 + (e >> 2), q1 - 1);
            const float4 d = reinterpret_cast<const float4*>(dz)[(size_t)p * 4 + (e & 3)];
            dv[i] = c0 + (e >> 2) < q1 ? d : f4(0.f);
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int e = t + i * 128;
            if (e < STEM_WPC * 27) xs[e / 27][e % 27] = xv[i];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = t + i * 128;
            ds[e >> 2][e & 3] = dv[i];
        }
        __syncthreads();
        if (m < 27) {
#pragma unroll 8
            for (int px = 0; px < STEM_WPC; ++px) {
                const float a = xs[px][m];
                const float4 d = ds[px][co4];
                acc.x = fmaf(a, d.x, acc.x);
                acc.y = fmaf(a, d.y, acc.y);
                acc.z = fmaf(a, d.z, acc.z);
                acc.w = fmaf(a, d.w, acc.w);
            }
        }
        __syncthreads();
    }
    if (m < 27) reinterpret_cast<float4*>(slab)[((size_t)blockIdx.x * 27 + m) * 4 + co4] = acc;
}

// DUMMY extractor backward: dz[b][p] = dg[b] / HWo for every output pixel (global average pool of a
// 1-channel map): dW[ky][kx][c] = sum_b dg[b]/HWo sum_p x[b][iy][ix][c], d bias = sum_b dg[b].
// One block per weight.
__global__ __launch_bounds__(256) void dummy_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dg,
                                                          int B, int H, int W, int C, int Ho, int Wo, int pad_t,
                                                          int pad_l, float* __restrict__ dw, float* __restrict__ db) {
    __shared__ float red[256];
    const int wi = blockIdx.x, t = threadIdx.x;
    const int tap = wi / C, c = wi - tap * C, ky = tap / 9, kx = tap % 9;
    float tot = 0.f;
    for (int b = 0; b < B; ++b) {
        float s = 0.f;
        for (int p = t; p < Ho * Wo; p += 256) {
            const int oy = p / Wo, ox = p - oy * Wo;
            const int iy = oy * 5 - pad_t + ky, ix = ox * 5 - pad_l + kx;
            const float v = x[(((size_t)b * H + min(max(iy, 0), H - 1)) * W + min(max(ix, 0), W - 1)) * C + c];
            s += (iy >= 0 && iy < H && ix >= 0 && ix < W) ? v : 0.f;
        }
        red[t] = s;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (t < o) red[t] += red[t + o];
            __syncthreads();
        }
        tot += red[0] * (dg[b] / (float)(Ho * Wo));
        __syncthreads();
    }
    if (t == 0) {
        dw[wi] = tot;
        if (wi == 0) {
            float s = 0.f;
            for (int b = 0; b < B; ++b) s += dg[b];
            db[0] = s;
        }
    }
}

// ----------------------------------------------------------------------------- SE / heads bwd
constexpr int FCT = 1024;

// out[j] = sum_k W[j][k] in[k] (W row-major [N][K]); threads (j, slice); fixed-order slice merge
__device__ void rowdot(const float* in, int K, const float* __restrict__ Wm, int N, float* out, float* red) {
    const int t = threadIdx.x;
    for (int j0 = 0; j0 < N; j0 += FCT) {
        const int n = min(N - j0, FCT);
        const int Q = max(1, min(32, FCT / n));
        const int j = t % n, qq = t / n;
        if (qq < Q) {
            const int k0 = (K * qq) / Q, k1 = (K * (qq + 1)) / Q;
            const float* row = Wm + (size_t)(j0 + j) * K;
            float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            int k = k0;
            for (; k + 8 <= k1; k += 8)
#pragma unroll
                for (int u = 0; u < 8; ++u) s[u] = fmaf(in[k + u], row[k + u], s[u]);
            for (; k < k1; ++k) s[0] = fmaf(in[k], row[k], s[0]);
            red[qq * n + j] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        }
        __syncthreads();
        for (int jj = t; jj < n; jj += FCT) {
            float s = 0.f;
            for (int q2 = 0; q2 < Q; ++q2) s += red[q2 * n + jj];
            out[j0 + jj] = s;
        }
        __syncthreads();
    }
}

// SE backward, one workgroup per image. dse partials [b][tile][C] (sums of dxin * u) -> dse;
// ds2 = dse hsig'(s2); dh = W2 ds2; ds1 = dh [s1 > 0]; dg = W1 ds1. Writes ds2, ds1 and
// dg / hw (the broadcast gradient of the squeezed map).
__global__ __launch_bounds__(FCT) void se_bwd_kernel(const float* __restrict__ part, int n_part, int C, int R, int hw,
                                                     const float* __restrict__ w1, const float* __restrict__ w2,
                                                     const float* __restrict__ s1, const float* __restrict__ s2,
                                                     float* __restrict__ ds1_out, float* __restrict__ ds2_out,
                                                     float* __restrict__ dgb) {
    __shared__ float v_c[1024];
    __shared__ float v_r[1024];
    __shared__ float red[FCT];
    const int b = blockIdx.x, t = threadIdx.x;
    // dse[c] = sum over tiles (fixed order), then ds2
    for (int c = t; c < C; c += FCT) {
        // four accumulators (partial k -> k mod 4), combined in a fixed order: deterministic, and 8 loads in
        // flight per lane instead of one dependent add chain over the tiles (58 us per call at B=4)
        const float* pc = part + (size_t)b * n_part * C + c;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int k = 0;
#pragma unroll 2
        for (; k + 4 <= n_part; k += 4) {
            a0 += pc[(size_t)k * C];
            a1 += pc[(size_t)(k + 1) * C];
            a2 += pc[(size_t)(k + 2) * C];
            a3 += pc[(size_t)(k + 3) * C];
        }
        for (; k < n_part; ++k) a0 += pc[(size_t)k * C];
        const float s = (a0 + a1) + (a2 + a3);
        const float u = s2[(size_t)b * C + c] + 3.f;
        const float d = (u > 0.f && u < 6.f) ? s * (1.f / 6.f) : 0.f;
        v_c[c] = d;
        ds2_out[(size_t)b * C + c] = d;
    }
    __syncthreads();
    rowdot(v_c, C, w2, R, v_r, red);          // dh[r] = sum_c W2[r][c] ds2[c]
    for (int r = t; r < R; r += FCT) {
        const float d = s1[(size_t)b * R + r] > 0.f ? v_r[r] : 0.f;
        v_r[r] = d;
        ds1_out[(size_t)b * R + r] = d;
    }
    __syncthreads();
    rowdot(v_r, R, w1, C, v_c, red);          // dg[c] = sum_r W1[c][r] ds1[r]
    for (int c = t; c < C; c += FCT) dgb[(size_t)b * C + c] = v_c[c] / (float)hw;
}

// dse partials: per-(image, tile) channel sums of dxin * u (u = the depthwise output the SE scaled)
__global__ __launch_bounds__(256) void se_dscale_kernel(const float* __restrict__ dxin, const float* __restrict__ u,
                                                        int HW, int C, int ppw, int slots, float* __restrict__ part) {
    __shared__ float4 red[256];
    const int cg = C >> 2, t = threadIdx.x, q = t % cg, slot = t / cg, b = blockIdx.y;
    const int p0 = blockIdx.x * ppw, p1 = min(p0 + ppw, HW);
    const size_t base = (size_t)b * HW * cg;
    const float4* d4 = reinterpret_cast<const float4*>(dxin) + base;
    const float4* u4 = reinterpret_cast<const float4*>(u) + base;
    float4 s = f4(0.f);
    for (int p = p0 + slot; p < p1; p += slots) s = add4(s, mul4(d4[(size_t)p * cg + q], u4[(size_t)p * cg + q]));
    red[t] = s;
    __syncthreads();
    if (slot == 0) {
        for (int k = 1; k < slots; ++k) s = add4(s, red[k * cg + q]);
        reinterpret_cast<float4*>(part)[((size_t)b * gridDim.x + blockIdx.x) * cg + q] = s;
    }
}

// heads backward step, one workgroup per image: out[b][j] = scale * sum_k W[j][k] in[b][k]
__global__ __launch_bounds__(FCT) void rowdot_kernel(const float* __restrict__ in, int K, const float* __restrict__ Wm,
                                                     int N, float scale, float* __restrict__ out) {
    __shared__ float v_in[4096];
    __shared__ float v_out[4096];
    __shared__ float red[FCT];
    const int b = blockIdx.x, t = threadIdx.x;
    for (int k = t; k < K; k += FCT) v_in[k] = in[(size_t)b * K + k];
    __syncthreads();
    rowdot(v_in, K, Wm, N, v_out, red);
    for (int j = t; j < N; j += FCT) out[(size_t)b * N + j] = v_out[j] * scale;
}

// dW[m][n] = sum_b f(a[b][m]) d[b][n] (f = relu when relu_a), db[n] = sum_b d[b][n] (optional)
__global__ __launch_bounds__(256) void outer_kernel(const float* __restrict__ a, int M, const float* __restrict__ d,
                                                    int N, int B, int relu_a, float* __restrict__ dW,
                                                    float* __restrict__ db) {
    const size_t n = (size_t)M * N;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int m = (int)(i / N), j = (int)(i % N);
        float s = 0.f;
        for (int b = 0; b < B; ++b) {
            float av = a[(size_t)b * M + m];
            if (relu_a) av = fmaxf(av, 0.f);
            s = fmaf(av, d[(size_t)b * N + j], s);
        }
        dW[i] = s;
        if (db != nullptr && m == 0) {
            float t2 = 0.f;
            for (int b = 0; b < B; ++b) t2 += d[(size_t)b * N + j];
            db[j] = t2;
        }
    }
}

// ------------------------------------------------------------------------------------ launchers
static unsigned grid1d(size_t n, unsigned cap) {
    unsigned g = (unsigned)((n + 255) / 256);
    return g < 1 ? 1 : (g > cap ? cap : g);
}

void elem_geometry(int C, int HW, int* block, int* slots, int* ppw, int* n_tiles) {
    dw_geometry(C, HW, block, slots, ppw, n_tiles);
}

hipError_t bn_forward_launch(const float* z, int B, int HW, int C, float* gamma_beta_mm_mv, float eps, float momentum,
                             float4* part, float2* ab, float2* mr, const float* res, float* y, int act,
                             float* y_part, hipStream_t st) {
    int block, slots, ppw, nt;
    elem_geometry(C, HW, &block, &slots, &ppw, &nt);
    if (C % 4 != 0) return hipErrorInvalidValue;   // channel quads (bn_stats / bn_finalize)
    bn_stats_kernel<<<dim3(nt, B), block, 0, st>>>(z, HW, C, ppw, slots, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    bn_finalize_kernel<<<C / 4, 256, 0, st>>>(part, nt, B, HW, C, ppw, gamma_beta_mm_mv, eps, momentum, ab, mr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    bn_apply_kernel<<<dim3(nt, B), block, 0, st>>>(z, ab, res, y, HW, C, ppw, slots, act, y_part);
    return hipGetLastError();
}

hipError_t bn_backward_launch(BnBwdArgs a, hipStream_t st) {
    int block;
    elem_geometry(a.C, a.HW, &block, &a.slots, &a.ppw, &a.n_tiles);
    bn_bwd_reduce_kernel<<<dim3(a.n_tiles, a.B), block, 0, st>>>(a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    bn_bwd_finalize_kernel<<<a.C, 64, 0, st>>>(a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    bn_bwd_apply_kernel<<<dim3(a.n_tiles, a.B), block, 0, st>>>(a);
    return hipGetLastError();
}

int pw_wgrad_splits(int B, int HW, int cin, int cout, int* pps) {
    const long N = (long)B * HW;
    const int tiles = ((cin + 15) / 16) * ((cout + 63) / 64);
    long S = (512 + tiles - 1) / tiles;
    const long smax = (N + 63) / 64;
    S = S < 1 ? 1 : (S > smax ? smax : S);
    long per = (N + S - 1) / S;
    per = (per + WG_PC - 1) / WG_PC * WG_PC;
    *pps = (int)per;
    return (int)((N + per - 1) / per);
}

hipError_t pw_wgrad_launch(const float* x, const float* se, const float* dz, int B, int HW, int cin, int cout,
                           float* slab, float* dW, hipStream_t st) {
    if ((cout & 3) != 0) return hipErrorInvalidValue;
    int pps;
    const int S = pw_wgrad_splits(B, HW, cin, cout, &pps);
    pw_wgrad_kernel<<<dim3((cin + 15) / 16, (cout + 63) / 64, S), 256, 0, st>>>(x, se, dz, B, HW, cin, cout, pps, slab);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t n = (size_t)cin * cout;
    slab_sum_kernel<<<(unsigned)((n + 63) / 64), 256, 0, st>>>(slab, S, n, dW);
    return hipGetLastError();
}

hipError_t transpose_batch_launch(const float* w, const TransposeJobs& jobs, float* wt, hipStream_t st) {
    if (jobs.n <= 0 || jobs.n > TransposeJobs::MAX) return hipErrorInvalidValue;
    transpose_batch_kernel<<<grid1d((size_t)jobs.end[jobs.n - 1], 1024), 256, 0, st>>>(w, jobs, wt);
    return hipGetLastError();
}

hipError_t transpose_launch(const float* w, int rows, int cols, float* wt, hipStream_t st) {
    transpose_kernel<<<grid1d((size_t)rows * cols, 1024), 256, 0, st>>>(w, rows, cols, wt);
    return hipGetLastError();
}

hipError_t dw_dgrad_launch(const float* dz, const float* w, float* dx, int B, int H, int W, int C, int Ho, int Wo,
                           int k, int stride, int pad_t, int pad_l, hipStream_t st) {
    int block, slots, ppw, nt;
    dw_geometry(C, H * W, &block, &slots, &ppw, &nt);
    dim3 grid(nt, B);
#define DWD(KK, SS)                                                                                              \
    if (k == KK && stride == SS) {                                                                               \
        dw_dgrad_kernel<KK, SS><<<grid, block, 0, st>>>(dz, w, dx, H, W, C, Ho, Wo, pad_t, pad_l, ppw, slots);   \
        return hipGetLastError();                                                                                \
    }
    DWD(3, 1) DWD(3, 2) DWD(5, 1) DWD(5, 2)
#undef DWD
    return hipErrorInvalidValue;
}

int dw_wgrad_splits(int B, int HWo, int C, int* pps, int* block, int* slots) {
    const int cg = C / 4;
    *slots = cg >= 256 ? 1 : 256 / cg;
    *block = cg * *slots;
    const long N = (long)B * HWo;
    long S = (N + *slots * 8 - 1) / (*slots * 8);   // ~8 pixels per thread
    S = S < 1 ? 1 : (S > 512 ? 512 : S);
    long per = (N + S - 1) / S;
    *pps = (int)per;
    return (int)((N + per - 1) / per);
}

hipError_t dw_wgrad_launch(const float* x, const float* dz, int B, int H, int W, int C, int Ho, int Wo, int k,
                           int stride, int pad_t, int pad_l, float* slab, float* dW, hipStream_t st) {
    int pps, block, slots;
    const int S = dw_wgrad_splits(B, Ho * Wo, C, &pps, &block, &slots);
#define DWW(KK, SS)                                                                                                   \
    if (k == KK && stride == SS) {                                                                                    \
        dw_wgrad_kernel<KK, SS><<<S, block, 0, st>>>(x, dz, B, H, W, C, Ho, Wo, pad_t, pad_l, pps, slots, slab);      \
    } else
    DWW(3, 1) DWW(3, 2) DWW(5, 1) DWW(5, 2) { return hipErrorInvalidValue; }
#undef DWW
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t n = (size_t)k * k * C;
    slab_sum_kernel<<<(unsigned)((n + 63) / 64), 256, 0, st>>>(slab, S, n, dW);
    return hipGetLastError();
}

int stem_wgrad_splits(int B, int HWo, int* pps) {
    const long N = (long)B * HWo;
    long S = (N + STEM_WPC * 8 - 1) / (STEM_WPC * 8);
    S = S < 1 ? 1 : (S > 1024 ? 1024 : S);
    long per = (N + S - 1) / S;
    per = (per + STEM_WPC - 1) / STEM_WPC * STEM_WPC;
    *pps = (int)per;
    return (int)((N + per - 1) / per);
}

hipError_t stem_wgrad_launch(const float* x, const float* dz, int B, int H, int W, int Ho, int Wo, int pad_t,
                             int pad_l, float* slab, float* dW, hipStream_t st) {
    int pps;
    const int S = stem_wgrad_splits(B, Ho * Wo, &pps);
    stem_wgrad_kernel<<<S, 128, 0, st>>>(x, dz, B, H, W, Ho, Wo, pad_t, pad_l, pps, slab);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    slab_sum_kernel<<<(432 + 63) / 64, 256, 0, st>>>(slab, S, 432, dW);
    return hipGetLastError();
}

hipError_t dummy_wgrad_launch(const float* x, const float* dg, int B, int H, int W, int C, int Ho, int Wo, int pad_t,
                              int pad_l, float* dW, float* db, hipStream_t st) {
    dummy_wgrad_kernel<<<81 * C, 256, 0, st>>>(x, dg, B, H, W, C, Ho, Wo, pad_t, pad_l, dW, db);
    return hipGetLastError();
}

hipError_t se_dscale_launch(const float* dxin, const float* u, int B, int HW, int C, float* part, int* n_part,
                            hipStream_t st) {
    int block, slots, ppw, nt;
    dw_geometry(C, HW, &block, &slots, &ppw, &nt);
    *n_part = nt;
    se_dscale_kernel<<<dim3(nt, B), block, 0, st>>>(dxin, u, HW, C, ppw, slots, part);
    return hipGetLastError();
}

hipError_t se_bwd_launch(const float* part, int n_part, int B, int C, int R, int hw, const float* w1, const float* w2,
                         const float* s1, const float* s2, float* ds1, float* ds2, float* dgb, hipStream_t st) {
    if (C > 1024 || R > 1024) return hipErrorInvalidValue;
    se_bwd_kernel<<<B, FCT, 0, st>>>(part, n_part, C, R, hw, w1, w2, s1, s2, ds1, ds2, dgb);
    return hipGetLastError();
}

hipError_t rowdot_launch(const float* in, int B, int K, const float* Wm, int N, float scale, float* out,
                         hipStream_t st) {
    if (K > 4096 || N > 4096) return hipErrorInvalidValue;
    rowdot_kernel<<<B, FCT, 0, st>>>(in, K, Wm, N, scale, out);
    return hipGetLastError();
}

hipError_t outer_launch(const float* a, int M, const float* d, int N, int B, int relu_a, float* dW, float* db,
                        hipStream_t st) {
    outer_kernel<<<grid1d((size_t)M * N, 4096), 256, 0, st>>>(a, M, d, N, B, relu_a, dW, db);
    return hipGetLastError();
}

}  // namespace rst
