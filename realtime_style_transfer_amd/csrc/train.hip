// train.hip — backward-pass and optimizer kernels of the training step (BASELINE config 4,
// train_network.py:102-138: Keras fit with RMSprop; loss styleLoss.py:295-369).
//
// Norm backward (CIN styleTransfer.py:57-71, BatchNorm training mode styleTransfer.py:201):
//   n = a z + b (a = scale*rstd, b = bias - mean*a), x^ = (z - mean) rstd, post in {relu, none, sigmoid}
//   dn = post'(G)                      (G = gradient w.r.t. the post-activation output)
//   S1 = sum dn, S2 = sum dn x^        (over HW per (image, channel); over B*HW for BN)
//   d bias = S1, d scale = S2          (style-parameter / beta, gamma gradients)
//   dz = a (dn - S1/N - x^ S2/N) [z > 0 when the conv carries a built-in ReLU]
// reduce -> finalize (f64, fixed order) -> apply, no atomics.
//
// The conv bias gradient (sum of dz) is accumulated by the apply pass itself (per-tile partials).
// Weight gradients: wgrad.hip.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "train.h"

namespace rst {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float post_grad(int post, float g, float z, float2 ab) {
    const float n = fmaf(ab.x, z, ab.y);
    if (post == 0) return n > 0.f ? g : 0.f;                      // relu
    if (post == 2) {                                               // sigmoid
        const float s = 1.f / (1.f + __expf(-n));
        return g * s * (1.f - s);
    }
    return g;                                                      // none
}

// ---------------------------------------------------------------------------------------------
// norm backward: per-tile partial {S1, S2}; layout [b][c][tile]
__global__ __launch_bounds__(256) void norm_bwd_reduce_kernel(NormBwdArgs a) {
    __shared__ float2 red[256];
    const int tile = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int C = a.C;
    const int R = 256 / C;                 // pixel lanes per channel
    const int c = tid % C, r = tid / C;
    float s1 = 0.f, s2 = 0.f;
    if (r < R) {
        const float2 ab = a.ab[b * C + c];
        const float2 mr = a.mr[b * C + c];
        const long p0 = (long)tile * a.tile, p1 = min((long)a.hw, p0 + a.tile);
        for (long p = p0 + r; p < p1; p += R) {
            const size_t i = ((size_t)b * a.hw + p) * C + c;
            const float z = a.z[i];
            const float dn = post_grad(a.post, a.g[i], z, ab);
            s1 += dn;
            s2 = fmaf(dn, (z - mr.x) * mr.y, s2);
        }
    }
    red[tid] = make_float2(s1, s2);
    __syncthreads();
    if (tid < C) {
        float t1 = 0.f, t2 = 0.f;
        for (int k = 0; k < R; ++k) {
            t1 += red[k * C + tid].x;
            t2 += red[k * C + tid].y;
        }
        a.part[((size_t)b * C + tid) * a.n_tiles + tile] = make_float2(t1, t2);
    }
}

// The same two passes with 16-B vectors (C % 4 == 0: every layer but expand_last): thread = (pixel lane,
// channel quad), 32-bit pixel indices; per channel the partial sums keep a fixed order (deterministic).
// The scalar forms above spent more issue on 64-bit index math than on their loads.
typedef float nf4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void norm_bwd_reduce4_kernel(NormBwdArgs a) {
    __shared__ float2 red[256 * 4];
    const int tile = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int C = a.C, C4 = C / 4;
    const int R = 256 / C4;
    const int c4 = tid % C4, r = tid / C4;
    nf4 s1 = nf4{0.f, 0.f, 0.f, 0.f}, s2 = s1;
    if (r < R) {
        float2 ab[4], mr[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ab[k] = a.ab[b * C + 4 * c4 + k];
            mr[k] = a.mr[b * C + 4 * c4 + k];
        }
        const int p0 = tile * a.tile, p1 = min(a.hw, p0 + a.tile);
        const float* zb = a.z + (size_t)b * a.hw * C + 4 * c4;
        const float* gb = a.g + (size_t)b * a.hw * C + 4 * c4;
        for (int p = p0 + r; p < p1; p += R) {
            const nf4 z = *reinterpret_cast<const nf4*>(zb + (size_t)p * C);
            const nf4 g = *reinterpret_cast<const nf4*>(gb + (size_t)p * C);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float dn = post_grad(a.post, g[k], z[k], ab[k]);
                s1[k] += dn;
                s2[k] = fmaf(dn, (z[k] - mr[k].x) * mr[k].y, s2[k]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[tid * 4 + k] = make_float2(s1[k], s2[k]);
    __syncthreads();
    if (tid < C) {
        const int q4 = tid / 4, k = tid % 4;
        float t1 = 0.f, t2 = 0.f;
        for (int q = 0; q < R; ++q) {
            const float2 v = red[(q * C4 + q4) * 4 + k];
            t1 += v.x;
            t2 += v.y;
        }
        a.part[((size_t)b * C + tid) * a.n_tiles + tile] = make_float2(t1, t2);
    }
}

__global__ __launch_bounds__(256) void norm_bwd_apply4_kernel(NormBwdArgs a) {
    __shared__ float red[256 * 4];
    const int tile = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int C = a.C, C4 = C / 4;
    const int R = 256 / C4;
    const int c4 = tid % C4, r = tid / C4;
    nf4 sdz = nf4{0.f, 0.f, 0.f, 0.f};
    if (r < R) {
        float2 ab[4], mr[4], kk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ab[k] = a.ab[b * C + 4 * c4 + k];
            mr[k] = a.mr[b * C + 4 * c4 + k];
            kk[k] = a.consts[b * C + 4 * c4 + k];
        }
        const int p0 = tile * a.tile, p1 = min(a.hw, p0 + a.tile);
        const size_t base = (size_t)b * a.hw * C + 4 * c4;
        for (int p = p0 + r; p < p1; p += R) {
            const size_t i = base + (size_t)p * C;
            const nf4 z = *reinterpret_cast<const nf4*>(a.z + i);
            const nf4 g = *reinterpret_cast<const nf4*>(a.g + i);
            nf4 dz;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float dn = post_grad(a.post, g[k], z[k], ab[k]);
                const float xh = (z[k] - mr[k].x) * mr[k].y;
                float d = ab[k].x * (dn - kk[k].x - xh * kk[k].y);
                if (a.conv_relu && !(z[k] > 0.f)) d = 0.f;
                dz[k] = d;
            }
            *reinterpret_cast<nf4*>(a.dz + i) = dz;
            sdz += dz;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[tid * 4 + k] = sdz[k];
    __syncthreads();
    if (tid < C) {
        const int q4 = tid / 4, k = tid % 4;
        float t = 0.f;
        for (int q = 0; q < R; ++q) t += red[(q * C4 + q4) * 4 + k];
        a.part[((size_t)b * C + tid) * a.n_tiles + tile].x = t;
    }
}

// per (b, c) [per c when merge_images]: S1, S2 in f64 -> consts (S1/N, S2/N), and the parameter grads
__global__ __launch_bounds__(64) void norm_bwd_finalize_kernel(NormBwdArgs a) {
    const int c = blockIdx.x, b = blockIdx.y;
    double s1 = 0.0, s2 = 0.0;
    const int b0 = a.merge_images ? 0 : b, b1 = a.merge_images ? a.batch : b + 1;
    for (int bb = b0; bb < b1; ++bb) {
        const float2* p = a.part + ((size_t)bb * a.C + c) * a.n_tiles;
        for (int t = threadIdx.x; t < a.n_tiles; t += 64) {
            s1 += (double)p[t].x;
            s2 += (double)p[t].y;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    if (threadIdx.x == 0) {
        const double n = (double)a.hw * (a.merge_images ? a.batch : 1);
        a.consts[b * a.C + c] = make_float2((float)(s1 / n), (float)(s2 / n));
        if (a.dscale != nullptr && (!a.merge_images || b == 0)) {
            // CIN: style-param grads per image; BN: gamma/beta grads (accumulated once)
            const size_t o = a.merge_images ? (size_t)c : (size_t)b * a.dstride + c;
            a.dscale[o] = (float)s2;
            a.dbias[o] = (float)s1;
        }
    }
}

// dz per element, plus per-tile sums of dz -> part[b][c][tile].x (the conv bias gradient's partials;
// part's {S1, S2} were consumed by finalize, which ran before this kernel on the same stream)
__global__ __launch_bounds__(256) void norm_bwd_apply_kernel(NormBwdArgs a) {
    __shared__ float red[256];
    const int tile = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int C = a.C;
    const int R = 256 / C;
    const int c = tid % C, r = tid / C;
    float sdz = 0.f;
    if (r < R) {
        const float2 ab = a.ab[b * C + c];
        const float2 mr = a.mr[b * C + c];
        const float2 k = a.consts[b * C + c];
        const long p0 = (long)tile * a.tile, p1 = min((long)a.hw, p0 + a.tile);
        for (long p = p0 + r; p < p1; p += R) {
            const size_t i = ((size_t)b * a.hw + p) * C + c;
            const float z = a.z[i];
            const float dn = post_grad(a.post, a.g[i], z, ab);
            const float xh = (z - mr.x) * mr.y;
            float dz = ab.x * (dn - k.x - xh * k.y);
            if (a.conv_relu && !(z > 0.f)) dz = 0.f;
            a.dz[i] = dz;
            sdz += dz;
        }
    }
    red[tid] = sdz;
    __syncthreads();
    if (tid < C) {
        float t = 0.f;
        for (int q = 0; q < R; ++q) t += red[q * C + tid];
        a.part[((size_t)b * C + tid) * a.n_tiles + tile].x = t;
    }
}

// conv bias gradient db[c] = sum over images and tiles of the dz partials (f64, fixed order)
__global__ __launch_bounds__(64) void norm_bwd_bias_kernel(NormBwdArgs a) {
    const int c = blockIdx.x;
    double s = 0.0;
    for (int b = 0; b < a.batch; ++b) {
        const float2* p = a.part + ((size_t)b * a.C + c) * a.n_tiles;
        for (int t = threadIdx.x; t < a.n_tiles; t += 64) s += (double)p[t].x;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) a.dconv_bias[c] = (float)s;
}

hipError_t norm_bwd_launch(const NormBwdArgs& a0, hipStream_t st) {
    NormBwdArgs a = a0;
    if (a.C > 256) return hipErrorInvalidValue;
    const bool v4 = a.C % 4 == 0 && (size_t)a.hw * a.C < ((size_t)1 << 31);
    if (v4) hipLaunchKernelGGL(norm_bwd_reduce4_kernel, dim3(a.n_tiles, a.batch), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(norm_bwd_reduce_kernel, dim3(a.n_tiles, a.batch), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(norm_bwd_finalize_kernel, dim3(a.C, a.batch), dim3(64), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (v4) hipLaunchKernelGGL(norm_bwd_apply4_kernel, dim3(a.n_tiles, a.batch), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(norm_bwd_apply_kernel, dim3(a.n_tiles, a.batch), dim3(256), 0, st, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.dconv_bias != nullptr) {
        hipLaunchKernelGGL(norm_bwd_bias_kernel, dim3(a.C), dim3(64), 0, st, a);
        e = hipGetLastError();
    }
    return e;
}

// ---------------------------------------------------------------------------------------------
// y = x1 + x2 (skip-connection gradient chains)
__global__ __launch_bounds__(256) void add_kernel(const float* __restrict__ x1, const float* __restrict__ x2,
                                                  float* __restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = x1[i] + x2[i];
}

hipError_t add_launch(const float* x1, const float* x2, float* y, size_t n, hipStream_t st) {
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(add_kernel, dim3(blocks), dim3(256), 0, st, x1, x2, y, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// max-pool 2x2 backward: gradient to the first maximum of each window (TF MaxPoolGrad order)
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                                           float* __restrict__ gx, int B, int H, int W, int C,
                                                           int accumulate) {
    const int Ho = H / 2, Wo = W / 2;
    const size_t total = (size_t)B * H * W * C;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const int c = (int)(i % C);
        size_t p = i / C;
        const int xx = (int)(p % W);
        p /= W;
        const int yy = (int)(p % H);
        const int b = (int)(p / H);
        const int oy = yy / 2, ox = xx / 2;
        float g = 0.f;
        if (oy < Ho && ox < Wo) {
            const float* base = x + (((size_t)b * H + 2 * oy) * W + 2 * ox) * C + c;
            const float v0 = base[0], v1 = base[C], v2 = base[(size_t)W * C], v3 = base[(size_t)W * C + C];
            const float m = fmaxf(fmaxf(v0, v1), fmaxf(v2, v3));
            const int first = (v0 == m) ? 0 : (v1 == m) ? 1 : (v2 == m) ? 2 : 3;
            const int mine = (yy - 2 * oy) * 2 + (xx - 2 * ox);
            if (mine == first) g = gy[(((size_t)b * Ho + oy) * Wo + ox) * C + c];
        }
        gx[i] = accumulate ? gx[i] + g : g;
    }
}

// Even H, W and C % 4 == 0 (every VGG16 pool here): one thread per (pooled pixel, channel quad) reads the
// window's four pixels and the pooled gradient as 16-B vectors once and writes the four gradient pixels
// (the element-per-thread form above re-read each window four times through 64-bit index math: 2.3 TB/s).
// XBF16: the forward activations x are stored as bf16 bits (the plain-bf16 VGG16): four 8-B window loads.
// GBF16: the gradients gy, gx are bf16 bits too (mixed_bfloat16 gradients); acc (optional, f32, not aliasing gx): the
// Gram backward's f32 gradient of the same activations, added before the single rounding: gx = bf16(acc + routed gy)
template <bool XBF16, bool GBF16>
__global__ __launch_bounds__(256) void maxpool2_bwd4_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                                            float* __restrict__ gx, int B, int H, int W, int C,
                                                            int accumulate, const float* __restrict__ acc) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int Ho = H / 2, Wo = W / 2, C4 = C / 4;
    const int total = B * Ho * Wo * C4;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        const int c4 = i % C4;
        int p = i / C4;
        const int ox = p % Wo;
        p /= Wo;
        const int oy = p % Ho;
        const int b = p / Ho;
        const size_t r0 = (((size_t)b * H + 2 * oy) * W + 2 * ox) * C + 4 * c4, r1 = r0 + (size_t)W * C;
        f4 v0, v1, v2, v3;
        if constexpr (XBF16) {
            const float4 u0 = ld_bf16x4(x, r0), u1 = ld_bf16x4(x, r0 + C), u2 = ld_bf16x4(x, r1), u3 = ld_bf16x4(x, r1 + C);
            v0 = f4{u0.x, u0.y, u0.z, u0.w};
            v1 = f4{u1.x, u1.y, u1.z, u1.w};
            v2 = f4{u2.x, u2.y, u2.z, u2.w};
            v3 = f4{u3.x, u3.y, u3.z, u3.w};
        } else {
            v0 = *reinterpret_cast<const f4*>(x + r0);
            v1 = *reinterpret_cast<const f4*>(x + r0 + C);
            v2 = *reinterpret_cast<const f4*>(x + r1);
            v3 = *reinterpret_cast<const f4*>(x + r1 + C);
        }
        f4 g;
        if constexpr (GBF16) {
            const float4 u = ld_bf16x4(gy, (size_t)i * 4);
            g = f4{u.x, u.y, u.z, u.w};
        } else {
            g = *reinterpret_cast<const f4*>(gy + (size_t)i * 4);
        }
        f4 o0, o1, o2, o3;
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // gradient to the first maximum (TF MaxPoolGrad order), as above
            const float m = fmaxf(fmaxf(v0[k], v1[k]), fmaxf(v2[k], v3[k]));
            const int first = (v0[k] == m) ? 0 : (v1[k] == m) ? 1 : (v2[k] == m) ? 2 : 3;
            o0[k] = first == 0 ? g[k] : 0.f;
            o1[k] = first == 1 ? g[k] : 0.f;
            o2[k] = first == 2 ? g[k] : 0.f;
            o3[k] = first == 3 ? g[k] : 0.f;
        }
        if constexpr (GBF16) {
            const size_t r[4] = {r0, r0 + C, r1, r1 + C};
            f4* const o[4] = {&o0, &o1, &o2, &o3};
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                f4 v = *o[w];
                if (acc != nullptr) v += *reinterpret_cast<const f4*>(acc + r[w]);
                *reinterpret_cast<uint2*>(reinterpret_cast<unsigned short*>(gx) + r[w]) = pack_bf16x4(v[0], v[1], v[2], v[3]);
            }
            continue;
        }
        f4* d0 = reinterpret_cast<f4*>(gx + r0);
        f4* d1 = reinterpret_cast<f4*>(gx + r0 + C);
        f4* d2 = reinterpret_cast<f4*>(gx + r1);
        f4* d3 = reinterpret_cast<f4*>(gx + r1 + C);
        if (accumulate) {
            o0 += *d0;
            o1 += *d1;
            o2 += *d2;
            o3 += *d3;
        }
        *d0 = o0;
        *d1 = o1;
        *d2 = o2;
        *d3 = o3;
    }
}

hipError_t maxpool2_bwd_launch(const float* x, const float* gy, float* gx, int B, int H, int W, int C, int accumulate,
                               hipStream_t st, bool x_bf16, bool g_bf16, const float* acc) {
    if (g_bf16 && accumulate) return hipErrorInvalidValue;   // (bf16 gradients sum through acc, rounded once)
    if (H % 2 == 0 && W % 2 == 0 && C % 4 == 0 && (size_t)B * H * W * C < ((size_t)1 << 31)) {
        const size_t n = (size_t)B * (H / 2) * (W / 2) * (C / 4);
        unsigned blocks = (unsigned)((n + 255) / 256);
        if (blocks > 32768) blocks = 32768;
        if (x_bf16 && g_bf16)
            hipLaunchKernelGGL((maxpool2_bwd4_kernel<true, true>), dim3(blocks), dim3(256), 0, st, x, gy, gx, B, H, W, C,
                               accumulate, acc);
        else if (x_bf16 && acc == nullptr)
            hipLaunchKernelGGL((maxpool2_bwd4_kernel<true, false>), dim3(blocks), dim3(256), 0, st, x, gy, gx, B, H, W, C,
                               accumulate, nullptr);
        else if (!g_bf16 && acc == nullptr)
            hipLaunchKernelGGL((maxpool2_bwd4_kernel<false, false>), dim3(blocks), dim3(256), 0, st, x, gy, gx, B, H, W, C,
                               accumulate, nullptr);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (x_bf16 || g_bf16 || acc) return hipErrorInvalidValue;   // the bf16 VGG16 pools are all even-sized, C % 4 == 0
    const size_t n = (size_t)B * H * W * C;
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(blocks), dim3(256), 0, st, x, gy, gx, B, H, W, C, accumulate);
    return hipGetLastError();
}

// g (+)= scale * (a - b)   (feature-loss gradient; accumulate into an existing gradient; BF16: a, b bf16 bits)
// (GBF16: g is stored as bf16 bits, rounded once from the f32 value; no accumulate)
template <bool BF16, bool GBF16 = false>
__global__ __launch_bounds__(256) void scaled_diff_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                          float scale, float* __restrict__ g, size_t n, int accumulate) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float v = scale * (BF16 ? ld_bf16(a, i) - ld_bf16(b, i) : a[i] - b[i]);
        if constexpr (GBF16)
            reinterpret_cast<unsigned short*>(g)[i] = (unsigned short)(bf16_last_piece(v, 0.f) & 0xFFFFu);
        else
            g[i] = accumulate ? g[i] + v : v;
    }
}

hipError_t scaled_diff_launch(const float* a, const float* b, float scale, float* g, size_t n, int accumulate,
                              hipStream_t st, bool in_bf16, bool g_bf16) {
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 16384) blocks = 16384;
    if (g_bf16 && (accumulate || !in_bf16)) return hipErrorInvalidValue;
    if (g_bf16)
        hipLaunchKernelGGL((scaled_diff_kernel<true, true>), dim3(blocks), dim3(256), 0, st, a, b, scale, g, n, accumulate);
    else if (in_bf16)
        hipLaunchKernelGGL(scaled_diff_kernel<true>, dim3(blocks), dim3(256), 0, st, a, b, scale, g, n, accumulate);
    else
        hipLaunchKernelGGL(scaled_diff_kernel<false>, dim3(blocks), dim3(256), 0, st, a, b, scale, g, n, accumulate);
    return hipGetLastError();
}

// VGG16 conv0 input gradient, second half (train_api.hip vgg_backward): the 3x3 conv 64 -> 3 runs as a
// 1x1 conv 64 -> 27 (+5 zero) columns P[q][(tap, c)] on conv_mfma (a 3-column output tile idled 29 of the
// MFMA's 32 columns: 681 us per B=4 step), and out[y][x][c] = sum over the 9 taps (ky, kx) of
// P[y + ky - 1][x + kx - 1][(3 ky + kx) 3 + c] (SAME, pad 1; zero outside), fixed tap order.
// Workgroup = 4 output rows x 64 columns (one pixel per thread): the (4+2) x (64+2) x 32 source rows of
// P are staged into LDS with coalesced 16-B loads (a pixel-per-thread gather of 12 B from each of nine
// 128-B rows ran at 274 us per B=4 step for 240 MB), then each thread sums its 9 taps from LDS.
constexpr int T3_TH = 4, T3_TW = 64, T3_SH = T3_TH + 2, T3_SW = T3_TW + 2, T3_PS = 33;   // pixel stride (floats)
__global__ __launch_bounds__(256) void tap3_sum_kernel(const float* __restrict__ p, float* __restrict__ out, int B,
                                                       int H, int W) {
    __shared__ float tile[T3_SH * T3_SW * T3_PS];
    const int tiles_x = (W + T3_TW - 1) / T3_TW, tiles_y = (H + T3_TH - 1) / T3_TH;
    const int t = blockIdx.x;
    const int b = t / (tiles_x * tiles_y), rem = t % (tiles_x * tiles_y);
    const int y0 = (rem / tiles_x) * T3_TH, x0 = (rem % tiles_x) * T3_TW;
    for (int i = threadIdx.x; i < T3_SH * T3_SW * 8; i += 256) {
        const int q = i & 7, px = i >> 3;
        const int r = px / T3_SW, c = px % T3_SW;
        const int gy = y0 - 1 + r, gx = x0 - 1 + c;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gy >= 0 && gy < H && gx >= 0 && gx < W)
            v = *reinterpret_cast<const float4*>(p + (((size_t)b * H + gy) * W + gx) * 32 + 4 * q);
        float* d = tile + px * T3_PS + 4 * q;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    __syncthreads();
    const int ty = threadIdx.x / T3_TW, tx = threadIdx.x % T3_TW;
    const int y = y0 + ty, x = x0 + tx;
    if (y >= H || x >= W) return;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {   // zero-padded halo: out-of-image taps add 0
            const float* q = tile + ((ty + ky) * T3_SW + tx + kx) * T3_PS + (3 * ky + kx) * 3;
            s0 += q[0];
            s1 += q[1];
            s2 += q[2];
        }
    const size_t o = (((size_t)b * H + y) * W + x) * 3;
    out[o + 0] = s0;
    out[o + 1] = s1;
    out[o + 2] = s2;
}

hipError_t tap3_sum_launch(const float* p, float* out, int B, int H, int W, hipStream_t st) {
    const long n = (long)B * ((H + T3_TH - 1) / T3_TH) * ((W + T3_TW - 1) / T3_TW);
    hipLaunchKernelGGL(tap3_sum_kernel, dim3((unsigned)n), dim3(256), 0, st, p, out, B, H, W);
    return hipGetLastError();
}

// total variation backward: d/dx of factor * (sum |x[y+1]-x[y]| + sum |x[:,x+1]-x[:,x]|), added to g
__global__ __launch_bounds__(256) void tv_bwd_kernel(const float* __restrict__ x, float factor, float* __restrict__ g,
                                                     int B, int H, int W, int C) {
    const size_t total = (size_t)B * H * W * C;
    auto sgn = [](float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); };
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        size_t p = i / C;
        const int xx = (int)(p % W);
        p /= W;
        const int yy = (int)(p % H);
        const float v = x[i];
        float d = 0.f;
        const size_t row = (size_t)W * C;
        if (yy + 1 < H) d -= sgn(x[i + row] - v);
        if (yy > 0) d += sgn(v - x[i - row]);
        if (xx + 1 < W) d -= sgn(x[i + C] - v);
        if (xx > 0) d += sgn(v - x[i - C]);
        g[i] += factor * d;
    }
}

hipError_t tv_bwd_launch(const float* x, float factor, float* g, int B, int H, int W, int C, hipStream_t st) {
    const size_t n = (size_t)B * H * W * C;
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(tv_bwd_kernel, dim3(blocks), dim3(256), 0, st, x, factor, g, B, H, W, C);
    return hipGetLastError();
}

// Gram backward: dF = F (dG + dG^T) / HW = F M with M = 2 coef (Gp - Gs) / HW (symmetric).
// Written straight into the packed 1x1-conv weight image (gather through a host-built map).
__global__ __launch_bounds__(256) void gram_bwd_weights_kernel(const float* __restrict__ gp, const float* __restrict__ gs,
                                                               const int* __restrict__ map, int n_packed, int CC,
                                                               float scale, float* __restrict__ packed) {
    const int b = blockIdx.y;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n_packed; i += gridDim.x * 256) {
        const int m = map[i];
        packed[(size_t)b * n_packed + i] =
            m < 0 ? 0.f : scale * (gp[(size_t)b * CC + m] - gs[(size_t)b * CC + m]);
    }
}

// plain-bf16 loss: the same weights rounded to bf16 (RNE) into conv_bf3's one-plane image (n16 elements/image)
__global__ __launch_bounds__(256) void gram_bwd_weights_bf16_kernel(const float* __restrict__ gp,
                                                                    const float* __restrict__ gs,
                                                                    const int* __restrict__ map, int n16, int CC,
                                                                    float scale, unsigned short* __restrict__ packed) {
    const int b = blockIdx.y;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) {
        const int m = map[i];
        const float v = m < 0 ? 0.f : scale * (gp[(size_t)b * CC + m] - gs[(size_t)b * CC + m]);
        const unsigned u = __float_as_uint(v);
        packed[(size_t)b * n16 + i] = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
    }
}

hipError_t gram_bwd_weights_bf16_launch(const float* gp, const float* gs, const int* map, int n16, int C, float scale,
                                        unsigned short* packed, int B, hipStream_t st) {
    hipLaunchKernelGGL(gram_bwd_weights_bf16_kernel, dim3((n16 + 255) / 256, B), dim3(256), 0, st, gp, gs, map, n16,
                       C * C, scale, packed);
    return hipGetLastError();
}

hipError_t gram_bwd_weights_launch(const float* gp, const float* gs, const int* map, int n_packed, int C, float scale,
                                   float* packed, int B, hipStream_t st) {
    hipLaunchKernelGGL(gram_bwd_weights_kernel, dim3((n_packed + 255) / 256, B), dim3(256), 0, st, gp, gs, map,
                       n_packed, C * C, scale, packed);
    return hipGetLastError();
}

// preprocess backward: x_pre[c'] = 255 x[2 - c'] - mean  ->  g_x[c] = 255 g_pre[2 - c]
__global__ __launch_bounds__(256) void preprocess_bwd_kernel(const float* __restrict__ gpre, float* __restrict__ gx,
                                                             size_t pixels, int accumulate) {
    for (size_t p = blockIdx.x * 256ull + threadIdx.x; p < pixels; p += (size_t)gridDim.x * 256) {
        for (int c = 0; c < 3; ++c) {
            const float v = 255.f * gpre[p * 3 + (2 - c)];
            gx[p * 3 + c] = accumulate ? gx[p * 3 + c] + v : v;
        }
    }
}

hipError_t preprocess_bwd_launch(const float* gpre, float* gx, size_t pixels, int accumulate, hipStream_t st) {
    unsigned blocks = (unsigned)((pixels + 255) / 256);
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(preprocess_bwd_kernel, dim3(blocks), dim3(256), 0, st, gpre, gx, pixels, accumulate);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// RMSprop (Keras OptimizerV2, centered=False, momentum=0): ms = rho ms + (1-rho) g^2;
// w -= lr g / (sqrt(ms) + eps)
__global__ __launch_bounds__(256) void rmsprop_kernel(float* __restrict__ w, float* __restrict__ ms,
                                                      const float* __restrict__ g, size_t n, float lr, float rho,
                                                      float eps) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float gi = g[i];
        const float m = rho * ms[i] + (1.f - rho) * gi * gi;
        ms[i] = m;
        w[i] -= lr * gi / (sqrtf(m) + eps);
    }
}

hipError_t rmsprop_launch(float* w, float* ms, const float* g, size_t n, float lr, float rho, float eps, hipStream_t st) {
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(rmsprop_kernel, dim3(blocks), dim3(256), 0, st, w, ms, g, n, lr, rho, eps);
    return hipGetLastError();
}

// dst[index[i]] = src[i] / divisor: writes a few canonical weight entries (the cross-rank average of the BN
// moving statistics) without touching the packed kernel images that are derived from the others
__global__ __launch_bounds__(256) void scatter_div_kernel(const float* __restrict__ src, const int* __restrict__ index,
                                                          float* __restrict__ dst, size_t n, float divisor) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[index[i]] = src[i] / divisor;
}

hipError_t scatter_div_launch(const float* src, const int* index, float* dst, size_t n, float divisor, hipStream_t st) {
    if (n == 0) return hipSuccess;
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(scatter_div_kernel, dim3(blocks), dim3(256), 0, st, src, index, dst, n, divisor);
    return hipGetLastError();
}

// packed[i] = map[i] < 0 ? 0 : src[map[i]]  (re-pack canonical weights into kernel stage images)
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ src, const int* __restrict__ map,
                                                     float* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int m = map[i];
        dst[i] = m < 0 ? 0.f : src[m];
    }
}

hipError_t gather_launch(const float* src, const int* map, float* dst, size_t n, hipStream_t st) {
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, st, src, map, dst, n);
    return hipGetLastError();
}

// Many gathers from one source in one launch (the trainer's re-pack after every update: ~40 index maps of 10^2 -
// 10^6 entries, which as separate launches spent more time between kernels than in them). Job j owns blocks
// [first[j], first[j + 1]); inside a job the same element loop as gather_kernel.
__global__ __launch_bounds__(256) void gather_batch_kernel(const float* __restrict__ src, GatherJobs jobs) {
    int j = 0;
    while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.first[j + 1]) ++j;
    const int nb = jobs.first[j + 1] - jobs.first[j];
    const int* __restrict__ map = jobs.map[j];
    float* __restrict__ dst = jobs.dst[j];
    const size_t n = jobs.count[j];
    for (size_t i = (size_t)((int)blockIdx.x - jobs.first[j]) * 256 + threadIdx.x; i < n; i += (size_t)nb * 256) {
        const int m = map[i];
        dst[i] = m < 0 ? 0.f : src[m];
    }
}

hipError_t gather_batch_launch(const float* src, GatherJobs& jobs, hipStream_t st) {
    if (jobs.n == 0) return hipSuccess;
    int blocks = 0;
    for (int j = 0; j < jobs.n; ++j) {
        jobs.first[j] = blocks;
        long b = (long)((jobs.count[j] + 255) / 256);
        blocks += (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
    }
    jobs.first[jobs.n] = blocks;
    hipLaunchKernelGGL(gather_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, jobs);
    jobs.n = 0;
    return hipGetLastError();
}


namespace {
constexpr int POISON_LDS_BYTES = 160 * 1024;
__global__ __launch_bounds__(1024) void lds_poison_kernel(unsigned bits, unsigned* sink) {
    extern __shared__ unsigned poison_lds[];
    for (int i = threadIdx.x; i < POISON_LDS_BYTES / 4; i += 1024) poison_lds[i] = bits;
    __syncthreads();
    // a read the compiler cannot drop the stores for (sink is null: the condition never holds on a real pattern)
    if (sink != nullptr && poison_lds[(threadIdx.x * 37) % (POISON_LDS_BYTES / 4)] == ~bits) sink[0] = 1u;
}
}  // namespace

hipError_t lds_poison_launch(unsigned bits, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)lds_poison_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, POISON_LDS_BYTES);
        if (e != hipSuccess) return e;
        attr = true;
    }
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    // one 160 KB workgroup fits a CU at a time: four rounds per CU cover every CU whatever the dispatch order
    hipLaunchKernelGGL(lds_poison_kernel, dim3(4 * cus), dim3(1024), POISON_LDS_BYTES, st, bits, (unsigned*)nullptr);
    return hipGetLastError();
}

}  // namespace rst
