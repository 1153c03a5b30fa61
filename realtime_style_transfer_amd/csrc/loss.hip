// loss.hip — element-wise / reduction kernels of the VGG16 style loss
// (realtime_style_transfer/models/styleLoss.py:69-109, 290-369).
//
//   maxpool2            keras VGG16 block*_pool (2x2, stride 2, valid), NHWC
//   sqdiff_partial      per-image partial sums of (a - b)^2 (mean_l2_loss_on_batch, :290-292)
//   tv_partial          per-image partial sums of |dy| + |dx| (tf.image.total_variation, :337)
//   loss_finalize       fixed-order f64 sum of the partials, scaled: factor * 0.5 * S / N (l2 terms)
//                       or factor * S (TV) — written per image into the loss table
// All reductions are two-level with a fixed order (no atomics) so the loss is bitwise reproducible.
// Memory-bound: each reads its inputs once with 16-B loads where the channel count allows.
#include <hip/hip_runtime.h>
#include "kernels.h"

namespace rst {

__global__ __launch_bounds__(256) void maxpool2_kernel(const float* __restrict__ x, float* __restrict__ y, int B,
                                                       int H, int W, int C) {
    const int Ho = H / 2, Wo = W / 2, C4 = C / 4;
    const int total = B * Ho * Wo * C4;   // < 2^31 (maxpool2_launch): 32-bit index math (a 64-bit division
                                          // chain per element cost more than the loads)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        const int c4 = i % C4;
        int p = i / C4;
        const int ox = p % Wo;
        p /= Wo;
        const int oy = p % Ho;
        const int b = p / Ho;
        const float4* base = reinterpret_cast<const float4*>(x + (((size_t)b * H + 2 * oy) * W + 2 * ox) * C) + c4;
        const float4 a0 = base[0], a1 = base[C4], a2 = base[(size_t)W * C4], a3 = base[(size_t)W * C4 + C4];
        float4 m;
        m.x = fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x));
        m.y = fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y));
        m.z = fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z));
        m.w = fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w));
        reinterpret_cast<float4*>(y)[i] = m;
    }
}

hipError_t maxpool2_launch(const float* x, float* y, int B, int H, int W, int C, hipStream_t st) {
    if (C % 4 != 0 || (long)B * (H / 2) * (W / 2) * (C / 4) >= (1L << 31)) return hipErrorInvalidValue;
    const long total = (long)B * (H / 2) * (W / 2) * (C / 4);
    long blocks = (total + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(maxpool2_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, y, B, H, W, C);
    return hipGetLastError();
}

__device__ __forceinline__ float block_sum_f(float v, float* scratch) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    return (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
}

// partial[b * nblk + blk] = sum over this block's slice of image b of (a - b)^2
// (BF16: a and c hold bf16 bits — the plain-bf16 VGG16's stored features — widened exactly to f32)
template <bool BF16>
__global__ __launch_bounds__(256) void sqdiff_partial_kernel(const float* __restrict__ a, const float* __restrict__ c,
                                                             float* __restrict__ partial, long n, int nblk) {
    __shared__ float scratch[4];
    const int blk = blockIdx.x, b = blockIdx.y;
    const long per = (n + nblk - 1) / nblk;
    const long s = (long)blk * per, e = (s + per < n) ? s + per : n;
    float acc = 0.f;
    for (long i = s + threadIdx.x; i < e; i += 256) {
        const size_t k = (size_t)b * n + i;
        const float d = BF16 ? ld_bf16(a, k) - ld_bf16(c, k) : a[k] - c[k];
        acc = fmaf(d, d, acc);
    }
    acc = block_sum_f(acc, scratch);
    if (threadIdx.x == 0) partial[(size_t)b * nblk + blk] = acc;
}

// partial[b * nblk + blk] = sum |x[y+1]-x[y]| + |x[:, x+1]-x[:, x]| over rows [r0, r1) of image b
__global__ __launch_bounds__(256) void tv_partial_kernel(const float* __restrict__ x, float* __restrict__ partial, int H,
                                                         int W, int C, int nblk) {
    __shared__ float scratch[4];
    const int blk = blockIdx.x, b = blockIdx.y;
    const int per = (H + nblk - 1) / nblk;
    const int r0 = blk * per, r1 = min(H, r0 + per);
    const float* px = x + (size_t)b * H * W * C;
    const long row = (long)W * C;
    float acc = 0.f;
    for (int r = r0; r < r1; ++r) {
        const float* pr = px + (size_t)r * row;
        for (long i = threadIdx.x; i < row; i += 256) {
            const float v = pr[i];
            if (r + 1 < H) acc += fabsf(pr[i + row] - v);
            if (i + C < row) acc += fabsf(pr[i + C] - v);
        }
    }
    acc = block_sum_f(acc, scratch);
    if (threadIdx.x == 0) partial[(size_t)b * nblk + blk] = acc;
}

// out[b * out_stride + out_col] (+)= scale * sum(partial[b][:])   (f64, fixed order)
__global__ __launch_bounds__(64) void loss_finalize_kernel(const float* __restrict__ partial, int nblk, double scale,
                                                           float* __restrict__ out, int out_stride, int out_col,
                                                           int accumulate) {
    const int b = blockIdx.x;
    double s = 0.0;
    for (int i = threadIdx.x; i < nblk; i += 64) s += (double)partial[(size_t)b * nblk + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) {
        float* dst = out + (size_t)b * out_stride + out_col;
        *dst = accumulate ? *dst + (float)(s * scale) : (float)(s * scale);
    }
}

int loss_partial_blocks(long n) {
    long nb = n / 16384;
    if (nb < 1) nb = 1;
    if (nb > 512) nb = 512;
    return (int)nb;
}

hipError_t sqdiff_loss_launch(const float* a, const float* c, int B, long n, float* partial, double scale, float* out,
                              int out_stride, int out_col, int accumulate, hipStream_t st, bool in_bf16) {
    const int nblk = loss_partial_blocks(n);
    if (in_bf16)
        hipLaunchKernelGGL(sqdiff_partial_kernel<true>, dim3(nblk, B), dim3(256), 0, st, a, c, partial, n, nblk);
    else
        hipLaunchKernelGGL(sqdiff_partial_kernel<false>, dim3(nblk, B), dim3(256), 0, st, a, c, partial, n, nblk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(B), dim3(64), 0, st, partial, nblk, scale, out, out_stride, out_col,
                       accumulate);
    return hipGetLastError();
}

hipError_t tv_loss_launch(const float* x, int B, int H, int W, int C, float* partial, double scale, float* out,
                          int out_stride, int out_col, hipStream_t st) {
    int nblk = H < 256 ? H : 256;
    hipLaunchKernelGGL(tv_partial_kernel, dim3(nblk, B), dim3(256), 0, st, x, partial, H, W, C, nblk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(B), dim3(64), 0, st, partial, nblk, scale, out, out_stride, out_col,
                       0);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void bf16_to_f32_kernel(const unsigned short* __restrict__ x, float* __restrict__ y,
                                                          size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        y[i] = __uint_as_float((unsigned)x[i] << 16);
}

hipError_t bf16_to_f32_launch(const void* x, float* y, size_t n, hipStream_t st) {
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(blocks), dim3(256), 0, st, static_cast<const unsigned short*>(x), y, n);
    return hipGetLastError();
}

// loss[b] = feature + style + tv   (columns 1..3 -> column 0 of a [B][4] table)
__global__ void loss_combine_kernel(float* table, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B) table[b * 4 + 0] = table[b * 4 + 1] + table[b * 4 + 2] + table[b * 4 + 3];
}

hipError_t loss_combine_launch(float* table, int B, hipStream_t st) {
    hipLaunchKernelGGL(loss_combine_kernel, dim3((B + 63) / 64), dim3(64), 0, st, table, B);
    return hipGetLastError();
}

}  // namespace rst
