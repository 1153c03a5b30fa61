// conv_small.hip — the final 9x9 stride-1 Conv2DTranspose with 3 output channels
// (realtime_style_transfer/models/styleTransfer.py:269-276, "expand_last").
//
// A SAME 9x9 s1 transposed conv is a 9x9 correlation with the spatially flipped kernel and
// pad 4 (adjoint of the SAME forward conv). With N = 3 an MFMA tile would idle 29/32 (32x32)
// or 13/16 (16x16) of its columns, so this layer runs on the f32 VALU (same 64 FLOP/clk/SIMD
// peak as f32 MFMA on gfx950): each thread owns RX=4 consecutive pixels x 3 channels, the
// input halo is staged channel-planar in LDS (fused CIN-apply + ReLU of expand_1), the 27
// weights of each (ky, ci) are wave-uniform and come in through the scalar cache, and each
// 12-float input row segment (3 x ds_read_b128) feeds 108 FMAs. The epilogue writes the raw
// conv output plus per-tile {sum, M2, n} for the final CIN (sigmoid is applied after finalize).
#include <hip/hip_runtime.h>
#include "kernels.h"

namespace rst {

namespace small {
constexpr int K = 9, PAD = 4, RX = 4, TH = 32, TW = 32, CC = 4;
constexpr int HH = TH + K - 1, HWD = TW + K - 1;   // 40 x 40
constexpr int RS = HWD + 4;                          // padded row stride (floats), 16-B multiple
constexpr int SEGS = TW / RX;                        // 8 segments per row
}  // namespace small

__global__ __launch_bounds__(256) void small_conv_kernel(SmallConvArgs a) {
    using namespace small;
    __shared__ __attribute__((aligned(16))) float halo[CC * HH * RS];
    __shared__ float2 pab[256];
    __shared__ float red[4][8];

    const int tid = threadIdx.x;
    const int tx = blockIdx.x % a.tiles_x;
    const int ty = (blockIdx.x / a.tiles_x) % a.tiles_y;
    const int b = blockIdx.x / (a.tiles_x * a.tiles_y);
    const int y0 = ty * TH, x0 = tx * TW;
    const int r = tid / SEGS, seg = tid % SEGS;
    const int Cin = a.cin;
    const float* __restrict__ w = a.w;

    if (a.pro_ab != nullptr)
        for (int c = tid; c < Cin; c += 256) pab[c] = a.pro_ab[b * Cin + c];

    float acc[RX][3];
#pragma unroll
    for (int i = 0; i < RX; ++i) acc[i][0] = acc[i][1] = acc[i][2] = 0.f;

    for (int c0 = 0; c0 < Cin; c0 += CC) {
        __syncthreads();
        for (int it = tid; it < HH * HWD; it += 256) {
            const int hy = it / HWD, hx = it % HWD;
            const int iy = y0 - PAD + hy, ix = x0 - PAD + hx;
            float v[CC];
#pragma unroll
            for (int q = 0; q < CC; ++q) v[q] = 0.f;
            if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
                const float* src = a.in + (((size_t)b * a.H + iy) * a.W + ix) * Cin + c0;
#pragma unroll
                for (int q = 0; q < CC; ++q) {
                    if (c0 + q < Cin) {
                        float x = src[q];
                        if (a.pro_ab != nullptr) {
                            const float2 p = pab[c0 + q];
                            x = fmaxf(fmaf(p.x, x, p.y), 0.f);
                        }
                        v[q] = x;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < CC; ++q) halo[(q * HH + hy) * RS + hx] = v[q];
        }
        __syncthreads();
        for (int q = 0; q < CC; ++q) {
            const int ci = c0 + q;
            if (ci >= Cin) break;
            for (int ky = 0; ky < K; ++ky) {
                const float* row = halo + (q * HH + r + ky) * RS + seg * RX;
                float in[12];
                const float4 i0 = *reinterpret_cast<const float4*>(row);
                const float4 i1 = *reinterpret_cast<const float4*>(row + 4);
                const float4 i2 = *reinterpret_cast<const float4*>(row + 8);
                in[0] = i0.x; in[1] = i0.y; in[2] = i0.z; in[3] = i0.w;
                in[4] = i1.x; in[5] = i1.y; in[6] = i1.z; in[7] = i1.w;
                in[8] = i2.x; in[9] = i2.y; in[10] = i2.z; in[11] = i2.w;
                const float* wk = w + ((size_t)ky * Cin + ci) * (K * 3);
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
                    const float w0 = wk[kx * 3 + 0], w1 = wk[kx * 3 + 1], w2 = wk[kx * 3 + 2];
#pragma unroll
                    for (int i = 0; i < RX; ++i) {
                        acc[i][0] = fmaf(in[i + kx], w0, acc[i][0]);
                        acc[i][1] = fmaf(in[i + kx], w1, acc[i][1]);
                        acc[i][2] = fmaf(in[i + kx], w2, acc[i][2]);
                    }
                }
            }
        }
    }

    // epilogue: bias, raw store, per-tile statistics per channel
    const int oy = y0 + r;
    float s[3] = {0.f, 0.f, 0.f}, cnt = 0.f;
    bool ok[RX];
#pragma unroll
    for (int i = 0; i < RX; ++i) {
        const int ox = x0 + seg * RX + i;
        ok[i] = oy < a.H && ox < a.W;
#pragma unroll
        for (int co = 0; co < 3; ++co) acc[i][co] += a.bias[co];
        if (ok[i]) {
            float* o = a.out + (((size_t)b * a.H + oy) * a.W + ox) * 3;
            o[0] = acc[i][0];
            o[1] = acc[i][1];
            o[2] = acc[i][2];
            s[0] += acc[i][0];
            s[1] += acc[i][1];
            s[2] += acc[i][2];
            cnt += 1.f;
        }
    }
    const int wave = tid >> 6, lane = tid & 63;
    float tot[4] = {s[0], s[1], s[2], cnt};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot[k] += __shfl_xor(tot[k], o);
    }
    __syncthreads();
    if (lane == 0)
        for (int k = 0; k < 4; ++k) red[wave][k] = tot[k];
    __syncthreads();
    float mean[3];
    const float n = red[0][3] + red[1][3] + red[2][3] + red[3][3];
    float sums[3];
#pragma unroll
    for (int co = 0; co < 3; ++co) {
        sums[co] = red[0][co] + red[1][co] + red[2][co] + red[3][co];
        mean[co] = n > 0.f ? sums[co] / n : 0.f;
    }
    float m2[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RX; ++i)
        if (ok[i])
#pragma unroll
            for (int co = 0; co < 3; ++co) {
                const float d = acc[i][co] - mean[co];
                m2[co] = fmaf(d, d, m2[co]);
            }
#pragma unroll
    for (int co = 0; co < 3; ++co)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m2[co] += __shfl_xor(m2[co], o);
    if (lane == 0)
        for (int co = 0; co < 3; ++co) red[wave][4 + co] = m2[co];
    __syncthreads();
    if (tid < 3) {
        const float mm = red[0][4 + tid] + red[1][4 + tid] + red[2][4 + tid] + red[3][4 + tid];
        const int n_tiles = a.tiles_x * a.tiles_y;
        a.part[((size_t)b * 3 + tid) * n_tiles + ty * a.tiles_x + tx] = make_float4(sums[tid], mm, n, 0.f);
    }
}

int small_conv_tiles_y(int H) { return (H + small::TH - 1) / small::TH; }
int small_conv_tiles_x(int W) { return (W + small::TW - 1) / small::TW; }

hipError_t small_conv_launch(const SmallConvArgs& a, hipStream_t st) {
    if (a.cin > 256) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    hipLaunchKernelGGL(small_conv_kernel, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace rst
