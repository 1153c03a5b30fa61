// conv_small.hip — the final 9x9 stride-1 Conv2DTranspose with 3 output channels
// (realtime_style_transfer/models/styleTransfer.py:269-276, "expand_last").
//
// A SAME 9x9 s1 transposed conv is a 9x9 correlation with the spatially flipped kernel and
// pad 4 (adjoint of the SAME forward conv). With N = 3 an MFMA tile would idle 29/32 (32x32)
// or 13/16 (16x16) of its columns, so this layer runs on the f32 VALU (same 64 FLOP/clk/SIMD
// peak as f32 MFMA on gfx950):
//   * each thread owns RX=4 consecutive pixels x 3 channels (12 accumulators);
//   * the input halo is staged channel-planar in LDS, CC=4 channels at a time, double-buffered:
//     the next chunk is prefetched into registers while the current one is consumed, and the
//     CIN-apply + ReLU of expand_1 is fused into that LDS write;
//   * the 27 weights of each (ky, ci) are wave-uniform; they are staged in LDS once per
//     workgroup and read as broadcast ds_read_b128 (measured 67 us vs 79 us for the s_load
//     variant at B=1, tools/conv_bench; equal at B=8) — SOPT selects the variant;
//   * each 12-float input row segment (3 x ds_read_b128) feeds 108 FMAs.
// The epilogue writes the raw conv output plus per-tile {sum, M2, n} for the final CIN.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include "kernels.h"

namespace rst {

namespace small {
#ifndef RST_SMALL_RX
#define RST_SMALL_RX 4
#endif
// RX = 8 (64-wide tiles: 4 input + 7 weight ds_read_b128 per 108 packed FMAs instead of 3 + 7 per 54)
// measured slower at B=1 (77.7 vs 69.6 us): its 113 KB of LDS leaves one workgroup (4 waves) per CU
// and 225 workgroups for 256 CUs
constexpr int K = 9, PAD = 4, RX = RST_SMALL_RX, TW = RX == 8 ? 64 : 32, TH = 256 / (TW / RX), CC = 4;
constexpr int NX = RX + K - 1;                       // input row values per thread and (ci, ky)
constexpr int HH = TH + K - 1, HWD = TW + K - 1;   // 40 x 40
constexpr int RS = HWD + 4;                          // padded row stride (floats), 16-B multiple
constexpr int SEGS = TW / RX;                        // 8 segments per row
constexpr int PLANE = HH * RS;                       // floats per channel plane
constexpr int CHUNK_FLOATS = CC * PLANE;
constexpr int ITEMS = HH * HWD;                      // halo pixels per chunk (one float4 each)
constexpr int PREG = (ITEMS + 255) / 256;            // prefetch registers (float4) per thread
constexpr int WS = 28;                               // 27 weights per (ky, ci), padded
}  // namespace small

typedef float sf32x4 __attribute__((ext_vector_type(4)));
typedef float sf32x2 __attribute__((ext_vector_type(2)));

// SOPT bit0: unroll the 4 channels of a chunk (lets hipcc hoist the next channel's weight s_loads)
//      bit1: weights staged in LDS once and read as broadcast ds_read_b128 (instead of s_load)
#ifndef RST_SMALL_OPT
#define RST_SMALL_OPT 2
#endif
template <int SOPT>
__global__ __launch_bounds__(256, RST_SMALL_RX == 8 ? 1 : 2) void small_conv_kernel(SmallConvArgs a, const float* __restrict__ w,
                                                            const float* __restrict__ in) {
    using namespace small;
    constexpr bool WLDS = (SOPT & 2) != 0;
    __shared__ __attribute__((aligned(16))) float halo[2 * CHUNK_FLOATS];
    __shared__ __attribute__((aligned(16))) float wl[WLDS ? 9 * 16 * WS : 4];
    __shared__ float2 pab[256];
    __shared__ float red[4][8];

    const int tid = threadIdx.x;
    const int tx = blockIdx.x % a.tiles_x;
    const int ty = (blockIdx.x / a.tiles_x) % a.tiles_y;
    const int b = blockIdx.x / (a.tiles_x * a.tiles_y);
    const int y0 = ty * TH, x0 = tx * TW;
    const int r = tid / SEGS, seg = tid % SEGS;
    const int Cin = a.cin;
    const bool pro = a.pro_ab != nullptr;
    const size_t img = (size_t)b * a.H * a.W;

    if (pro)
        for (int c = tid; c < Cin; c += 256) pab[c] = a.pro_ab[b * Cin + c];
    if constexpr (WLDS)
        for (int i = tid; i < 9 * Cin * WS; i += 256) wl[i] = w[i];
    __syncthreads();

    auto item_src = [&](int it, int& hy, int& hx, bool& valid) __attribute__((always_inline)) {
        hy = it / HWD;
        hx = it - hy * HWD;
        const int iy = y0 - PAD + hy, ix = x0 - PAD + hx;
        valid = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const int cy = min(max(iy, 0), a.H - 1), cx = min(max(ix, 0), a.W - 1);
        return (img + (size_t)cy * a.W + cx) * Cin;
    };
    auto write_item = [&](float* buf, int hy, int hx, bool valid, sf32x4 v, int c0) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < CC; ++q) {
            float x = valid && (c0 + q < Cin) ? v[q] : 0.f;
            if (pro && valid && c0 + q < Cin) {
                const float2 p = pab[c0 + q];
                x = fmaxf(fmaf(p.x, x, p.y), 0.f);
            }
            buf[q * PLANE + hy * RS + hx] = x;
        }
    };
    const bool vec = (Cin % CC) == 0;
    // synchronous staging of one chunk (prologue; also the whole path when Cin % 4 != 0)
    auto stage_sync = [&](int c0, float* buf) __attribute__((always_inline)) {
        for (int it = tid; it < ITEMS; it += 256) {
            int hy, hx;
            bool valid;
            const size_t gi = item_src(it, hy, hx, valid) + c0;
            sf32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (vec) {
                v = *reinterpret_cast<const sf32x4*>(in + gi);
            } else {
#pragma unroll
                for (int q = 0; q < CC; ++q) v[q] = (c0 + q < Cin) ? in[gi + q] : 0.f;
            }
            write_item(buf, hy, hx, valid, v, c0);
        }
    };

    // accumulators as pixel pairs: acc2[p][co] = (pixel 2p, pixel 2p+1) of channel co, so every FMA
    // is a v_pk_fma_f32 (two lanes' worth per issue: the 64 FLOP/clk/SIMD VALU peak needs packed FMA)
    sf32x2 acc2[RX / 2][3];
#pragma unroll
    for (int i = 0; i < RX / 2; ++i) acc2[i][0] = acc2[i][1] = acc2[i][2] = sf32x2{0.f, 0.f};

    stage_sync(0, halo);
    __syncthreads();
    const int nchunks = (Cin + CC - 1) / CC;
    for (int ch = 0; ch < nchunks; ++ch) {
        const int c0 = ch * CC;
        const bool has_next = ch + 1 < nchunks;
        const float* cur = halo + (ch & 1) * CHUNK_FLOATS;
        sf32x4 pre[PREG];
        if (vec) {
            const int cn = has_next ? c0 + CC : c0;
#pragma unroll
            for (int k = 0; k < PREG; ++k) {
                const int it = min(k * 256 + tid, ITEMS - 1);
                int hy, hx;
                bool valid;
                pre[k] = *reinterpret_cast<const sf32x4*>(in + item_src(it, hy, hx, valid) + cn);
            }
        }
#pragma unroll((SOPT & 1) ? CC : 1)
        for (int q = 0; q < CC; ++q) {
            const int ci = c0 + q;
            if (ci >= Cin) break;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                const float* row = cur + q * PLANE + (r + ky) * RS + seg * RX;
                float x[NX];
#pragma unroll
                for (int j = 0; j < NX / 4; ++j) {
                    const sf32x4 t = *reinterpret_cast<const sf32x4*>(row + 4 * j);
                    x[4 * j] = t[0]; x[4 * j + 1] = t[1]; x[4 * j + 2] = t[2]; x[4 * j + 3] = t[3];
                }
                float wv[WS];
                if constexpr (WLDS) {
                    const float* wk = wl + (ky * Cin + ci) * WS;
#pragma unroll
                    for (int j = 0; j < WS / 4; ++j) {
                        const sf32x4 t = *reinterpret_cast<const sf32x4*>(wk + 4 * j);
                        wv[4 * j] = t[0]; wv[4 * j + 1] = t[1]; wv[4 * j + 2] = t[2]; wv[4 * j + 3] = t[3];
                    }
                } else {
                    const float* wk = w + ((size_t)ky * Cin + ci) * WS;
#pragma unroll
                    for (int j = 0; j < WS; ++j) wv[j] = wk[j];
                }
                // pairs of the NX row values: even-aligned (x0,x1),(x2,x3).. and odd-shifted (x1,x2),(x3,x4)..
                sf32x2 xe[NX / 2], xo[NX / 2 - 1];
#pragma unroll
                for (int j = 0; j < NX / 2; ++j) xe[j] = sf32x2{x[2 * j], x[2 * j + 1]};
#pragma unroll
                for (int j = 0; j < NX / 2 - 1; ++j) xo[j] = sf32x2{x[2 * j + 1], x[2 * j + 2]};
#pragma unroll
                for (int kx = 0; kx < K; ++kx) {
#pragma unroll
                    for (int co = 0; co < 3; ++co) {
                        const sf32x2 wp = sf32x2{wv[kx * 3 + co], wv[kx * 3 + co]};
#pragma unroll
                        for (int p = 0; p < RX / 2; ++p) {
                            const sf32x2 xv = (kx & 1) ? xo[p + kx / 2] : xe[p + kx / 2];
#ifdef RST_SMALL_PK   // the packed form (v_pk_fma_f32): see below
                            acc2[p][co] = __builtin_elementwise_fma(xv, wp, acc2[p][co]);
#else
                            // two scalar FMAs, not v_pk_fma_f32: with the packed accumulate chains, a few 8-lane
                            // groups of a workgroup took a wrong sum (one accumulator element) whenever bf16-VGG16
                            // waves of another stream shared the CU (profiles/r06/r06bf-r06bj); the
                            // scalar form is clean there and the training step is no slower (r06bk)
                            acc2[p][co][0] = fmaf(xv[0], wp[0], acc2[p][co][0]);
                            acc2[p][co][1] = fmaf(xv[1], wp[1], acc2[p][co][1]);
#endif
                        }
                    }
                }
            }
        }
        if (has_next) {
            float* nxt = halo + ((ch + 1) & 1) * CHUNK_FLOATS;
            if (vec) {
#pragma unroll
                for (int k = 0; k < PREG; ++k) {
                    const int it = k * 256 + tid;
                    if (it < ITEMS) {
                        int hy, hx;
                        bool valid;
                        item_src(it, hy, hx, valid);
                        write_item(nxt, hy, hx, valid, pre[k], c0 + CC);
                    }
                }
            } else {
                stage_sync(c0 + CC, nxt);
            }
        }
        __syncthreads();
    }

    // epilogue: bias, raw store, per-tile statistics per channel
    float acc[RX][3];
#pragma unroll
    for (int i = 0; i < RX; ++i)
#pragma unroll
        for (int co = 0; co < 3; ++co) acc[i][co] = acc2[i / 2][co][i & 1];
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
int small_conv_weight_stride() { return small::WS; }

hipError_t small_conv_launch(const SmallConvArgs& a, hipStream_t st) {
    if (a.cin > 256 || ((RST_SMALL_OPT & 2) && a.cin > 16)) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    // diagnostic (the targets race): RST_SMALL_EXCLUSIVE=1 pads the workgroup's LDS to the whole 160 KB, so
    // no other workgroup (of this or another kernel) shares its CU
    static const bool exclusive = [] {
        const char* v = getenv("RST_SMALL_EXCLUSIVE");
        return v != nullptr && atoi(v) != 0;
    }();
    size_t dyn = 0;
    if (exclusive) {
        hipFuncAttributes fa{};
        hipError_t e = hipFuncGetAttributes(&fa, (const void*)small_conv_kernel<RST_SMALL_OPT>);
        if (e != hipSuccess) return e;
        dyn = 160 * 1024 - fa.sharedSizeBytes;
        e = hipFuncSetAttribute((const void*)small_conv_kernel<RST_SMALL_OPT>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(small_conv_kernel<RST_SMALL_OPT>, dim3(grid), dim3(256), dyn, st, a, a.w, a.in);
    return hipGetLastError();
}

}  // namespace rst
