// wino.hip — the residual-block convolutions (3x3, stride 1, SAME, 128 output channels;
// realtime_style_transfer/models/styleTransfer.py:144-185) as a fused Winograd F(2x2, 3x3)
// implicit GEMM on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Y = A^T [ (G g G^T) (.) (B^T d B) ] A per 2x2 output tile (Lavin & Gray): 16 element-wise
// products per tile instead of 36 direct MACs, i.e. 2.25x fewer MFMA operations for the same
// convolution. Numerics: fp32 throughout (exact-f32 MFMA products, f32 accumulation); B and A have
// entries in {0, +-1} (input / output transforms are exact adds), G has entries in {0, +-1/2, 1}
// and U = G g G^T is formed on the host in f64 and rounded once.
//
// Workgroup = 4 waves, output tile 8 x 16 pixels = 4 x 8 = 32 Winograd tiles (one 32-row MFMA M
// tile) x 128 output channels; wave w owns channels [32w, 32w+32) for all 16 transform points xi,
// so each lane's accumulators hold, for 16 Winograd tiles, all 16 xi of one channel and the output
// transform is lane-local. 16 accumulators x 16 = 256 registers per lane (1 wave per SIMD).
// Per 8-channel input chunk:
//   prefetch (registers): the 10 x 18 x 8 input patch (+ residual source) and U[xi][co][8]
//   stage: prologue (CIN affine [+ ReLU | + residual], materialised block output) -> LDS patch;
//          U -> LDS
//   transform: one thread per (tile, channel): V = B^T d B -> LDS [xi][tile][8]
//   MFMA: per xi one ds_read_b128 of V and of U feeds 4 k-steps (k-step kk pairs channels kk and
//          kk+4 of the chunk across the two lane halves); the next chunk's loads are in flight.
// Epilogue: output transform, conv bias + ReLU, store, and per-(workgroup, channel) two-pass
// {sum, M2, n} for the conditional instance norm that follows (finalize_kernel merges them).
#include <hip/hip_runtime.h>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace rst {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WTH = 8, WTW = 16;                  // output pixels per workgroup
constexpr int WPH = WTH + 2, WPW = WTW + 2;       // input patch
constexpr int WNP = WPH * WPW;                    // 180 patch pixels
constexpr int WCK = 8;                            // input channels per chunk
constexpr int WPS = 9;                            // patch pixel stride (floats): conflict-free transform reads
constexpr int WVS = 12;                           // V / U row stride (floats): odd count of 16-B slots
constexpr int WN = 128;                           // output channels (4 waves x 32)
constexpr int WXI = 16;                           // transform points
constexpr int W_PATCH_F4 = WNP * WCK / 4;         // 360 float4 per chunk
constexpr int W_U_F4 = WXI * WN * WCK / 4;        // 4096 float4 per chunk
constexpr int W_MAX_CIN = 256;
constexpr size_t W_LDS_BYTES =
    (size_t)(WNP * WPS + WXI * 32 * WVS + WXI * WN * WVS) * 4 + W_MAX_CIN * sizeof(float2);

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

__device__ __forceinline__ float pro_apply(int mode, float x, float2 ab, float r) {
    float y = fmaf(ab.x, x, ab.y);
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}

}  // namespace

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void wino_conv_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* patch = smem;                               // [180][9]
    float* vs = patch + WNP * WPS;                     // [16][32][12]
    float* us = vs + WXI * 32 * WVS;                   // [16][128][12]
    float2* pab = reinterpret_cast<float2*>(us + WXI * WN * WVS);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    int bid = blockIdx.x;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * WTH, x0 = tx * WTW;
    const int H = a.H, W = a.W, Cin = a.cin;
    const int pro = a.pro_mode;
    const size_t img = (size_t)b * H * W;
    const float* res_src = pro == PRO_AFF_RES ? a.res : a.in;
    const int nchunks = Cin / WCK;

    if (pro != PRO_NONE) {
        for (int c = tid; c < Cin; c += 256) pab[c] = a.pro_ab[(size_t)b * Cin + c];
    }

    // ---- prefetch registers (compile-time indexed only) -------------------------------------
    f32x4 xr[2], rr[2], ur[16];
    auto load = [&](int chunk) __attribute__((always_inline)) {
        const int c0 = chunk * WCK;
        sfor<0, 2>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = min(tid + k * 256, W_PATCH_F4 - 1);
            const int px = it >> 1, q = it & 1;
            const int iy = min(max(y0 - 1 + px / WPW, 0), H - 1), ix = min(max(x0 - 1 + px % WPW, 0), W - 1);
            const size_t gi = (img + (size_t)iy * W + ix) * Cin + c0 + 4 * q;
            xr[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
            rr[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
        });
        const f32x4* usrc = reinterpret_cast<const f32x4*>(a.U) + (size_t)chunk * W_U_F4;
        sfor<0, 16>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            ur[k] = usrc[k * 256 + tid];
        });
    };
    auto stage = [&](int chunk) __attribute__((always_inline)) {
        const int c0 = chunk * WCK;
        sfor<0, 2>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = tid + k * 256;
            if (it < W_PATCH_F4) {
                const int px = it >> 1, q = it & 1;
                const int iy = y0 - 1 + px / WPW, ix = x0 - 1 + px % WPW;
                const int c = c0 + 4 * q;
                f32x4 v = xr[k];
                const bool inside = iy >= 0 && iy < H && ix >= 0 && ix < W;
                if (pro != PRO_NONE) {
                    const f32x4 r = rr[k];
                    v.x = pro_apply(pro, v.x, pab[c], r.x);
                    v.y = pro_apply(pro, v.y, pab[c + 1], r.y);
                    v.z = pro_apply(pro, v.z, pab[c + 2], r.z);
                    v.w = pro_apply(pro, v.w, pab[c + 3], r.w);
                    if (a.mat != nullptr && inside && iy >= y0 && iy < y0 + WTH && ix >= x0 && ix < x0 + WTW)
                        *reinterpret_cast<f32x4*>(a.mat + (img + (size_t)iy * W + ix) * Cin + c) = v;
                }
                if (!inside) v = f32x4{0.f, 0.f, 0.f, 0.f};
                float* d = patch + px * WPS + 4 * q;
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
        });
        // U[xi][co][8] (global, contiguous) -> LDS [xi][co][12]
        sfor<0, 16>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = k * 256 + tid;         // float4 index: ((xi * 128 + co) * 2 + half)
            const int row = it >> 1, half = it & 1;
            *reinterpret_cast<f32x4*>(us + row * WVS + 4 * half) = ur[k];
        });
    };

    floatx16 acc[WXI];
#pragma unroll
    for (int x = 0; x < WXI; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

    // transform thread role: (tile, channel)
    const int tt = tid & 31, tc = tid >> 5;
    const int twy = tt >> 3, twx = tt & 7;

    if (pro != PRO_NONE) __syncthreads();   // pab visible before the first staging
    load(0);
    for (int chunk = 0; chunk < nchunks; ++chunk) {
        stage(chunk);
        __syncthreads();
        // ---- input transform: V = B^T d B for tile tt, channel tc -----------------------------
        {
            float d[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int s = 0; s < 4; ++s) d[r][s] = patch[((2 * twy + r) * WPW + 2 * twx + s) * WPS + tc];
            float t[4][4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {   // rows: B^T d
                t[0][s] = d[0][s] - d[2][s];
                t[1][s] = d[1][s] + d[2][s];
                t[2][s] = d[2][s] - d[1][s];
                t[3][s] = d[1][s] - d[3][s];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {   // columns: (B^T d) B
                const float v0 = t[r][0] - t[r][2], v1 = t[r][1] + t[r][2];
                const float v2 = t[r][2] - t[r][1], v3 = t[r][1] - t[r][3];
                vs[((r * 4 + 0) * 32 + tt) * WVS + tc] = v0;
                vs[((r * 4 + 1) * 32 + tt) * WVS + tc] = v1;
                vs[((r * 4 + 2) * 32 + tt) * WVS + tc] = v2;
                vs[((r * 4 + 3) * 32 + tt) * WVS + tc] = v3;
            }
        }
        __syncthreads();
        if (chunk + 1 < nchunks) load(chunk + 1);   // in flight during the MFMAs
        // ---- 16 batched GEMMs: acc[xi] (32 tiles x 32 channels) += V[xi] (32 x 8) U[xi] (8 x 32) ----
        // operands of point x+1 are read from LDS before the MFMAs of point x (order pinned with
        // sched_barrier: without it the compiler reuses one register set and waits on every read)
        {
            const float* va = vs + li * WVS + 4 * lh;
            const float* ub = us + (wave * 32 + li) * WVS + 4 * lh;
            f32x4 av[2], bv[2];
            av[0] = *reinterpret_cast<const f32x4*>(va);
            bv[0] = *reinterpret_cast<const f32x4*>(ub);
#pragma unroll
            for (int x = 0; x < WXI; ++x) {
                if (x + 1 < WXI) {
                    av[(x + 1) & 1] = *reinterpret_cast<const f32x4*>(va + (x + 1) * 32 * WVS);
                    bv[(x + 1) & 1] = *reinterpret_cast<const f32x4*>(ub + (x + 1) * WN * WVS);
                }
                __builtin_amdgcn_sched_barrier(0);
                const f32x4 a4 = av[x & 1], b4 = bv[x & 1];
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4.x, acc[x], 0, 0, 0);
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4.y, acc[x], 0, 0, 0);
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4.z, acc[x], 0, 0, 0);
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4.w, acc[x], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();   // V / U / patch free for the next chunk
    }

    // ---- epilogue: output transform, bias + ReLU, store, tile statistics -----------------------
    const int co = wave * 32 + li;
    const float bias = a.bias[co];
    float yv[64];
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * lh;   // Winograd tile of this accumulator row
        const int wy = row >> 3, wx = row & 7;
        float m[16];
#pragma unroll
        for (int x = 0; x < WXI; ++x) m[x] = acc[x][j];
        // T = A^T M (2 x 4), Y = T A (2 x 2); A^T = [[1,1,1,0],[0,1,-1,-1]]
        float t0[4], t1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            t0[c] = m[0 * 4 + c] + m[1 * 4 + c] + m[2 * 4 + c];
            t1[c] = m[1 * 4 + c] - m[2 * 4 + c] - m[3 * 4 + c];
        }
        const float yy[4] = {t0[0] + t0[1] + t0[2], t0[1] - t0[2] - t0[3], t1[0] + t1[1] + t1[2],
                             t1[1] - t1[2] - t1[3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int oy = y0 + 2 * wy + (q >> 1), ox = x0 + 2 * wx + (q & 1);
            const float v = fmaxf(yy[q] + bias, 0.f);
            const bool ok = oy < H && ox < W;
            yv[j * 4 + q] = ok ? v : 0.f;
            if (ok) {
                a.out[(img + (size_t)oy * W + ox) * WN + co] = v;
                s += v;
                cnt += 1.f;
            }
        }
    }
    if (a.part != nullptr) {
        s += __shfl_xor(s, 32);
        cnt += __shfl_xor(cnt, 32);
        const float mean = cnt > 0.f ? s / cnt : 0.f;
        float m2 = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = (j & 3) + 8 * (j >> 2) + 4 * lh;
            const int wy = row >> 3, wx = row & 7;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int oy = y0 + 2 * wy + (q >> 1), ox = x0 + 2 * wx + (q & 1);
                const float dd = yv[j * 4 + q] - mean;
                if (oy < H && ox < W) m2 = fmaf(dd, dd, m2);
            }
        }
        m2 += __shfl_xor(m2, 32);
        if (lh == 0) {
            const int n_part = a.tiles_y * a.tiles_x;
            a.part[((size_t)b * WN + co) * n_part + ty * a.tiles_x + tx] = make_float4(s, m2, cnt, 0.f);
        }
    }
}

bool wino_supported(int kh, int stride, int cin, int cout) {
    return kh == 3 && stride == 1 && cout == WN && cin % WCK == 0 && cin <= W_MAX_CIN;
}

int wino_tiles_y(int H) { return (H + WTH - 1) / WTH; }
int wino_tiles_x(int W) { return (W + WTW - 1) / WTW; }

// U[chunk][xi][co][8] = (G g G^T)[xi] for input channel chunk*8 + c; g = Keras HWIO kernel (3,3,cin,128)
std::vector<float> wino_pack_weights(const float* kern, int cin) {
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    std::vector<float> U((size_t)cin / WCK * WXI * WN * WCK);
    for (int ci = 0; ci < cin; ++ci)
        for (int co = 0; co < WN; ++co) {
            double g[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) g[i][j] = kern[(((size_t)i * 3 + j) * cin + ci) * WN + co];
            for (int p = 0; p < 4; ++p)
                for (int q = 0; q < 4; ++q) {
                    double u = 0.0;
                    for (int i = 0; i < 3; ++i)
                        for (int j = 0; j < 3; ++j) u += G[p][i] * g[i][j] * G[q][j];
                    const int chunk = ci / WCK, c = ci % WCK, xi = p * 4 + q;
                    U[(((size_t)chunk * WXI + xi) * WN + co) * WCK + c] = (float)u;
                }
        }
    return U;
}

hipError_t wino_prepare() {
    return hipFuncSetAttribute((const void*)wino_conv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)W_LDS_BYTES);
}

hipError_t wino_launch(const WinoArgs& a, hipStream_t st) {
    if (a.cin % WCK != 0 || a.cin > W_MAX_CIN) return hipErrorInvalidValue;
    if (!(a.pro_mode == PRO_NONE || a.pro_mode == PRO_AFF_RELU || a.pro_mode == PRO_AFF ||
          a.pro_mode == PRO_AFF_RES))
        return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    hipLaunchKernelGGL(wino_conv_kernel, dim3(grid), dim3(256), W_LDS_BYTES, st, a);
    return hipGetLastError();
}

}  // namespace rst
