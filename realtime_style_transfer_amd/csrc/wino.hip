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
// Per 8-channel input chunk c the loop body is ONE software-pipelined step with a single barrier:
//   64 MFMAs per wave on V(c) (LDS, operands for point xi+1 read during the MFMAs of xi) x U(c)
//   (registers: U is packed on the host in MFMA B-operand order, so each lane loads its own
//   operands straight from global/L2 -- no LDS round trip; U(c+1)[xi] is loaded into the registers
//   of U(c)[xi] as soon as the MFMAs of point xi have issued), interleaved with
//   - the input transform of chunk c+1: one thread per (tile, channel), V = B^T d B from the LDS
//     patch of c+1 into the other V buffer,
//   - the staging of chunk c+2's patch (prologue: CIN affine [+ ReLU | + residual], materialised
//     block output) from registers into the free patch buffer, and the global loads of chunk c+3.
// Measured before this pipeline (tools/wino_bench.hip phase profile): 45 % of a chunk in MFMA issue,
// the rest in staging U through LDS, load issue, the transform and three barriers.
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
constexpr int WVS = 12;                           // V row stride (floats): odd count of 16-B slots
constexpr int WN = 128;                           // output channels (4 waves x 32)
constexpr int WXI = 16;                           // transform points
constexpr int W_PATCH_F4 = WNP * WCK / 4;         // 360 float4 per chunk
constexpr int W_MAX_CIN = 256;
constexpr int W_PATCH_FL = WNP * WPS;             // one patch buffer (floats)
constexpr int W_V_FL = WXI * 32 * WVS;            // one V buffer (floats)
constexpr size_t W_LDS_BYTES = (size_t)(2 * W_PATCH_FL + 2 * W_V_FL) * 4 + W_MAX_CIN * sizeof(float2);

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

// RST_WINO_OPT bit0: stage the patch of chunk c+2 (prologue + LDS write) and issue the loads of
// chunk c+3 inside the MFMA loop of chunk c instead of before it (one wave per SIMD: work outside
// the MFMA loop leaves the MFMA pipe idle); bit1: issue those HBM patch loads first in the chunk,
// ahead of the chunk's L2 U loads (vmcnt drains in order)
#ifndef RST_WINO_OPT
#define RST_WINO_OPT 1
#endif

#ifdef WINO_PROF
// phase timestamps per (workgroup, wave, chunk) for tools/wino_bench.hip (never in the library build)
__device__ unsigned long long wino_prof[WINO_PROF][4][16][8];
// timeline per (workgroup, wave) on the constant 100 MHz clock: start, pipeline filled, chunk loop done, end
__device__ unsigned long long wino_tl[WINO_PROF][4][4];
#define WPROF(c, k) \
    if (blockIdx.x < WINO_PROF && lane == 0) wino_prof[blockIdx.x][wave][(c)][(k)] = __builtin_amdgcn_s_memtime()
#define WTL(k) \
    if (blockIdx.x < WINO_PROF && lane == 0) wino_tl[blockIdx.x][wave][(k)] = __builtin_amdgcn_s_memrealtime()
#else
#define WPROF(c, k)
#define WTL(k)
#endif

// PRO (the prologue mode) is a template parameter: a runtime mode turned the per-element prologue
// inside the MFMA loop into a branch tree with an lgkmcnt(0) wait per branch
template <int PRO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void wino_conv_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* const patch = smem;                         // [2][180][9]
    float* const vs = patch + 2 * W_PATCH_FL;          // [2][16][32][12]
    float2* const pab = reinterpret_cast<float2*>(vs + 2 * W_V_FL);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    WTL(0);
    int bid = xcd_tile_order(blockIdx.x, gridDim.x);   // XCD-contiguous tile runs (halo reuse in L2)
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * WTH, x0 = tx * WTW;
    const int H = a.H, W = a.W, Cin = a.cin;
    constexpr int pro = PRO;
    const size_t img = (size_t)b * H * W;
    const float* res_src = pro == PRO_AFF_RES ? a.res : a.in;
    const int nchunks = Cin / WCK;

    if constexpr (pro != PRO_NONE) {
        for (int c = tid; c < Cin; c += 256) pab[c] = a.pro_ab[(size_t)b * Cin + c];
    }

    // ---- patch: global -> registers (clamped, branch-free) -> prologue -> LDS -----------------
    f32x4 xr[2], rr[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    auto load_patch = [&](int chunk) __attribute__((always_inline)) {
        const int c0 = chunk * WCK;
        sfor<0, 2>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = min(tid + k * 256, W_PATCH_F4 - 1);
            const int px = it >> 1, q = it & 1;
            const int iy = min(max(y0 - 1 + px / WPW, 0), H - 1), ix = min(max(x0 - 1 + px % WPW, 0), W - 1);
            const size_t gi = (img + (size_t)iy * W + ix) * Cin + c0 + 4 * q;
            xr[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
            if constexpr (pro == PRO_AFF_RES) rr[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
        });
    };
    auto stage = [&](int chunk, float* pbuf) __attribute__((always_inline)) {
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
                if constexpr (pro != PRO_NONE) {
                    const f32x4 r = rr[k];
                    const f32x4 p01 = *reinterpret_cast<const f32x4*>(pab + c);       // (a,b) of c, c+1
                    const f32x4 p23 = *reinterpret_cast<const f32x4*>(pab + c + 2);   // (a,b) of c+2, c+3
                    v.x = pro_apply(pro, v.x, float2{p01.x, p01.y}, r.x);
                    v.y = pro_apply(pro, v.y, float2{p01.z, p01.w}, r.y);
                    v.z = pro_apply(pro, v.z, float2{p23.x, p23.y}, r.z);
                    v.w = pro_apply(pro, v.w, float2{p23.z, p23.w}, r.w);
                    if (a.mat != nullptr && inside && iy >= y0 && iy < y0 + WTH && ix >= x0 && ix < x0 + WTW)
                        *reinterpret_cast<f32x4*>(a.mat + (img + (size_t)iy * W + ix) * Cin + c) = v;
                }
                if (!inside) v = f32x4{0.f, 0.f, 0.f, 0.f};
                float* d = pbuf + px * WPS + 4 * q;
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
        });
    };

    // ---- U: lane (li, lh) of wave w reads U[chunk][xi][32w + li][4lh .. 4lh+3] = its B operand ----
    // buffer loads: one VGPR lane offset, the (chunk, xi) part in the scalar offset
    const __amdgpu_buffer_rsrc_t usrd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, nchunks * WXI * WN * WCK * 4, 0x00020000);
    const int uvoff = ((wave * 32 + li) * 2 + lh) * 16;
    auto load_u = [&](f32x4* u, int chunk, auto X) __attribute__((always_inline)) {
        constexpr int x = decltype(X)::value;
        u[x] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              usrd, uvoff, (chunk * WXI + x) * (WN * WCK * 4), 0));
    };

    // ---- input transform, one thread per (tile tt, channel tc), in pieces -----------------------
    const int tt = tid & 31, tc = tid >> 5;
    const int twy = tt >> 3, twx = tt & 7;
    float d[4][4], t[4][4];
    auto tr_read = [&](const float* pbuf) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) d[r][c] = pbuf[((2 * twy + r) * WPW + 2 * twx + c) * WPS + tc];
    };
    auto tr_rows = [&]() __attribute__((always_inline)) {   // B^T d
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            t[0][c] = d[0][c] - d[2][c];
            t[1][c] = d[1][c] + d[2][c];
            t[2][c] = d[2][c] - d[1][c];
            t[3][c] = d[1][c] - d[3][c];
        }
    };
    auto tr_cols = [&](float* vbuf, int r) __attribute__((always_inline)) {   // (B^T d) B, row r
        const float v0 = t[r][0] - t[r][2], v1 = t[r][1] + t[r][2];
        const float v2 = t[r][2] - t[r][1], v3 = t[r][1] - t[r][3];
        vbuf[((r * 4 + 0) * 32 + tt) * WVS + tc] = v0;
        vbuf[((r * 4 + 1) * 32 + tt) * WVS + tc] = v1;
        vbuf[((r * 4 + 2) * 32 + tt) * WVS + tc] = v2;
        vbuf[((r * 4 + 3) * 32 + tt) * WVS + tc] = v3;
    };

    floatx16 acc[WXI];
#pragma unroll
    for (int x = 0; x < WXI; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

    f32x4 ur[WXI];   // U operands: point xi of chunk c+1 is loaded as soon as the MFMAs of chunk c consumed xi

    // ---- pipeline fill: V(0) in vs[0], patch(1) in patch[1], patch(2) and U(0) loads in flight --
    if constexpr (pro != PRO_NONE) __syncthreads();   // pab visible before the first staging
    load_patch(0);
    sfor<0, WXI>([&](auto X) __attribute__((always_inline)) { load_u(ur, 0, X); });
    stage(0, patch);
    if (nchunks > 1) load_patch(1);
    __syncthreads();
    tr_read(patch);
    tr_rows();
#pragma unroll
    for (int r = 0; r < 4; ++r) tr_cols(vs, r);
    if (nchunks > 1) {
        stage(1, patch + W_PATCH_FL);
        if (nchunks > 2) load_patch(2);
    }
    __syncthreads();
    WTL(1);

    // one chunk: P = chunk parity (V(c) in vs[P], patch(c+1) in patch[1-P], patch[P] free)
    for (int c = 0; c < nchunks; ++c) {
        const int P = c & 1;
        const bool has2 = c + 2 < nchunks, has3 = c + 3 < nchunks;
        const int c1 = min(c + 1, nchunks - 1);
        const float* va = vs + P * W_V_FL + li * WVS + 4 * lh;
        float* const vnext = vs + (1 - P) * W_V_FL;
        const float* const pnext = patch + (1 - P) * W_PATCH_FL;
        WPROF(c, 0);
        if constexpr (!(RST_WINO_OPT & 1)) {
            if (has2) stage(c + 2, patch + P * W_PATCH_FL);   // patch(c+2): its loads landed during chunk c-1
            if (has3) load_patch(c + 3);
        }
        WPROF(c, 1);
        f32x4 av[2];
        av[0] = *reinterpret_cast<const f32x4*>(va);
        __builtin_amdgcn_sched_barrier(0);
        sfor<0, WXI>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            if constexpr (x + 1 < WXI) av[(x + 1) & 1] = *reinterpret_cast<const f32x4*>(va + (x + 1) * 32 * WVS);
            __builtin_amdgcn_sched_barrier(0);   // the read of point x+1 issues before the MFMAs of x
            const f32x4 a4 = av[x & 1], b4 = ur[x];
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4.x, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4.y, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4.z, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4.w, acc[x], 0, 0, 0);
            // chunk c+1 (clamped: past the last chunk this re-reads and writes buffers nobody reads)
            load_u(ur, c1, X);
            if constexpr (x == 1) tr_read(pnext);
            if constexpr (x == 3) tr_rows();
            if constexpr (x >= 4 && x < 8) tr_cols(vnext, x - 4);
            if constexpr ((RST_WINO_OPT & 1) && x == 9) {   // patch(c+2) -> patch[P] (free since chunk c-1's transform)
                if (has2) stage(c + 2, patch + P * W_PATCH_FL);
            }
            if constexpr ((RST_WINO_OPT & 1) && x == ((RST_WINO_OPT & 2) ? 0 : 11)) {
                if (has3) load_patch(c + 3);
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        WPROF(c, 2);
        __syncthreads();
        WPROF(c, 3);
    }
    WTL(2);

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
            const float v = a.linear ? yy[q] + bias : fmaxf(yy[q] + bias, 0.f);
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
    WTL(3);
}

// ---- 8-wave variant: two waves per SIMD ------------------------------------------------------------
// Same tile, transforms and operand layouts as wino_conv_kernel, but 8 waves: wave w owns output
// channels 32(w&3)..+32 for the transform points 8(w>>2)..+8 only (128 accumulator registers), so
// two waves share each SIMD and one's LDS/L2 waits and barrier skew hide behind the other's MFMAs
// (with one wave per SIMD the MFMA issue inside the chunk loop was ~77 %). Waves 0-3 run the input
// transform of chunk c+1, waves 4-7 the staging of chunk c+2 (each SIMD holds one of each), both
// interleaved with their 32 MFMAs per chunk. Epilogue: A^T M A is linear in M, so the waves holding
// points 8..15 (M rows 2, 3) push their partial 2x2 outputs through LDS to the waves holding 0..7,
// which add them and finish bias + ReLU + store + tile statistics.
constexpr int W8_EXCH_FL = 4 * 16 * 4 * 64;                              // [cg][j][q][lane]
constexpr size_t W8_LDS_BYTES = (size_t)W8_EXCH_FL * 4;                  // aliases patch + V + pab
static_assert(W8_LDS_BYTES >= W_LDS_BYTES, "exchange buffer covers the main-loop LDS");

template <int PRO>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_conv8_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* const patch = smem;                         // [2][180][9]
    float* const vs = patch + 2 * W_PATCH_FL;          // [2][16][32][12]
    float2* const pab = reinterpret_cast<float2*>(vs + 2 * W_V_FL);
    float* const exch = smem;                          // after the main loop

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cg = wave & 3, xh = wave >> 2;           // channel group, transform-point half
    const int li = lane & 31, lh = lane >> 5;
    int bid = xcd_tile_order(blockIdx.x, gridDim.x);   // XCD-contiguous tile runs (halo reuse in L2)
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * WTH, x0 = tx * WTW;
    const int H = a.H, W = a.W, Cin = a.cin;
    constexpr int pro = PRO;
    const size_t img = (size_t)b * H * W;
    const float* res_src = pro == PRO_AFF_RES ? a.res : a.in;
    const int nchunks = Cin / WCK;

    if constexpr (pro != PRO_NONE) {
        for (int c = tid; c < Cin; c += 512) pab[c] = a.pro_ab[(size_t)b * Cin + c];
    }

    // ---- staging role (waves 4-7): items st and st + 256 of the 360 float4 of a chunk's patch ----
    const int st = tid - 256;
    f32x4 xr[2], rr[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    auto load_patch = [&](int chunk) __attribute__((always_inline)) {
        const int c0 = chunk * WCK;
        sfor<0, 2>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = min(st + k * 256, W_PATCH_F4 - 1);
            const int px = it >> 1, q = it & 1;
            const int iy = min(max(y0 - 1 + px / WPW, 0), H - 1), ix = min(max(x0 - 1 + px % WPW, 0), W - 1);
            const size_t gi = (img + (size_t)iy * W + ix) * Cin + c0 + 4 * q;
            xr[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
            if constexpr (pro == PRO_AFF_RES) rr[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
        });
    };
    auto stage = [&](int chunk, float* pbuf) __attribute__((always_inline)) {
        const int c0 = chunk * WCK;
        sfor<0, 2>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = st + k * 256;
            if (it < W_PATCH_F4) {
                const int px = it >> 1, q = it & 1;
                const int iy = y0 - 1 + px / WPW, ix = x0 - 1 + px % WPW;
                const int c = c0 + 4 * q;
                f32x4 v = xr[k];
                const bool inside = iy >= 0 && iy < H && ix >= 0 && ix < W;
                if constexpr (pro != PRO_NONE) {
                    const f32x4 r = rr[k];
                    const f32x4 p01 = *reinterpret_cast<const f32x4*>(pab + c);
                    const f32x4 p23 = *reinterpret_cast<const f32x4*>(pab + c + 2);
                    v.x = pro_apply(pro, v.x, float2{p01.x, p01.y}, r.x);
                    v.y = pro_apply(pro, v.y, float2{p01.z, p01.w}, r.y);
                    v.z = pro_apply(pro, v.z, float2{p23.x, p23.y}, r.z);
                    v.w = pro_apply(pro, v.w, float2{p23.z, p23.w}, r.w);
                    if (a.mat != nullptr && inside && iy >= y0 && iy < y0 + WTH && ix >= x0 && ix < x0 + WTW)
                        *reinterpret_cast<f32x4*>(a.mat + (img + (size_t)iy * W + ix) * Cin + c) = v;
                }
                if (!inside) v = f32x4{0.f, 0.f, 0.f, 0.f};
                float* d = pbuf + px * WPS + 4 * q;
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
        });
    };

    // ---- U operands of this wave's points 8xh..8xh+7 -------------------------------------------
    const __amdgpu_buffer_rsrc_t usrd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, nchunks * WXI * WN * WCK * 4, 0x00020000);
    const int uvoff = ((cg * 32 + li) * 2 + lh) * 16;
    auto load_u = [&](f32x4* u, int chunk, auto X) __attribute__((always_inline)) {
        constexpr int x = decltype(X)::value;
        u[x] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              usrd, uvoff, (chunk * WXI + 8 * xh + x) * (WN * WCK * 4), 0));
    };

    // ---- transform role (waves 0-3): one thread per (tile tt, channel tc) ------------------------
    const int tt = tid & 31, tc = (tid >> 5) & 7;
    const int twy = tt >> 3, twx = tt & 7;
    float d[4][4];   // input tile, transformed in place (B^T d) to keep the register count <= 256
    auto tr_read = [&](const float* pbuf) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) d[r][c] = pbuf[((2 * twy + r) * WPW + 2 * twx + c) * WPS + tc];
    };
    auto tr_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float a0 = d[0][c], a1 = d[1][c], a2 = d[2][c], a3 = d[3][c];
            d[0][c] = a0 - a2;
            d[1][c] = a1 + a2;
            d[2][c] = a2 - a1;
            d[3][c] = a1 - a3;
        }
    };
    auto tr_cols = [&](float* vbuf, int r) __attribute__((always_inline)) {
        const float v0 = d[r][0] - d[r][2], v1 = d[r][1] + d[r][2];
        const float v2 = d[r][2] - d[r][1], v3 = d[r][1] - d[r][3];
        vbuf[((r * 4 + 0) * 32 + tt) * WVS + tc] = v0;
        vbuf[((r * 4 + 1) * 32 + tt) * WVS + tc] = v1;
        vbuf[((r * 4 + 2) * 32 + tt) * WVS + tc] = v2;
        vbuf[((r * 4 + 3) * 32 + tt) * WVS + tc] = v3;
    };

    floatx16 acc[8];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;
    f32x4 ur[8];

    // ---- pipeline fill -----------------------------------------------------------------------
    if constexpr (pro != PRO_NONE) __syncthreads();
    if (xh == 1) load_patch(0);
    sfor<0, 8>([&](auto X) __attribute__((always_inline)) { load_u(ur, 0, X); });
    if (xh == 1) {
        stage(0, patch);
        if (nchunks > 1) load_patch(1);
    }
    __syncthreads();
    if (xh == 0) {
        tr_read(patch);
        tr_rows();
#pragma unroll
        for (int r = 0; r < 4; ++r) tr_cols(vs, r);
    } else if (nchunks > 1) {
        stage(1, patch + W_PATCH_FL);
        if (nchunks > 2) load_patch(2);
    }
    __syncthreads();

    for (int c = 0; c < nchunks; ++c) {
        const int P = c & 1;
        const bool has2 = c + 2 < nchunks, has3 = c + 3 < nchunks;
        const int c1 = min(c + 1, nchunks - 1);
        const float* va = vs + P * W_V_FL + (8 * xh * 32 + li) * WVS + 4 * lh;
        float* const vnext = vs + (1 - P) * W_V_FL;
        const float* const pnext = patch + (1 - P) * W_PATCH_FL;
        f32x4 av[2];
        av[0] = *reinterpret_cast<const f32x4*>(va);
        __builtin_amdgcn_sched_barrier(0);
        sfor<0, 8>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            if constexpr (x + 1 < 8) av[(x + 1) & 1] = *reinterpret_cast<const f32x4*>(va + (x + 1) * 32 * WVS);
            __builtin_amdgcn_sched_barrier(0);
            const f32x4 a4 = av[x & 1], b4 = ur[x];
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4.x, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4.y, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4.z, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4.w, acc[x], 0, 0, 0);
            load_u(ur, c1, X);
            if (xh == 0) {
                if constexpr (x == 0) tr_read(pnext);
                if constexpr (x == 2) tr_rows();
                if constexpr (x >= 3 && x < 7) tr_cols(vnext, x - 3);
            } else {
                if constexpr (x == 1) {
                    if (has2) stage(c + 2, patch + P * W_PATCH_FL);
                }
                if constexpr (x == 4) {
                    if (has3) load_patch(c + 3);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        });
        __syncthreads();
    }

    // ---- epilogue ------------------------------------------------------------------------------
    // T = A^T M (2 x 4) with A^T = [[1,1,1,0],[0,1,-1,-1]]: rows 0,1 of M come from xh == 0,
    // rows 2,3 from xh == 1; Y = T A (2 x 2).
    auto out_tf = [&](const float (&t0)[4], const float (&t1)[4], float (&yy)[4]) __attribute__((always_inline)) {
        yy[0] = t0[0] + t0[1] + t0[2];
        yy[1] = t0[1] - t0[2] - t0[3];
        yy[2] = t1[0] + t1[1] + t1[2];
        yy[3] = t1[1] - t1[2] - t1[3];
    };
    if (xh == 1) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            float t0[4], t1[4], yy[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                t0[q] = acc[q][j];                     // M[2][q]
                t1[q] = -acc[q][j] - acc[4 + q][j];    // -M[2][q] - M[3][q]
            }
            out_tf(t0, t1, yy);
#pragma unroll
            for (int q = 0; q < 4; ++q) exch[((cg * 16 + j) * 4 + q) * 64 + lane] = yy[q];
        }
    }
    __syncthreads();
    if (xh == 1) return;
    const int co = cg * 32 + li;
    const float bias = a.bias[co];
    float yv[64];
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * lh;
        const int wy = row >> 3, wx = row & 7;
        float t0[4], t1[4], yy[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            t0[q] = acc[q][j] + acc[4 + q][j];         // M[0][q] + M[1][q]
            t1[q] = acc[4 + q][j];                     // M[1][q]
        }
        out_tf(t0, t1, yy);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float y = yy[q] + exch[((cg * 16 + j) * 4 + q) * 64 + lane];
            const int oy = y0 + 2 * wy + (q >> 1), ox = x0 + 2 * wx + (q & 1);
            const float v = a.linear ? y + bias : fmaxf(y + bias, 0.f);
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
#pragma clang fp contract(off)   // same operation order as wino_transform_kernel
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

// Device form of wino_pack_weights (training re-packs after every optimizer step): one thread per
// (ci, co), U = G g G^T in float64 with the host's operation order and no contraction, so the image
// is bitwise the host's.
__global__ __launch_bounds__(256) void wino_transform_kernel(const float* __restrict__ kern, int cin,
                                                             float* __restrict__ U) {
#pragma clang fp contract(off)
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= cin * WN) return;
    const int ci = idx / WN, co = idx - (idx / WN) * WN;
    const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    double g[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[i][j] = kern[(((size_t)i * 3 + j) * cin + ci) * WN + co];
    const int chunk = ci / WCK, c = ci % WCK;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double u = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) u = u + G[p][i] * g[i][j] * G[q][j];
            U[(((size_t)chunk * WXI + p * 4 + q) * WN + co) * WCK + c] = (float)u;
        }
}

hipError_t wino_transform_launch(const float* kern, int cin, float* U, hipStream_t st) {
    if (cin % WCK != 0 || cin > W_MAX_CIN) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wino_transform_kernel, dim3((unsigned)((cin * WN + 255) / 256)), dim3(256), 0, st, kern, cin, U);
    return hipGetLastError();
}

// RST_WINO8: launch the 8-wave (two waves per SIMD) variant. Measured (tools/wino_bench.hip, residual
// conv at 120x240x128): 54.6 vs 54.0 us at B=1, 394 vs 382 us at B=8 — no gain over one wave per
// SIMD; the chunk loop is not latency-bound (interleaving the accumulators of two points, or
// issuing the HBM patch loads ahead of the L2 U loads, did not move it either), so the 4-wave
// kernel stays the default.
#ifndef RST_WINO8
#define RST_WINO8 0
#endif

hipError_t wino_prepare() {
    for (const void* k : {(const void*)wino_conv_kernel<PRO_NONE>, (const void*)wino_conv_kernel<PRO_AFF_RELU>,
                          (const void*)wino_conv_kernel<PRO_AFF>, (const void*)wino_conv_kernel<PRO_AFF_RES>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)W_LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    for (const void* k : {(const void*)wino_conv8_kernel<PRO_NONE>, (const void*)wino_conv8_kernel<PRO_AFF_RELU>,
                          (const void*)wino_conv8_kernel<PRO_AFF>, (const void*)wino_conv8_kernel<PRO_AFF_RES>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)W8_LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int PRO>
static void wino_launch_mode(const WinoArgs& a, unsigned grid, hipStream_t st) {
    if (RST_WINO8)
        hipLaunchKernelGGL(wino_conv8_kernel<PRO>, dim3(grid), dim3(512), W8_LDS_BYTES, st, a);
    else
        hipLaunchKernelGGL(wino_conv_kernel<PRO>, dim3(grid), dim3(256), W_LDS_BYTES, st, a);
}

hipError_t wino_launch(const WinoArgs& a, hipStream_t st) {
    if (a.cin % WCK != 0 || a.cin > W_MAX_CIN) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    switch (a.pro_mode) {
        case PRO_NONE: wino_launch_mode<PRO_NONE>(a, grid, st); break;
        case PRO_AFF_RELU: wino_launch_mode<PRO_AFF_RELU>(a, grid, st); break;
        case PRO_AFF: wino_launch_mode<PRO_AFF>(a, grid, st); break;
        case PRO_AFF_RES: wino_launch_mode<PRO_AFF_RES>(a, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rst
