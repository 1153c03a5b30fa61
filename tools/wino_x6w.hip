// wino_x6w.hip — EXPERIMENT (tools/wino_x6w_bench only, not in librst): measured slower than wino_x6 at every
// prologue mode (B=1, Cin 128: 39.7 vs 34.5 us ReLU prologue, 44.1 vs 35.8 skip-add; profiles/r03/x6w_u.log), so
// the U bytes per MFMA are not what bounds wino_x6. Kept with its bench as the record of that measurement.
//
// The residual-block convolutions (3x3, stride 1, SAME, 128 output channels;
// realtime_style_transfer/models/styleTransfer.py:144-185) as fused Winograd F(2x2, 3x3) with split-bf16 x6
// products on the bf16 MFMA pipe: wino_x6.hip's arithmetic on a wider workgroup tile that halves the L2 bytes of
// the transformed weights per MFMA.
//
// wino_x6 (8 x 16 pixels = 32 Winograd tiles x all 128 output channels per workgroup) streams the whole U image
// (1.57 MB at Cin 128) through every workgroup: 196 KB per 16-channel chunk against 96 MFMAs per SIMD, i.e.
// ~150 GB/s per CU at the MFMA rate, twice the 66-73 GB/s per CU that MI355X_MICROARCH.md measures for rows
// every workgroup of an XCD shares. Here a workgroup owns 16 x 16 pixels = 64 Winograd tiles (two 32-row MFMA
// M blocks) x 64 output channels (grid = 2 channel halves per spatial tile): the same MFMAs per workgroup, half
// the U bytes (786 KB), ~75 GB/s per CU at the MFMA rate.
//
// The V image of 64 tiles would be 96 KB per 16-channel chunk (192 KB double-buffered), so chunks are 8 input
// channels and the six split terms are packed into the MFMA's K = 16 (lanes 0-31 carry K rows 0-7, lanes 32-63
// rows 8-15, both over the same 8 channels):
//     MFMA 1: A = [v0 | v0], B = R1 = [u0 | u1]  ->  v0 u0 + v0 u1
//     MFMA 2: A = [v1 | v1], B = R1             ->  v1 u0 + v1 u1
//     MFMA 3: A = [v0 | v2], B = R2 = [u2 | u0]  ->  v0 u2 + v2 u0
// i.e. exactly the six terms a0b0 a0b1 a1b0 a0b2 a1b1 a2b0 of wino_x6 (the same pieces, the same fp32
// accumulation), with two 16-B U loads per lane and point (R1, R2: the lane half selects the piece) feeding
// six MFMAs (both M blocks). Wave (nb, pq) owns output channels [32 nb, 32 nb + 32) of the workgroup's 64 and
// the transform points of row pq (4 points x 2 M blocks = 8 accumulators); the U ring holds a whole chunk.
// Epilogue: each wave forms T_pq = M[pq][.] A (two columns) into an LDS image [p][c][tile][channel]; the final
// pass sums Y = A^T T per pixel, adds bias (+ ReLU), stores the workgroup's 64 channels of each pixel and
// reduces the per-(workgroup, channel) two-pass {sum, M2, n} for the CIN that follows.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace rst {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int WTH = 16, WTW = 16;                 // output pixels per workgroup
constexpr int WPH = WTH + 2, WPW = WTW + 2;       // input patch 18 x 18
constexpr int WNP = WPH * WPW;                    // 324 patch pixels
constexpr int WCK = 8;                            // input channels per chunk
constexpr int WPS = 12;                           // patch pixel stride (floats): conflict-free ds_read_b64 columns
constexpr int WN = 64;                            // output channels per workgroup (2 waves x 32)
constexpr int WCO = 128;                          // output channels of the layer
constexpr int WXI = 16;                           // transform points
constexpr int WPF4 = WNP * WCK / 4;               // 648 float4 per chunk patch
constexpr int WMAX_CIN = 256;
constexpr int WPATCH_FL = WNP * WPS + 4;          // one patch buffer (floats) + a 16-B sink for idle staging items
constexpr int WVROW = 16;                         // bytes per (piece, xi, tile) row: 8 bf16
constexpr int WV_BYTES = 3 * WXI * 64 * WVROW;    // one V buffer: 48 KB
constexpr int WPIECE = WXI * 64 * WVROW;          // 16 KB between V pieces
constexpr int WUPIECE = WCO * WVROW;              // 2 KB between U pieces of one (chunk, point)
constexpr int WT = 512;                           // threads per workgroup
constexpr int WST = (WPF4 + WT - 1) / WT;         // 2 staging float4 per thread
constexpr int WPT = 4;                            // transform points per wave
constexpr int WRING = 4;                          // U ring: points in flight (a whole chunk)
constexpr size_t WLOOP_BYTES = (size_t)2 * WPATCH_FL * 4 + 2 * WV_BYTES + WMAX_CIN * sizeof(float2);
constexpr size_t WIMG_BYTES = (size_t)4 * 2 * 64 * WN * 4;      // epilogue: T [p][c][tile][channel] (128 KB)
constexpr size_t WRED_BYTES = (size_t)2 * 8 * 16 * 16;          // statistics reduction [2][8 waves][16] float4
constexpr size_t WEPI_BYTES = WIMG_BYTES + WRED_BYTES + 2 * WN * 8;   // + [2][64] f64 (accumulator adds)
constexpr size_t WLDS_BYTES = WLOOP_BYTES > WEPI_BYTES ? WLOOP_BYTES : WEPI_BYTES;
constexpr size_t WLDS_BLEND_BYTES = WLDS_BYTES + WMAX_CIN * sizeof(float2);   // + the second style's affine
static_assert(WLDS_BLEND_BYTES <= 160 * 1024, "LDS budget");
static_assert(WPT % WRING == 0 || WRING % WPT == 0, "ring");

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

__device__ __forceinline__ float pro_apply_blend(int mode, float x, float2 ab, float2 ab1, float w, float r) {
    float y = style_blend(w, fmaf(ab.x, x, ab.y), fmaf(ab1.x, x, ab1.y));
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}

}  // namespace

template <int PRO, bool BLEND = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_x6w_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* const patch = smem;                                                                 // [2][324 * 12 + 4]
    unsigned char* const vbytes = reinterpret_cast<unsigned char*>(smem + 2 * WPATCH_FL);      // [2][3][16][64][16 B]
    float2* const pab = reinterpret_cast<float2*>(vbytes + 2 * WV_BYTES);
    float2* const pab1 = reinterpret_cast<float2*>(reinterpret_cast<unsigned char*>(smem) + WLDS_BYTES);

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 31, lh = lane >> 5;
    const int nb = wave & 1, pq = wave >> 1;   // channel block (of the workgroup's two), transform-point row
    int bid = xcd_tile_order(blockIdx.x, gridDim.x);
    const int ch = bid & 1;                    // channel half: the two halves of a tile are neighbours (same XCD)
    bid >>= 1;
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

    auto load_affine = [&]() __attribute__((always_inline)) {
        if constexpr (pro != PRO_NONE) {
            if (a.pro_stat.acc != nullptr) {
                const bool store = tx == 0 && ty == 0 && ch == 0;   // one workgroup per image keeps the host copy
                const CinSrc& ps = a.pro_stat;
                cin_affine_table<WT>(ps, b, 1, pab, BLEND ? pab1 : nullptr,
                                     store && ps.ab_out ? ps.ab_out + (size_t)b * Cin : nullptr,
                                     store && ps.ab1_out ? ps.ab1_out + (size_t)b * Cin : nullptr);
            } else {
                for (int c = tid; c < Cin; c += WT) pab[c] = a.pro_ab[(size_t)b * Cin + c];
                if constexpr (BLEND)
                    for (int c = tid; c < Cin; c += WT) pab1[c] = a.pro_ab1[(size_t)b * Cin + c];
            }
        }
    };
    static_assert(!BLEND || PRO != PRO_NONE, "the blend is a prologue");

    // ---- staging descriptors: item k = float4 tid + 512k of a chunk's 648-float4 patch (pixel, channel quad) ----
    int sg_goff[WST], sg_lf[WST], sg_moff[WST];
#pragma unroll
    for (int k = 0; k < WST; ++k) {
        const int it = tid + k * WT, itc = min(it, WPF4 - 1);
        const int px = itc >> 1, q = itc & 1;
        const int iy = y0 - 1 + px / WPW, ix = x0 - 1 + px % WPW;
        const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
        sg_goff[k] = (int)((img + (size_t)cy * W + cx) * Cin) + 4 * q;
        const bool inside = iy >= 0 && iy < H && ix >= 0 && ix < W;
        const int loff = it < WPF4 ? px * WPS + 4 * q : WNP * WPS;   // idle items write the sink
        sg_lf[k] = loff | (inside ? 1 << 16 : 0);
        // one of the two channel halves materialises the block output (interior pixels of its tile)
        const bool interior = ch == 0 && it < WPF4 && inside && iy >= y0 && iy < y0 + WTH && ix >= x0 && ix < x0 + WTW;
        sg_moff[k] = interior ? (int)(((img + (size_t)iy * W + ix) * Cin + 4 * q) * 4) : 0x7F000000;
    }
    const __amdgpu_buffer_rsrc_t msrd = __builtin_amdgcn_make_buffer_rsrc(
        a.mat, 0, a.mat != nullptr ? (int)((size_t)a.batch * H * W * Cin * 4) : 0, 0x00020000);
    f32x4 xr[WST], rr[WST];
    float wr[WST];
    const int cq4 = 4 * (tid & 1);   // channel quad of every staging item of this thread
#pragma unroll
    for (int k = 0; k < WST; ++k) {
        rr[k] = xr[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        wr[k] = 0.f;
        if constexpr (BLEND) wr[k] = a.pro_w[(sg_goff[k] - cq4) / Cin];
    }
    auto gload = [&](int k, int chunk) __attribute__((always_inline)) {
        const int gi = sg_goff[k] + chunk * WCK;
        xr[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
        if constexpr (pro == PRO_AFF_RES) rr[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
    };
    auto stage_math = [&](int k, int chunk, f32x4 p01, f32x4 p23) __attribute__((always_inline)) {
        f32x4 v = xr[k];
        if constexpr (pro != PRO_NONE) {
            const f32x4 r = rr[k];
            if constexpr (BLEND) {
                const f32x4 q01 = *reinterpret_cast<const f32x4*>(pab1 + chunk * WCK + cq4);
                const f32x4 q23 = *reinterpret_cast<const f32x4*>(pab1 + chunk * WCK + cq4 + 2);
                const float w = wr[k];
                v.x = pro_apply_blend(pro, v.x, float2{p01.x, p01.y}, float2{q01.x, q01.y}, w, r.x);
                v.y = pro_apply_blend(pro, v.y, float2{p01.z, p01.w}, float2{q01.z, q01.w}, w, r.y);
                v.z = pro_apply_blend(pro, v.z, float2{p23.x, p23.y}, float2{q23.x, q23.y}, w, r.z);
                v.w = pro_apply_blend(pro, v.w, float2{p23.z, p23.w}, float2{q23.z, q23.w}, w, r.w);
            } else {
                v.x = pro_apply(pro, v.x, float2{p01.x, p01.y}, r.x);
                v.y = pro_apply(pro, v.y, float2{p01.z, p01.w}, r.y);
                v.z = pro_apply(pro, v.z, float2{p23.x, p23.y}, r.z);
                v.w = pro_apply(pro, v.w, float2{p23.z, p23.w}, r.w);
            }
            if (a.mat != nullptr)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), msrd,
                                                       sg_moff[k] + chunk * WCK * 4, 0, 0);
        }
        return v;
    };
    auto stage_write = [&](int k, float* pbuf, f32x4 v) __attribute__((always_inline)) {
        const bool inside = (sg_lf[k] >> 16) != 0;
        v.x = inside ? v.x : 0.f;
        v.y = inside ? v.y : 0.f;
        v.z = inside ? v.z : 0.f;
        v.w = inside ? v.w : 0.f;
        *reinterpret_cast<f32x4*>(pbuf + (sg_lf[k] & 0xFFFF)) = v;
    };
    auto stage_all = [&](int chunk, float* pbuf) __attribute__((always_inline)) {
        sfor<0, WST>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            f32x4 p01 = f32x4{0.f, 0.f, 0.f, 0.f}, p23 = p01;
            if constexpr (pro != PRO_NONE) {
                p01 = *reinterpret_cast<const f32x4*>(pab + chunk * WCK + cq4);
                p23 = *reinterpret_cast<const f32x4*>(pab + chunk * WCK + cq4 + 2);
            }
            stage_write(k, pbuf, stage_math(k, chunk, p01, p23));
        });
    };

    // ---- U: lane (li, lh) of wave (nb, pq) reads U[chunk][4pq + x][piece][64ch + 32nb + li][0..7] ---------------
    // R1 = [u0 | u1] (piece lh), R2 = [u2 | u0] (piece 2 - 2lh); the chunk/point part is a scalar offset
    const __amdgpu_buffer_rsrc_t usrd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.U), 0, nchunks * WXI * 3 * WUPIECE, 0x00020000);
    const int uco = (WN * ch + 32 * nb + li) * WVROW;
    const int uoff1 = uco + lh * WUPIECE, uoff2 = uco + (2 - 2 * lh) * WUPIECE;
    short8 ur[WRING][2];
    auto load_u = [&](int chunk, int x, int s, int r) __attribute__((always_inline)) {
        ur[s][r] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(
                                                  usrd, r ? uoff2 : uoff1, (chunk * WXI + 4 * pq + x) * 3 * WUPIECE, 0));
    };

    // ---- input transform + split: thread = (half h, tile tt, channel pair cp) --------------------------------
    // rows 2h, 2h+1 of B^T d from patch rows f0, f1, f2 = (d0, d2, d1) for h = 0, (d2, d1, d3) for h = 1 (wino_x6.hip)
    const int h = tid >> 8;   // wave-uniform
    const int tt = (tid >> 2) & 63, cp = tid & 3;
    const int twy = tt >> 3, twx = tt & 7;
    const int rd0 = ((2 * twy) * WPW + 2 * twx) * WPS + 2 * cp;
    const int rofs0 = (2 * h) * WPW * WPS, rofs1 = (2 - h) * WPW * WPS, rofs2 = (1 + 2 * h) * WPW * WPS;
    const float sgn = h ? -1.f : 1.f;
    const int vwoff = tt * WVROW + 4 * cp + 8 * h * 64 * WVROW;
    float fx[3][4], fy[3][4];
    auto tr_read_col = [&](const float* pbuf, int c) __attribute__((always_inline)) {
        const f32x2 v0 = *reinterpret_cast<const f32x2*>(pbuf + rd0 + rofs0 + c * WPS);
        const f32x2 v1 = *reinterpret_cast<const f32x2*>(pbuf + rd0 + rofs1 + c * WPS);
        const f32x2 v2 = *reinterpret_cast<const f32x2*>(pbuf + rd0 + rofs2 + c * WPS);
        fx[0][c] = v0.x; fy[0][c] = v0.y;
        fx[1][c] = v1.x; fy[1][c] = v1.y;
        fx[2][c] = v2.x; fy[2][c] = v2.y;
    };
    auto tr_rows_col = [&](int c) __attribute__((always_inline)) {   // row 2h -> f0, row 2h+1 -> f2
        fx[2][c] = fmaf(sgn, fx[2][c], fx[1][c]);
        fy[2][c] = fmaf(sgn, fy[2][c], fy[1][c]);
        fx[0][c] = fx[0][c] - fx[1][c];
        fy[0][c] = fy[0][c] - fy[1][c];
    };
    auto piece = [&](float& x, float& y, unsigned& p) __attribute__((always_inline)) {
        p = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
        x = x - __uint_as_float(p << 16);
        y = y - __uint_as_float(p & 0xFFFF0000u);
    };
    auto last_piece = [&](float x, float y) __attribute__((always_inline)) {
        return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
    };
    auto vwrite = [&](unsigned char* vbuf, int lx, unsigned p0, unsigned p1, unsigned p2) __attribute__((always_inline)) {
        *reinterpret_cast<unsigned*>(vbuf + 0 * WPIECE + lx * 64 * WVROW + vwoff) = p0;
        *reinterpret_cast<unsigned*>(vbuf + 1 * WPIECE + lx * 64 * WVROW + vwoff) = p1;
        *reinterpret_cast<unsigned*>(vbuf + 2 * WPIECE + lx * 64 * WVROW + vwoff) = p2;
    };
    float w0x = 0.f, w0y = 0.f, w1x = 0.f, w1y = 0.f;
    auto cols = [&](int rs, int q0) __attribute__((always_inline)) {
        const float* rx = rs ? fx[2] : fx[0];
        const float* ry = rs ? fy[2] : fy[0];
        if (q0 == 0) {
            w0x = rx[0] - rx[2];
            w0y = ry[0] - ry[2];
            w1x = rx[1] + rx[2];
            w1y = ry[1] + ry[2];
        } else {
            w0x = rx[2] - rx[1];
            w0y = ry[2] - ry[1];
            w1x = rx[1] - rx[3];
            w1y = ry[1] - ry[3];
        }
    };
    auto transform_all = [&](const float* pbuf, unsigned char* vbuf) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < 4; ++c) tr_read_col(pbuf, c);
#pragma unroll
        for (int c = 0; c < 4; ++c) tr_rows_col(c);
#pragma unroll
        for (int rs = 0; rs < 2; ++rs)
#pragma unroll
            for (int q0 = 0; q0 < 4; q0 += 2) {
                cols(rs, q0);
                unsigned p0, p1;
                piece(w0x, w0y, p0);
                piece(w0x, w0y, p1);
                vwrite(vbuf, 4 * rs + q0, p0, p1, last_piece(w0x, w0y));
                piece(w1x, w1y, p0);
                piece(w1x, w1y, p1);
                vwrite(vbuf, 4 * rs + q0 + 1, p0, p1, last_piece(w1x, w1y));
            }
    };

    floatx16 acc[2][WPT];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int x = 0; x < WPT; ++x)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][x][r] = 0.f;

    // ---- pipeline fill: V(0) in V[0], patch(1) in patch[1], patch(2) loads and U(0, all points) in flight ------
    sfor<0, WST>([&](auto K) __attribute__((always_inline)) { gload(decltype(K)::value, 0); });
    sfor<0, WRING>([&](auto X) __attribute__((always_inline)) {
        constexpr int x = decltype(X)::value;
        load_u(x / WPT, x % WPT, x, 0);
        load_u(x / WPT, x % WPT, x, 1);
    });
    load_affine();
    if constexpr (pro != PRO_NONE) lds_barrier();
    stage_all(0, patch);
    if (nchunks > 1) sfor<0, WST>([&](auto K) __attribute__((always_inline)) { gload(decltype(K)::value, 1); });
    lds_barrier();
    transform_all(patch, vbytes);
    if (nchunks > 1) {
        stage_all(1, patch + WPATCH_FL);
        if (nchunks > 2) sfor<0, WST>([&](auto K) __attribute__((always_inline)) { gload(decltype(K)::value, 2); });
    }
    lds_barrier();

    // A operands of lane (li, lh): A0 = v0, A1 = v1, A2 = lh ? v2 : v0 at [piece][4pq + x][32 mb + li]
    const int varow = li * WVROW + 4 * pq * 64 * WVROW;
    const int va2 = varow + lh * 2 * WPIECE;
    unsigned qa0 = 0, qa1 = 0, qb0 = 0, qb1 = 0;
    f32x4 sp01 = f32x4{0.f, 0.f, 0.f, 0.f}, sp23 = sp01, sv = sp01;

    for (int c = 0; c < nchunks; ++c) {
        const int P = c & 1;
        const int c1 = min(c + 1, nchunks - 1), c2 = min(c + 2, nchunks - 1), c3 = min(c + 3, nchunks - 1);
        const unsigned char* const vb = vbytes + P * WV_BYTES;
        unsigned char* const vnext = vbytes + (1 - P) * WV_BYTES;
        const float* const pnext = patch + (1 - P) * WPATCH_FL;
        float* const pstage = patch + P * WPATCH_FL;
        short8 av[2][3];   // [buffer][A0, A1, A2]
        auto read_a = [&](int buf, int x, int mb) __attribute__((always_inline)) {
            const int o = x * 64 * WVROW + mb * 32 * WVROW;
            av[buf][0] = *reinterpret_cast<const short8*>(vb + varow + o);
            av[buf][1] = *reinterpret_cast<const short8*>(vb + WPIECE + varow + o);
            av[buf][2] = *reinterpret_cast<const short8*>(vb + va2 + o);
        };
        read_a(0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // slot s = 6x + 3mb + k: MFMA k of block mb at point x
        sfor<0, WPT>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            constexpr int s = x % WRING;
            sfor<0, 2>([&](auto MB) __attribute__((always_inline)) {
                constexpr int mb = decltype(MB)::value;
                constexpr int buf = (2 * x + mb) & 1;
                sfor<0, 3>([&](auto K) __attribute__((always_inline)) {
                    constexpr int k = decltype(K)::value;
                    constexpr int slot = 6 * x + 3 * mb + k;
                    acc[mb][x] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[buf][k], ur[s][k == 2 ? 1 : 0],
                                                                         acc[mb][x], 0, 0, 0);
                    if constexpr (k == 0 && slot + 3 < 6 * WPT) {   // A operands of the next (point, block)
                        constexpr int nx = mb ? x + 1 : x, nmb = 1 - mb;
                        read_a(1 - buf, nx, nmb);
                    }
                    // U ring refill: R1 last read by (mb 1, k 1), R2 by (mb 1, k 2)
                    if constexpr (mb == 1 && k >= 1) {
                        constexpr int xn = x + WRING;
                        load_u(xn < WPT ? c : c1, xn % WPT, s, k - 1);
                    }
                    // transform + split of chunk c+1 into V[1-P]: slots 0..15
                    if constexpr (slot < 2) {
                        tr_read_col(pnext, 2 * slot);
                        tr_read_col(pnext, 2 * slot + 1);
                    }
                    if constexpr (slot >= 2 && slot < 4) {
                        tr_rows_col(2 * (slot - 2));
                        tr_rows_col(2 * (slot - 2) + 1);
                    }
                    if constexpr (slot >= 4 && slot < 16) {
                        constexpr int grp = (slot - 4) / 3, ph = (slot - 4) % 3;
                        constexpr int rs = grp >> 1, q0 = (grp & 1) * 2, lx0 = 4 * rs + q0;
                        if constexpr (ph == 0) {
                            cols(rs, q0);
                            piece(w0x, w0y, qa0);
                        }
                        if constexpr (ph == 1) {
                            piece(w0x, w0y, qa1);
                            vwrite(vnext, lx0, qa0, qa1, last_piece(w0x, w0y));
                            piece(w1x, w1y, qb0);
                        }
                        if constexpr (ph == 2) {
                            piece(w1x, w1y, qb1);
                            vwrite(vnext, lx0 + 1, qb0, qb1, last_piece(w1x, w1y));
                        }
                    }
                    // staging of chunk c+2 into patch[P], then the loads of chunk c+3: slots 16..23
                    if constexpr (slot >= 16) {
                        constexpr int ks = (slot - 16) >> 2, ph = (slot - 16) & 3;
                        if constexpr (ph == 0 && pro != PRO_NONE && ks == 0) {
                            sp01 = *reinterpret_cast<const f32x4*>(pab + c2 * WCK + cq4);
                            sp23 = *reinterpret_cast<const f32x4*>(pab + c2 * WCK + cq4 + 2);
                        }
                        if constexpr (ph == 1) sv = stage_math(ks, c2, sp01, sp23);
                        if constexpr (ph == 2) stage_write(ks, pstage, sv);
                        if constexpr (ph == 3) gload(ks, c3);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                });
            });
        });
        lds_barrier();
    }

    // ---- epilogue: T_pq[c] = sum_q M[pq][q] A[q][c] per (tile, channel) -> LDS [p][c][tile][64] -----------------
    {
        float* const timg = smem;
        const int col = 32 * nb + li;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int row = 32 * mb + (j & 3) + 8 * (j >> 2) + 4 * lh;   // tile of this accumulator row
                const float m0 = acc[mb][0][j], m1 = acc[mb][1][j], m2 = acc[mb][2][j], m3 = acc[mb][3][j];
                timg[((pq * 2 + 0) * 64 + row) * WN + col] = m0 + m1 + m2;
                timg[((pq * 2 + 1) * 64 + row) * WN + col] = m1 - m2 - m3;
            }
    }
    lds_barrier();
    // thread = (channel quad cq, pixel column px, row half rh): rows 8rh .. 8rh+7 of the tile
    const int cq = tid & 15, px = (tid >> 4) & 15, rh = tid >> 8;
    const int cc = px & 1, twc = px >> 1;
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bias + WN * ch + 4 * cq);
    const bool col_ok = x0 + px < W;
    f32x4 yv[8];
    f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int trow = 4 * rh + i, tile = trow * 8 + twc;
        f32x4 t[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) t[p] = *reinterpret_cast<const f32x4*>(smem + ((p * 2 + cc) * 64 + tile) * WN + 4 * cq);
        f32x4 y2[2] = {t[0] + t[1] + t[2], t[1] - t[2] - t[3]};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            f32x4 v = y2[r] + b4;
            if (!a.linear) {
                v.x = fmaxf(v.x, 0.f);
                v.y = fmaxf(v.y, 0.f);
                v.z = fmaxf(v.z, 0.f);
                v.w = fmaxf(v.w, 0.f);
            }
            const int yy = y0 + 2 * trow + r;
            const bool ok = col_ok && yy < H;
            if (ok) *reinterpret_cast<f32x4*>(a.out + (img + (size_t)yy * W + x0 + px) * WCO + WN * ch + 4 * cq) = v;
            yv[2 * i + r] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
            s4 += yv[2 * i + r];
        }
    }
    if (a.part != nullptr || a.stat.acc != nullptr) {
        f32x4* const red = reinterpret_cast<f32x4*>(reinterpret_cast<unsigned char*>(smem) + WIMG_BYTES);   // [2][8][16]
        double* const dred = reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(smem) + WIMG_BYTES + WRED_BYTES);
        const float cnt = (float)(min(WTH, H - y0) * min(WTW, W - x0));
        auto xsum = [&](f32x4 v) __attribute__((always_inline)) {   // over the wave's 4 pixel columns
#pragma unroll
            for (int o = 16; o < 64; o <<= 1) {
                v.x += __shfl_xor(v.x, o);
                v.y += __shfl_xor(v.y, o);
                v.z += __shfl_xor(v.z, o);
                v.w += __shfl_xor(v.w, o);
            }
            return v;
        };
        s4 = xsum(s4);
        if (lane < 16) red[wave * 16 + cq] = s4;
        lds_barrier();
        f32x4 S = red[cq];
#pragma unroll
        for (int w = 1; w < 8; ++w) S += red[w * 16 + cq];
        const f32x4 mean = S / cnt;
        f32x4 m2 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const bool ok = col_ok && y0 + 2 * (4 * rh + (i >> 1)) + (i & 1) < H;
            const f32x4 d = yv[i] - mean;
            if (ok) m2 += d * d;
        }
        m2 = xsum(m2);
        if (lane < 16) red[128 + wave * 16 + cq] = m2;
        lds_barrier();
        if (tid < 16) {
            f32x4 M = red[128 + cq];
#pragma unroll
            for (int w = 1; w < 8; ++w) M += red[128 + w * 16 + cq];
            if (a.stat.acc != nullptr) {   // {S, M2 + S^2 / n} as f64 (finalize_kernel's merge quantity)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const double dS = (double)S[k];
                    dred[4 * cq + k] = dS;
                    dred[WN + 4 * cq + k] = (double)M[k] + dS * dS / (double)cnt;
                }
            } else {
                const int n_part = a.tiles_y * a.tiles_x;
                float4* const dst = a.part + ((size_t)b * WCO + WN * ch + 4 * cq) * n_part + ty * a.tiles_x + tx;
                dst[0] = make_float4(S.x, M.x, cnt, 0.f);
                dst[n_part] = make_float4(S.y, M.y, cnt, 0.f);
                dst[2 * n_part] = make_float4(S.z, M.z, cnt, 0.f);
                dst[3 * n_part] = make_float4(S.w, M.w, cnt, 0.f);
            }
        }
        if (a.stat.acc != nullptr) {
            lds_barrier();
            if (tid < WN)
                cin_acc_add(a.stat, a.batch, WCO, b, WN * ch + tid, (int)blockIdx.x % a.stat.nslot, dred[tid], dred[WN + tid]);
        }
    }
}

bool wino_x6w_supported(int kh, int stride, int cin, int cout) {
    return kh == 3 && stride == 1 && cout == WCO && cin % WCK == 0 && cin <= WMAX_CIN;
}

static uint16_t bf16_rne_host(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static float bf16_val_host(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// U pieces [cin/8][xi][piece][co][8] bf16 (returned as the float-sized buffer holding the bits): the values and
// pieces of wino_x6_pack_weights (U = G g G^T in f64 rounded to f32, three RNE bf16 pieces), 8-channel chunks
std::vector<float> wino_x6w_pack_weights(const float* kern, int cin) {
#pragma clang fp contract(off)
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    const size_t n16 = (size_t)cin / WCK * WXI * 3 * WCO * WCK;
    std::vector<uint16_t> U(n16);
    for (int ci = 0; ci < cin; ++ci)
        for (int co = 0; co < WCO; ++co) {
            double g[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) g[i][j] = kern[(((size_t)i * 3 + j) * cin + ci) * WCO + co];
            for (int p = 0; p < 4; ++p)
                for (int q = 0; q < 4; ++q) {
                    double u = 0.0;
                    for (int i = 0; i < 3; ++i)
                        for (int j = 0; j < 3; ++j) u += G[p][i] * g[i][j] * G[q][j];
                    const float uf = (float)u;
                    uint16_t pc[3];
                    pc[0] = bf16_rne_host(uf);
                    const float r = uf - bf16_val_host(pc[0]);
                    pc[1] = bf16_rne_host(r);
                    pc[2] = bf16_rne_host(r - bf16_val_host(pc[1]));
                    const int chunk = ci / WCK, c = ci % WCK, xi = p * 4 + q;
                    for (int k = 0; k < 3; ++k)
                        U[((((size_t)chunk * WXI + xi) * 3 + k) * WCO + co) * WCK + c] = pc[k];
                }
        }
    std::vector<float> out((n16 + 1) / 2);
    std::memcpy(out.data(), U.data(), n16 * 2);
    return out;
}

hipError_t wino_x6w_prepare() {
    for (const void* k : {(const void*)wino_x6w_kernel<PRO_NONE>, (const void*)wino_x6w_kernel<PRO_AFF_RELU>,
                          (const void*)wino_x6w_kernel<PRO_AFF>, (const void*)wino_x6w_kernel<PRO_AFF_RES>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WLDS_BYTES);
        if (e != hipSuccess) return e;
    }
    for (const void* k : {(const void*)wino_x6w_kernel<PRO_AFF_RELU, true>, (const void*)wino_x6w_kernel<PRO_AFF, true>,
                          (const void*)wino_x6w_kernel<PRO_AFF_RES, true>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WLDS_BLEND_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

static thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
void wino_x6w_set_timing_events(hipEvent_t start, hipEvent_t stop) {
    g_ev_start = start;
    g_ev_stop = stop;
}

int wino_x6w_tiles_y(int H) { return (H + WTH - 1) / WTH; }
int wino_x6w_tiles_x(int W) { return (W + WTW - 1) / WTW; }

hipError_t wino_x6w_launch(const WinoArgs& a, hipStream_t st) {
    const hipEvent_t e0 = g_ev_start, e1 = g_ev_stop;
    g_ev_start = g_ev_stop = nullptr;
    if (a.cin % WCK != 0 || a.cin > WMAX_CIN || a.tiles_y != (a.H + WTH - 1) / WTH ||
        a.tiles_x != (a.W + WTW - 1) / WTW || (size_t)a.batch * a.H * a.W * a.cin * 4 >= (size_t)0x7F000000)
        return hipErrorInvalidValue;   // 32-bit staging offsets; the out-of-range store offset must stay out of range
    if (a.stat.acc != nullptr && (a.stat.nslot < 1 || a.stat.nslot > CIN_ACC_MAX_SLOTS))
        return hipErrorInvalidValue;
    const bool src_acc = a.pro_stat.acc != nullptr;
    if (src_acc && (a.pro_stat.nslot < 1 || a.pro_stat.nslot > CIN_ACC_MAX_SLOTS || a.pro_stat.C != a.cin ||
                    a.pro_stat.batch != a.batch || a.pro_stat.style == nullptr || a.pro_mode == PRO_NONE))
        return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(2 * a.batch * a.tiles_y * a.tiles_x);
    if (a.pro_w != nullptr) {
        if (src_acc ? a.pro_stat.style1_offset < 0 : (a.pro_ab1 == nullptr || a.pro_ab == nullptr))
            return hipErrorInvalidValue;
        switch (a.pro_mode) {
            case PRO_AFF_RELU: hipExtLaunchKernelGGL((wino_x6w_kernel<PRO_AFF_RELU, true>), dim3(grid), dim3(WT), WLDS_BLEND_BYTES, st, e0, e1, 0, a); break;
            case PRO_AFF: hipExtLaunchKernelGGL((wino_x6w_kernel<PRO_AFF, true>), dim3(grid), dim3(WT), WLDS_BLEND_BYTES, st, e0, e1, 0, a); break;
            case PRO_AFF_RES: hipExtLaunchKernelGGL((wino_x6w_kernel<PRO_AFF_RES, true>), dim3(grid), dim3(WT), WLDS_BLEND_BYTES, st, e0, e1, 0, a); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (a.pro_mode) {
        case PRO_NONE: hipExtLaunchKernelGGL(wino_x6w_kernel<PRO_NONE>, dim3(grid), dim3(WT), WLDS_BYTES, st, e0, e1, 0, a); break;
        case PRO_AFF_RELU: hipExtLaunchKernelGGL(wino_x6w_kernel<PRO_AFF_RELU>, dim3(grid), dim3(WT), WLDS_BYTES, st, e0, e1, 0, a); break;
        case PRO_AFF: hipExtLaunchKernelGGL(wino_x6w_kernel<PRO_AFF>, dim3(grid), dim3(WT), WLDS_BYTES, st, e0, e1, 0, a); break;
        case PRO_AFF_RES: hipExtLaunchKernelGGL(wino_x6w_kernel<PRO_AFF_RES>, dim3(grid), dim3(WT), WLDS_BYTES, st, e0, e1, 0, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rst
