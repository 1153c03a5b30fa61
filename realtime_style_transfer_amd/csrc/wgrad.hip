// wgrad.hip — weight gradients of the transfer network's convs on f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// dW[r][c] = sum_q S(q, r) * U(q, c), a GEMM with M = rows r = (tap, channel of the shifted operand),
// N = columns c, K = pixels q (all images):
//   conv  (styleTransfer.py:170,194):  S = X at q*s + tap - pad  (r = (tap, ci)),  U = dZ at q
//   convT (styleTransfer.py:115-119):  S = dZ at q*s + tap - pad (r = (tap, co)),  U = X at q
// Both land directly in the canonical Keras kernel layout ((kh,kw,in,out) resp. (kh,kw,out,in)).
//
// Workgroup = 4 waves, output tile TR x TC, K split over pixel ranges (split-K) so every layer
// fills the chip; per-split slabs are reduced in a fixed order (bitwise reproducible, no atomics).
// Per stage KP = 32 pixels: each thread owns a fixed row vector of S (its tap / channel decode is
// done once per kernel) and a fixed column vector of U (U is linear in q: no decode at all); the
// next stage's loads are issued into registers before this stage's MFMAs (register prefetch),
// then written to LDS behind one barrier. LDS reads are ds_read_b32 with 32 consecutive rows per
// lane half: conflict-free (banks (a/4)%32 per 32-lane half).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "train.h"

namespace rst {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace wg {
constexpr int KP = 32;   // pixels per stage
}

struct WgradGeom {
    int Cs, Cu, R, SH, SW;
    const float* S;
    const float* U;
};

__device__ __forceinline__ WgradGeom wgrad_geom(const WgradArgs& a) {
    WgradGeom g;
    const bool tr = a.transposed != 0;
    g.Cs = tr ? a.C2 : a.C1;
    g.Cu = tr ? a.C1 : a.C2;
    g.R = a.kh * a.kw * g.Cs;
    g.SH = tr ? a.DH : a.XH;
    g.SW = tr ? a.DW : a.XW;
    g.S = tr ? a.D : a.X;
    g.U = tr ? a.X : a.D;
    return g;
}

template <int TR, int TC, int WR, int WC, bool VS>
__global__ __launch_bounds__(256) void wgrad_mfma_kernel(WgradArgs a) {
    using wg::KP;
    constexpr int MR = TR / WR / 32, MC = TC / WC / 32;
    constexpr int AV = VS ? 4 : 1;
    constexpr int RA = TR / AV;          // S vectors per pixel
    constexpr int PSA = 256 / RA;        // pixel step of one thread's S loads
    constexpr int NA = KP / PSA;         // S loads per thread per stage
    constexpr int CB = TC / 4;           // U float4 per pixel
    constexpr int PSB = 256 / CB;
    constexpr int NB = KP / PSB;
    static_assert(WR * WC == 4 && MR >= 1 && MC >= 1, "4 waves");
    static_assert(256 % RA == 0 && KP % PSA == 0 && 256 % CB == 0 && KP % PSB == 0, "load mapping");
    typedef typename std::conditional<VS, f32x4, float>::type sT;

    __shared__ float la[KP * TR];
    __shared__ float lb[KP * TC];

    const WgradGeom g = wgrad_geom(a);
    const int nr = (g.R + TR - 1) / TR, nc = (g.Cu + TC - 1) / TC;
    int bid = blockIdx.x;
    const int split = bid % a.nsplit;
    bid /= a.nsplit;
    const int tc = bid % nc;
    const int trw = bid / nc;
    const int r0 = trw * TR, c0 = tc * TC;
    const long qhw = (long)a.Qh * a.Qw;
    const long total = (long)a.batch * qhw;
    const long q_begin = (long)split * a.span;
    const long q_end = min(total, q_begin + a.span);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WC, wc = wave % WC;
    const int li = lane & 31, lh = lane >> 5;

    // fixed S row vector of this thread: rows r .. r+AV-1 share one tap (Cs % AV == 0)
    const int ra = tid % RA, pa0 = tid / RA;
    const int r = r0 + ra * AV;
    const bool rvalid = r < g.R;
    const int tap = rvalid ? r / g.Cs : 0;
    const int ch = rvalid ? r - tap * g.Cs : 0;
    const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
    const int dy = ky - a.pad_t, dx = kx - a.pad_l;
    // fixed U column vector
    const int cb = tid % CB, pb0 = tid / CB;
    const int c = c0 + cb * 4;
    const bool cvalid = c < g.Cu;

    sT sreg[NA];
    f32x4 ureg[NB];
    auto load_stage = [&](long q0) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const long q = q0 + pa0 + k * PSA;
            sT v = sT(0.f);
            if (rvalid && q < q_end) {
                // 32-bit index math (B*Qh*Qw < 2^31; a 64-bit division per load dominated this loop)
                const int qi = (int)q, qhw_i = (int)qhw;
                const int b = qi / qhw_i;
                const int rem = qi - b * qhw_i;
                const int qy = rem / a.Qw, qx = rem - qy * a.Qw;
                const int sy = qy * a.stride + dy, sx = qx * a.stride + dx;
                if (sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW)
                    v = *reinterpret_cast<const sT*>(g.S + (((size_t)b * g.SH + sy) * g.SW + sx) * g.Cs + ch);
            }
            sreg[k] = v;
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const long q = q0 + pb0 + k * PSB;
            f32x4 v = f32x4(0.f);
            if (cvalid && q < q_end) v = *reinterpret_cast<const f32x4*>(g.U + (size_t)q * g.Cu + c);
            ureg[k] = v;
        }
    };
    auto store_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NA; ++k) *reinterpret_cast<sT*>(&la[(pa0 + k * PSA) * TR + ra * AV]) = sreg[k];
#pragma unroll
        for (int k = 0; k < NB; ++k) *reinterpret_cast<f32x4*>(&lb[(pb0 + k * PSB) * TC + cb * 4]) = ureg[k];
    };

    floatx16 acc[MR][MC];
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < MC; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

    const int arow = wr * (TR / WR) + li, bcol = wc * (TC / WC) + li;
    if (q_begin < q_end) {
        load_stage(q_begin);
        store_stage();
        __syncthreads();
        for (long q0 = q_begin; q0 < q_end; q0 += KP) {
            const bool more = q0 + KP < q_end;
            if (more) load_stage(q0 + KP);
#pragma unroll 4
            for (int s = 0; s < KP / 2; ++s) {
                const int p = 2 * s + lh;
                float av[MR], bv[MC];
#pragma unroll
                for (int m = 0; m < MR; ++m) av[m] = la[p * TR + arow + m * 32];
#pragma unroll
                for (int n = 0; n < MC; ++n) bv[n] = lb[p * TC + bcol + n * 32];
#pragma unroll
                for (int m = 0; m < MR; ++m)
#pragma unroll
                    for (int n = 0; n < MC; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m], bv[n], acc[m][n], 0, 0, 0);
            }
            __syncthreads();
            if (more) {
                store_stage();
                __syncthreads();
            }
        }
    }
    const int Rp = nr * TR, Cp = nc * TC;
    float* out = a.slab + (size_t)split * Rp * Cp;
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < MC; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * lh;
                out[(size_t)(r0 + wr * (TR / WR) + m * 32 + row) * Cp + c0 + wc * (TC / WC) + n * 32 + li] =
                    acc[m][n][i];
            }
}

// ---- residual convs (3x3 s1, 128 -> 128): the same GEMM with exact split-bf16 products ----------------
// Both operands are split exactly into three bf16 pieces when a stage is written to LDS (x = x0 + x1 + x2,
// round-to-nearest-even at each step) and every 32x32 output tile accumulates the six terms a0b0 a0b1
// a1b0 a0b2 a1b1 a2b0 on v_mfma_f32_32x32x16_bf16 (dropped terms <= 2^-25 of each product; the scheme of
// wino_x6.hip): 6 bf16 MFMAs of 32 cycles per 16 pixels instead of 8 f32 ones of 64. LDS holds one stage
// of KP = 32 pixels as [piece][row or column][pixel] bf16, rows padded to 80 B (odd 16-B slots: the
// ds_read_b128 of 32 consecutive rows hit distinct bank groups); a staging thread owns 4 consecutive rows
// (or columns) x 4 consecutive pixels, so its f32x4 loads (4 channels of one pixel) transpose into
// pixel-pair bf16 words. Register prefetch of the next stage as in wgrad_mfma_kernel; slabs and the
// fixed-order reduction are shared with it.
namespace wx6 {
constexpr int TR = 128, TC = 128, KP = 32;
constexpr int RSB = 80;                       // bytes per LDS row (32 bf16 + 16 B pad)
constexpr int PLANE = TR * RSB;               // bytes per piece plane (TR == TC)
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned piece(float& x, float& y) { return bf16_piece(x, y); }   // nearest bf16 pair; (x, y) -= it (exact)
}  // namespace wx6

__global__ __launch_bounds__(256, 2) void wgrad_x6_kernel(WgradArgs a) {
    using namespace wx6;
    __shared__ __attribute__((aligned(16))) unsigned char la[3 * PLANE], lb[3 * PLANE];
    const WgradGeom g = wgrad_geom(a);
    const int nr = (g.R + TR - 1) / TR, nc = (g.Cu + TC - 1) / TC;
    int bid = blockIdx.x;
    const int split = bid % a.nsplit;
    bid /= a.nsplit;
    const int tc = bid % nc;
    const int trw = bid / nc;
    const int r0 = trw * TR, c0 = tc * TC;
    const long qhw = (long)a.Qh * a.Qw;
    const long total = (long)a.batch * qhw;
    const long q_begin = (long)split * a.span;
    const long q_end = min(total, q_begin + a.span);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int li = lane & 31, lh = lane >> 5;

    // staging: rows r0 + 4 rg .. +3 (one tap: Cs % 4 == 0) and columns c0 + 4 rg .. +3, pixels 4 pq .. +3
    const int rg = tid >> 3, pq = tid & 7;   // pixel quad fastest: 8 lanes write 64 contiguous LDS bytes
    const int r = r0 + 4 * rg;
    const bool rvalid = r < g.R;
    const int tap = rvalid ? r / g.Cs : 0;
    const int ch = rvalid ? r - tap * g.Cs : 0;
    const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
    const int dy = ky - a.pad_t, dx = kx - a.pad_l;
    const int c = c0 + 4 * rg;
    const bool cvalid = c < g.Cu;
    f32x4 sreg[2][4], ureg[2][4];   // two stages in flight (one stage of MFMAs is shorter than the load latency)
    // the thread's first pixel q0 + 4 pq as (image, row, column), advanced by KP per stage without
    // divisions (the per-load decode cost as much VALU as the split)
    int pb = 0, py = 0, px = 0;
    {
        const int qi = (int)(q_begin + 4 * pq), qhw_i = (int)qhw;
        pb = qi / qhw_i;
        const int rem = qi - pb * qhw_i;
        py = rem / a.Qw;
        px = rem - py * a.Qw;
    }
    auto advance = [&](int d) __attribute__((always_inline)) {
        px += d;
        while (px >= a.Qw) {
            px -= a.Qw;
            if (++py == a.Qh) {
                py = 0;
                ++pb;
            }
        }
    };
    auto load_stage = [&](long q0, auto SET) __attribute__((always_inline)) {
        constexpr int st = decltype(SET)::value;
        int b = pb, qy = py, qx = px;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long q = q0 + 4 * pq + k;
            f32x4 v = f32x4(0.f), u = f32x4(0.f);
            if (q < q_end) {
                const int sy = qy * a.stride + dy, sx = qx * a.stride + dx;
                if (rvalid && sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW)
                    v = *reinterpret_cast<const f32x4*>(g.S + (((size_t)b * g.SH + sy) * g.SW + sx) * g.Cs + ch);
                if (cvalid) u = *reinterpret_cast<const f32x4*>(g.U + (size_t)q * g.Cu + c);
            }
            sreg[st][k] = v;
            ureg[st][k] = u;
            if (++qx == a.Qw) {
                qx = 0;
                if (++qy == a.Qh) {
                    qy = 0;
                    ++b;
                }
            }
        }
        advance(KP);
    };
    // f32x4 x 4 pixels -> rows 4rg + j, pixels 4pq .. 4pq+3 of the three piece planes (8 B per row and piece)
    auto put = [&](unsigned char* base, const f32x4 (&v)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float x0 = v[0][j], y0 = v[1][j], x1 = v[2][j], y1 = v[3][j];
            unsigned p[3][2];
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
                p[pc][0] = piece(x0, y0);
                p[pc][1] = piece(x1, y1);
            }
            unsigned char* dst = base + (4 * rg + j) * RSB + 8 * pq;
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) *reinterpret_cast<uint2*>(dst + pc * PLANE) = make_uint2(p[pc][0], p[pc][1]);
        }
    };

    floatx16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

    auto mfma_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int ks = 0; ks < KP / 16; ++ks) {
            short8 A[2][3], B[2][3];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) {
                    A[m][pc] = *reinterpret_cast<const short8*>(la + pc * PLANE + (wr * 64 + m * 32 + li) * RSB +
                                                                (16 * ks + 8 * lh) * 2);
                    B[m][pc] = *reinterpret_cast<const short8*>(lb + pc * PLANE + (wc * 64 + m * 32 + li) * RSB +
                                                                (16 * ks + 8 * lh) * 2);
                }
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    floatx16& C = acc[m][n];
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[m][0], B[n][0], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[m][0], B[n][1], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[m][1], B[n][0], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[m][0], B[n][2], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[m][1], B[n][1], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[m][2], B[n][0], C, 0, 0, 0);
                }
        }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    const int nst = q_begin < q_end ? (int)((q_end - q_begin + KP - 1) / KP) : 0;
    // stage k sits in register set k & 1: loaded two stages ahead, written to LDS one stage ahead
    if (nst > 0) {
        load_stage(q_begin, S0{});
        if (nst > 1) load_stage(q_begin + KP, S1{});
        put(la, sreg[0]);
        put(lb, ureg[0]);
        __syncthreads();
    }
    for (int k = 0; k < nst; k += 2) {
        if (k + 2 < nst) load_stage(q_begin + (long)(k + 2) * KP, S0{});
        mfma_stage();
        __syncthreads();
        if (k + 1 < nst) {
            put(la, sreg[1]);
            put(lb, ureg[1]);
            __syncthreads();
            if (k + 3 < nst) load_stage(q_begin + (long)(k + 3) * KP, S1{});
            mfma_stage();
            __syncthreads();
            if (k + 2 < nst) {
                put(la, sreg[0]);
                put(lb, ureg[0]);
                __syncthreads();
            }
        }
    }
    const int Rp = nr * TR, Cp = nc * TC;
    float* out = a.slab + (size_t)split * Rp * Cp;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * lh;
                out[(size_t)(r0 + wr * 64 + m * 32 + row) * Cp + c0 + wc * 64 + n * 32 + li] = acc[m][n][i];
            }
}

// ---- residual convs, tap-row tiles (wgrad_x6r): one kernel row ky per workgroup ----------------------------
// wgrad_x6_kernel's 128-row tiles are one tap each, so every tile re-reads the 32 stage pixels of both operands:
// 9 x (X + dZ) per launch, 1.06 GB at B = 4 (120 x 240 x 128), which bounds it (~4 TB/s L2/MALL -> CU).
// Here a workgroup owns the three taps (ky, 0..2) of one kernel row (384 rows = kx x 128 ci) x all 128 columns:
// per stage of 32 pixels it loads the 34-pixel window of X row-shifted by ky - 1 once (17 KB contiguous) and the
// 32 dZ pixels once, and forms the three column-shifted S images in LDS (masked where x + kx - 1 or y + ky - 1
// leaves the image: SAME zero padding). 3 x (X + dZ) per launch. 8 waves (two per SIMD), wave (wr, wc) owns rows
// 96 wr .. +95 (3 M tiles) x columns 64 wc .. +63 (2 N tiles): 72 MFMAs of 32x32x16 bf16 per stage, the same
// six split terms as wgrad_x6_kernel. Stage k+1's loads are issued before stage k's MFMAs (register prefetch) and
// split into bf16 pieces right after them; the masked / shifted pieces go to LDS behind the stage's barrier.
namespace wx6r {
constexpr int TAPS = 3, CI = 128, CO = 128, TR = TAPS * CI, KP = 32;
constexpr int RSB = 80;                       // bytes per LDS row (32 bf16 + 16 B pad: conflict-free b128 reads)
constexpr int SPLANE = TR * RSB, UPLANE = CO * RSB;
constexpr size_t LDS_BYTES = (size_t)3 * SPLANE + 3 * UPLANE;   // 122880
typedef short short8 __attribute__((ext_vector_type(8)));
}  // namespace wx6r

__global__ __launch_bounds__(512, 1) void wgrad_x6r_kernel(WgradArgs a) {
    using namespace wx6r;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_x6r[];
    unsigned char* const ls = lds_x6r;                   // [piece][384 rows (kx, ci)][80 B]
    unsigned char* const lu = lds_x6r + 3 * SPLANE;      // [piece][128 rows co][80 B]
    // blockIdx -> (split, ky): the three kernel rows of one pixel split on one XCD (xcd_tile_order: contiguous runs)
    const int t3 = xcd_tile_order(blockIdx.x, gridDim.x);
    const int ky = t3 % TAPS, split = t3 / TAPS;
    const int H = a.Qh, W = a.Qw;
    const long qhw = (long)H * W;
    const long total = (long)a.batch * qhw;
    const long q_begin = (long)split * a.span;
    const long q_end = min(total, q_begin + a.span);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int li = lane & 31, lh = lane >> 5;
    const int dy = ky - a.pad_t;

    // staging: every thread builds both operands for (channel quad cq, pixel pair pp), pp fastest (a wave's b32 LDS
    // writes of one channel cover 4 rows x 64 contiguous bytes: 64 distinct banks). S: the window pixels 2 pp .. 2 pp + 3
    // (= stage pixels 2 pp - 1 .. 2 pp + 2) are split once into two bf16 pair words per channel and piece; tap kx of
    // LDS pixels (2 pp, 2 pp + 1) is window pixels (kx, kx + 1): pair word A (kx 0), B (kx 2) or the v_perm of A's high
    // and B's low half (kx 1), masked per pixel. U: stage pixels 2 pp, 2 pp + 1.
    const int pp = tid & 15, cq = tid >> 4;
    // the stage's first pixel of this thread's pair as (row, column), advanced by KP per stage
    int py, px;
    {
        const long q0 = q_begin + 2 * pp;
        const int rem = (int)(q0 % qhw);
        py = rem / W;
        px = rem - py * W;
    }
    auto advance = [&]() __attribute__((always_inline)) {
        px += KP;
        while (px >= W) {
            px -= W;
            if (++py == H) py = 0;
        }
    };
    f32x4 sreg[4], ureg[2];
    auto load_stage = [&](long q0) __attribute__((always_inline)) {
        const long qt = q0 + 2 * pp;
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // window pixel j <-> X linear index qt - 1 + j + dy W (clamped; masked later)
            long xi = qt - 1 + j + (long)dy * W;
            xi = xi < 0 ? 0 : (xi >= total ? total - 1 : xi);
            sreg[j] = *reinterpret_cast<const f32x4*>(a.X + (size_t)xi * CI + 4 * cq);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const long q = qt + j;
            ureg[j] = *reinterpret_cast<const f32x4*>(a.D + (size_t)(q < q_end ? q : q_begin) * CO + 4 * cq);
        }
    };
    unsigned sw[4][3][2], uw[4][3];   // [channel][piece][pair A / B], [channel][piece]
    auto split_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float x0 = sreg[0][c], y0 = sreg[1][c], x1 = sreg[2][c], y1 = sreg[3][c], xu = ureg[0][c], yu = ureg[1][c];
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
                sw[c][pc][0] = bf16_piece(x0, y0);
                sw[c][pc][1] = bf16_piece(x1, y1);
                uw[c][pc] = bf16_piece(xu, yu);
            }
        }
    };
    auto write_stage = [&](long q0) __attribute__((always_inline)) {
        // masks of the pair's two pixels (low / high bf16 half) per tap; U: inside the split
        const long qt = q0 + 2 * pp;
        int y1 = py, x1 = px + 1;
        if (x1 == W) {
            x1 = 0;
            if (++y1 == H) y1 = 0;
        }
        const bool in0 = qt < q_end && py + dy >= 0 && py + dy < H, in1 = qt + 1 < q_end && y1 + dy >= 0 && y1 + dy < H;
        unsigned ms[TAPS];
#pragma unroll
        for (int kx = 0; kx < TAPS; ++kx) {
            const int d = kx - a.pad_l;
            ms[kx] = (in0 && px + d >= 0 && px + d < W ? 0x0000FFFFu : 0u) | (in1 && x1 + d >= 0 && x1 + d < W ? 0xFFFF0000u : 0u);
        }
        const unsigned mu = (qt < q_end ? 0x0000FFFFu : 0u) | (qt + 1 < q_end ? 0xFFFF0000u : 0u);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
                const unsigned A = sw[c][pc][0], Bw = sw[c][pc][1];
                unsigned char* dst = ls + pc * SPLANE + (4 * cq + c) * RSB + 4 * pp;
                *reinterpret_cast<unsigned*>(dst) = A & ms[0];
                *reinterpret_cast<unsigned*>(dst + CI * RSB) = __builtin_amdgcn_perm(Bw, A, 0x05040302u) & ms[1];
                *reinterpret_cast<unsigned*>(dst + 2 * CI * RSB) = Bw & ms[2];
                *reinterpret_cast<unsigned*>(lu + pc * UPLANE + (4 * cq + c) * RSB + 4 * pp) = uw[c][pc] & mu;
            }
    };

    floatx16 acc[3][2];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;
    auto mfma_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int ks = 0; ks < KP / 16; ++ks) {
            short8 B[2][3];
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int pc = 0; pc < 3; ++pc)
                    B[n][pc] = *reinterpret_cast<const short8*>(lu + pc * UPLANE + (wc * 64 + n * 32 + li) * RSB +
                                                                (16 * ks + 8 * lh) * 2);
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                short8 A[3];
#pragma unroll
                for (int pc = 0; pc < 3; ++pc)
                    A[pc] = *reinterpret_cast<const short8*>(ls + pc * SPLANE + (wr * 96 + m * 32 + li) * RSB +
                                                             (16 * ks + 8 * lh) * 2);
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    floatx16& C = acc[m][n];
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[n][0], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[n][1], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[n][0], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[n][2], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[n][1], C, 0, 0, 0);
                    C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[n][0], C, 0, 0, 0);
                }
            }
        }
    };
    const int nst = q_begin < q_end ? (int)((q_end - q_begin + KP - 1) / KP) : 0;
    if (nst > 0) {
        load_stage(q_begin);
        split_stage();
        write_stage(q_begin);
        advance();
        __syncthreads();
    }
    for (int k = 0; k < nst; ++k) {
        const long qn = q_begin + (long)(k + 1) * KP;
        if (k + 1 < nst) load_stage(qn);
        mfma_stage();
        split_stage();   // (after the last stage: on stale registers, never written)
        // one MFMA, then three VALU, 72 times: the split's VALU issues between this wave's MFMAs (197 -> 192 us at
        // B = 4, two VALU per MFMA the same, profiles/r06/r06ap)
#pragma unroll
        for (int i = 0; i < 72; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        }
        __syncthreads();
        if (k + 1 < nst) {
            write_stage(qn);
            advance();
            __syncthreads();
        }
    }
    // slab rows [ky * 384, +384) = taps (ky, 0..2) x ci, all 128 columns
    float* out = a.slab + (size_t)split * (9 * CI) * CO;
    const int r0 = ky * TR;
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * lh;
                out[(size_t)(r0 + wr * 96 + m * 32 + row) * CO + wc * 64 + n * 32 + li] = acc[m][n][i];
            }
}

// ---- contract_start (9x9 s1 SAME, cin <= 17 -> 32): LDS-patch weight gradient --------------------------
// The generic kernel above reads its S operand (the shifted input, R = 81 taps x 17 channels = 1377
// rows) straight from global memory with 4-byte loads (17 channels: no 16-B vectors): every input
// element is fetched 81 times, 6.4 ms per B=4 step at 480x960. Here a workgroup walks over 8 x 16
// output-pixel tiles; per tile the 16 x 24 x 17 input patch (planar [ci][row][col] in LDS) and the
// 128 x 32 output-gradient tile ([co][pixel]) are staged once, and
//   dW^T[co][(tap, ci)] += dZ^T[co][pixel] X[pixel + tap][ci]
// runs as MFMA with M = the 32 output channels (A operand = dZ, one ds_read_b128 per 4 k-steps) and
// N = the 1377 (tap, ci) columns (44 column tiles, 11 per wave; each lane's column decode is done
// once per kernel). K = pixels; k-step s pairs pixel s (lane half 0) with s + 64 (lane half 1), so a
// lane's 4 consecutive k-steps are 4 consecutive pixels of one tile row. Each workgroup writes one
// partial [1408][32] slab; wgrad_reduce_kernel sums the slabs in a fixed order.
namespace w9 {
constexpr int TH = 8, TW = 16, NPX = TH * TW;          // output pixels per tile
// Strides chosen by an exhaustive search over the bank mapping of the B-operand reads (lane = column (tap, ci),
// lane half = pixel row + 4): row stride 24 and plane stride 401 (= 17 mod 64) put the 64 lanes of a
// ds_read_b32 in at most 2 passes (1.18 on average over the 44 column tiles) instead of 5 (4.8) with 25 / 400
// (SQ: lds_conflict 0.88 of the LDS cycles at 25 / 400)
constexpr int PR = TH + 8, PC = TW + 8, PRS = 24;      // patch rows / cols / row stride (floats)
constexpr int PL = 401;                                // plane stride (floats), >= PR * PRS
constexpr int CMAX = 17, NCOL = 81 * CMAX, NCOLP = 1408, NT = NCOLP / 32, NTW = NT / 4;   // 44 tiles, 11 per wave
constexpr int DZS = NPX + 4;                           // dZ^T row stride (floats)
constexpr int ZERO = CMAX * PL;                        // a zero word after the planes (padding columns)
constexpr int DZOFF = (CMAX * PL + 8 + 3) / 4 * 4;     // dZ^T offset (16-B aligned)
constexpr int LDS_FL = DZOFF + 32 * DZS;
static_assert(PL >= PR * PRS && PRS >= PC, "patch planes");
}  // namespace w9

__global__ __launch_bounds__(256, 2) void wgrad9_kernel(WgradArgs a) {
    using namespace w9;
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];
    float* const patch = lds;                    // [ci][PR][PRS] + zero word
    float* const dzt = lds + DZOFF;              // [co][DZS]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    constexpr int C = CMAX;   // wgrad9_applies: cin == 17 (the slab rows are (tap, ci) with stride 17)
    const int tiles_x = (a.Qw + TW - 1) / TW, tiles_y = (a.Qh + TH - 1) / TH;
    const int ntiles = a.batch * tiles_x * tiles_y;

    // per-lane column decode of this wave's 11 column tiles: LDS offset of (tap, ci) at pixel (0, 0)
    int coff[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave + 4 * j) * 32 + li;   // wave w owns column tiles w, w+4, ...
        if (n < NCOL) {
            const int tap = n / CMAX, ci = n % CMAX;
            coff[j] = ci * PL + (tap / 9) * PRS + tap % 9;
        } else {
            coff[j] = -1;                         // padding column / channel >= cin
        }
    }
    floatx16 acc[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    if (tid < 8) patch[ZERO + tid] = 0.f;

    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int b = t / (tiles_x * tiles_y), rem = t % (tiles_x * tiles_y);
        const int y0 = (rem / tiles_x) * TH, x0 = (rem % tiles_x) * TW;
        __syncthreads();   // previous tile's operands consumed
        // input patch rows y0-4 .. y0+11, cols x0-4 .. x0+19 (SAME pad 4), NHWC -> planar
        for (int i = tid; i < PR * PC * C; i += 256) {
            const int c = i % C, px = i / C;
            const int r = px / PC, q = px % PC;
            const int gy = y0 - a.pad_t + r, gx = x0 - a.pad_l + q;
            float v = 0.f;
            if (gy >= 0 && gy < a.XH && gx >= 0 && gx < a.XW) v = a.X[(((size_t)b * a.XH + gy) * a.XW + gx) * C + c];
            patch[c * PL + r * PRS + q] = v;
        }
        // output-gradient tile, transposed to [co][pixel]
        for (int i = tid; i < NPX * 32; i += 256) {
            const int co = i & 31, p = i >> 5;
            const int oy = y0 + p / TW, ox = x0 + p % TW;
            float v = 0.f;
            if (oy < a.Qh && ox < a.Qw) v = a.D[(((size_t)b * a.DH + oy) * a.DW + ox) * 32 + co];
            dzt[co * DZS + p] = v;
        }
        __syncthreads();
        // 16 groups of 4 k-steps: pixels 4g..4g+3 (lane half 0) / 64+4g.. (lane half 1)
#pragma unroll 2
        for (int g = 0; g < 16; ++g) {
            const int p0 = 4 * g + 64 * lh;
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(dzt + li * DZS + p0);
            const int pixoff = (p0 / TW) * PRS + p0 % TW;
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const float* src = patch + (coff[j] >= 0 ? coff[j] + pixoff : ZERO);
                const int st = coff[j] >= 0 ? 1 : 0;
                const float b0 = src[0], b1 = src[st], b2 = src[2 * st], b3 = src[3 * st];
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b0, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b1, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b2, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b3, acc[j], 0, 0, 0);
            }
        }
    }
    // partial slab [blockIdx][column n][co]: accumulator r of lane (li, lh) is co = (r&3) + 8(r>>2) + 4lh, n = tile*32 + li
    float* slab = a.slab + (size_t)blockIdx.x * NCOLP * 32;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave + 4 * j) * 32 + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) slab[(size_t)n * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] = acc[j][r];
    }
}

// ---- contract_start weight gradient on split-bf16 x6 (the x6 trainer's start conv) --------------------------
// As wgrad9_kernel (M = the 32 output channels, N = the 1377 (tap, ci) columns, K = pixels, one [1408][32] slab per
// workgroup) with the products on v_mfma_f32_32x32x16_bf16: dZ^T and the input patch are split once at staging into
// three exact bf16 pieces, six product terms per k-step (fp32-level, the wgrad_x6 scheme). K-step = one 16-pixel tile
// row: lane half lh takes pixels 8lh .. 8lh + 7. The B operand of column (ky, kx, ci) is 8 consecutive patch
// pixels starting at column kx + 8lh — kx odd is not 4-byte aligned in a bf16 row, so the patch is kept twice, as
// written (copy 0) and shifted one element left (copy 1): column kx reads copy kx & 1 at the even offset kx & ~1,
// four ds_read_b32 per piece.
namespace w9x {
constexpr int TH = 8, TW = 16, NPX = TH * TW;
constexpr int PR = TH + 8, PC = TW + 8, PRS = 24;           // patch rows / cols / row stride (bf16 elements)
// one channel's plane, padded to an odd number of dwords (193): the 32 columns of a B read are mostly consecutive
// channels, which an even-dword pitch (192 = 0 mod 64 banks) put on one bank
constexpr int CMAX = 17, PLANE = PR * PRS + 2;
constexpr int PIECE = CMAX * PLANE, COPY = 3 * PIECE;        // elements per piece / per copy
constexpr int DZS = NPX + 8;                                 // dZ^T row stride (elements; 16-B aligned rows)
constexpr int DZOFF = (2 * COPY + 7) / 8 * 8;                // dZ^T [piece][co][DZS] after the two copies, 16-B aligned
constexpr int LDS_EL = DZOFF + 3 * 32 * DZS;
constexpr size_t LDS_BYTES = (size_t)LDS_EL * 2;
constexpr int NCOL = 81 * CMAX, NCOLP = 1408, NTW = NCOLP / 32 / 4;   // 11 column tiles per wave
static_assert(LDS_BYTES <= 160 * 1024 && (COPY % 2) == 0 && (PLANE % 2) == 0, "layout");
// the A operand (dZ^T, short8 per lane and piece) is read with ds_read_b128: every row 16-B aligned
static_assert((DZOFF * 2) % 16 == 0 && (DZS * 2) % 16 == 0, "16-B aligned dZ^T rows");
}  // namespace w9x

__global__ __launch_bounds__(256, 1) void wgrad9_x6_kernel(WgradArgs a) {
    using namespace w9x;
    typedef short short8 __attribute__((ext_vector_type(8)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned short lds9x[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    constexpr int C = CMAX;
    const int tiles_x = (a.Qw + TW - 1) / TW, tiles_y = (a.Qh + TH - 1) / TH;
    const int ntiles = a.batch * tiles_x * tiles_y;
    // per-lane column decode: element offset of (copy, piece 0, ci, ky, kx & ~1) for this wave's column tiles
    int coff[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave + 4 * j) * 32 + li;
        if (n < NCOL) {
            const int tap = n / C, ci = n % C, ky = tap / 9, kx = tap % 9;
            coff[j] = (kx & 1) * COPY + ci * PLANE + ky * PRS + (kx & ~1);
        } else {
            coff[j] = -1;
        }
    }
    floatx16 acc[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    auto split = [](float v, unsigned short (&p)[3]) __attribute__((always_inline)) {   // exact: v = p0 + p1 + p2
        float y = 0.f;
        const unsigned q0 = bf16_piece(v, y), q1 = bf16_piece(v, y), q2 = bf16_last_piece(v, y);
        p[0] = (unsigned short)(q0 & 0xFFFFu);
        p[1] = (unsigned short)(q1 & 0xFFFFu);
        p[2] = (unsigned short)(q2 & 0xFFFFu);
    };
    // the next tile's global values are loaded into registers while this tile's MFMAs run (one workgroup per CU:
    // no other workgroup hides the load latency), split and stored after the barrier
    constexpr int NXL = (PR * PC * C + 255) / 256, NDL = NPX * 32 / 256;
    float xs[NXL], dz[NDL];
    auto load_tile = [&](int t) __attribute__((always_inline)) {
        const int b = t / (tiles_x * tiles_y), rem = t % (tiles_x * tiles_y);
        const int y0 = (rem / tiles_x) * TH, x0 = (rem % tiles_x) * TW;
#pragma unroll
        for (int k = 0; k < NXL; ++k) {
            const int i = tid + 256 * k;
            const int c = i % C, px = i / C;
            const int r = px / PC, q = px % PC;
            const int gy = y0 - a.pad_t + r, gx = x0 - a.pad_l + q;
            xs[k] = (i < PR * PC * C && gy >= 0 && gy < a.XH && gx >= 0 && gx < a.XW)
                        ? a.X[(((size_t)b * a.XH + gy) * a.XW + gx) * C + c] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NDL; ++k) {
            const int i = tid + 256 * k;
            const int co = i & 31, px = i >> 5;
            const int oy = y0 + px / TW, ox = x0 + px % TW;
            dz[k] = (oy < a.Qh && ox < a.Qw) ? a.D[(((size_t)b * a.DH + oy) * a.DW + ox) * 32 + co] : 0.f;
        }
    };
    auto store_tile = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NXL; ++k) {
            const int i = tid + 256 * k;
            if (i < PR * PC * C) {
                const int c = i % C, px = i / C;
                const int r = px / PC, q = px % PC;
                unsigned short pcs[3];
                split(xs[k], pcs);
                const int e = c * PLANE + r * PRS + q;
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) {
                    lds9x[pc * PIECE + e] = pcs[pc];
                    if (q > 0) lds9x[COPY + pc * PIECE + e - 1] = pcs[pc];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NDL; ++k) {
            const int i = tid + 256 * k;
            const int co = i & 31, px = i >> 5;
            unsigned short pcs[3];
            split(dz[k], pcs);
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) lds9x[DZOFF + (pc * 32 + co) * DZS + px] = pcs[pc];
        }
    };
    if ((int)blockIdx.x < ntiles) load_tile(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        __syncthreads();   // previous tile's operands consumed
        store_tile();
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) load_tile(t + gridDim.x);
#pragma unroll 1
        for (int ks = 0; ks < TH; ++ks) {   // k-step = tile row ks, pixels 16 ks + 8 lh ..
            short8 A[3];
#pragma unroll
            for (int pc = 0; pc < 3; ++pc)
                A[pc] = *reinterpret_cast<const short8*>(lds9x + DZOFF + (pc * 32 + li) * DZS + 16 * ks + 8 * lh);
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                short8 B[3];
#pragma unroll
                for (int pc = 0; pc < 3; ++pc) {
                    if (coff[j] >= 0) {
                        const unsigned* src =
                            reinterpret_cast<const unsigned*>(lds9x + coff[j] + pc * PIECE + ks * PRS + 8 * lh);
                        B[pc] = __builtin_bit_cast(short8, u32x4{src[0], src[1], src[2], src[3]});
                    } else {
                        B[pc] = short8{0, 0, 0, 0, 0, 0, 0, 0};
                    }
                }
                floatx16& Cc = acc[j];
                Cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], Cc, 0, 0, 0);
                Cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], Cc, 0, 0, 0);
                Cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], Cc, 0, 0, 0);
                Cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], Cc, 0, 0, 0);
                Cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], Cc, 0, 0, 0);
                Cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], Cc, 0, 0, 0);
            }
        }
    }
    float* slab = a.slab + (size_t)blockIdx.x * NCOLP * 32;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave + 4 * j) * 32 + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) slab[(size_t)n * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] = acc[j][r];
    }
}

static bool wgrad9_applies(const WgradArgs& a) {
    return !a.transposed && a.kh == 9 && a.kw == 9 && a.stride == 1 && a.C1 == w9::CMAX && a.C2 == 32 &&
           a.pad_t == 4 && a.pad_l == 4 && a.Qh == a.XH && a.Qw == a.XW;
}

// ---- expand_last (9x9 s1 SAME Conv2DTranspose, 16 -> 3): LDS-patch weight gradient ---------------------
// The generic kernel's shifted operand here is dZ with 3 channels (no 16-B vectors: 4-byte global loads,
// every element fetched once per tap) and its 256 x 32 tile idles half of N (Cu = 16): 1.1 ms per B=4
// step for 14 GFLOP. As wgrad9 for the start conv: a workgroup walks 8 x 16 pixel tiles, stages the
// 16 x 24 x 3 dZ patch (planar [co][row][col]) and the 128-pixel X tile transposed to [ci][pixel] once, and
//   dW[(tap, co)][ci] += sum_p X[p][ci] dZ[p + tap - pad][co]
// runs on v_mfma_f32_16x16x4_f32 with M = the 16 input channels (A = X^T, one ds_read_b128 per 4 k-steps),
// N = the 243 (tap, co) columns (16 tiles of 16, 4 per wave; column decode once per kernel), K = pixels:
// k-step s of lane group kg is pixel 32 kg + s, so a lane's 4 consecutive k-steps are 4 consecutive pixels
// of one tile row. Each workgroup writes one [256][16] slab; wgrad_reduce_kernel sums them in a fixed order.
namespace wt9 {
constexpr int TH = 8, TW = 16, NPX = TH * TW;         // pixels per tile
// strides from the same bank search as w9 (lane = column (tap, co), lane group = pixel row + 2): row stride
// 24 and plane stride 395 give at most 2 passes per ds_read_b32 (1.5 average) instead of 3 (2.9) with 25 / 400
constexpr int PR = TH + 8, PC = TW + 8, PRS = 24;     // dZ patch rows / cols / row stride (floats)
constexpr int PL = 395;                               // plane stride (floats), >= PR * PRS
constexpr int CS = 3, CU = 16, NCOL = 81 * CS, NTW = 4;   // 243 columns: 16 tiles of 16, 4 per wave
constexpr int RP = 16 * 16, CP = CU;                  // slab rows (padded columns) x slab columns
constexpr int XS = NPX + 4;                           // X^T row stride (floats)
constexpr int ZERO = CS * PL;                         // zero words after the planes (padding columns)
constexpr int XOFF = (CS * PL + 8 + 3) / 4 * 4;       // X^T offset (16-B aligned)
static_assert(PL >= PR * PRS && PRS >= PC, "patch planes");
constexpr int LDS_FL = XOFF + CU * XS;
}  // namespace wt9

__global__ __launch_bounds__(256, 2) void wgradT9_kernel(WgradArgs a) {
    using namespace wt9;
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];
    float* const patch = lds;           // [co][PR][PRS] + zero words
    float* const xt = lds + XOFF;       // [ci][XS]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, kg = lane >> 4;
    const int tiles_x = (a.Qw + TW - 1) / TW, tiles_y = (a.Qh + TH - 1) / TH;
    const int ntiles = a.batch * tiles_x * tiles_y;

    int coff[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave + 4 * j) * 16 + l16;   // wave w owns column tiles w, w+4, w+8, w+12
        if (n < NCOL) {
            const int tap = n / CS, co = n % CS;
            coff[j] = co * PL + (tap / 9) * PRS + tap % 9;
        } else {
            coff[j] = -1;
        }
    }
    f32x4 acc[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (tid < 8) patch[ZERO + tid] = 0.f;

    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int b = t / (tiles_x * tiles_y), rem = t % (tiles_x * tiles_y);
        const int y0 = (rem / tiles_x) * TH, x0 = (rem % tiles_x) * TW;
        __syncthreads();   // previous tile's operands consumed
        for (int i = tid; i < PR * PC * CS; i += 256) {
            const int c = i % CS, px = i / CS;
            const int r = px / PC, q = px % PC;
            const int gy = y0 - a.pad_t + r, gx = x0 - a.pad_l + q;
            float v = 0.f;
            if (gy >= 0 && gy < a.DH && gx >= 0 && gx < a.DW) v = a.D[(((size_t)b * a.DH + gy) * a.DW + gx) * CS + c];
            patch[c * PL + r * PRS + q] = v;
        }
        for (int i = tid; i < NPX * (CU / 4); i += 256) {   // X tile, one float4 (4 channels) per item
            const int cq = i & 3, p = i >> 2;
            const int oy = y0 + p / TW, ox = x0 + p % TW;
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (oy < a.Qh && ox < a.Qw)
                v = *reinterpret_cast<const f32x4*>(a.X + (((size_t)b * a.XH + oy) * a.XW + ox) * CU + 4 * cq);
            xt[(4 * cq + 0) * XS + p] = v.x;
            xt[(4 * cq + 1) * XS + p] = v.y;
            xt[(4 * cq + 2) * XS + p] = v.z;
            xt[(4 * cq + 3) * XS + p] = v.w;
        }
        __syncthreads();
#pragma unroll 2
        for (int g = 0; g < 8; ++g) {
            const int p0 = 32 * kg + 4 * g;
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(xt + l16 * XS + p0);
            const int pixoff = (p0 / TW) * PRS + p0 % TW;
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const float* src = patch + (coff[j] >= 0 ? coff[j] + pixoff : ZERO);
                const int st = coff[j] >= 0 ? 1 : 0;
                const float b0 = src[0], b1 = src[st], b2 = src[2 * st], b3 = src[3 * st];
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b0, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b1, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b2, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b3, acc[j], 0, 0, 0);
            }
        }
    }
    // slab [blockIdx][row n = (tap, co)][ci]: accumulator i of lane (l16, kg) is ci = 4 kg + i, n = tile*16 + l16
    float* slab = a.slab + (size_t)blockIdx.x * RP * CP;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave + 4 * j) * 16 + l16;
        *reinterpret_cast<f32x4*>(slab + (size_t)n * CP + 4 * kg) = acc[j];
    }
}

static bool wgradT9_applies(const WgradArgs& a) {
    return a.transposed && a.kh == 9 && a.kw == 9 && a.stride == 1 && a.C2 == wt9::CS && a.C1 == wt9::CU &&
           a.Qh == a.XH && a.Qw == a.XW && a.DH == a.XH && a.DW == a.XW;
}

// dW[r][c] = sum over splits (fixed order)
// dW = sum over the nsplit slabs, in a fixed order: a workgroup owns 64 float4 columns of dW; its four
// waves sum contiguous quarters of the slab range (8 loads in flight per lane), then wave 0 adds the
// quarters in order. (Cu % 4 == 0 and Cp % 4 == 0 on every path that reaches here.)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(WgradArgs a, int Rp, int Cp) {
    const WgradGeom g = wgrad_geom(a);
    const int cu4 = g.Cu / 4, lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const long total4 = (long)g.R * cu4;
    const long i = (long)blockIdx.x * 64 + lane;
    __shared__ float4 part[3][64];
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < total4) {
        const long r = i / cu4, c4 = i - r * cu4;
        const float4* base = reinterpret_cast<const float4*>(a.slab) + (size_t)r * (Cp / 4) + c4;
        const size_t ks = (size_t)Rp * Cp / 4;
        const int k0 = (a.nsplit * q) / 4, k1 = (a.nsplit * (q + 1)) / 4;
#pragma unroll 8
        for (int k = k0; k < k1; ++k) {
            const float4 v = base[(size_t)k * ks];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
    }
    if (q > 0) part[q - 1][lane] = s;
    __syncthreads();
    if (q == 0 && i < total4) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float4 v = part[j][lane];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        float* o = a.dW + 4 * i;   // dW may sit at any float offset of the gradient bucket
        o[0] = s.x;
        o[1] = s.y;
        o[2] = s.z;
        o[3] = s.w;
    }
}

// ---- host side -------------------------------------------------------------------------------
namespace {
struct WTile {
    int tr, tc;
};

WTile wgrad_tile(const WgradArgs& a) {
    const int Cu = a.transposed ? a.C1 : a.C2;
    return Cu > 32 ? WTile{128, 128} : WTile{256, 32};
}

void wgrad_dims(const WgradArgs& a, int& R, int& Cu, int& Cs) {
    Cs = a.transposed ? a.C2 : a.C1;
    Cu = a.transposed ? a.C1 : a.C2;
    R = a.kh * a.kw * Cs;
}
}  // namespace

constexpr int W9_BLOCKS = 512;   // two workgroups per CU, each a persistent walk over the pixel tiles

// the split-bf16 start-conv kernel for the x6 trainer (RST_WGRAD9_X6=0: the f32 kernel). Config-4 step 24.97 -> 24.29 ms
// same box (profiles/r04/trainab_wgrad9_x6_prefetch.log); the first form, before the odd channel pitch and the
// register prefetch, ran 29.6 ms (trainab_wgrad9_x6.log)
static bool wgrad9_x6_enabled() {
    static const bool ok = [] {
        const char* v = getenv("RST_WGRAD9_X6");
        if (v != nullptr && v[0] == '0') return false;
        return hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad9_x6_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)w9x::LDS_BYTES) == hipSuccess;
    }();
    return ok;
}

static int wgrad_cu_count() {
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    return n_cu;
}

// the tap-row kernel (wgrad_x6r_kernel): the residual convs of the split-bf16 trainer (3x3 s1 SAME, 128 -> 128);
// RST_WGRAD_X6R=0: wgrad_x6_kernel
static bool wgrad_x6r_applies(const WgradArgs& a) {
    static const bool ok = [] {
        const char* v = getenv("RST_WGRAD_X6R");
        if (v != nullptr && v[0] == '0') return false;
        return hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad_x6r_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)wx6r::LDS_BYTES) == hipSuccess;
    }();
    return ok && a.x6 && !a.transposed && a.kh == 3 && a.kw == 3 && a.stride == 1 && a.pad_t == 1 && a.pad_l == 1 &&
           a.C1 == wx6r::CI && a.C2 == wx6r::CO && a.XH == a.Qh && a.XW == a.Qw;
}

int wgrad_choose_splits(const WgradArgs& a) {
    if (wgrad_x6r_applies(a)) {
        // one workgroup per CU: 3 kernel rows x splits, each split >= 8 stages
        const long total = (long)a.batch * a.Qh * a.Qw;
        long ns = wgrad_cu_count() / wx6r::TAPS;
        const long max_ns = (total + 8 * wx6r::KP - 1) / (8 * wx6r::KP);
        if (ns > max_ns) ns = max_ns;
        return (int)(ns < 1 ? 1 : ns);
    }
    if (wgrad9_applies(a) && a.x6 && wgrad9_x6_enabled()) {
        // one workgroup per CU (104 KB of LDS, launch_bounds(256, 1)): one round of persistent workgroups, never more
        // than the pixel tiles (each writes a slab the reduce then reads)
        const int ntiles = a.batch * ((a.Qh + w9x::TH - 1) / w9x::TH) * ((a.Qw + w9x::TW - 1) / w9x::TW);
        // minus 3/8 of the CUs (RST_WGRAD9_FREE_CUS=k: k): the kernel runs beside the style predictor's backward, whose
        // small launches found no CU while it held all of them (config-4 step, free 0 / 32 / 64 / 96 / 128 / 160 of
        // 256: 20.9 / 20.8 / 20.7 / 20.3 / 20.3 / 21.2 ms, profiles/r06/r06k, r06n, r06q)
        static const int free_cus = [] {
            const char* v = getenv("RST_WGRAD9_FREE_CUS");
            return v != nullptr ? atoi(v) : wgrad_cu_count() * 3 / 8;
        }();
        int n = wgrad_cu_count() - free_cus;
        if (n < 8) n = 8;
        return ntiles < n ? (ntiles < 1 ? 1 : ntiles) : n;
    }
    if (wgrad9_applies(a) || wgradT9_applies(a)) return W9_BLOCKS;
    int R, Cu, Cs;
    wgrad_dims(a, R, Cu, Cs);
    const WTile t = wgrad_tile(a);
    const long tiles = (long)((R + t.tr - 1) / t.tr) * ((Cu + t.tc - 1) / t.tc);
    const long total = (long)a.batch * a.Qh * a.Qw;
    long ns = 1024 / tiles;                      // ~4 workgroups per CU
    const long max_ns = (total + 8 * wg::KP - 1) / (8 * wg::KP);   // >= 8 stages per split
    if (ns > max_ns) ns = max_ns;
    return (int)(ns < 1 ? 1 : ns);
}

size_t wgrad_slab_bytes(const WgradArgs& a) {
    if (wgrad_x6r_applies(a)) return (size_t)a.nsplit * 9 * wx6r::CI * wx6r::CO * sizeof(float);
    if (wgrad9_applies(a)) return (size_t)a.nsplit * w9::NCOLP * 32 * sizeof(float);
    if (wgradT9_applies(a)) return (size_t)a.nsplit * wt9::RP * wt9::CP * sizeof(float);
    int R, Cu, Cs;
    wgrad_dims(a, R, Cu, Cs);
    const WTile t = wgrad_tile(a);
    const size_t Rp = (size_t)((R + t.tr - 1) / t.tr) * t.tr, Cp = (size_t)((Cu + t.tc - 1) / t.tc) * t.tc;
    return (size_t)a.nsplit * Rp * Cp * sizeof(float);
}

hipError_t wgrad_launch(WgradArgs a, hipStream_t st) {
    int R, Cu, Cs;
    wgrad_dims(a, R, Cu, Cs);
    if (wgrad9_applies(a)) {
        if (a.nsplit < 1) return hipErrorInvalidValue;
        if (a.x6 && wgrad9_x6_enabled())
            hipLaunchKernelGGL(wgrad9_x6_kernel, dim3((unsigned)a.nsplit), dim3(256), w9x::LDS_BYTES, st, a);
        else
            hipLaunchKernelGGL(wgrad9_kernel, dim3((unsigned)a.nsplit), dim3(256), 0, st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const size_t n4 = (size_t)R * Cu / 4;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, a, w9::NCOLP, 32);
        return hipGetLastError();
    }
    if (wgradT9_applies(a)) {
        if (a.nsplit < 1) return hipErrorInvalidValue;
        hipLaunchKernelGGL(wgradT9_kernel, dim3((unsigned)a.nsplit), dim3(256), 0, st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const size_t n4 = (size_t)R * Cu / 4;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, a, wt9::RP, wt9::CP);
        return hipGetLastError();
    }
    if (wgrad_x6r_applies(a)) {
        if (a.nsplit < 1) return hipErrorInvalidValue;
        const long total = (long)a.batch * a.Qh * a.Qw;
        long span = (total + a.nsplit - 1) / a.nsplit;
        a.span = ((span + wx6r::KP - 1) / wx6r::KP) * wx6r::KP;
        hipLaunchKernelGGL(wgrad_x6r_kernel, dim3((unsigned)(wx6r::TAPS * a.nsplit)), dim3(512), wx6r::LDS_BYTES, st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const size_t n4 = (size_t)R * Cu / 4;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, a, 9 * wx6r::CI,
                           wx6r::CO);
        return hipGetLastError();
    }
    if (Cu % 4 != 0) return hipErrorInvalidValue;
    const WTile t = wgrad_tile(a);
    const long total = (long)a.batch * a.Qh * a.Qw;
    long span = (total + a.nsplit - 1) / a.nsplit;
    span = ((span + wg::KP - 1) / wg::KP) * wg::KP;
    a.span = span;
    const int nr = (R + t.tr - 1) / t.tr, nc = (Cu + t.tc - 1) / t.tc;
    const dim3 grid((unsigned)(nr * nc * a.nsplit));
    const bool vs = Cs % 4 == 0;
    if (a.x6 && !a.transposed && vs && t.tr == 128 && t.tc == 128 && wx6::KP == wg::KP) {
        hipLaunchKernelGGL(wgrad_x6_kernel, grid, dim3(256), 0, st, a);
    } else if (t.tr == 128) {
        if (vs) hipLaunchKernelGGL((wgrad_mfma_kernel<128, 128, 2, 2, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((wgrad_mfma_kernel<128, 128, 2, 2, false>), grid, dim3(256), 0, st, a);
    } else {
        if (vs) hipLaunchKernelGGL((wgrad_mfma_kernel<256, 32, 4, 1, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((wgrad_mfma_kernel<256, 32, 4, 1, false>), grid, dim3(256), 0, st, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t n4 = (size_t)R * Cu / 4;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, a, nr * t.tr, nc * t.tc);
    return hipGetLastError();
}

}  // namespace rst
