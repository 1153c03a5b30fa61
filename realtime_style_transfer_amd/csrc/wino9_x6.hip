// wino9_x6.hip — the network's first layer ("contract_start": Conv2D 9x9 s1 SAME, 17 -> 32 channels,
// built-in ReLU, then BatchNormalization and ReLU; realtime_style_transfer/models/styleTransfer.py:
// 188-205, 225-226) as the composite Winograd F(2x2, 3x3) of wino9.hip (nine 3x3 sub-kernels g_ab
// sharing one accumulator per transform point) with the transform-domain products on the bf16 MFMA
// pipe at fp32-level accuracy: every operand of the 16 batched GEMMs (V_ab = B^T d_ab B and
// U_ab = G g_ab G^T) split exactly into three bf16 pieces, six product terms, fp32 accumulation
// (dropped terms <= 2^-25 of each product; the scheme of wino_x6.hip).
//
// Workgroup = 8 waves (two per SIMD), output block 16 x 16 pixels = 8 x 8 = 64 Winograd tiles (two
// 32-row MFMA M blocks) x 32 output channels. Wave w owns transform-point row p = w & 3 and the two
// points q = 2(w >> 2), +1 of it (ξ = 4p + q), for both M blocks: four accumulators (64 registers).
// The V operands never touch LDS: lane (li, lh) of a wave computes exactly the A-operand values it feeds
// its MFMAs — row p of B^T d for tile 32h + li and channels 8lh..8lh+7 (two 32-B patch reads per point
// of the 4x4 input tile, ds_read_b128), the two points' V, the exact 3-piece split, packed straight into
// the short8 operands. K per sub-kernel: channels 0..15 = one K-step of the 32x32x16 MFMA (6 terms);
// channel 16 of all nine sub-kernels is gathered into one more K-step at the end (K index = ab), its V
// kept in registers by the lanes that feed it. The loop over the nine sub-kernels has no barrier.
// Each U element (B operand, L2) is loaded by one wave and serves 64 tiles.
// Epilogue, per M block: M -> LDS [xi][tile][co], output transform per (tile, channel), bias -> ReLU ->
// BN (folded moving statistics) -> ReLU. Training (Wino9Args.part set): the raw ReLU output and a two-pass
// {sum, M2, n} per (channel, 16 x 8 M block) for the batch-statistics BatchNorm (finalize_kernel).
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

constexpr int TH = 16, TW = 16;                // output pixels per workgroup
constexpr int PH = TH + 8, PW = TW + 8;        // input patch (pad 4 each side): 24 x 24
constexpr int NPX = PH * PW;                   // 576 patch pixels
constexpr int PS = 20;                         // patch pixel stride (floats): 17 channels + 3 (80 B, 16-B aligned)
// A patch row holds the even pixels, then the odd ones (tiles step 2 pixels in x, so a wave's tiles read
// consecutive pixels of one parity plane), padded to 496 floats: with that pitch the 16 lanes of every
// ds_read_b128 lane group hit 16 distinct 4-bank groups (searched exhaustively; stride 2 x 80 B could use
// only 8 of them)
constexpr int PLANE = (PW / 2) * PS;           // 240 floats: one parity plane of a row
constexpr int RP = 2 * PLANE + 16;             // 496 floats: row pitch
constexpr int NT = 32;                         // output channels
constexpr int NXI = 16;                        // transform points
constexpr int VROW = 32;                       // bytes per (co, 16 channels) U row: 16 bf16
constexpr int PATCH_FL = PH * RP;              // 11904 floats
constexpr int MS = 33;                         // M exchange row stride (floats)
constexpr int MEX_FL = NXI * 32 * MS;          // one M block: [16][32 tiles][33]
constexpr int V16S = 12;                       // channel-16 V row: ab 0..8 + 3 pad (48 B)
constexpr int V16_FL = NXI * 64 * V16S;        // [xi][tile][12] f32
// LDS: [patch 0][v16][patch 1]. A tile computes from patch (t & 1) while the next tile's patch is staged
// into the other one; the epilogue's M exchange uses the current patch + v16 (contiguous either way).
constexpr int LDS_FL = 2 * PATCH_FL + V16_FL;
constexpr int LDS_BYTES = LDS_FL * 4;          // 140 KB
static_assert(MEX_FL + 3 * 256 <= PATCH_FL + V16_FL, "M exchange + statistics scratch fit in one patch + v16");
constexpr int UBLK = NT * VROW;                // bytes per (ab, xi, piece) U block: 32 co x 16 bf16
constexpr int NTHR = 512;

__host__ __device__ constexpr int pix_off(int r, int x) { return r * RP + (x & 1) * PLANE + (x >> 1) * PS; }

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

// (x, y) -> the bf16 pair nearest them; (x, y) -= its value (exact in fp32)
__device__ __forceinline__ unsigned piece(float& x, float& y) { return bf16_piece(x, y); }

// eight fp32 values -> the three short8 bf16 pieces (v = p0 + p1 + p2 exactly)
__device__ __forceinline__ void split8(const float (&v)[8], short8 (&A)[3]) {
    unsigned pk[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float x = v[2 * j], y = v[2 * j + 1];
        pk[0][j] = piece(x, y);
        pk[1][j] = piece(x, y);
        pk[2][j] = piece(x, y);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) A[p] = __builtin_bit_cast(short8, (u32x4){pk[p][0], pk[p][1], pk[p][2], pk[p][3]});
}

}  // namespace

// (The knock-out measurements of DESIGN.md §3 were built from this file as of commit 94f9b44; the product kernel
// carries no such switches.)
// (Measured and removed, round 4: a software-pipelined unit loop with the next unit's operand preparation beside
// the MFMAs, and an s_sleep stagger of the qh = 1 waves at each tile start — both slower,
// profiles/r04/w9_stagger_pipe_slp.log.)
#ifdef W9_PROF
// timeline per (workgroup, wave) on the constant 100 MHz clock: start, staged, loop done, end
__device__ unsigned long long w9_tl[W9_PROF][8][9][4];   // [workgroup][wave][tile iteration][stamp]
#define W9TL(k) \
    if (blockIdx.x < W9_PROF && lane == 0 && w9_it < 9) w9_tl[blockIdx.x][wave][w9_it][(k)] = __builtin_amdgcn_s_memrealtime()
#else
#define W9TL(k)
#endif

template <int CINT, bool TRAIN>
// Work units: units 0 .. n_full-1 are whole tiles; the n_tiles - n_full tiles of the last, partial round
// are split into two units each (one 32-tile M block, i.e. 8 output rows), so that round occupies twice
// as many CUs for about half as long (1800 tiles on 256 CUs: 7 full rounds + 8 tiles -> 16 half units).
__global__ __launch_bounds__(NTHR, 1) void wino9_x6_kernel(Wino9Args a, int n_units, int n_full) {
    extern __shared__ __attribute__((aligned(16))) float smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar U offsets, no waterfall)
    if (a.zero != nullptr)   // the frame's CIN accumulators (no separate memset launch; no layer before this one)
        for (long i = (long)blockIdx.x * NTHR + tid; i < a.zero_n2; i += (long)gridDim.x * NTHR)
            reinterpret_cast<uint4*>(a.zero)[i] = make_uint4(0u, 0u, 0u, 0u);
    const int li = lane & 31, lh = lane >> 5;
    const int p = wave & 3, qh = wave >> 2;   // point row p, points q = 2qh, 2qh + 1
    int w9_it = 0;
    (void)w9_it;
    const int H = a.H, W = a.W, Cin = CINT > 0 ? CINT : a.cin;
    const int ROW = PW * Cin;   // <= 408 <= NTHR (cin <= 17, wino9_supported)
    static_assert(CINT == 17 || CINT == 0, "");

    // ---- U pieces: lane (li, lh) reads U[ab][4p + q][piece][co = li][8lh .. 8lh+7] ------------------
    const __amdgpu_buffer_rsrc_t usrd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, (9 + 1) * NXI * 3 * UBLK, 0x00020000);
    const int uvoff = li * VROW + 16 * lh;
    short8 ub[2][2][3];   // [buffer][q of the pair][piece]
    auto load_u = [&](auto BUF, int ab) __attribute__((always_inline)) {   // ab == 9: the channel-16 K-step
        constexpr int buf = decltype(BUF)::value;
        sfor<0, 2>([&](auto Q) __attribute__((always_inline)) {
            constexpr int q = decltype(Q)::value;
            sfor<0, 3>([&](auto Pc) __attribute__((always_inline)) {
                constexpr int pc = decltype(Pc)::value;
                ub[buf][q][pc] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(
                    usrd, uvoff, ((ab * NXI + 4 * p + 2 * qh + q) * 3 + pc) * UBLK, 0));
            });
        });

    };
    load_u(std::integral_constant<int, 0>{}, 0);

    // ---- persistent tile loop: workgroup g takes tiles g, g + G, ... The next tile's patch is staged into
    // the other patch buffer in two halves during the current tile's sub-kernel loop (loads issued a few
    // sub-kernels before their LDS stores, so their latency hides behind the MFMAs). ----
    auto unit_tile = [&](int u) __attribute__((always_inline)) { return u < n_full ? u : n_full + ((u - n_full) >> 1); };
    auto unit_mask = [&](int u) __attribute__((always_inline)) { return u < n_full ? 3 : 1 << ((u - n_full) & 1); };
    auto tile_coords = [&](int u, int& y0, int& x0, size_t& img) __attribute__((always_inline)) {
        int t = unit_tile(u);
        const int tx = t % a.tiles_x;
        t /= a.tiles_x;
        const int ty = t % a.tiles_y;
        img = (size_t)(t / a.tiles_y) * H * W;
        y0 = ty * TH;
        x0 = tx * TW;
    };
    // Staging: a patch row (24 pixels x Cin channels = PW*Cin <= 408 floats) is contiguous in NHWC, so thread
    // j < PW*Cin owns element j of every row (pixel j / Cin, channel j % Cin) and walks the 24 rows: its LDS
    // destination and column part of the source offset are per-thread constants, the row part is scalar
    // (one multiply-add per element instead of the two divisions and 64-bit address math of a flat index)
    constexpr int NPART = 3, NH = PH / NPART;   // staged in three parts of 8 rows
    const int sj = tid < ROW ? tid : 0, spx = sj / Cin, sc = sj - spx * Cin;
    const int sloff = pix_off(0, spx) + sc;   // LDS offset of the thread's element in row 0
    const bool sact = tid < ROW;
    const __amdgpu_buffer_rsrc_t insrd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.in), 0, (int)((size_t)a.batch * H * W * Cin * 4), 0x00020000);
    float pf[NH];
    auto load_half = [&](int t, auto HALF) __attribute__((always_inline)) {   // clamped addresses
        constexpr int hf = decltype(HALF)::value;
        int y0, x0;
        size_t img;
        tile_coords(t, y0, x0, img);
        const int gx = min(max(x0 - 4 + spx, 0), W - 1);
        const int voff = sact ? (gx * Cin + sc) * 4 : 0x7FFFFFF0;   // idle threads read out of range (-> 0)
        sfor<0, NH>([&](auto K) __attribute__((always_inline)) {
            constexpr int r = hf * NH + decltype(K)::value;
            const int gy = min(max(y0 - 4 + r, 0), H - 1);
            const int soff = __builtin_amdgcn_readfirstlane((int)((img + (size_t)gy * W) * Cin * 4));
            pf[decltype(K)::value] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(insrd, voff, soff, 0));
        });
    };
    auto store_half = [&](int t, float* pbuf, auto HALF) __attribute__((always_inline)) {   // zero outside
        constexpr int hf = decltype(HALF)::value;
        int y0, x0;
        size_t img;
        tile_coords(t, y0, x0, img);
        const int gx = x0 - 4 + spx;
        const bool inx = gx >= 0 && gx < W;
        if (sact) {
            sfor<0, NH>([&](auto K) __attribute__((always_inline)) {
                constexpr int r = hf * NH + decltype(K)::value;
                const int gy = y0 - 4 + r;
                const bool inside = inx && gy >= 0 && gy < H;
                pbuf[r * RP + sloff] = inside ? pf[decltype(K)::value] : 0.f;
            });
        }
        if constexpr (hf == NPART - 1)   // channels cin..19 (the previous M exchange overwrote them)
            for (int i = tid; i < NPX * (PS - Cin); i += NTHR) {
                const int px = i / (PS - Cin);
                pbuf[pix_off(px / PW, px % PW) + Cin + i % (PS - Cin)] = 0.f;
            }
    };
    auto patch_buf = [&](int parity) __attribute__((always_inline)) { return smem + parity * (PATCH_FL + V16_FL); };
    float* const v16s = smem + PATCH_FL;   // [16][64][12]: channel-16 V of every sub-kernel (K index ab)

    // B^T d row p = Y + s X from the d rows (rY, rX), s = +-1 (one exact fma per element):
    // p0: d0 - d2, p1: d1 + d2, p2: d2 - d1, p3: d1 - d3
    const int rX = p == 0 ? 2 : (p == 1 ? 2 : (p == 2 ? 1 : 3));
    const int rY = p == 0 ? 0 : (p == 2 ? 2 : 1);
    const float sx = p == 1 ? 1.f : -1.f;
    auto mfma6 = [&](floatx16& C, const short8 (&A)[3], const short8 (&B)[3]) __attribute__((always_inline)) {
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], C, 0, 0, 0);   // a0 b0
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], C, 0, 0, 0);   // a0 b1
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], C, 0, 0, 0);   // a1 b0
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], C, 0, 0, 0);   // a0 b2
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], C, 0, 0, 0);   // a1 b1
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], C, 0, 0, 0);   // a2 b0

    };
    const int co = tid & 31, g = tid >> 5;   // epilogue thread: output channel co, tiles 2g, 2g + 1 of a block
    const float bias = a.bias[co];
    constexpr bool train = TRAIN;            // training: raw ReLU output + per-(tile, M block) statistics
    const float2 bn = train ? make_float2(1.f, 0.f) : a.bn_ab[co];
    const int n_tile_img = a.tiles_y * a.tiles_x, n_part = 2 * n_tile_img;

    unsigned l2f = 0;     // the next layer's weights into this XCD's L2, touched during the last unit (speed only)
    // work units: the first two of each workgroup static (blockIdx.x, + gridDim.x), the rest from a queue (a.queue):
    // the partial last round's half units go to the workgroups that finish their whole units first, not to the
    // first 16 by index (their spread of finishing times is several microseconds). Thread 0 fetches the unit after
    // next at the top of each unit and publishes it at the end (the atomic's latency hides behind the unit).
    __shared__ int w9_next;
    const bool dyn = a.queue != nullptr;
    unsigned qv = 0u;
    int t = blockIdx.x;   // work unit
    int tn = t + (int)gridDim.x;   // the next one (its patch is staged during this one)
    if (t < n_units) {
        sfor<0, NPART>([&](auto PART) __attribute__((always_inline)) {
            load_half(t, PART);
            store_half(t, patch_buf(0), PART);
        });
    }
    for (int it = 0; t < n_units; ++it) {
        w9_it = it;
        W9TL(0);
        if (dyn && tid == 0) qv = 2u * gridDim.x + atomicAdd(a.queue, 1u);
        if (tn >= n_units) l2f = l2_touch_xcd_slice<NTHR, 1>(a.w_next, a.w_next_bytes).x;   // late: stays in L2
        const int hmask = __builtin_amdgcn_readfirstlane(unit_mask(t));   // M blocks of this unit
        int y0, x0;
        size_t img;
        tile_coords(t, y0, x0, img);
        float* const patch = patch_buf(it & 1);
        float* const pnext = patch_buf((it & 1) ^ 1);
        // patch element at the top-left of the epilogue's M exchange: the current patch + v16
        float* const ms = (it & 1) ? smem + PATCH_FL : smem;   // [16][32][33], one M block at a time
        // per-lane row pointers (tile li of block 0, rows rX / rY of the 4x4 input tile, channels 8lh..);
        // every read below adds a compile-time offset (sub-kernel shift, block, column) to one of them
        const float* const bx = patch + pix_off(2 * (li >> 3) + rX, 2 * (li & 7)) + 8 * lh;
        const float* const by = patch + pix_off(2 * (li >> 3) + rY, 2 * (li & 7)) + 8 * lh;
        const float* const bx16 = patch + pix_off(2 * (li >> 3) + rX, 2 * (li & 7)) + 16;
        const float* const by16 = patch + pix_off(2 * (li >> 3) + rY, 2 * (li & 7)) + 16;
        for (int i = tid; i < NXI * 64 * (V16S - 9); i += NTHR)   // channel-16 rows: ab 9..11 are zero
            v16s[(i / (V16S - 9)) * V16S + 9 + i % (V16S - 9)] = 0.f;
        floatx16 acc[2][2];   // [q of the pair][M block]
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[q][h][r] = 0.f;
        lds_barrier();   // patch + pads visible
        W9TL(1);
        // The q pair is a compile-time parameter (one code path per wave-uniform value): pair 0 uses the
        // columns 0..2 of B^T d (V0 = T0 - T2, V1 = T1 + T2), pair 1 the columns 1..3 (V2 = T2 - T1,
        // V3 = T1 - T3).
        // MASK (compile time: a runtime branch per block stops the scheduler from overlapping one block's
        // MFMAs with the next block's transform): the M blocks this unit computes
        auto main_loop = [&](auto QH, auto MK) __attribute__((always_inline)) {
            constexpr int QHC = decltype(QH)::value, MASK = decltype(MK)::value;
            // sub-kernel loop fully unrolled (the U double buffer is indexed at compile time); no barriers
            sfor<0, 9>([&](auto AB) __attribute__((always_inline)) {
                constexpr int ab = decltype(AB)::value, cur = ab & 1, sa = ab / 3, sb = ab % 3;
                load_u(std::integral_constant<int, cur ^ 1>{}, ab + 1);   // ab + 1 == 9: the channel-16 step's U
                // the next tile's patch in three parts: loads at sub-kernels 1, 3, 5, LDS stores two later (3, 5, 7;
                // each store before the next part's loads reuse its registers)
                if constexpr (ab == 3 || ab == 5 || ab == 7) {
                    if (tn < n_units) store_half(tn, pnext, std::integral_constant<int, (ab - 3) / 2>{});
                }
                if constexpr (ab == 1 || ab == 3 || ab == 5) {
                    if (tn < n_units) load_half(tn, std::integral_constant<int, (ab - 1) / 2>{});
                }
                sfor<0, 2>([&](auto Hh) __attribute__((always_inline)) {
                    constexpr int h = decltype(Hh)::value;
                    if constexpr (!(MASK & (1 << h))) return;   // half unit: the other M block only
                    const int tile = 32 * h + li;
                    float tv[3][8], t16[3];
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) {
                        // pixel (8h + 3sa, 3sb + QHC + cc) relative to the lane's tile origin (even x)
                        const int off = (8 * h + 3 * sa) * RP + ((3 * sb + QHC + cc) & 1) * PLANE +
                                        ((3 * sb + QHC + cc) >> 1) * PS;
                        const f32x4 x0v = *reinterpret_cast<const f32x4*>(bx + off);
                        const f32x4 x1v = *reinterpret_cast<const f32x4*>(bx + off + 4);
                        const f32x4 y0v = *reinterpret_cast<const f32x4*>(by + off);
                        const f32x4 y1v = *reinterpret_cast<const f32x4*>(by + off + 4);
                        const float xv[8] = {x0v.x, x0v.y, x0v.z, x0v.w, x1v.x, x1v.y, x1v.z, x1v.w};
                        const float yv[8] = {y0v.x, y0v.y, y0v.z, y0v.w, y1v.x, y1v.y, y1v.z, y1v.w};
#pragma unroll
                        for (int k = 0; k < 8; ++k) tv[cc][k] = fmaf(sx, xv[k], yv[k]);
                        t16[cc] = fmaf(sx, bx16[off], by16[off]);   // channel 16 (the K-step gathered over ab)
                    }

                    float v0[8], v1[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        v0[k] = QHC == 0 ? tv[0][k] - tv[2][k] : tv[1][k] - tv[0][k];
                        v1[k] = QHC == 0 ? tv[1][k] + tv[2][k] : tv[0][k] - tv[2][k];
                    }
                    // channel 16 -> LDS (lane half lh stores the point q = lh of the pair)
                    {
                        const float w0 = QHC == 0 ? t16[0] - t16[2] : t16[1] - t16[0];
                        const float w1 = QHC == 0 ? t16[1] + t16[2] : t16[0] - t16[2];
                        v16s[((4 * p + 2 * QHC + lh) * 64 + tile) * V16S + ab] = lh ? w1 : w0;
                    }
                    short8 A0[3], A1[3];
                    split8(v0, A0);
                    split8(v1, A1);

                    mfma6(acc[0][h], A0, ub[cur][0]);
                    mfma6(acc[1][h], A1, ub[cur][1]);
                });
            });
        };
        auto main_loop_q = [&](auto MK) __attribute__((always_inline)) {
            if (__builtin_amdgcn_readfirstlane(qh) == 0) main_loop(std::integral_constant<int, 0>{}, MK);
            else main_loop(std::integral_constant<int, 1>{}, MK);
        };
        if (hmask == 3) main_loop_q(std::integral_constant<int, 3>{});
        else if (hmask == 1) main_loop_q(std::integral_constant<int, 1>{});
        else main_loop_q(std::integral_constant<int, 2>{});
        // channel-16 K-step: lane (li, lh) supplies K = 8lh .. 8lh+7 (ab; 9..15 are zero)
        lds_barrier();   // every wave's channel-16 V in LDS
        sfor<0, 2>([&](auto Hh) __attribute__((always_inline)) {
            constexpr int h = decltype(Hh)::value;
            if (!(hmask & (1 << h))) return;
            float w[2][8];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float* r = v16s + ((4 * p + 2 * qh + q) * 64 + 32 * h + li) * V16S + 8 * lh;
                const f32x4 r0 = *reinterpret_cast<const f32x4*>(r);
                const f32x4 r1 = lh ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(r + 4);
                w[q][0] = r0.x; w[q][1] = r0.y; w[q][2] = r0.z; w[q][3] = r0.w;
                w[q][4] = r1.x; w[q][5] = r1.y; w[q][6] = r1.z; w[q][7] = r1.w;
            }
            short8 A0[3], A1[3];
            split8(w[0], A0);
            split8(w[1], A1);
            mfma6(acc[0][h], A0, ub[1][0]);   // 9 sub-kernels: the last load_u (ab + 1 == 9) went to buffer 1
            mfma6(acc[1][h], A1, ub[1][1]);
        });
        if (tn < n_units) load_u(std::integral_constant<int, 0>{}, 0);   // the next tile's first U
        W9TL(2);

        // ---- epilogue, one M block at a time: M -> LDS [xi][tile][co], output transform, store -------
        const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
        sfor<0, 2>([&](auto Hh) __attribute__((always_inline)) {
            constexpr int h = decltype(Hh)::value;
            if (!(hmask & (1 << h))) return;   // uniform over the workgroup (barriers inside)
            lds_barrier();   // patch / v16 reads (h = 0) / the previous block's M reads (h = 1) done
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int row = (j & 3) + 8 * (j >> 2) + 4 * lh;   // accumulator j of lane (li, lh): tile row, co li
                    ms[((4 * p + 2 * qh + q) * 32 + row) * MS + li] = acc[q][h][j];
                }
            lds_barrier();
            float vals[8];
            float vs = 0.f, vn = 0.f;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int tl = 2 * g + k, tile = 32 * h + tl;
                const int wy = tile >> 3, wx = tile & 7;
                float m[16];
#pragma unroll
                for (int x = 0; x < NXI; ++x) m[x] = ms[(x * 32 + tl) * MS + co];
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
                    const bool inside = oy < H && ox < W;
                    const float v = fmaxf(yy[q] + bias, 0.f);                     // Conv2D(..., activation='relu')
                    vals[4 * k + q] = inside ? v : 0.f;
                    vs += vals[4 * k + q];
                    vn += inside ? 1.f : 0.f;
                    if (inside) {   // inference: BN (folded moving statistics) -> ReLU; training: the raw ReLU output
                        const float o = train ? v : fmaxf(fmaf(bn.x, v, bn.y), 0.f);
                        const size_t oi = (img + (size_t)oy * W + ox) * NT + co;
                        if (a.wt_stores)   // write-through (sc1): no dirty lines left for the end-of-kernel write-back
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), osrd, (int)(oi * 4), 0, 16);
                        else
                            a.out[oi] = o;
                    }
                }
            }
            if constexpr (train) {
                // two-pass {sum, M2, n} of channel co over this M block (32 tiles = 8 output rows x 16 columns):
                // lanes co / co + 32 of a wave hold groups 2w, 2w + 1; the eight waves meet in LDS just past
                // the M exchange image (disjoint from it, inside the same dead patch + v16 span)
                float* const red = ms + MEX_FL;   // [3][8 waves][32]
                vs = lane_xor_sum<32>(vs);
                vn = lane_xor_sum<32>(vn);
                if (lh == 0) {
                    red[wave * 32 + co] = vs;
                    red[256 + wave * 32 + co] = vn;
                }
                lds_barrier();
                float S = 0.f, N = 0.f;
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    S += red[w * 32 + co];
                    N += red[256 + w * 32 + co];
                }
                const float mean = N > 0.f ? S / N : 0.f;
                float m2 = 0.f;
#pragma unroll
                for (int k = 0; k < 2; ++k)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int tl = 2 * g + k, tile = 32 * h + tl;
                        const int oy = y0 + 2 * (tile >> 3) + (q >> 1), ox = x0 + 2 * (tile & 7) + (q & 1);
                        const float d = vals[4 * k + q] - mean;
                        if (oy < H && ox < W) m2 = fmaf(d, d, m2);
                    }
                m2 = lane_xor_sum<32>(m2);
                if (lh == 0) red[512 + wave * 32 + co] = m2;
                lds_barrier();
                if (tid < 32) {
                    float M2 = 0.f;
#pragma unroll
                    for (int w = 0; w < 8; ++w) M2 += red[512 + w * 32 + co];
                    const int tt = unit_tile(t), bi = tt / n_tile_img, tli = tt - bi * n_tile_img;
                    a.part[((size_t)bi * NT + co) * n_part + 2 * tli + h] = make_float4(S, M2, N, 0.f);
                }
            }
        });
        if (dyn && tid == 0) w9_next = (int)min(qv, 0x7FFFFFFFu);
        lds_barrier();   // M reads done before the next tile's v16 pads / computations; w9_next published
        W9TL(3);
        t = tn;
        tn = dyn ? __builtin_amdgcn_readfirstlane(w9_next) : tn + (int)gridDim.x;   // uniform: an SGPR
    }
    if (dyn && tid == 0) {   // the last workgroup out (all fetches done) resets the queue for the next launch
        if (atomicAdd(a.queue + 1, 1u) == gridDim.x - 1) {
            atomicExch(a.queue, 0u);
            atomicExch(a.queue + 1, 0u);
        }
    }
    l2_touch_keep(l2_touch_t{l2f, 0u}, a.batch < 0, smem);
}

#ifdef W9_PROF
void w9_timeline_print(int nwg) {
    std::vector<unsigned long long> tl((size_t)W9_PROF * 8 * 9 * 4, 0);
    if (hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(w9_tl), tl.size() * 8) != hipSuccess) return;
    if (nwg > W9_PROF) nwg = W9_PROF;
    double ph[4] = {0, 0, 0, 0};
    int n = 0;
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 8; ++w)
            for (int it = 0; it + 1 < 7; ++it) {
                const unsigned long long* q = &tl[(((size_t)g * 8 + w) * 9 + it) * 4];
                const unsigned long long nx = q[4];   // next iteration's stamp 0
                ph[0] += (double)(q[1] - q[0]);
                ph[1] += (double)(q[2] - q[1]);
                ph[2] += (double)(q[3] - q[2]);
                ph[3] += (double)(nx - q[3]);
                ++n;
            }
    printf("  per tile (us, iterations 0..5): top %.2f, loop %.2f, epilogue %.2f, gap %.2f\n", ph[0] / n * 0.01,
           ph[1] / n * 0.01, ph[2] / n * 0.01, ph[3] / n * 0.01);
    // per workgroup (wave 0): first stamp, end of its last unit; the span of the whole grid
    unsigned long long t0 = ~0ull, tmax = 0;
    for (int g = 0; g < nwg; ++g) {
        const unsigned long long* q = &tl[((size_t)g * 8) * 9 * 4];
        if (q[0] && q[0] < t0) t0 = q[0];
    }
    int gmax = -1;
    for (int g = 0; g < nwg; ++g) {
        const unsigned long long* q = &tl[((size_t)g * 8) * 9 * 4];
        unsigned long long e = 0;
        int last = -1;
        for (int it = 0; it < 9; ++it)
            if (q[it * 4 + 3]) { e = q[it * 4 + 3]; last = it; }
        if (g < 20 || g % 32 == 0)
            printf("    wg %3d: start +%.2f, %d units, end +%.2f us\n", g, (q[0] - t0) * 0.01, last + 1, (e - t0) * 0.01);
        if (e > tmax) { tmax = e; gmax = g; }
    }
    printf("  grid span %.2f us (last workgroup to finish: %d)\n", (tmax - t0) * 0.01, gmax);
}
#endif

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

// U pieces, bf16 [ab 0..8 | 9 = channel 16][xi][piece][co][16] (returned as the float-sized buffer holding
// the bits): blocks ab < 9 hold (G g_ab G^T)[xi] of channels 0..15 (K = channel); block 9 holds channel 16
// of every sub-kernel (K = ab; 9..15 zero). U rounded from f64 to f32 exactly as wino9_pack_weights, then
// split into three bf16 pieces, round-to-nearest-even at each step. Channels >= cin are zero.
std::vector<float> wino9_x6_pack_weights(const float* kern, int cin) {
#pragma clang fp contract(off)
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    const size_t n16 = (size_t)10 * NXI * 3 * NT * 16;
    std::vector<uint16_t> U(n16, 0);
    for (int ab = 0; ab < 9; ++ab) {
        const int sa = ab / 3, sb = ab % 3;
        for (int ci = 0; ci < cin; ++ci)
            for (int co = 0; co < NT; ++co) {
                double gg[3][3];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        gg[i][j] = kern[(((size_t)(3 * sa + i) * 9 + (3 * sb + j)) * cin + ci) * NT + co];
                for (int p = 0; p < 4; ++p)
                    for (int q = 0; q < 4; ++q) {
                        double u = 0.0;
                        for (int i = 0; i < 3; ++i)
                            for (int j = 0; j < 3; ++j) u += G[p][i] * gg[i][j] * G[q][j];
                        const float uf = (float)u;
                        uint16_t pc[3];
                        pc[0] = bf16_rne_host(uf);
                        const float r = uf - bf16_val_host(pc[0]);
                        pc[1] = bf16_rne_host(r);
                        pc[2] = bf16_rne_host(r - bf16_val_host(pc[1]));
                        const int xi = p * 4 + q;
                        const int blk = ci < 16 ? ab : 9, k = ci < 16 ? ci : ab;
                        for (int pi = 0; pi < 3; ++pi)
                            U[((((size_t)blk * NXI + xi) * 3 + pi) * NT + co) * 16 + k] = pc[pi];
                    }
            }
    }
    std::vector<float> out(n16 / 2);
    std::memcpy(out.data(), U.data(), n16 * 2);
    return out;
}

// Device form of wino9_x6_pack_weights (training re-packs after every optimizer step): one thread per
// (block, co, K index) writes its 16 points x 3 pieces, zeros included (no reliance on a cleared buffer);
// f64 with the host's operation order and no contraction, the host's RNE bit formula: bitwise the host image.
__global__ __launch_bounds__(256) void wino9_x6_transform_kernel(const float* __restrict__ kern, int cin,
                                                                 unsigned short* __restrict__ U) {
#pragma clang fp contract(off)
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= 10 * NT * 16) return;
    const int k = idx & 15, co = (idx >> 4) % NT, blk = idx / (16 * NT);
    const int ab = blk < 9 ? blk : k, ci = blk < 9 ? k : 16;
    const bool valid = ci < cin && ab < 9;
    const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    const int sa = ab / 3, sb = ab % 3;
    double gg[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            gg[i][j] = valid ? (double)kern[(((size_t)(3 * sa + i) * 9 + (3 * sb + j)) * cin + ci) * NT + co] : 0.0;
    auto rne = [](float x) -> unsigned short {
        const unsigned u = __float_as_uint(x);
        return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
    };
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double u = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) u = u + G[p][i] * gg[i][j] * G[q][j];
            const float uf = (float)u;
            unsigned short pc[3];
            pc[0] = rne(uf);
            const float r = uf - __uint_as_float((unsigned)pc[0] << 16);
            pc[1] = rne(r);
            pc[2] = rne(r - __uint_as_float((unsigned)pc[1] << 16));
#pragma unroll
            for (int pi = 0; pi < 3; ++pi)
                U[((((size_t)blk * NXI + p * 4 + q) * 3 + pi) * NT + co) * 16 + k] = valid ? pc[pi] : (unsigned short)0;
        }
}

hipError_t wino9_x6_transform_launch(const float* kern, int cin, float* U, hipStream_t st) {
    if (cin > 17 || cin <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wino9_x6_transform_kernel, dim3((10 * NT * 16 + 255) / 256), dim3(256), 0, st, kern, cin,
                       reinterpret_cast<unsigned short*>(U));
    return hipGetLastError();
}

size_t wino9_x6_weight_floats() { return (size_t)10 * NXI * 3 * NT * 16 / 2; }

hipError_t wino9_x6_prepare() {
    for (const void* k : {(const void*)wino9_x6_kernel<17, false>, (const void*)wino9_x6_kernel<0, false>,
                          (const void*)wino9_x6_kernel<17, true>, (const void*)wino9_x6_kernel<0, true>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int wino9_x6_tiles_y(int H) { return (H + TH - 1) / TH; }
int wino9_x6_tiles_x(int W) { return (W + TW - 1) / TW; }

hipError_t wino9_x6_launch(const Wino9Args& a, hipStream_t st) {
    if (a.cin > 17 || a.cin <= 0 || a.tiles_y != (a.H + TH - 1) / TH || a.tiles_x != (a.W + TW - 1) / TW ||
        (a.part == nullptr && a.bn_ab == nullptr))
        return hipErrorInvalidValue;   // inference: folded BN affine; training: statistics partials
    if ((size_t)a.batch * a.H * a.W * a.cin * 4 >= (size_t)0x7FFFFFF0)
        return hipErrorInvalidValue;   // 32-bit staging offsets; the idle threads' offset must stay out of range
    // persistent: one workgroup per CU (LDS and registers allow one), each looping over tiles
    const int n_tiles = a.batch * a.tiles_y * a.tiles_x;
    static int n_cu = 0;   // queried once (not per launch: graph capture replays the recorded arguments)
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    const unsigned grid = (unsigned)(n_tiles < n_cu ? n_tiles : n_cu);
    // a last round that fills at most half the grid runs as half-tile units (see the kernel)
    const int tail = n_tiles % (int)grid;
    const int n_full = (tail > 0 && 2 * tail <= (int)grid) ? n_tiles - tail : n_tiles;
    const int n_units = n_full + 2 * (n_tiles - n_full);
    if (a.part != nullptr) {   // training
        if (a.cin == 17)
            hipLaunchKernelGGL((wino9_x6_kernel<17, true>), dim3(grid), dim3(NTHR), LDS_BYTES, st, a, n_units, n_full);
        else
            hipLaunchKernelGGL((wino9_x6_kernel<0, true>), dim3(grid), dim3(NTHR), LDS_BYTES, st, a, n_units, n_full);
    } else if (a.cin == 17) {
        hipLaunchKernelGGL((wino9_x6_kernel<17, false>), dim3(grid), dim3(NTHR), LDS_BYTES, st, a, n_units, n_full);
    } else {
        hipLaunchKernelGGL((wino9_x6_kernel<0, false>), dim3(grid), dim3(NTHR), LDS_BYTES, st, a, n_units, n_full);
    }
    return hipGetLastError();
}

}  // namespace rst
