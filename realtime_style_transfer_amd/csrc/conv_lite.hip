// conv_lite.hip — the narrow-channel convolutions of the transfer network on f32 MFMA, exact f32:
//   contract_0/1   Conv2D 3x3 s2 'same' + bias + ReLU -> BatchNorm -> ReLU     styleTransfer.py:194-203
//   expand_0/1     Conv2DTranspose 3x3 s2 'same' + bias (+ CIN stats)         styleTransfer.py:115-119
// (Cin 16..128, Cout 16 or 32). The general implicit-GEMM kernel (conv_mfma.hip) ran these at
// 0.17-0.25 of their rooflines: 32-wide N tiles half empty for Cout = 16, and the 4-phase transposed
// form issued all 16 (tap, phase) products of which 7 multiply structural zeros.
//
// Mapping (one workgroup = 4 waves = 4 rows of MS pixels of the GEMM grid; MS = Cout = MFMA M = N):
//   * Cout 16 -> v_mfma_f32_16x16x4_f32, Cout 32 -> v_mfma_f32_32x32x2_f32: no idle columns;
//   * the input halo of the tile (all channels of a Cin chunk) is staged once into LDS, stride-2
//     columns split by parity so a wave's 16/32 pixels read consecutive 16-B slots, each pixel padded
//     to an odd number of 16-B slots: every operand read is one conflict-free ds_read_b128 whose four
//     channels feed four MFMAs;
//   * weights are host-packed in the LDS image order [chunk][slot][r][kslot][n][4];
//   * transposed conv: out[2p+py][2q+px] = sum over the taps of phase (py,px) of in[p+ty-1][q+tx-1] .
//     w[py+2(1-ty)][px+2(1-tx)] — phase (0,0) has 4 taps, (0,1) and (1,0) two, (1,1) one: the nine
//     (phase, tap) slots issue exactly the 9 x Cin x Cout MACs per input pixel, and the four operand
//     positions (ty, tx) are read once and shared by the phases that use them;
//   * the CIN statistics {sum, M2, n} of a tile merge its four phases (finalize sees one partial per
//     tile and channel), two-pass inside the tile, fixed order: deterministic.
// Multi-chunk layers (expand_0, Cin 128 in 4 chunks of 32): chunk c+1 is loaded into registers while chunk c's
// MFMAs run and written to the (single) halo + weight image after.
// (Measured and removed, round 4: a double-buffered 16-channel chunk pipeline for expand_0 — equal at B = 8, 3.5 us
// slower at B = 1, profiles/r04/lite_pipe.log; a bank-conflict-free staging map — LDS conflicts 0.56 -> 0.10 with no
// layer faster, lite_remap.log; the prologue affine formed before the first input loads — neutral in the frame,
// ab_table_first.log; a deeper B-operand ring — neutral.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kernels.h"

// x6 transposed convs: full tiles' output staged through LDS and stored as whole lines (0: per-accumulator stores)
#ifndef LITE_OSTAGE
#define LITE_OSTAGE 1
#endif
#ifndef LITE_OSTAGE0
#define LITE_OSTAGE0 1   // the same for the x6 strided convs
#endif

namespace rst {

#ifdef LITE_PROF
// s_memtime per (workgroup < 64, wave, step < 16, point): 0 step top, 1 after staging + barrier,
// 2 after the MFMAs, 3 after the epilogue (tools/lite_bench)
__device__ unsigned long long lite_tl[64][8][16][4];
__device__ unsigned long long lite_t0[64][8][2];   // kernel start, end of the last step
#define LTL(st, pt) \
    if (blockIdx.x < 64 && lane == 0 && (st) < 16) lite_tl[blockIdx.x][wave][(st)][(pt)] = __builtin_amdgcn_s_memtime()
#define LT0(k) \
    if (blockIdx.x < 64 && lane == 0) lite_t0[blockIdx.x][wave][(k)] = __builtin_amdgcn_s_memtime()
#else
#define LTL(st, pt)
#define LT0(k)
#endif

namespace lite {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// (x, y) -> three packed bf16 pairs, x = x0 + x1 + x2 exactly (round-to-nearest-even at each step)
__device__ __forceinline__ void split3(float x, float y, unsigned& p0, unsigned& p1, unsigned& p2) {
    p0 = bf16_piece(x, y);
    p1 = bf16_piece(x, y);
    p2 = bf16_last_piece(x, y);
}

template <int MODE, int CIN, int NC, int CKC, int X6 = 0, int KSP = 1>
struct Cfg {
    static constexpr int MS = NC;                           // MFMA M = N = Cout
    static constexpr int TW = MS, TH = 4;                   // GEMM-grid tile: 4 rows x MS pixels
    static constexpr int KS = 64 / MS;                      // k slots per MFMA (lane groups)
    static constexpr int NCH = CIN / CKC;                   // Cin chunks
    static constexpr int QC = CKC / 4;                      // channel quads per pixel and chunk
    static constexpr int R = QC / KS;                       // operand reads per slot and chunk
    static constexpr int HR = MODE == 0 ? 2 * TH + 1 : TH + 1;
    static constexpr int HC = MODE == 0 ? 2 * TW + 1 : TW + 1;
    static constexpr int NPIX = HR * HC;
    static constexpr int CS = CKC + 4;                      // floats per halo pixel (odd 16-B slots)
    // split-bf16 x6: the bf16 MFMA of the Cout (32: 32x32x16, K step 16 = two 8-channel lane groups; 16: 16x16x32,
    // K step 32 = four groups). Halo [piece][K step][group][pixel][8 bf16] (pixels padded to a multiple of 16: the
    // four groups of a ds_read_b128 lane set then hit disjoint banks), weights [slot][K step][piece][group][n][8 bf16]
    // — the MFMA operand layouts. Single-chunk layers (Cin <= CKC) hold the split weights in VGPRs (9 slots x 3 pieces
    // x 4 registers): no weight image in LDS, no B-operand LDS reads.
    static constexpr int KSTEP = MS == 32 ? 16 : 32;
    static constexpr int G = KSTEP / 8;                     // 8-channel lane groups per K step
    static constexpr int KS2 = X6 ? CKC / KSTEP : 1;        // K steps per chunk (x6)
    static constexpr int NPIXP = (NPIX + 15) / 16 * 16;
    static constexpr bool WIN_REGS = X6 && NCH == 1;        // x6 weights in registers
    // K split (expand_0): waves w and w + 4 compute pixel row w & 3 over the even / odd K steps of every chunk, then
    // trade accumulators so that each finishes one output row (two phases): two waves per SIMD hide each other's LDS
    // operand latency and the staging work per thread halves (one workgroup per CU either way: 240 tiles, 256 CUs)
    // The K split's weights come by LDS-DMA (global_load_lds, no staging registers: two waves per SIMD leave 256
    // registers a wave) into two weight buffers, chunk c + 1's landing while chunk c's MFMAs read the other.
    static constexpr int KSPLIT = KSP;
    static_assert(KSP == 1 || (KSP == 2 && X6 && MODE == 1 && NCH > 1 && KS2 % 2 == 0), "K split: x6 multi-chunk transposed");
    static constexpr bool WDMA = KSPLIT == 2;
    static constexpr int NW = 4 * KSPLIT, NT = 64 * NW;     // waves, threads per workgroup
    static constexpr int HALO = X6 ? 3 * KS2 * G * NPIXP * 4 : NPIX * CS;   // floats per halo buffer
    static constexpr int WCH = WIN_REGS ? 0 : (X6 ? 9 * CKC * NC * 3 / 2 : 9 * CKC * NC);   // floats per chunk of weights in LDS
    static constexpr int WBUF = WDMA ? 2 : 1;               // weight buffers
    static constexpr int WITEMS = WCH / 4;
    static constexpr int WREG = (WITEMS + NT - 1) / NT;
    static_assert(!WDMA || (WITEMS % 64 == 0 && NCH % 2 == 0), "LDS-DMA: whole wave instructions, chunk parity = buffer");
    static constexpr int NACC = MS == 16 ? 4 : 16;          // accumulator floats per MFMA tile and lane
    static constexpr int NPH = MODE == 0 ? 1 : 4;           // output phases
    static constexpr int OST_FL = 4 * TW * NC;              // floats of one pixel row's output (4 phases)
    static constexpr int XCH = KSPLIT == 2 ? NW * 2 * NACC * 64 : 0;   // K-split accumulator exchange (floats)
    // LDS body: the halo + weight images; at the end of a tile the K split's exchange, then its output staging, in it
    static constexpr int IMG = HALO + WBUF * WCH;
    static constexpr int BODY = IMG > 4 * OST_FL && IMG > XCH ? IMG : (4 * OST_FL > XCH ? 4 * OST_FL : XCH);
    static constexpr int RED = MODE == 1 ? 4 * NW * NC : 0; // statistics scratch (floats): [NW][NC] f64 pairs
    static constexpr size_t LDS_BYTES = (size_t)BODY * 4 + RED * 4;
    static_assert(CIN % CKC == 0 && CKC % (4 * KS) == 0, "chunking");
    static_assert(MS == 16 || MS == 32, "MFMA shape");
    static_assert(((CS / 4) & 1) == 1, "odd 16-B slots per halo pixel");
    static_assert(!X6 || CKC % KSTEP == 0, "x6: whole K steps per chunk");
    static_assert(!WIN_REGS || KS2 == 1, "x6 weights in registers: one K step");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

template <int MS>
struct Mfma;
template <>
struct Mfma<16> {
    typedef f32x4 acc_t;
    static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // accumulator entry j of lane l: row (pixel) and column (channel)
    static __device__ __forceinline__ int row(int j, int lane) { return 4 * (lane >> 4) + j; }
    static __device__ __forceinline__ int col(int lane) { return lane & 15; }
};
template <>
struct Mfma<32> {
    typedef f32x16 acc_t;
    static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int j, int lane) { return (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5); }
    static __device__ __forceinline__ int col(int lane) { return lane & 31; }
};

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

// sum of N per-wave values p[0], p[stride], ... as a pairwise tree (fixed order; N = 4: (p0 + p1) + (p2 + p3))
template <int N, typename T>
__device__ __forceinline__ T wave_sum(const T* p, int stride) {
    if constexpr (N == 1) return p[0];
    else return wave_sum<N / 2>(p, stride) + wave_sum<N / 2>(p + (N / 2) * stride, stride);
}

// transposed-conv slots: (phase, operand position ty*2+tx); the kernel tap is ky = py + 2(1-ty), kx = px + 2(1-tx)
__host__ __device__ constexpr int t_phase(int s) { return s < 4 ? 0 : (s < 6 ? 1 : (s < 8 ? 2 : 3)); }
__host__ __device__ constexpr int t_pos(int s) {
    return s < 4 ? s : (s == 4 ? 1 : (s == 5 ? 3 : (s == 6 ? 2 : 3)));
}
}  // namespace lite

// PROF: the prologue mode (kernels.h ProMode) | LITE_BLEND (two styles: the per-pixel blend of the two CIN
// affines, styleTransfer.py:36-44, as conv_mfma.hip's prologue)
constexpr int LITE_BLEND = 8;

template <int MODE, int CIN, int NC, int CKC, int PROF, int X6, int KSP>
__global__ __launch_bounds__((lite::Cfg<MODE, CIN, NC, CKC, X6, KSP>::NT)) void conv_lite_kernel(ConvArgs a, int n_tiles) {
    using namespace lite;
    constexpr int PRO = PROF & 7;
    constexpr bool BLEND = (PROF & LITE_BLEND) != 0;
    using C = Cfg<MODE, CIN, NC, CKC, X6, KSP>;
    using M = Mfma<C::MS>;
    typedef typename M::acc_t acc_t;
    constexpr int MS = C::MS, TW = C::TW, TH = C::TH, KS = C::KS, CS = C::CS, HC = C::HC, HR = C::HR, R = C::R;
    constexpr int QC = C::QC, NCH = C::NCH;

    extern __shared__ __attribute__((aligned(16))) float smem[];
    // [HALO] one Cin chunk of the tile's input halo, then [WCH] its weights. LDS-DMA weights (K split): [WCH] weight
    // buffer 1, [HALO], [WCH] buffer 0 — chunk c uses buffer c & 1, so a tile's last chunk reads buffer 1 and the next
    // tile's first chunk lands in buffer 0 while the epilogue's exchange / output staging use [0, 64 KB)
    float* const halo = smem + (C::WDMA ? C::WCH : 0);
    float* const wts = smem + C::HALO;   // (not LDS-DMA)
    auto wbase = [&](int buf) __attribute__((always_inline)) {
        return C::WDMA ? (buf == 0 ? smem + C::WCH + C::HALO : smem) : wts;
    };
    int wbuf = 0;   // LDS-DMA weights: the buffer the current step's MFMAs read
    // [3][NW][NC] statistics: S, n, M2 per wave (partials path) / [NW][NC][2] f64 (accumulator flush)
    float* const red = smem + C::BODY;
    static_assert(C::BODY % 2 == 0, "f64-aligned statistics scratch");
    constexpr int NT = C::NT, NW = C::NW;
    float2* const tab = reinterpret_cast<float2*>(red + C::RED);   // prologue affine [batch][CIN] (+ second style)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rw = wave & 3, kh = C::KSPLIT == 2 ? wave >> 2 : 0;   // pixel row of the tile, K half
    LT0(0);
    const int H = a.H, W = a.W;
    auto halo_off = [&](int hy, int hx) __attribute__((always_inline)) {
        if constexpr (MODE == 0) return (hy * HC + (hx & 1) * (TW + 1) + (hx >> 1)) * CS;
        else return (hy * HC + hx) * CS;
    };

    // ---- persistent schedule: this workgroup's k-th tile is xcd_tile_order(blockIdx.x + k grid) (the
    // grid is a multiple of 8, so every tile of a workgroup stays on its XCD's contiguous range) ------
    struct Tile { int b, ty, tx, y0, x0, iy0, ix0; };
    auto tile_of = [&](int k) __attribute__((always_inline)) {
        Tile T;
        int t = xcd_tile_order(blockIdx.x + k * gridDim.x, n_tiles);
        T.tx = t % a.tiles_x;
        t /= a.tiles_x;
        T.ty = t % a.tiles_y;
        T.b = t / a.tiles_y;
        T.y0 = T.ty * TH;
        T.x0 = T.tx * TW;
        T.iy0 = MODE == 0 ? 2 * T.y0 - a.pad_t : T.y0 - 1;
        T.ix0 = MODE == 0 ? 2 * T.x0 - a.pad_l : T.x0 - 1;
        return T;
    };

    // ---- staging map -----------------------------------------------------------------------------
    // Thread t stages channel quad q = t % QC of main column col = (t / QC) % (HC - 1) in rows
    // rsub + RPP k, and (t < HR QC) the last halo column in row t / QC: the global and LDS offsets
    // advance by a constant per row (a per-item (pixel, quad) decode cost as much VALU as the MFMAs).
    constexpr int HCM = HC - 1, TPR = HCM * QC, RPP = NT / TPR, NMAIN = (HR + RPP - 1) / RPP;
    constexpr int NEXTRA = HR * QC;
    static_assert(NT % TPR == 0 && NEXTRA <= NT, "staging map");
    const int q = tid % QC;
    const int col = (tid / QC) % HCM;
    const int rsub = tid / TPR;
    const bool ext = tid < NEXTRA;   // stages the last halo column
    const int ehy = min(tid / QC, HR - 1);
    const int lcm = halo_off(0, col) + 4 * q, lce = halo_off(0, HCM) + 4 * q;
    // two register sets of staged input (single-chunk layers prefetch two tiles ahead: the HBM latency
    // under load exceeds one tile's MFMAs); multi-chunk layers use set 0 only
    // (x6 single-chunk layers hold their weights in VGPRs instead: one set, two workgroups per CU cover the latency)
    constexpr int NSET = NCH == 1 && !C::WIN_REGS ? 2 : 1;
    f32x4 hreg[NSET][NMAIN + 1], rreg[NSET][NMAIN + 1], wreg[NCH > 1 && !C::WDMA ? C::WREG : 1], pa01[NSET], pa23[NSET];
    f32x4 pb01[NSET], pb23[NSET];   // BLEND: the second style's affine of the thread's channel quad
    float bw[NSET][NMAIN + 1];      // BLEND: the second style's weight at each staged pixel
    // one chunk's weight image (multi-chunk layers, one register set)
    auto load_w = [&](int ch, int buf) __attribute__((always_inline)) {
        sfor<0, C::WREG>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            if constexpr (C::WDMA) {   // 1 KB per wave instruction into the lane-linear image (the packed order)
                const int i0 = NT * k + wave * 64;   // wave-uniform
                if (C::WITEMS % NT == 0 || i0 < C::WITEMS)
                    __builtin_amdgcn_global_load_lds(
                        (const void*)(reinterpret_cast<const f32x4*>(a.wpk) + (size_t)ch * C::WITEMS + i0 + lane),
                        (__attribute__((address_space(3))) void*)(wbase(buf) + i0 * 4), 16, 0, 0);
            } else {
                const int it = min(tid + NT * k, C::WITEMS - 1);
                wreg[k] = reinterpret_cast<const f32x4*>(a.wpk)[(size_t)ch * C::WITEMS + it];
            }
        });
    };
    auto load_in = [&](const Tile& T, int ch, auto SET, int buf = 0) __attribute__((always_inline)) {
        constexpr int st = decltype(SET)::value;
        const int co = ch * CKC;
        const int ixm = min(max(T.ix0 + col, 0), W - 1), ixe = min(max(T.ix0 + HCM, 0), W - 1);
        const int rb = T.b * H;
        sfor<0, NMAIN + 1>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int hy = k < NMAIN ? min(rsub + RPP * k, HR - 1) : ehy;
            const int gi = ((rb + min(max(T.iy0 + hy, 0), H - 1)) * W + (k < NMAIN ? ixm : ixe)) * CIN + co + 4 * q;
            hreg[st][k] = *reinterpret_cast<const f32x4*>(a.in + gi);
            if constexpr (PRO == PRO_AFF_RES) rreg[st][k] = *reinterpret_cast<const f32x4*>(a.res + gi);
            if constexpr (BLEND) bw[st][k] = a.pro_w[(rb + min(max(T.iy0 + hy, 0), H - 1)) * W + (k < NMAIN ? ixm : ixe)];
        });
        if constexpr (NCH > 1) load_w(ch, buf);
    };
    auto load_aff = [&](const Tile& T, int ch, auto SET) __attribute__((always_inline)) {   // from the LDS table
        constexpr int st = decltype(SET)::value;
        if constexpr (PRO != PRO_NONE) {
            const int co = ch * CKC;
            const f32x4* pa = reinterpret_cast<const f32x4*>(tab + T.b * CIN + co + 4 * q);
            pa01[st] = pa[0];
            pa23[st] = pa[1];
            if constexpr (BLEND) {
                const f32x4* pb = reinterpret_cast<const f32x4*>(tab + (a.batch + T.b) * CIN + co + 4 * q);
                pb01[st] = pb[0];
                pb23[st] = pb[1];
            }
        }
    };
    auto load_step = [&](const Tile& T, int ch, auto SET, int buf = 0) __attribute__((always_inline)) {
        load_in(T, ch, SET, buf);
        load_aff(T, ch, SET);
    };
    auto xform = [&](f32x4 v, f32x4 r, const f32x4& p01, const f32x4& p23, float w, const f32x4& q01,
                     const f32x4& q23) __attribute__((always_inline)) {
        if constexpr (PRO != PRO_NONE) {
            if constexpr (BLEND) {
                v.x = style_blend(w, fmaf(p01.x, v.x, p01.y), fmaf(q01.x, v.x, q01.y));
                v.y = style_blend(w, fmaf(p01.z, v.y, p01.w), fmaf(q01.z, v.y, q01.w));
                v.z = style_blend(w, fmaf(p23.x, v.z, p23.y), fmaf(q23.x, v.z, q23.y));
                v.w = style_blend(w, fmaf(p23.z, v.w, p23.w), fmaf(q23.z, v.w, q23.w));
            } else {
                v.x = fmaf(p01.x, v.x, p01.y);
                v.y = fmaf(p01.z, v.y, p01.w);
                v.z = fmaf(p23.x, v.z, p23.y);
                v.w = fmaf(p23.z, v.w, p23.w);
            }
            if constexpr (PRO == PRO_AFF_RELU) {
                v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
            } else if constexpr (PRO == PRO_AFF_RES) {
                v += r;
            }
        }
        return v;
    };
    // x6: channel quad q of the chunk = K step q / (KSTEP / 4), lane group (q % (KSTEP / 4)) >> 1, bf16 slots
    // 4 (q & 1) .. +3 of the group's 8; pixels in halo_off's order (stride-2 columns parity-split)
    auto hbytes_r = [&]() __attribute__((always_inline)) { return reinterpret_cast<const unsigned char*>(halo); };
    constexpr int QPS = C::KSTEP / 4;                                                  // channel quads per K step
    const int xq = (((q / QPS) * C::G + ((q % QPS) >> 1)) * C::NPIXP) * 16 + (q & 1) * 8;   // + piece + pixel
    constexpr int XPIECE = C::KS2 * C::G * C::NPIXP * 16;                             // bytes per piece plane
    auto hpix = [&](int hy, int hx) __attribute__((always_inline)) {                  // x6 halo pixel index
        if constexpr (MODE == 0) return hy * HC + (hx & 1) * (TW + 1) + (hx >> 1);
        else return hy * HC + hx;
    };
    auto put = [&](int hy, int hx, int lf, f32x4 v) __attribute__((always_inline)) {
        if constexpr (X6) {
            unsigned p0[2], p1[2], p2[2];
            split3(v.x, v.y, p0[0], p1[0], p2[0]);
            split3(v.z, v.w, p0[1], p1[1], p2[1]);
            unsigned char* dst = reinterpret_cast<unsigned char*>(halo) + xq + hpix(hy, hx) * 16;
            *reinterpret_cast<uint2*>(dst) = make_uint2(p0[0], p0[1]);
            *reinterpret_cast<uint2*>(dst + XPIECE) = make_uint2(p1[0], p1[1]);
            *reinterpret_cast<uint2*>(dst + 2 * XPIECE) = make_uint2(p2[0], p2[1]);
        } else {
            *reinterpret_cast<f32x4*>(halo + lf + hy * (HC * CS)) = v;
        }
    };
    // staging of one chunk into LDS, as NSTORE items: the NMAIN main-column rows, the last halo column, then the WREG
    // weight float4s
    constexpr int NSTORE = NMAIN + 1 + (NCH > 1 && !C::WDMA ? C::WREG : 0);
    auto store_item = [&](const Tile& T, auto SET, auto IDX) __attribute__((always_inline)) {
        constexpr int st = decltype(SET)::value, idx = decltype(IDX)::value;
        auto row_ok = [&](int hy) __attribute__((always_inline)) { return T.iy0 + hy >= 0 && T.iy0 + hy < H; };
        if constexpr (idx < NMAIN) {
            constexpr int k = idx;
            const bool okm = T.ix0 + col >= 0 && T.ix0 + col < W;
            const int hy = rsub + RPP * k;
            if (HR % RPP == 0 || k < NMAIN - 1 || hy < HR) {
                const f32x4 v = okm && row_ok(hy) ? xform(hreg[st][k], rreg[st][k], pa01[st], pa23[st], bw[st][k],
                                                          pb01[st], pb23[st])
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
                put(hy, col, lcm, v);
            }
        } else if constexpr (idx == NMAIN) {
            const bool oke = T.ix0 + HCM >= 0 && T.ix0 + HCM < W;
            if (ext) {
                const f32x4 v = oke && row_ok(ehy) ? xform(hreg[st][NMAIN], rreg[st][NMAIN], pa01[st], pa23[st],
                                                           bw[st][NMAIN], pb01[st], pb23[st])
                                                   : f32x4{0.f, 0.f, 0.f, 0.f};
                put(ehy, HCM, lce, v);
            }
        } else if constexpr (NCH > 1) {
            constexpr int k = idx - NMAIN - 1;
            const int it = tid + NT * k;
            if (C::WITEMS % NT == 0 || it < C::WITEMS) reinterpret_cast<f32x4*>(wts)[it] = wreg[k];
        }
    };
    auto store_step = [&](const Tile& T, auto SET) __attribute__((always_inline)) {
        sfor<0, NSTORE>([&](auto I) __attribute__((always_inline)) { store_item(T, SET, I); });
    };

    // ---- operands: A = pixel m of this wave's row, quad g + KS r; B = row (slot, r, g), column m ------
    const int m = lane % MS, g = lane / MS;
    auto a_off = [&](int pos) __attribute__((always_inline)) {   // pos: tap (MODE 0) / operand position (MODE 1)
        if constexpr (MODE == 0) return halo_off(2 * rw + pos / 3, 2 * m + pos % 3);
        else return halo_off(rw + (pos >> 1), m + (pos & 1));
    };
    // software pipeline: the operands of step u+1 are read before the MFMAs of step u issue. Steps:
    // MODE 0 one (r, kernel row) = 3 taps, 12 MFMAs into 3 accumulators (one per kx: no back-to-back
    // dependent MFMAs); MODE 1 one r = 4 operand positions x 9 slots, 36 MFMAs into the 4 phase
    // accumulators (phase 0's four slots alternate between two).
    constexpr int NA = MODE == 0 ? 3 : 4, NB = MODE == 0 ? 3 : 9, NSTEP = MODE == 0 ? 3 * R : R;
    // (x6 strided conv with Cout 32: one 32x32x16 accumulator chain, which issues back to back, MI355X_MICROARCH.md)
    // (K split: one accumulator per phase — two waves per SIMD interleave their MFMA chains — for the registers)
    constexpr int NACCS = MODE == 0 ? (X6 && MS == 32 ? 1 : 3) : (C::KSPLIT == 2 ? 4 : 5);
    acc_t acc[NACCS];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < NACCS; ++p)
#pragma unroll
            for (int j = 0; j < C::NACC; ++j) acc[p][j] = 0.f;
    };
    auto read_step = [&](auto U, f32x4 (&A)[NA], f32x4 (&Bv)[NB]) __attribute__((always_inline)) {
        constexpr int u = decltype(U)::value;
        if constexpr (MODE == 0) {
            constexpr int r = u / 3, ky = u % 3;
            const int qo = 4 * (g + KS * r);
            sfor<0, 3>([&](auto X) __attribute__((always_inline)) {
                constexpr int kx = decltype(X)::value, t = ky * 3 + kx;
                A[kx] = *reinterpret_cast<const f32x4*>(halo + a_off(t) + qo);
                Bv[kx] = *reinterpret_cast<const f32x4*>(wts + (((t * R + r) * KS + g) * MS + m) * 4);
            });
        } else {
            constexpr int r = u;
            const int qo = 4 * (g + KS * r);
            sfor<0, 4>([&](auto P) __attribute__((always_inline)) {
                constexpr int pos = decltype(P)::value;
                A[pos] = *reinterpret_cast<const f32x4*>(halo + a_off(pos) + qo);
            });
            sfor<0, 9>([&](auto S) __attribute__((always_inline)) {
                constexpr int sl = decltype(S)::value;
                Bv[sl] = *reinterpret_cast<const f32x4*>(wts + (((sl * R + r) * KS + g) * MS + m) * 4);
            });
        }
    };
    auto mfma_step = [&](const f32x4 (&A)[NA], const f32x4 (&Bv)[NB]) __attribute__((always_inline)) {
        sfor<0, 4>([&](auto I) __attribute__((always_inline)) {
            constexpr int i = decltype(I)::value;
            if constexpr (MODE == 0) {
                sfor<0, 3>([&](auto X) __attribute__((always_inline)) {
                    constexpr int kx = decltype(X)::value;
                    acc[kx] = M::op(A[kx][i], Bv[kx][i], acc[kx]);
                });
            } else {
                constexpr int order[9] = {0, 4, 6, 8, 1, 5, 7, 2, 3};
                sfor<0, 9>([&](auto S) __attribute__((always_inline)) {
                    constexpr int sl = order[decltype(S)::value];
                    constexpr int ai = (sl == 1 || sl == 3) ? 4 : t_phase(sl);
                    acc[ai] = M::op(A[t_pos(sl)][i], Bv[sl][i], acc[ai]);
                });
            }
        });
    };
    // x6: per K step, MODE 1 reads the 4 operand positions x 3 pieces of A once and walks the slots in
    // phase-interleaved order; MODE 0 walks the 9 taps with A read one tap ahead. B (3 pieces) comes from the
    // weight registers (single-chunk layers) or from LDS one slot ahead; 6 terms per slot.
    const int kg = lane / MS;   // the lane's 8-channel group of a K step
    short8 wr6[C::WIN_REGS ? 9 : 1][3];
    if constexpr (C::WIN_REGS) {   // [slot][piece] B fragments of this lane (n = m, group kg)
        const u32x4* wp = reinterpret_cast<const u32x4*>(a.wpk);
        sfor<0, 9>([&](auto S) __attribute__((always_inline)) {
            constexpr int sl = decltype(S)::value;
            sfor<0, 3>([&](auto PC) __attribute__((always_inline)) {
                constexpr int pc = decltype(PC)::value;
                wr6[sl][pc] = __builtin_bit_cast(short8, wp[((sl * 3 + pc) * C::G + kg) * MS + m]);
            });
        });
    }
    auto mfma6 = [&](acc_t& acc_, const short8 (&A)[3], const short8 (&Bv)[3]) __attribute__((always_inline)) {
        constexpr int ap[6] = {0, 0, 1, 0, 1, 2}, bp[6] = {0, 1, 0, 2, 1, 0};
        sfor<0, 6>([&](auto T6) __attribute__((always_inline)) {
            constexpr int t6 = decltype(T6)::value;
            if constexpr (MS == 32)
                acc_ = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[ap[t6]], Bv[bp[t6]], acc_, 0, 0, 0);
            else
                acc_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ap[t6]], Bv[bp[t6]], acc_, 0, 0, 0);
        });
    };
    auto compute_x6 = [&]() __attribute__((always_inline)) {
      if constexpr (X6) {   // discarded (not instantiated) for the f32 configurations
        const unsigned char* wbytes = reinterpret_cast<const unsigned char*>(wbase(wbuf));
        const unsigned char* hbytes = hbytes_r();
        auto readB = [&](int sl, int ks, short8 (&Bv)[3]) __attribute__((always_inline)) {
            sfor<0, 3>([&](auto PC) __attribute__((always_inline)) {
                constexpr int pc = decltype(PC)::value;
                Bv[pc] = *reinterpret_cast<const short8*>(wbytes + ((((sl * C::KS2 + ks) * 3 + pc) * C::G + kg) * MS + m) * 16);
            });
        };
        auto readA = [&](int pix, int ks, short8 (&A)[3]) __attribute__((always_inline)) {
            sfor<0, 3>([&](auto PC) __attribute__((always_inline)) {
                constexpr int pc = decltype(PC)::value;
                A[pc] = *reinterpret_cast<const short8*>(hbytes + pc * XPIECE + ((ks * C::G + kg) * C::NPIXP + pix) * 16);
            });
        };
        sfor<0, C::KS2 / C::KSPLIT>([&](auto KSI) __attribute__((always_inline)) {
            const int ks = decltype(KSI)::value * C::KSPLIT + kh;   // this wave's K steps
            if constexpr (MODE == 1 && C::KSPLIT == 2) {
                // each operand position read one or two slots before its first use and dead after its last (slot order
                // 0 1 4 2 6 3 5 7 8: position 0 | 1 1 | 2 2 | 3 3 3 3): two positions live instead of four
                constexpr int order[9] = {0, 1, 4, 2, 6, 3, 5, 7, 8};
                short8 A[4][3];
                auto rdA = [&](auto P) __attribute__((always_inline)) {
                    constexpr int pos = decltype(P)::value;
                    readA((rw + (pos >> 1)) * HC + m + (pos & 1), ks, A[pos]);
                };
                rdA(std::integral_constant<int, 0>{});
                rdA(std::integral_constant<int, 1>{});
                constexpr int BD = 2;   // B operand one slot ahead
                short8 Bq[BD][3];
                readB(order[0], ks, Bq[0]);
                sfor<0, 9>([&](auto J) __attribute__((always_inline)) {
                    constexpr int j = decltype(J)::value, sl = order[j];
                    if constexpr (j == 1) rdA(std::integral_constant<int, 2>{});
                    if constexpr (j == 3) rdA(std::integral_constant<int, 3>{});
                    if constexpr (j + 1 < 9) readB(order[j + 1], ks, Bq[(j + 1) % BD]);
                    __builtin_amdgcn_sched_barrier(0);
                    mfma6(acc[t_phase(sl)], A[t_pos(sl)], Bq[j % BD]);
                    __builtin_amdgcn_sched_barrier(0);
                });
            } else if constexpr (MODE == 1) {
                constexpr int order[9] = {0, 4, 6, 8, 1, 5, 7, 2, 3};
                short8 A[4][3];
                sfor<0, 4>([&](auto P) __attribute__((always_inline)) {
                    constexpr int pos = decltype(P)::value;
                    readA((rw + (pos >> 1)) * HC + m + (pos & 1), ks, A[pos]);
                });
                constexpr int BD = 2;   // B operand one slot ahead
                short8 Bq[BD][3];
                if constexpr (!C::WIN_REGS)
                    sfor<0, BD - 1>([&](auto P) __attribute__((always_inline)) {
                        readB(order[decltype(P)::value], ks, Bq[decltype(P)::value]);
                    });
                sfor<0, 9>([&](auto J) __attribute__((always_inline)) {
                    constexpr int j = decltype(J)::value, sl = order[j];
                    constexpr int ai = (sl == 1 || sl == 3) ? 4 : t_phase(sl), pos = t_pos(sl);
                    if constexpr (!C::WIN_REGS && j + BD - 1 < 9) readB(order[j + BD - 1], ks, Bq[(j + BD - 1) % BD]);
                    __builtin_amdgcn_sched_barrier(0);
                    if constexpr (C::WIN_REGS) mfma6(acc[ai], A[pos], wr6[sl]);
                    else mfma6(acc[ai], A[pos], Bq[j % BD]);
                    __builtin_amdgcn_sched_barrier(0);
                });
            } else {   // taps t = 3 ky + kx into acc[kx]; A of tap t + 1 read while tap t's MFMAs run
                static_assert(MODE != 0 || C::WIN_REGS, "x6 strided conv: single-chunk layers");
                short8 A0[3], A1[3];
                readA(hpix(2 * rw, 2 * m), ks, A0);
                sfor<0, 9>([&](auto T) __attribute__((always_inline)) {
                    constexpr int t = decltype(T)::value, ky = t / 3, kx = t % 3;
                    if constexpr (t + 1 < 9) {
                        constexpr int ky1 = (t + 1) / 3, kx1 = (t + 1) % 3;
                        if constexpr ((t & 1) == 0) readA(hpix(2 * rw + ky1, 2 * m + kx1), ks, A1);
                        else readA(hpix(2 * rw + ky1, 2 * m + kx1), ks, A0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    constexpr int ai = NACCS == 1 ? 0 : kx;
                    if constexpr ((t & 1) == 0) mfma6(acc[ai], A0, wr6[t]);
                    else mfma6(acc[ai], A1, wr6[t]);
                    __builtin_amdgcn_sched_barrier(0);
                });
            }
        });
      }
    };
    auto compute = [&]() __attribute__((always_inline)) {
        if constexpr (X6) {
            compute_x6();
        } else {
            f32x4 A0[NA], B0[NB], A1[NA], B1[NB];
            read_step(std::integral_constant<int, 0>{}, A0, B0);
            sfor<0, NSTEP>([&](auto U) __attribute__((always_inline)) {
                constexpr int u = decltype(U)::value;
                if constexpr (u + 1 < NSTEP) {
                    if constexpr (((u + 1) & 1) == 0) read_step(std::integral_constant<int, u + 1>{}, A0, B0);
                    else read_step(std::integral_constant<int, u + 1>{}, A1, B1);
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr ((u & 1) == 0) mfma_step(A0, B0);
                else mfma_step(A1, B1);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
    };

    // ---- epilogue of one tile ----------------------------------------------------------------------
    const int n = M::col(lane);
    const float bias = a.bias[n];
    const float2 bn = MODE == 0 ? a.bn_ab[n] : float2{1.f, 0.f};
    // CIN statistics into fixed-point accumulators (a.stat): per wave and tile a two-pass {S, M2} over the wave's
    // pixel row, summed per image as {S, M2 + S^2/n} (finalize_kernel's merge quantity: the sum of squares formed
    // around the row mean) in the wave's lanes < MS (lane = channel) — no cross-wave exchange per tile. At an
    // image change / the end (every thread, uniform) the four waves' sums meet in LDS in a fixed order and lanes
    // tid < NC add them to the accumulators.
    const bool to_acc = a.stat.acc != nullptr;
    double accS = 0.0, accQ = 0.0;
    int acc_b = -1;
    double* const red_d = reinterpret_cast<double*>(red);   // [NW waves][NC][2] at the flush
    auto acc_flush = [&]() __attribute__((always_inline)) {
        if (acc_b >= 0) {
            if (lane < MS) {
                red_d[(wave * NC + lane) * 2] = accS;
                red_d[(wave * NC + lane) * 2 + 1] = accQ;
            }
            lds_barrier();   // (the next write of red_d comes after the next step's top barrier)
            if (tid < NC) {
                const double S = wave_sum<NW>(red_d + tid * 2, 2 * NC);
                const double Q = wave_sum<NW>(red_d + tid * 2 + 1, 2 * NC);
                cin_acc_add(a.stat, a.batch, NC, acc_b, tid, (int)blockIdx.x % a.stat.nslot, S, Q);
            }
        }
        accS = accQ = 0.0;
    };
    const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
    // x6 transposed convs stage full tiles' output through LDS
    constexpr bool OSTAGE = X6 && MODE == 1 && LITE_OSTAGE;
    constexpr int OST_FL = C::OST_FL;   // floats per pixel row
    // x6 strided convs (contract_0 / _1, weights in VGPRs): the same for their one output row per wave
    constexpr bool OSTAGE0 = X6 && MODE == 0 && C::WIN_REGS && LITE_OSTAGE0;
    static_assert(!OSTAGE0 || 4 * TW * NC <= C::HALO, "output staging fits the halo image");
    static_assert(!OSTAGE || 4 * OST_FL <= C::BODY, "output staging fits the LDS body");
    auto epilogue = [&](const Tile& T) __attribute__((always_inline)) {
        if constexpr (MODE == 0) {   // bias + ReLU -> BatchNorm (inference affine) -> ReLU, NHWC store
            acc_t y;
            if constexpr (NACCS == 1) y = acc[0];
            else y = (acc[0] + acc[1]) + acc[2];
            const int oy = T.y0 + rw;
            const bool full = T.y0 + TH <= a.Ho && T.x0 + TW <= a.Wo;
            float* const orow = a.out + ((size_t)(T.b * a.Ho + oy) * a.Wo) * NC + n;
            if (OSTAGE0 && full) {   // the wave's TW x NC output row segment through LDS, 16 B per lane
#pragma unroll
                for (int j = 0; j < C::NACC; ++j) {
                    float v = fmaxf(y[j] + bias, 0.f);
                    y[j] = fmaxf(fmaf(bn.x, v, bn.y), 0.f);
                }
                lds_barrier();   // every wave's MFMA operand reads are done
                float* const ob = smem + rw * (TW * NC);
#pragma unroll
                for (int j = 0; j < C::NACC; ++j) ob[M::row(j, lane) * NC + n] = y[j];
                const size_t obase = ((size_t)(T.b * a.Ho + oy) * a.Wo + T.x0) * NC;
#pragma unroll
                for (int it = 0; it < TW * NC / 256; ++it) {
                    const int e = (it * 64 + lane) * 4;
                    const f32x4 v = *reinterpret_cast<const f32x4*>(ob + e);
                    if (a.wt_stores)
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), osrd, (int)((obase + e) * 4),
                                                               0, 16);
                    else
                        *reinterpret_cast<f32x4*>(a.out + obase + e) = v;
                }
                return;
            }
#pragma unroll
            for (int j = 0; j < C::NACC; ++j) {
                const int ox = T.x0 + M::row(j, lane);
                float v = fmaxf(y[j] + bias, 0.f);
                v = fmaxf(fmaf(bn.x, v, bn.y), 0.f);
                if (full || (oy < a.Ho && ox < a.Wo)) {
                    if (a.wt_stores)   // write-through (sc1): no dirty lines left for the end-of-kernel write-back
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), osrd,
                                                              (int)((orow + (size_t)ox * NC - a.out) * 4), 0, 16);
                    else
                        orow[(size_t)ox * NC] = v;
                }
            }
        } else {   // bias, pixel-shuffle store, per-tile CIN statistics over the four phases
            if constexpr (NACCS == 5) acc[0] = acc[0] + acc[4];
            const int p = T.y0 + rw;
            const int Ho2 = 2 * a.Ho, Wo2 = 2 * a.Wo;
            // interior tiles (every pixel inside) store without per-element guards
            const bool full = T.y0 + TH <= a.Ho && T.x0 + TW <= a.Wo;
            float* const orow = a.out + ((size_t)(T.b * Ho2 + 2 * p) * Wo2) * NC + n;
            // the phases [P0, P0 + NPHW) this wave finishes: all four, or (K split) output row py = kh's two
            constexpr int NPHW = 4 / C::KSPLIT;
            if constexpr (C::KSPLIT == 2) {
                // the two K halves of a pixel row meet: wave (rw, kh) hands its partial sums of the partner's output row
                // (phases 2 - 2 kh, 3 - 2 kh) to the partner through LDS (the halo / weight images are dead after the
                // barrier) and adds the partner's partials of its own row, which it keeps in acc[0..1]; float adds
                // commute, so both sides form the same sums. Selects on values, not on accumulator indices: a
                // kh-dependent index would put the accumulators in scratch.
                lds_barrier();   // every wave's MFMA operand reads are done
                f32x4* const xw = reinterpret_cast<f32x4*>(smem) + (size_t)wave * (2 * C::NACC / 4) * 64 + lane;
                const f32x4* const xr = reinterpret_cast<const f32x4*>(smem) + (size_t)(wave ^ 4) * (2 * C::NACC / 4) * 64 + lane;
                const bool hi = kh != 0;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j4 = 0; j4 < C::NACC / 4; ++j4) {
                        f32x4 v;
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = hi ? acc[i][4 * j4 + e] : acc[2 + i][4 * j4 + e];
                        xw[(i * (C::NACC / 4) + j4) * 64] = v;
                    }
                lds_barrier();
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j4 = 0; j4 < C::NACC / 4; ++j4) {
                        const f32x4 v = xr[(i * (C::NACC / 4) + j4) * 64];
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            acc[i][4 * j4 + e] = (hi ? acc[2 + i][4 * j4 + e] : acc[i][4 * j4 + e]) + v[e];
                    }
                lds_barrier();   // the output staging below reuses the exchange area
            }
            // output row (0 / 1 of the pixel row's two) of this wave's local phase ph: K split, all in row kh
            auto prow = [&](int ph) __attribute__((always_inline)) { return C::KSPLIT == 2 ? kh : ph >> 1; };
            auto finish = [&](auto PH0) __attribute__((always_inline)) {
            constexpr int P0 = decltype(PH0)::value;
            float s = 0.f, cnt = 0.f;
            if (full && OSTAGE) {
                // x6: the wave's output rows x 2 TW pixels x NC channels through LDS (the tile's halo / weight
                // images are dead after the barrier), then stored as whole 128-B lines, 16 B per lane: 4x fewer
                // store instructions than the per-accumulator dword stores, no half-line writes
#pragma unroll
                for (int ph = P0; ph < P0 + NPHW; ++ph)
#pragma unroll
                    for (int j = 0; j < C::NACC; ++j) {
                        acc[ph][j] += bias;
                        s += acc[ph][j];
                    }
                cnt = (float)NPHW * C::NACC;
                if constexpr (C::KSPLIT == 1) lds_barrier();   // every wave's MFMA operand reads are done
                float* const ob = smem + rw * OST_FL;
#pragma unroll
                for (int ph = P0; ph < P0 + NPHW; ++ph)
#pragma unroll
                    for (int j = 0; j < C::NACC; ++j)
                        ob[(prow(ph) * 2 * TW + 2 * M::row(j, lane) + (ph & 1)) * NC + n] = acc[ph][j];
                constexpr int ROWF = 2 * TW * NC;   // floats of one output row segment (contiguous in NHWC)
#pragma unroll
                for (int pr = 0; pr < NPHW / 2; ++pr) {
                    const int py = C::KSPLIT == 2 ? kh : pr;
                    const size_t obase = ((size_t)(T.b * Ho2 + 2 * p + py) * Wo2 + 2 * T.x0) * NC;
#pragma unroll
                    for (int it = 0; it < ROWF / 256; ++it) {
                        const int e = (it * 64 + lane) * 4;
                        const f32x4 v = *reinterpret_cast<const f32x4*>(ob + py * ROWF + e);
                        if (a.wt_stores)
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), osrd,
                                                                   (int)((obase + e) * 4), 0, 16);
                        else
                            *reinterpret_cast<f32x4*>(a.out + obase + e) = v;
                    }
                }
            } else if (full) {
#pragma unroll
                for (int ph = P0; ph < P0 + NPHW; ++ph)
#pragma unroll
                    for (int j = 0; j < C::NACC; ++j) {
                        const int qq = T.x0 + M::row(j, lane);
                        const float v = acc[ph][j] + bias;
                        acc[ph][j] = v;
                        if (a.wt_stores)
                            __builtin_amdgcn_raw_buffer_store_b32(
                                __builtin_bit_cast(unsigned, v), osrd,
                                (int)((orow + ((size_t)prow(ph) * Wo2 + 2 * qq + (ph & 1)) * NC - a.out) * 4), 0, 16);
                        else
                            orow[((size_t)prow(ph) * Wo2 + 2 * qq + (ph & 1)) * NC] = v;
                        s += v;
                    }
                cnt = (float)NPHW * C::NACC;
            } else {
#pragma unroll
                for (int ph = P0; ph < P0 + NPHW; ++ph)
#pragma unroll
                    for (int j = 0; j < C::NACC; ++j) {
                        const int qq = T.x0 + M::row(j, lane);
                        const float v = acc[ph][j] + bias;
                        acc[ph][j] = v;
                        if (p < a.Ho && qq < a.Wo) {
                            orow[((size_t)prow(ph) * Wo2 + 2 * qq + (ph & 1)) * NC] = v;
                            s += v;
                            cnt += 1.f;
                        }
                    }
            }
            if (to_acc) {   // per-wave two-pass partials (see acc_flush)
                if constexpr (MS == 16) {
                    s = lane_xor_sum<16>(s);
                    cnt = lane_xor_sum<16>(cnt);
                }
                s = lane_xor_sum<32>(s);
                cnt = lane_xor_sum<32>(cnt);
                const float mean = cnt > 0.f ? s / cnt : 0.f;
                float m2 = 0.f;
#pragma unroll
                for (int ph = P0; ph < P0 + NPHW; ++ph)
#pragma unroll
                    for (int j = 0; j < C::NACC; ++j) {
                        const int qq = T.x0 + M::row(j, lane);
                        const float d = acc[ph][j] - mean;
                        if (full || (p < a.Ho && qq < a.Wo)) m2 = fmaf(d, d, m2);
                    }
                if constexpr (MS == 16) m2 = lane_xor_sum<16>(m2);
                m2 = lane_xor_sum<32>(m2);
                if (T.b != acc_b) {   // uniform over the workgroup
                    acc_flush();
                    acc_b = T.b;
                }
                if (lane < MS) {
                    const double dS = (double)s;
                    accS += dS;
                    if (cnt > 0.f) accQ += (double)m2 + dS * dS / (double)cnt;
                }
            } else if (a.part != nullptr) {
                // lanes n, n + MS, ... hold column n: reduce over them, then over the NW waves (fixed order)
                if constexpr (MS == 16) {
                    s = lane_xor_sum<16>(s);
                    cnt = lane_xor_sum<16>(cnt);
                }
                s = lane_xor_sum<32>(s);
                cnt = lane_xor_sum<32>(cnt);
                if (lane < MS) {
                    red[wave * NC + n] = s;
                    red[NW * NC + wave * NC + n] = cnt;
                }
                lds_barrier();
                const float S = wave_sum<NW>(red + n, NC);
                const float N = wave_sum<NW>(red + NW * NC + n, NC);
                const float mean = N > 0.f ? S / N : 0.f;
                float m2 = 0.f;
#pragma unroll
                for (int ph = P0; ph < P0 + NPHW; ++ph)
#pragma unroll
                    for (int j = 0; j < C::NACC; ++j) {
                        const int qq = T.x0 + M::row(j, lane);
                        const float d = acc[ph][j] - mean;
                        if (full || (p < a.Ho && qq < a.Wo)) m2 = fmaf(d, d, m2);
                    }
                if constexpr (MS == 16) m2 = lane_xor_sum<16>(m2);
                m2 = lane_xor_sum<32>(m2);
                if (lane < MS) red[2 * NW * NC + wave * NC + n] = m2;   // its own rows: no barrier before the write
                lds_barrier();
                if (tid < NC) {   // lane tid < NC holds column tid
                    const float M2 = wave_sum<NW>(red + 2 * NW * NC + tid, NC);
                    const int n_part = a.tiles_y * a.tiles_x;
                    a.part[((size_t)T.b * NC + tid) * n_part + T.ty * a.tiles_x + T.tx] = make_float4(S, M2, N, 0.f);
                }
            }
            };
            finish(std::integral_constant<int, 0>{});   // (K split: the wave's own phases sit in acc[0..1])
        }
    };

    // ---- main loop over (tile, chunk) steps: step s+1's global loads are in flight while step s
    // computes and (last chunk) stores its tile ---------------------------------------------------------
    if constexpr (NCH == 1 && !C::WIN_REGS) {   // one weight image for every tile: staged once
        for (int it = tid; it < C::WITEMS; it += NT)
            reinterpret_cast<f32x4*>(wts)[it] = reinterpret_cast<const f32x4*>(a.wpk)[it];
    }
    // the prologue affine of every image into the LDS table: given, or formed from the producer's fixed-point
    // accumulators (no finalize ran). One image: the accumulator loads go out first (fill_issue, CinAffineSplit) and
    // are merged after the first tiles' input loads are issued (fill_table), so their wait excludes those loads'
    // latency (vmcnt retires in issue order); more images: cin_affine_table after the input loads
    // (not the x6 single-chunk layers, whose weights live in VGPRs: the split form's 24 registers held across the
    // first input loads took expand_1 from 2 waves per SIMD to 1, 21.2 -> 28.3 us in the frame, profiles/r05)
    constexpr bool SPLIT_OK = !C::WIN_REGS;
    const bool split_aff = SPLIT_OK && PRO != PRO_NONE && a.pro_stat.acc != nullptr && a.batch == 1 &&
                           CinAffineSplit<NT, 2>::usable(a.pro_stat);
    CinAffineSplit<NT, 2> aff;
    auto fill_issue = [&]() __attribute__((always_inline)) {
        if constexpr (PRO != PRO_NONE)
            if constexpr (SPLIT_OK)
                if (split_aff) aff.issue(a.pro_stat, 0, BLEND);
    };
    auto fill_table = [&]() __attribute__((always_inline)) {
    if constexpr (PRO != PRO_NONE) {
        const CinSrc& ps = a.pro_stat;
        if (ps.acc != nullptr) {
            const bool store = blockIdx.x == 0;   // the host-visible copy (rst_copy_activation)
            if (SPLIT_OK && split_aff)
                aff.finish(ps, tab, BLEND ? tab + CIN : nullptr, store ? ps.ab_out : nullptr, store ? ps.ab1_out : nullptr);
            else
                cin_affine_table<NT, SPLIT_OK ? 8 : 1>(ps, 0, a.batch, tab, BLEND ? tab + a.batch * CIN : nullptr,
                                      store ? ps.ab_out : nullptr, store ? ps.ab1_out : nullptr);
        } else {
            for (int i = tid; i < a.batch * CIN; i += NT) {
                tab[i] = a.pro_ab[i];
                if constexpr (BLEND) tab[a.batch * CIN + i] = a.pro_ab1[i];
            }
        }
        lds_barrier();
    }
    };
    const int my_tiles = (n_tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    // the next layer's weights into this XCD's L2, touched as the workgroup starts its last tile(s) so that this
    // kernel's own stream does not evict them again (speed only)
    l2_touch_t l2f = {0u, 0u};
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, NSET - 1>;
    zero_acc();
    if constexpr (NCH == 1 && NSET == 2) {
        // tile k's input sits in register set k & 1, loaded two tiles ahead
        Tile T0 = tile_of(0), T1 = T0;
        fill_issue();
        load_in(T0, 0, S0{});
        if (my_tiles > 1) {
            T1 = tile_of(1);
            load_in(T1, 0, S1{});
        }
        fill_table();
        load_aff(T0, 0, S0{});
        if (my_tiles > 1) load_aff(T1, 0, S1{});
        for (int k = 0; k < my_tiles; k += 2) {
            LTL(k, 0);
            if (k + 2 >= my_tiles) l2f = l2_touch_xcd_slice<NT, 2>(a.w_next, a.w_next_bytes);
            if (k > 0) lds_barrier();
            store_step(T0, S0{});
            lds_barrier();
            LTL(k, 1);
            Tile T2 = T0;
            if (k + 2 < my_tiles) {
                T2 = tile_of(k + 2);
                load_step(T2, 0, S0{});
            }
            compute();
            LTL(k, 2);
            epilogue(T0);
            zero_acc();
            LTL(k, 3);
            if (k + 1 < my_tiles) {
                lds_barrier();
                store_step(T1, S1{});
                lds_barrier();
                Tile T3 = T1;
                if (k + 3 < my_tiles) {
                    T3 = tile_of(k + 3);
                    load_step(T3, 0, S1{});
                }
                compute();
                epilogue(T1);
                zero_acc();
                T1 = T3;
            }
            T0 = T2;
        }
    } else {   // multi-chunk layers, and single-chunk layers with one register set (x6: weights in VGPRs)
        const int n_steps = my_tiles * NCH;
        Tile cur = tile_of(0);
        fill_issue();
        load_in(cur, 0, S0{});
        fill_table();
        load_aff(cur, 0, S0{});
        for (int s = 0; s < n_steps; ++s) {
            const int ch = s % NCH;
            LTL(s, 0);
            if (s == n_steps - NCH) l2f = l2_touch_xcd_slice<NT, 2>(a.w_next, a.w_next_bytes);
            if (s > 0) lds_barrier();        // the previous step's operand reads are done
            store_step(cur, S0{});
            if constexpr (C::WDMA) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this chunk's weights have landed
            lds_barrier();
            LTL(s, 1);
            Tile nxt = cur;
            if (s + 1 < n_steps) {
                const int ch1 = (s + 1) % NCH;
                if (ch1 == 0) nxt = tile_of((s + 1) / NCH);
                load_step(nxt, ch1, S0{}, ch1 & 1);
            }
            wbuf = ch & 1;
            compute();
            LTL(s, 2);
            if (ch == NCH - 1) {
                epilogue(cur);
                zero_acc();
            }
            LTL(s, 3);
            cur = nxt;
        }
    }
    if (to_acc) acc_flush();
    LT0(1);
    l2_touch_keep(l2f, a.batch < 0, smem);
    tl_stamp_end(a.tl);
}

// ------------------------------------------------------------------------------------------------
// host side: the instantiated layer shapes
// ------------------------------------------------------------------------------------------------
#define RST_LITE_CONFIGS(X)        \
    X(1, 0, 32, 16, 32, 0)         \
    X(2, 0, 16, 32, 16, 0)         \
    X(3, 1, 128, 32, 32, 0)        \
    X(4, 1, 32, 16, 32, 0)         \
    X(5, 1, 128, 32, 32, 1)        \
    X(6, 0, 32, 16, 32, 1)         \
    X(7, 0, 16, 32, 16, 1)         \
    X(8, 1, 32, 16, 32, 1)

bool conv_lite_select(int keras_kind, int k, int stride, int cin, int cout, bool x6, LiteTile* t) {
    if (k != 3 || stride != 2) return false;
    // split-bf16 x6 where an instantiation exists (expand_0), the f32 form otherwise
    for (int pass = x6 ? 1 : 0; pass >= 0; --pass) {
#define X(ID, MODE, CIN, NC, CKC, X6)                                              \
        if (X6 == pass && keras_kind == MODE && cin == CIN && cout == NC) {            \
            using C = lite::Cfg<MODE, CIN, NC, CKC, X6>;                               \
            t->id = ID; t->mode = MODE; t->cin = CIN; t->nc = NC; t->ckc = CKC;        \
            t->th = C::TH; t->tw = C::TW; t->lds_bytes = (int)C::LDS_BYTES; t->x6 = X6; \
            return true;                                                               \
        }
        RST_LITE_CONFIGS(X)
#undef X
    }
    return false;
}

// weights: Conv2D HWIO [ky][kx][ci][co]; Conv2DTranspose [ky][kx][co][ci] (Keras layouts) ->
// [chunk][slot][r][kslot][n][4], the LDS image of one chunk
static uint16_t lite_bf16_rne(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static float lite_bf16_val(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static float lite_slot_weight(const LiteTile& t, const float* kern, int s, int ci, int n) {
    if (t.mode == 0) return kern[((size_t)s * t.cin + ci) * t.nc + n];
    const int ph = lite::t_phase(s), pos = lite::t_pos(s);
    const int py = ph >> 1, px = ph & 1, tyy = pos >> 1, txx = pos & 1;
    const int ky = py + 2 * (1 - tyy), kx = px + 2 * (1 - txx);
    return kern[(((size_t)ky * 3 + kx) * t.nc + n) * t.cin + ci];
}

std::vector<float> conv_lite_pack_weights(const LiteTile& t, const float* kern) {
    if (t.x6) {   // [chunk][slot][K step][piece][lane group][n][8] bf16, each weight split into 3 RNE pieces
        const int kstep = t.nc == 32 ? 16 : 32, ng = kstep / 8, nch = t.cin / t.ckc, ks2 = t.ckc / kstep;
        std::vector<uint16_t> img((size_t)nch * 9 * ks2 * 3 * ng * t.nc * 8);
        size_t idx = 0;
        for (int ch = 0; ch < nch; ++ch)
            for (int s = 0; s < 9; ++s)
                for (int k2 = 0; k2 < ks2; ++k2)
                    for (int pc = 0; pc < 3; ++pc)
                        for (int kg = 0; kg < ng; ++kg)
                            for (int n = 0; n < t.nc; ++n)
                                for (int e = 0; e < 8; ++e) {
                                    const float v = lite_slot_weight(t, kern, s, ch * t.ckc + k2 * kstep + kg * 8 + e, n);
                                    uint16_t p[3];
                                    p[0] = lite_bf16_rne(v);
                                    const float r = v - lite_bf16_val(p[0]);
                                    p[1] = lite_bf16_rne(r);
                                    p[2] = lite_bf16_rne(r - lite_bf16_val(p[1]));
                                    img[idx++] = p[pc];
                                }
        std::vector<float> out(img.size() / 2);
        std::memcpy(out.data(), img.data(), img.size() * 2);
        return out;
    }
    const int ks = 64 / t.nc, nch = t.cin / t.ckc, R = t.ckc / 4 / ks;
    std::vector<float> out((size_t)nch * 9 * t.ckc * t.nc);
    size_t idx = 0;
    for (int ch = 0; ch < nch; ++ch)
        for (int s = 0; s < 9; ++s)
            for (int r = 0; r < R; ++r)
                for (int g = 0; g < ks; ++g)
                    for (int n = 0; n < t.nc; ++n)
                        for (int i = 0; i < 4; ++i) {
                            const int ci = ch * t.ckc + 4 * (g + ks * r) + i;
                            if (t.mode == 0) {
                                out[idx++] = kern[((size_t)s * t.cin + ci) * t.nc + n];
                            } else {
                                const int ph = lite::t_phase(s), pos = lite::t_pos(s);
                                const int py = ph >> 1, px = ph & 1, tyy = pos >> 1, txx = pos & 1;
                                const int ky = py + 2 * (1 - tyy), kx = px + 2 * (1 - txx);
                                out[idx++] = kern[(((size_t)ky * 3 + kx) * t.nc + n) * t.cin + ci];
                            }
                        }
    return out;
}

#ifdef LITE_PROF
void lite_timeline_print(int nsteps) {
    std::vector<unsigned long long> tl((size_t)64 * 8 * 16 * 4);
    if (hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(lite_tl), tl.size() * 8) != hipSuccess) return;
    double d[3] = {0, 0, 0}, gap = 0;
    int n = 0, ng = 0;
    for (int g = 0; g < 64; ++g)
        for (int w = 0; w < 8; ++w)
            for (int st = 0; st < nsteps && st < 16; ++st) {
                const unsigned long long* q = &tl[(((size_t)g * 8 + w) * 16 + st) * 4];
                if (q[0] == 0 || q[3] < q[0]) continue;
                for (int k = 0; k < 3; ++k) d[k] += (double)(q[k + 1] - q[k]);
                ++n;
                if (st + 1 < nsteps && st + 1 < 16) {
                    const unsigned long long* q1 = q + 4;
                    if (q1[0] >= q[3] && q1[0] != 0) { gap += (double)(q1[0] - q[3]); ++ng; }
                }
            }
    if (n) printf("    per step (100 cycles): staging+barrier %.2f, MFMA %.2f, epilogue %.2f (n=%d)\n", d[0] / n * 0.01,
                  d[1] / n * 0.01, d[2] / n * 0.01, n);
    std::vector<unsigned long long> t0((size_t)64 * 8 * 2);
    if (hipMemcpyFromSymbol(t0.data(), HIP_SYMBOL(lite_t0), t0.size() * 8) == hipSuccess) {
        double fill = 0, span = 0;
        int nw = 0;
        for (int g = 0; g < 64; ++g)
            for (int w = 0; w < 8; ++w) {
                const unsigned long long s0 = t0[(g * 8 + w) * 2], s1 = t0[(g * 8 + w) * 2 + 1];
                const unsigned long long f = tl[(((size_t)g * 8 + w) * 16) * 4];
                if (s0 == 0 || s1 < s0 || f < s0) continue;
                fill += (double)(f - s0);
                span += (double)(s1 - s0);
                ++nw;
            }
        if (nw) printf("    per wave (100 cycles): start -> first step %.2f, start -> end %.2f\n", fill / nw * 0.01,
                       span / nw * 0.01);
    }
    std::vector<unsigned long long> z(tl.size(), 0);   // clear for the next measured launch
    (void)hipMemcpyToSymbol(HIP_SYMBOL(lite_tl), z.data(), z.size() * 8);
}
#endif

// persistent grid: every CU holds as many workgroups as LDS and registers allow (queried once per
// instantiation at prepare time), rounded to a multiple of the 8 XCDs; never more than the tiles
static int lite_cu_count() {
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    return n_cu;
}

// LDS past the kernel's fixed image: the prologue affine table [batch][CIN] (two styles: both)
static size_t lite_tab_bytes(int pro, int cin, int batch) {
    const int p = pro & 7;
    return p == PRO_NONE ? 0 : (size_t)batch * cin * sizeof(float2) * ((pro & LITE_BLEND) ? 2 : 1);
}
constexpr int LITE_MAX_TAB_BATCH = LITE_MAX_BATCH;

template <int MODE, int CIN, int NC, int CKC, int PRO, int X6, int KSP>
static int lite_slots() {
    static int slots = 0;
    if (slots == 0) {
        using C = lite::Cfg<MODE, CIN, NC, CKC, X6, KSP>;
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_lite_kernel<MODE, CIN, NC, CKC, PRO, X6, KSP>, C::NT,
                                                         C::LDS_BYTES + lite_tab_bytes(PRO, CIN, 1)) != hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        slots = ((lite_cu_count() * per_cu) / 8) * 8;
        if (slots <= 0) slots = 8;
    }
    return slots;
}

template <int MODE, int CIN, int NC, int CKC, int PRO, int X6, int KSP>
static void lite_launch_pro(const ConvArgs& a, int n_tiles, hipStream_t st) {
    using C = lite::Cfg<MODE, CIN, NC, CKC, X6, KSP>;
    const int grid = std::min(n_tiles, lite_slots<MODE, CIN, NC, CKC, PRO, X6, KSP>());
    hipLaunchKernelGGL((conv_lite_kernel<MODE, CIN, NC, CKC, PRO, X6, KSP>), dim3(grid), dim3(C::NT),
                       C::LDS_BYTES + lite_tab_bytes(PRO, CIN, a.batch), st, a, n_tiles);
}

// the K-split form (x6 multi-chunk transposed convs) exists, and its LDS with the prologue table of `batch` images fits
template <int MODE, int CIN, int NC, int CKC, int X6>
static constexpr bool lite_ksplit_ok() {
    return X6 && MODE == 1 && CIN / CKC > 1 && CIN / CKC % 2 == 0 && CKC % (2 * (NC == 32 ? 16 : 32)) == 0;
}
static bool lite_ksplit_env() {   // RST_LITE_KSPLIT=0: the four-wave form everywhere (A/B measurements)
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("RST_LITE_KSPLIT");
        v = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

template <int MODE, int CIN, int NC, int CKC, int X6, int KSP>
static void lite_launch_sel(const ConvArgs& a, int n_tiles, int pro, hipStream_t st) {
    switch (pro) {
        case PRO_NONE: lite_launch_pro<MODE, CIN, NC, CKC, PRO_NONE, X6, KSP>(a, n_tiles, st); break;
        case PRO_AFF_RELU: lite_launch_pro<MODE, CIN, NC, CKC, PRO_AFF_RELU, X6, KSP>(a, n_tiles, st); break;
        case PRO_AFF_RES: lite_launch_pro<MODE, CIN, NC, CKC, PRO_AFF_RES, X6, KSP>(a, n_tiles, st); break;
        case PRO_AFF_RELU | LITE_BLEND: lite_launch_pro<MODE, CIN, NC, CKC, PRO_AFF_RELU | LITE_BLEND, X6, KSP>(a, n_tiles, st); break;
        case PRO_AFF_RES | LITE_BLEND: lite_launch_pro<MODE, CIN, NC, CKC, PRO_AFF_RES | LITE_BLEND, X6, KSP>(a, n_tiles, st); break;
    }
}

template <int MODE, int CIN, int NC, int CKC, int X6>
static hipError_t lite_launch_cfg(const ConvArgs& a, hipStream_t st) {
    using C = lite::Cfg<MODE, CIN, NC, CKC, X6>;
    if (a.cin != CIN || a.cout != NC || a.tiles_y != (a.Ho + C::TH - 1) / C::TH ||
        a.tiles_x != (a.Wo + C::TW - 1) / C::TW || (size_t)a.batch * a.H * a.W * CIN >= ((size_t)1 << 31))
        return hipErrorInvalidValue;   // 32-bit staging offsets
    if (a.batch > LITE_MAX_TAB_BATCH && a.pro_mode != PRO_NONE) return hipErrorInvalidValue;   // LDS affine table
    if (a.stat.acc != nullptr && (MODE != 1 || a.stat.nslot < 1 || a.stat.nslot > CIN_ACC_MAX_SLOTS))
        return hipErrorInvalidValue;
    const bool src_acc = a.pro_stat.acc != nullptr;
    if (src_acc && (a.pro_stat.nslot < 1 || a.pro_stat.nslot > CIN_ACC_MAX_SLOTS || a.pro_stat.C != CIN ||
                    a.pro_stat.batch != a.batch || a.pro_stat.style == nullptr || a.pro_mode == PRO_NONE))
        return hipErrorInvalidValue;
    const int n_tiles = a.batch * a.tiles_y * a.tiles_x;
    int pro = a.pro_mode;
    if (a.pro_w != nullptr) {   // two styles
        if (src_acc ? a.pro_stat.style1_offset < 0 : (a.pro_ab1 == nullptr || a.pro_ab == nullptr))
            return hipErrorInvalidValue;
        if (pro != PRO_AFF_RELU && pro != PRO_AFF_RES) return hipErrorInvalidValue;
        pro |= LITE_BLEND;
    } else if (pro != PRO_NONE && pro != PRO_AFF_RELU && pro != PRO_AFF_RES) {
        return hipErrorInvalidValue;
    }
    if constexpr (lite_ksplit_ok<MODE, CIN, NC, CKC, X6>()) {
        using K = lite::Cfg<MODE, CIN, NC, CKC, X6, 2>;
        if (lite_ksplit_env() && K::LDS_BYTES + lite_tab_bytes(pro, CIN, a.batch) <= 160 * 1024) {
            lite_launch_sel<MODE, CIN, NC, CKC, X6, 2>(a, n_tiles, pro, st);
            return hipGetLastError();
        }
    }
    lite_launch_sel<MODE, CIN, NC, CKC, X6, 1>(a, n_tiles, pro, st);
    return hipGetLastError();
}

template <int MODE, int CIN, int NC, int CKC, int X6, int KSP>
static hipError_t lite_prepare_ksp() {
    using C = lite::Cfg<MODE, CIN, NC, CKC, X6, KSP>;
    for (const void* k : {(const void*)conv_lite_kernel<MODE, CIN, NC, CKC, PRO_NONE, X6, KSP>,
                          (const void*)conv_lite_kernel<MODE, CIN, NC, CKC, PRO_AFF_RELU, X6, KSP>,
                          (const void*)conv_lite_kernel<MODE, CIN, NC, CKC, PRO_AFF_RES, X6, KSP>,
                          (const void*)conv_lite_kernel<MODE, CIN, NC, CKC, PRO_AFF_RELU | LITE_BLEND, X6, KSP>,
                          (const void*)conv_lite_kernel<MODE, CIN, NC, CKC, PRO_AFF_RES | LITE_BLEND, X6, KSP>}) {
        const size_t bytes = std::min<size_t>(C::LDS_BYTES + lite_tab_bytes(PRO_AFF_RELU | LITE_BLEND, CIN, LITE_MAX_TAB_BATCH),
                                              160 * 1024);
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return e;
    }
    // occupancy queries outside any graph capture
    lite_slots<MODE, CIN, NC, CKC, PRO_NONE, X6, KSP>();
    lite_slots<MODE, CIN, NC, CKC, PRO_AFF_RELU, X6, KSP>();
    lite_slots<MODE, CIN, NC, CKC, PRO_AFF_RES, X6, KSP>();
    lite_slots<MODE, CIN, NC, CKC, PRO_AFF_RELU | LITE_BLEND, X6, KSP>();
    lite_slots<MODE, CIN, NC, CKC, PRO_AFF_RES | LITE_BLEND, X6, KSP>();
    return hipSuccess;
}

template <int MODE, int CIN, int NC, int CKC, int X6>
static hipError_t lite_prepare_cfg() {
    const hipError_t e = lite_prepare_ksp<MODE, CIN, NC, CKC, X6, 1>();
    if (e != hipSuccess) return e;
    if constexpr (lite_ksplit_ok<MODE, CIN, NC, CKC, X6>()) return lite_prepare_ksp<MODE, CIN, NC, CKC, X6, 2>();
    return hipSuccess;
}

hipError_t conv_lite_launch(const LiteTile& t, const ConvArgs& a, hipStream_t st) {
    switch (t.id) {
#define X(ID, MODE, CIN, NC, CKC, X6) \
    case ID: return lite_launch_cfg<MODE, CIN, NC, CKC, X6>(a, st);
        RST_LITE_CONFIGS(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

hipError_t conv_lite_prepare(const LiteTile& t) {
    switch (t.id) {
#define X(ID, MODE, CIN, NC, CKC, X6) \
    case ID: return lite_prepare_cfg<MODE, CIN, NC, CKC, X6>();
        RST_LITE_CONFIGS(X)
#undef X
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rst
