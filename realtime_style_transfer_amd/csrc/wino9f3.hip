// wino9f3.hip — the network's first layer ("contract_start": Conv2D 9x9 s1 SAME, cin <= 17 -> 32 channels, built-in
// ReLU, then the inference BatchNormalization (folded moving statistics) and ReLU; realtime_style_transfer/models/
// styleTransfer.py:188-205, 225-226) as nine 3x3 sub-kernels g_ab (taps 3a..3a+2, 3b..3b+2) on Winograd F(3x3, 3x3)
// tiles, with the transform-domain products on the bf16 MFMA pipe at fp32-level accuracy (every operand split exactly
// into three bf16 pieces, six product terms, fp32 accumulation; the scheme of wino_x6.hip / wino9_x6.hip).
//
// Why F(3x3, 3x3) here: the sub-kernels sit 3 pixels apart, which is exactly the F(3,3) tile pitch, so sub-kernel
// (a, b) of output tile T reads the input tile T + (a, b) of ONE tile grid. A workgroup's 8 x 8 output tiles (24 x 24
// pixels) need the input transforms V of a 10 x 10 tile grid once each (100 tile transforms serve 576 sub-kernel
// uses), where the F(2x2) composite of wino9_x6.hip transforms a tile per sub-kernel use (9 x 64 per 16 x 16 pixels):
// 8.3x less transform + split VALU per output pixel, and 25 products per 9 pixels instead of 16 per 4 (0.69x the
// MFMAs). The transform VALU bounded wino9_x6 (18 us of loop per 16 x 16 block against 10.5 us without it).
//
// Points {0, 1, -1, 2, inf} (Toom-Cook, transposed): B^T = [[2,-1,-2,1,0],[0,2,1,-1,0],[0,-2,3,-1,0],[0,-1,0,1,0],
// [0,2,-1,-2,1]] (integers: V = B^T d B in f32), G = [[1/2,0,0],[1/2,1/2,1/2],[1/6,-1/6,1/6],[1/6,1/3,2/3],[0,0,1]]
// (U = G g G^T formed on the host in f64, rounded once to f32, split), A^T = [[1,1,1,1,0],[0,1,-1,2,0],[0,1,1,4,1]].
// f32 emulation of the whole layer (round-off of V, of the accumulation and of the output transform): max relative
// error 5.5e-7 of the output range against f64, F(2x2) composite 1.8e-7 (both far below the 1e-5 start-conv bar).
//
// Workgroup = 8 waves (two per SIMD), persistent over 24 x 24-pixel blocks (two 32-tile M blocks of 4 x 8 tiles);
// lane li of an MFMA feeds tile (row li & 3, column li >> 2) of its M block (column-major: the V reads then hit at
// most two lanes per bank group with the dense 10-tile V row pitch). Accumulators: 25 points x 2 blocks = 50 32 x 32
// tiles; wave w owns points w, w + 8, w + 16 (both blocks), waves 6 / 7 also point 24 of block 0 / 1 (13 + 13 + 12 + 12
// per SIMD). Input channels in three chunks: A = 0..7, B = 8..15, C = 16. Per chunk: the patch (32 x 32 pixels x 8
// channels, f32) is staged in LDS, one thread per (V tile, channel pair) forms B^T d B for all 25 points, splits it into
// three bf16 pieces and writes the V image [piece][point][tile][8 ch] (120 KB); then the MFMA phase runs K-steps of
// 16 = two sub-kernels x 8 channels (lane half lh reads sub-kernel 2ks + lh at its shifted tile: one ds_read_b128 per
// piece). Chunk C (one channel) puts the nine sub-kernels into one K-step (V16 image [point][tile][3 pieces], eight
// 8-B reads per lane). U (825 KB, [K-step slot][point][piece][co][16 K] bf16) streams from L2, one 1 KB block per wave
// load feeding both M blocks. Epilogue per M block: accumulators -> LDS M image [point][tile][co], output transform per
// (tile, channel), bias -> ReLU -> BN -> ReLU, stores. The next block's input loads are issued at the epilogue start
// (no U loads behind them there: vmcnt retires in order).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace rst {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int FT = 24;                       // output pixels per block side (8 F(3,3) tiles)
constexpr int FP = 32;                       // input patch side (block + 8)
constexpr int NV = 10;                       // V tile grid side
constexpr int NVT = NV * NV;                 // 100 V tiles
constexpr int NXI = 25;                      // transform points
constexpr int NCO = 32;                      // output channels
constexpr int RP = 272;                      // patch row pitch (floats): 32 pixels x 8 channels + 16 (conflict-free reads)
constexpr int RPC = 33;                      // channel-16 patch row pitch (floats)
constexpr int VPLANE = NVT * 16;             // bytes per (piece, point): 100 tiles x 8 channels bf16
constexpr int VBYTES = 3 * NXI * VPLANE;     // 120000: the V image of one 8-channel chunk
constexpr int V16BYTES = NXI * NVT * 8;      // 20000: channel 16's V [point][tile] {p0 | p1, p2}
constexpr int PATCH_OFF = VBYTES;            // [32][272] f32
constexpr int PATCHC_OFF = PATCH_OFF + FP * RP * 4;   // [32][33] f32 (channel 16)
constexpr int PARAM_OFF = PATCHC_OFF + FP * RPC * 4;  // bias [32] + BN affine [32] float2 (the epilogue reads them
                                                      // from LDS: a global load there would wait, vmcnt being in
                                                      // order, for the next unit's input prefetch issued before it)
constexpr int LDS_BYTES = PARAM_OFF + NCO * 12;       // 159424
constexpr int MP = 36;                       // M image [xi][co][tile]: tile pitch (floats; 16-B aligned b128 writes)
static_assert(NXI * 32 * MP * 4 <= VBYTES, "M image of one block fits the V region");
static_assert(V16BYTES <= VBYTES, "V16 fits the V region");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
constexpr int UBLK = 1024;                   // bytes per U block: 32 co x 16 K (points 0..23) / 16 co x 32 K (24) bf16
constexpr int NSLOT = 11;                    // K-step slots: chunk A ks 0..4, chunk B ks 0..4, chunk C
constexpr int NXM = 24;                      // points on 32x32x16 tiles (point 24: 16x16x32 tiles)
constexpr int NSLOT24 = 7;                   // point 24's K-step slots: chunk A ks 0..2, chunk B ks 0..2, chunk C
constexpr int U24_OFF = NSLOT * NXM * 3 * UBLK;           // 792 KB
constexpr int U_BYTES = U24_OFF + NSLOT24 * 3 * 2 * UBLK;   // + 42 KB
constexpr int NTHR = 512;

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

// 1-D input transform t = B^T d (five values -> five), exact-integer coefficients as adds and fmas with +-2
template <typename T>
__device__ __forceinline__ void bt5(const T (&d)[5], T (&t)[5]) {
    const T a = d[3] - d[1], s = d[0] - d[2], b = d[2] - d[3], c = d[2] - d[1], e = d[4] - d[2];
    t[0] = (T)2.f * s + a;
    t[1] = (T)2.f * d[1] + b;
    t[2] = (T)2.f * c + b;
    t[3] = a;
    t[4] = e - (T)2.f * a;
}

// (x, y) pair -> three packed bf16 pieces (x = x0 + x1 + x2 exactly; kernels.h bf16_piece)
__device__ __forceinline__ void split_pair(f32x2 v, unsigned& p0, unsigned& p1, unsigned& p2) {
    float x = v.x, y = v.y;
    p0 = bf16_piece(x, y);
    p1 = bf16_piece(x, y);
    p2 = bf16_last_piece(x, y);
}

}  // namespace

// (The knock-out measurements of DESIGN.md §3 — no U loads, transforms, MFMAs or epilogue — were built from this file
// as of commit 94f9b44; the product kernel carries no such switches.)
#ifdef W9F3_PROF
// per (workgroup < W9F3_PROF, wave, unit iteration < 4) on the 100 MHz clock: 0 start, 1 staged, 2 transform A,
// 3 MFMA A, 4 transform B, 5 MFMA B, 6 transform C, 7 MFMA C, 8 epilogue block 0, 9 epilogue block 1
__device__ unsigned long long f3_tl[W9F3_PROF][8][4][10];
#define F3TL(k) \
    if (!HALF && blockIdx.x < W9F3_PROF && lane == 0 && f3_it < 4) f3_tl[blockIdx.x][wave][f3_it][(k)] = __builtin_amdgcn_s_memrealtime()
#else
#define F3TL(k)
#endif

// HALF: the launch for the last partial round's blocks, each as two half units (one 12-row M block): unit u is M block
// u & 1 of block blk0 + (u >> 1); the active block sits in accumulator slot 0 and its tile rows are an address offset
// wg / ngrid: this workgroup's index among the ngrid workgroups that share the units (blockIdx.x / gridDim.x of a
// launch of one kind; the fused launch below offsets its half-unit workgroups)
template <bool HALF>
__device__ __forceinline__ void wino9f3_body(const Wino9Args& a, int n_units, int blk0, int wg, int ngrid) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // LDS pointers, re-derived each unit from an opaque zero (the loop below): otherwise every LDS address of the unrolled
    // phases whose offset exceeds the 16-bit instruction offset is computed once before the persistent loop and kept
    // live in a register (which spilled)
    unsigned char* lbp = lds;
    float* patch = reinterpret_cast<float*>(lds + PATCH_OFF);
    float* patchc = reinterpret_cast<float*>(lds + PATCHC_OFF);

    const int tid = threadIdx.x, lane = tid & 63;
    // the thread index made opaque at a use site: thread-constant addresses derived from it are then recomputed in each
    // phase (a few VALU) instead of being hoisted before the persistent loop, kept live across the MFMA phases and spilled
    auto otid = [&]() __attribute__((always_inline)) {
        int v = tid;
        asm volatile("" : "+v"(v));
        return v;
    };
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (a.zero != nullptr)   // the frame's CIN accumulators (no separate memset launch; no layer before this one)
        for (long i = (long)wg * NTHR + tid; i < a.zero_n2; i += (long)ngrid * NTHR)
            reinterpret_cast<uint4*>(a.zero)[i] = make_uint4(0u, 0u, 0u, 0u);
    const int li = lane & 31, lh = lane >> 5;
    const int H = a.H, W = a.W, Cin = a.cin;
    const bool has_b = Cin > 8, has_c = Cin > 16;

    // ---- units: 24 x 24-pixel blocks; the last partial round's blocks as two half units (one 12-row M block each)
    auto unit_block = [&](int u) __attribute__((always_inline)) { return HALF ? blk0 + (u >> 1) : u; };
    auto block_coords = [&](int u, int& y0, int& x0, size_t& img) __attribute__((always_inline)) {
        int t = unit_block(u);
        const int tx = t % a.tiles_x;
        t /= a.tiles_x;
        const int ty = t % a.tiles_y;
        img = (size_t)(t / a.tiles_y) * H * W;
        y0 = ty * FT;
        x0 = tx * FT;
    };

    // ---- input staging: chunk A / B thread = (row parity rb, patch column col, channel ch of the chunk): rows
    // rb + 2m, m = 0..15 (a wave's 32-lane half covers 4 columns x 8 channels: 128 contiguous LDS bytes); chunk C
    // thread = pixels tid and tid + 512 of the 32 x 32 patch
    const __amdgpu_buffer_rsrc_t insrd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.in), 0, (int)((size_t)a.batch * H * W * Cin * 4), 0x00020000);
    const int s_rb = tid >> 8, s_col = (tid >> 3) & 31, s_ch = tid & 7;
    float ra[16], rb[16], rc[2];
    auto load_patch = [&](int u) __attribute__((always_inline)) {
        // opaque unit index: the loads cannot be hoisted above this point (global loads are not ordered by the LDS
        // barriers, and hoisted they kept 34 registers live through the MFMA phases)
        int rbo = s_rb, colo = s_col, cho = s_ch, tido = tid;   // (thread constants made opaque too: their products
        asm volatile("" : "+s"(u), "+v"(rbo), "+v"(colo), "+v"(cho), "+v"(tido));   // would be hoisted likewise)
        int y0, x0;
        size_t img;
        block_coords(u, y0, x0, img);
        const int gx = x0 - 4 + colo;
        const bool xin = gx >= 0 && gx < W;
        // 32-bit offsets (wino9f3_launch: the input is < 2^31 bytes); the row part is wave-uniform (s_rb = tid >> 8)
        const int img_fl = (int)img * Cin;
        const int xa = xin && cho < Cin ? (gx * Cin + cho) * 4 : 0x7FFFFFF0;
        const int xb = xin && 8 + cho < Cin ? (gx * Cin + 8 + cho) * 4 : 0x7FFFFFF0;
        sfor<0, 16>([&](auto M) __attribute__((always_inline)) {
            constexpr int m = decltype(M)::value;
            const int gy = __builtin_amdgcn_readfirstlane(y0 - 4 + rbo + 2 * m);
            const bool rin = gy >= 0 && gy < H;
            const int soff = rin ? (img_fl + gy * W * Cin) * 4 : 0;
            ra[m] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(insrd, rin ? xa : 0x7FFFFFF0, soff, 0));
            rb[m] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(insrd, rin ? xb : 0x7FFFFFF0, soff, 0));
        });
        sfor<0, 2>([&](auto M) __attribute__((always_inline)) {
            constexpr int m = decltype(M)::value;
            const int px = tido + NTHR * m, r = px >> 5, c = px & 31;
            const int gy = y0 - 4 + r, gxc = x0 - 4 + c;
            const bool in = has_c && gy >= 0 && gy < H && gxc >= 0 && gxc < W;
            const int off = in ? (img_fl + (gy * W + gxc) * Cin + 16) * 4 : 0x7FFFFFF0;
            rc[m] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(insrd, off, 0, 0));
        });
    };
    auto stage_ab = [&](const float (&r)[16]) __attribute__((always_inline)) {
        const int tt = otid();
        float* const dst = patch + (tt >> 8) * RP + ((tt >> 3) & 31) * 8 + (tt & 7);
#pragma unroll
        for (int m = 0; m < 16; ++m) dst[2 * m * RP] = r[m];
    };
    auto stage_c = [&]() __attribute__((always_inline)) {
        const int tt = otid();
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int px = tt + NTHR * m;
            patchc[(px >> 5) * RPC + (px & 31)] = rc[m];
        }
    };

    // ---- input transform of an 8-channel chunk: thread = (V tile vt, channel pair cp), vt < 100 (half units: the
    // six tile rows 4h .. 4h + 5 their M block reads)
    auto transform_ab = [&](int hmask) __attribute__((always_inline)) {
        const int r0 = hmask == 2 ? 4 : 0, nrow = hmask == 3 ? NV : 6;
        const int tt = otid();
        const int vt = (tt >> 2) + r0 * NV, cp = tt & 3;
        if ((tt >> 2) < nrow * NV) {
            const int vy = vt / NV, vx = vt - vy * NV;
            const float* src = patch + (3 * vy) * RP + (3 * vx) * 8 + 2 * cp;
            f32x2 t[5][5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {   // along the row (l), per input row k
                f32x2 d[5];
#pragma unroll
                for (int l = 0; l < 5; ++l) d[l] = *reinterpret_cast<const f32x2*>(src + k * RP + l * 8);
                bt5(d, t[k]);
            }
            unsigned char* const vdst = lbp + vt * 16 + cp * 4;
#pragma unroll
            for (int j = 0; j < 5; ++j) {   // along the column (k), per transformed column j
                const f32x2 c[5] = {t[0][j], t[1][j], t[2][j], t[3][j], t[4][j]};
                f32x2 v[5];
                bt5(c, v);
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    unsigned p0, p1, p2;
                    split_pair(v[i], p0, p1, p2);
                    const int xi = 5 * i + j;
                    *reinterpret_cast<unsigned*>(vdst + (0 * NXI + xi) * VPLANE) = p0;
                    *reinterpret_cast<unsigned*>(vdst + (1 * NXI + xi) * VPLANE) = p1;
                    *reinterpret_cast<unsigned*>(vdst + (2 * NXI + xi) * VPLANE) = p2;
                }
                __builtin_amdgcn_sched_barrier(0);   // one column at a time (register pressure: the MFMA accumulators are live)
            }
        }
    };
    // channel 16: one thread per V tile (threads 0..99: waves 0 and 1, two SIMDs), all 25 points (no per-lane
    // selection: a lane-dependent point row compiled to divergent branches); V16[xi][vt] = {p0 | p1 << 16, p2}
    auto transform_c = [&](int hmask) __attribute__((always_inline)) {
        const int r0 = hmask == 2 ? 4 : 0, nrow = hmask == 3 ? NV : 6;
        const int tt = otid();
        if (tt < nrow * NV) {
            const int vt = tt + r0 * NV, vy = vt / NV, vx = vt - vy * NV;
            const float* src = patchc + (3 * vy) * RPC + 3 * vx;
            float t[5][5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                float d[5];
#pragma unroll
                for (int l = 0; l < 5; ++l) d[l] = src[k * RPC + l];
                bt5(d, t[k]);
            }
            u32x2* const dst = reinterpret_cast<u32x2*>(lbp) + vt;
            float v[5][5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const float c[5] = {t[0][j], t[1][j], t[2][j], t[3][j], t[4][j]};
                float o[5];
                bt5(c, o);
#pragma unroll
                for (int i = 0; i < 5; ++i) v[i][j] = o[i];
            }
#pragma unroll
            for (int x = 0; x < NXI; x += 2) {   // points in pairs through the packed split
                const float y = x + 1 < NXI ? v[(x + 1) / 5][(x + 1) % 5] : 0.f;
                unsigned p0, p1, p2;
                split_pair(f32x2{v[x / 5][x % 5], y}, p0, p1, p2);
                dst[x * NVT] = u32x2{(p0 & 0xFFFFu) | (p1 << 16), p2 & 0xFFFFu};
                if (x + 1 < NXI) dst[(x + 1) * NVT] = u32x2{(p0 >> 16) | (p1 & 0xFFFF0000u), p2 >> 16};
            }
        }
    };

    // ---- MFMA phase -----------------------------------------------------------------------------------------
    // Points 0..23 on 32x32x16 tiles: wave w owns points w, w + 8, w + 16 of both M blocks (6 accumulators). U block
    // (slot, xi, piece): lane (li, lh) reads co = li, K = 8 lh .. 8 lh + 7. Point 24 on 16x16x32 tiles, one per wave
    // (block w >> 2, tiles 16 ((w >> 1) & 1) .. + 15, output channels 16 (w & 1) .. + 15): K-step = four sub-kernels
    // (lane group kg = lane >> 4: sub-kernel 4 ks + kg) x 8 channels; U24 block (slot24, piece, co half): lane reads
    // co = 16 nh + (lane & 15), K = 8 kg .. 8 kg + 7. Every wave runs the same instruction stream.
    const __amdgpu_buffer_rsrc_t usrd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, U_BYTES, 0x00020000);
    const int uvoff = li * 32 + 16 * lh;
    auto load_u = [&](short8 (&u)[3], int slot, int xi) __attribute__((always_inline)) {
        sfor<0, 3>([&](auto P) __attribute__((always_inline)) {
            constexpr int p = decltype(P)::value;
            u[p] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(usrd, uvoff, ((slot * NXM + xi) * 3 + p) * UBLK, 0));
        });
    };
    const int l16 = lane & 15, kg = lane >> 4;
    const int h24 = wave >> 2, mq = (wave >> 1) & 1, nh = wave & 1;
    const int u24off = l16 * 64 + kg * 16;
    auto load_u24 = [&](short8 (&u)[3], int slot24) __attribute__((always_inline)) {
        sfor<0, 3>([&](auto P) __attribute__((always_inline)) {
            constexpr int p = decltype(P)::value;
            u[p] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(
                                                  usrd, u24off, U24_OFF + ((slot24 * 3 + p) * 2 + nh) * UBLK, 0));
        });
    };
    // the lane's tile in M block h: row li & 3, column li >> 2 -> V tile (4h + (li & 3)) * 10 + (li >> 2)
    const int vt_l = (li & 3) * NV + (li >> 2);
    // point 24: M row 16 mq + l16 of block h24 -> tile (row l16 & 3, column 4 mq + (l16 >> 2))
    const int vt24 = (4 * h24 + (l16 & 3)) * NV + 4 * mq + (l16 >> 2);
    auto mfma6 = [&](floatx16& C, const short8 (&A)[3], const short8 (&B)[3]) __attribute__((always_inline)) {
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], C, 0, 0, 0);   // a0 b0
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], C, 0, 0, 0);   // a0 b1
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], C, 0, 0, 0);   // a1 b0
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], C, 0, 0, 0);   // a0 b2
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], C, 0, 0, 0);   // a1 b1
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], C, 0, 0, 0);   // a2 b0
    };
    auto mfma6s = [&](floatx4& C, const short8 (&A)[3], const short8 (&B)[3]) __attribute__((always_inline)) {
        C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], C, 0, 0, 0);
    };
    const int xi0 = wave;
    floatx16 acc[3][2];
    floatx4 acc24;
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j) acc[j][0][r] = acc[j][1][r] = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc24[r] = 0.f;
    };
    auto shift_of = [](int ab) __attribute__((always_inline)) { return (ab / 3) * NV + ab % 3; };
    // V read addresses: per-lane bases made opaque once per unit (asm barrier: otherwise every shifted address of the
    // unrolled phase is hoisted out of the persistent loop and kept live, which spilled); the shifts, blocks, points
    // and pieces are added as constants
    int vb_main = 0, vb_24 = 0, lhd = 0, vb24_16 = 0, shift24[3] = {0, 0, 0};
    auto read_v = [&](short8 (&A)[3], int base, int off) __attribute__((always_inline)) {
        const unsigned char* va = lbp + base + off;
        sfor<0, 3>([&](auto P) __attribute__((always_inline)) {
            constexpr int p = decltype(P)::value;
            A[p] = *reinterpret_cast<const short8*>(va + p * NXI * VPLANE);
        });
    };
    // sub-kernel 2 ks + lh of lane half lh (ks = 4: both halves sub-kernel 8): shift_of(2 ks) + lh d(ks)
    auto dks = [&](int ks) __attribute__((always_inline)) { return ks < 4 ? shift_of(2 * ks + 1) - shift_of(2 * ks) : 0; };
    // one 8-channel chunk c: main steps S = 3 ks + j (K-step ks: sub-kernels 2 ks (lh 0), 2 ks + 1 (lh 1; ks = 4: none,
    // its U half is zero and the A read repeats sub-kernel 8)); U two steps ahead (ring of 3); after the three steps of
    // ks < 3, point 24's K-step ks (sub-kernels 4 ks + kg; past 8: zero U, sub-kernel 8 re-read)
    // MK: the unit's M blocks (compile time: 3 whole block, 1 / 2 half unit); point 24's sub-tile runs when its block
    // h24 is in the unit (uniform)
    auto mfma_chunk = [&](auto CH, auto MK) __attribute__((always_inline)) {
        constexpr int c = decltype(CH)::value, MASK = decltype(MK)::value;
        const bool do24 = MASK == 3 || ((MASK >> h24) & 1);
        short8 ub[3][3], u24[3];
        load_u(ub[0], 5 * c, xi0);
        load_u(ub[1], 5 * c, xi0 + 8);
        sfor<0, 15>([&](auto SS) __attribute__((always_inline)) {
            constexpr int S = decltype(SS)::value, ks = S / 3, j = S % 3;
            if constexpr (S + 2 < 15) load_u(ub[(S + 2) % 3], 5 * c + (S + 2) / 3, xi0 + 8 * ((S + 2) % 3));
            if constexpr (j == 0 && ks < 3) load_u24(u24, 3 * c + ks);
            const int vb = vb_main + lhd * dks(ks);
            sfor<0, 2>([&](auto Hh) __attribute__((always_inline)) {
                constexpr int h = decltype(Hh)::value;
                if constexpr ((MASK >> h) & 1) {
                    short8 A[3];
                    read_v(A, vb, (8 * j) * VPLANE + (4 * h * NV + shift_of(2 * ks)) * 16);
                    mfma6(acc[j][h], A, ub[S % 3]);
                }
            });
            if constexpr (j == 2 && ks < 3) {
                // lane group kg: sub-kernel min(4 ks + kg, 8): kg-dependent shift from a table in registers
                if (do24) {
                    short8 A[3];
                    read_v(A, vb_24, shift24[ks] * 16);
                    mfma6s(acc24, A, u24);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    // channel 16: one K-step, K index = sub-kernel (32x32x16: lh 0 sub-kernels 0..7, lh 1 sub-kernel 8 then zero U;
    // 16x16x32: lane group kg = 0 sub-kernels 0..7, kg = 1 sub-kernel 8, the rest zero U)
    // V16 reads: K index k of lane half lh is sub-kernel 8 lh + k; past 8 the U is zero, so there any finite V16 serves:
    // k >= 1 reads sub-kernel k for both halves (constant offsets), k = 0 reads sub-kernel 8 lh
    auto read_v16 = [&](short8 (&A)[3], int base, int base0) __attribute__((always_inline)) {
        const unsigned char* v16 = lbp + base;
        u32x2 r[8];
        r[0] = *reinterpret_cast<const u32x2*>(lbp + base0);
#pragma unroll
        for (int k = 1; k < 8; ++k) r[k] = *reinterpret_cast<const u32x2*>(v16 + shift_of(k) * 8);
        u32x4 q0, q1, q2;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            q0[m] = __builtin_amdgcn_perm(r[2 * m + 1].x, r[2 * m].x, 0x05040100u);   // low halves: piece 0
            q1[m] = __builtin_amdgcn_perm(r[2 * m + 1].x, r[2 * m].x, 0x07060302u);   // high halves: piece 1
            q2[m] = __builtin_amdgcn_perm(r[2 * m + 1].y, r[2 * m].y, 0x05040100u);   // piece 2
        }
        A[0] = __builtin_bit_cast(short8, q0);
        A[1] = __builtin_bit_cast(short8, q1);
        A[2] = __builtin_bit_cast(short8, q2);
    };
    auto mfma_c = [&](auto MK) __attribute__((always_inline)) {
        constexpr int MASK = decltype(MK)::value;
        short8 ub[3][3], u24[3];
        load_u(ub[0], 10, xi0);
        load_u(ub[1], 10, xi0 + 8);
        load_u(ub[2], 10, xi0 + 16);
        load_u24(u24, 6);
        // V16 [xi][vt] 8 B: lane bases from the same opaque V-tile base (16 B per tile there, 8 B here)
        const int b16 = vb_main >> 1, b16_0 = b16 + lhd * 11;   // lh: + shift_of(8) = 22 tiles = 176 B
        sfor<0, 3>([&](auto J) __attribute__((always_inline)) {
            constexpr int j = decltype(J)::value;
            sfor<0, 2>([&](auto Hh) __attribute__((always_inline)) {
                constexpr int h = decltype(Hh)::value;
                if constexpr ((MASK >> h) & 1) {
                    constexpr int off = ((8 * j) * NVT + 4 * h * NV) * 8;
                    short8 A[3];
                    read_v16(A, b16 + off, b16_0 + off);
                    mfma6(acc[j][h], A, ub[j]);
                }
            });
            __builtin_amdgcn_sched_barrier(0);
        });
        // point 24: lane group kg: K index 8 kg + k -> sub-kernel 8 kg + k (kg = 0: 0..7; kg = 1: 8 at k = 0)
        if (MASK == 3 || ((MASK >> h24) & 1)) {
            short8 A[3];
            read_v16(A, vb24_16, vb24_16 + (kg == 1 ? 22 * 8 : 0));
            mfma6s(acc24, A, u24);
        }
    };

    // ---- epilogue of M block h: accumulators -> M image [xi][co][tile] (tile fastest, row pitch MP: a lane's four
    // consecutive accumulator rows are one ds_write_b128; a reader's two tiles one ds_read_b64), output transform,
    // bias -> ReLU -> BN -> ReLU, buffer stores (per-tile 32-bit base; the pixel row as the scalar offset)
    // epilogue thread: output channel eco = tid & 31, tiles 2 eg, 2 eg + 1 of the block (eg = tid >> 5)
    const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
    float* ms = reinterpret_cast<float*>(lds);
    auto epilogue = [&](int h, int hrow, int y0, int x0, size_t img) __attribute__((always_inline)) {
        const bool inside = y0 + FT <= H && x0 + FT <= W;   // uniform: no per-pixel bounds tests
        const int tt = otid(), eco = tt & 31, eg = tt >> 5;
        const float bias = reinterpret_cast<const float*>(lbp + PARAM_OFF)[eco];
        const float2 bn = reinterpret_cast<const float2*>(lbp + PARAM_OFF + NCO * 4)[eco];
        lds_barrier();   // every V / V16 read of the unit done (h = 0), the previous block's M reads done (h = 1)
        // lane base from the opaque thread index (see otid); accumulator register 4q + r of lane (li, lh) is tile row
        // 8q + 4lh + r, channel li
        const int lq = tt & 63;
        float* const mlane = ms + (lq & 31) * MP + 4 * (lq >> 5);
        auto put = [&](const floatx16& C, int xi) __attribute__((always_inline)) {
            float* const mp = mlane + xi * 32 * MP;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<f32x4*>(mp + 8 * q) = f32x4{C[4 * q], C[4 * q + 1], C[4 * q + 2], C[4 * q + 3]};
        };
        if (h == 0) {
            put(acc[0][0], xi0);
            put(acc[1][0], xi0 + 8);
            put(acc[2][0], xi0 + 16);
        } else {
            put(acc[0][1], xi0);
            put(acc[1][1], xi0 + 8);
            put(acc[2][1], xi0 + 16);
        }
        if (h == h24)   // point 24: lane holds tile rows 16 mq + 4 kg + r, channel 16 nh + l16
            *reinterpret_cast<f32x4*>(ms + (24 * 32 + 16 * nh + (lq & 15)) * MP + 16 * mq + 4 * (lq >> 4)) =
                f32x4{acc24[0], acc24[1], acc24[2], acc24[3]};
        lds_barrier();
        float M[2][25];
        const float* const mr = ms + eco * MP + 2 * eg;
#pragma unroll
        for (int x = 0; x < NXI; ++x) {
            const f32x2 v = *reinterpret_cast<const f32x2*>(mr + x * 32 * MP);
            M[0][x] = v.x;
            M[1][x] = v.y;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int m = 2 * eg + k;                    // M row = tile (row m & 3, column m >> 2) of the block
            const int ty = 4 * hrow + (m & 3), tx = m >> 2;
            // T = A^T M (3 x 5), Y = T A (3 x 3); A^T rows: [1,1,1,1,0], [0,1,-1,2,0], [0,1,1,4,1]
            float T[3][5];
#pragma unroll
            for (int c = 0; c < 5; ++c) {
                const float m0 = M[k][c], m1 = M[k][5 + c], m2 = M[k][10 + c], m3 = M[k][15 + c], m4 = M[k][20 + c];
                const float p = m1 + m2, q = m1 - m2;
                T[0][c] = (m0 + p) + m3;
                T[1][c] = fmaf(2.f, m3, q);
                T[2][c] = fmaf(4.f, m3, p) + m4;
            }
            float o[3][3];
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float p = T[r][1] + T[r][2], q = T[r][1] - T[r][2];
                const float yr[3] = {(T[r][0] + p) + T[r][3], fmaf(2.f, T[r][3], q), fmaf(4.f, T[r][3], p) + T[r][4]};
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float v = fmaxf(yr[c] + bias, 0.f);           // Conv2D(..., activation='relu')
                    o[r][c] = fmaxf(fmaf(bn.x, v, bn.y), 0.f);         // BN (folded moving statistics) -> ReLU
                }
            }
            const int oy0 = y0 + 3 * ty, ox0 = x0 + 3 * tx;
            const int base = (int)(((img + (size_t)oy0 * W + ox0) * NCO + eco) * 4);
            auto store = [&](auto WT) __attribute__((always_inline)) {
                constexpr int aux = decltype(WT)::value ? 16 : 0;   // 16: write-through (sc1)
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int so = __builtin_amdgcn_readfirstlane(r * W * NCO * 4);
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        if (inside || (oy0 + r < H && ox0 + c < W))
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[r][c]), osrd,
                                                                  base + c * NCO * 4, so, aux);
                }
            };
            if (a.wt_stores) store(std::true_type{});
            else store(std::false_type{});
        }
    };

    unsigned l2f = 0;     // the next layer's weights into this XCD's L2, touched during the last unit (speed only)
    int f3_it = 0;
    (void)f3_it;
    if (tid < NCO) {
        reinterpret_cast<float*>(lds + PARAM_OFF)[tid] = a.bias[tid];
        reinterpret_cast<float2*>(lds + PARAM_OFF + NCO * 4)[tid] = a.bn_ab[tid];
    }
    if (wg < n_units) load_patch(wg);
    for (int t = wg; t < n_units; t += ngrid, ++f3_it) {
        F3TL(0);
        const int tn = t + ngrid;
        if (tn >= n_units) l2f = l2_touch_xcd_slice<NTHR, 1>(a.w_next, a.w_next_bytes).x;
        int y0, x0;
        size_t img;
        block_coords(t, y0, x0, img);
        const int hb = HALF ? (t & 1) : 0;                 // a half unit's M block
        const int hmask = HALF ? 1 << hb : 3;               // (transform rows)
        constexpr int MASKC = HALF ? 1 : 3;                 // accumulator slots in use
        {
            int lb = 0;
            asm volatile("" : "+v"(lb));
            lbp = lds + lb;
            patch = reinterpret_cast<float*>(lbp + PATCH_OFF);
            patchc = reinterpret_cast<float*>(lbp + PATCHC_OFF);
            ms = reinterpret_cast<float*>(lbp);
        }
        {   // per-unit opaque lane bases of the V reads (see read_v); a half unit's block as a tile-row offset
            const int boff = HALF ? (t & 1) * 4 * NV : 0;
            int vbm = xi0 * VPLANE + (vt_l + boff) * 16, vb24b = 24 * VPLANE + (vt24 + boff) * 16, lh16 = lh * 16, kk = kg;
            asm volatile("" : "+v"(vbm), "+v"(vb24b), "+v"(lh16), "+v"(kk));
            vb_main = vbm;
            vb_24 = vb24b;
            vb24_16 = vb24b >> 1;
            lhd = lh16;
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) shift24[ks] = shift_of(min(4 * ks + kk, 8));
        }
        // chunk A: stage (with channel 16's patch), transform
        stage_ab(ra);
        stage_c();
        lds_barrier();
        F3TL(1);
        transform_ab(hmask);
        lds_barrier();
        F3TL(2);
        // chunk B's patch over A's (A is transformed); A's MFMAs
        if (has_b) stage_ab(rb);
        zero_acc();
        auto chunk_m = [&](auto CH) __attribute__((always_inline)) { mfma_chunk(CH, std::integral_constant<int, MASKC>{}); };
        chunk_m(std::integral_constant<int, 0>{});
        lds_barrier();
        F3TL(3);
        if (has_b) {
            transform_ab(hmask);
            lds_barrier();
            F3TL(4);
            chunk_m(std::integral_constant<int, 1>{});
            lds_barrier();
            F3TL(5);
        }
        if (has_c) {
            transform_c(hmask);
            lds_barrier();
            F3TL(6);
            mfma_c(std::integral_constant<int, MASKC>{});
            F3TL(7);
        }
        // the next unit's input, issued after the last U load (vmcnt retires in order) and consumed at the next unit's
        // staging: its HBM latency hides behind the epilogue
        __builtin_amdgcn_sched_barrier(0);   // (the MFMA phase's operand registers are dead before these loads)
        if (tn < n_units) load_patch(tn);
        epilogue(0, HALF ? hb : 0, y0, x0, img);
        F3TL(8);
        if (!HALF) epilogue(1, 1, y0, x0, img);

        F3TL(9);
        lds_barrier();   // M image reads done before the next unit's staging
    }
    l2_touch_keep(l2_touch_t{l2f, 0u}, a.batch < 0, reinterpret_cast<float*>(lds));
}

template <bool HALF>
__global__ __launch_bounds__(NTHR, 1) void wino9f3_kernel(Wino9Args a, int n_units, int blk0) {
    wino9f3_body<HALF>(a, n_units, blk0, (int)blockIdx.x, (int)gridDim.x);
}

// The last partial round inside the same launch: workgroups [0, n_main) walk the n_full whole blocks persistently, the
// n_half workgroups after them take one half unit each. One workgroup fits a CU (LDS), and workgroups are dispatched in
// index order as CUs free up, so the half units start on the first CUs whose persistent walk ends — while the other
// walks finish — instead of after the whole launch (the second launch of wino9f3_launch's split form). Speed only: a
// half unit's result does not depend on where or when it runs.
__global__ __launch_bounds__(NTHR, 1) void wino9f3_fused_kernel(Wino9Args a, int n_full, int n_main) {
    if ((int)blockIdx.x < n_main) {
        wino9f3_body<false>(a, n_full, 0, (int)blockIdx.x, n_main);
    } else {
        Wino9Args b = a;
        b.zero = nullptr;     // (cleared by the persistent workgroups)
        b.w_next = nullptr;   // (touched by the persistent workgroups' last units)
        wino9f3_body<true>(b, (int)gridDim.x - n_main, n_full, (int)blockIdx.x - n_main, (int)gridDim.x - n_main);
    }
}

#ifdef W9F3_PROF
void f3_timeline_print(int nwg) {
    std::vector<unsigned long long> tl((size_t)W9F3_PROF * 8 * 4 * 10, 0);
    if (hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(f3_tl), tl.size() * 8) != hipSuccess) return;
    if (nwg > W9F3_PROF) nwg = W9F3_PROF;
    const char* names[9] = {"stage", "T_A", "MFMA_A", "T_B", "MFMA_B", "T_C", "MFMA_C", "epi0", "epi1"};
    double ph[9] = {0};
    int n = 0;
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 8; ++w)
            for (int it = 0; it < 3; ++it) {
                const unsigned long long* q = &tl[(((size_t)g * 8 + w) * 4 + it) * 10];
                if (q[9] == 0) continue;
                for (int k = 0; k < 9; ++k) ph[k] += (double)(q[k + 1] - q[k]);
                ++n;
            }
    printf("  per unit (us, %d samples):", n);
    double tot = 0;
    for (int k = 0; k < 9; ++k) {
        printf(" %s %.2f", names[k], n ? ph[k] / n * 0.01 : 0.0);
        tot += ph[k];
    }
    printf(" | total %.2f\n", n ? tot / n * 0.01 : 0.0);
    // per workgroup: start of unit 0 relative to the earliest, gaps between units, end of the last unit
    unsigned long long t0 = ~0ull;
    for (int g = 0; g < nwg; ++g) {
        const unsigned long long v = tl[((size_t)g * 8) * 4 * 10];
        if (v && v < t0) t0 = v;
    }
    double gap = 0, span = 0, st0 = 0;
    int ng = 0, nsp = 0;
    for (int g = 0; g < nwg; ++g) {
        const unsigned long long* q = &tl[((size_t)g * 8) * 4 * 10];
        if (!q[0]) continue;
        st0 += (double)(q[0] - t0);
        unsigned long long e = 0;
        for (int it = 0; it < 4; ++it) {
            if (q[it * 10 + 9]) e = q[it * 10 + 9];
            if (it + 1 < 4 && q[(it + 1) * 10] && q[it * 10 + 9]) {
                gap += (double)(q[(it + 1) * 10] - q[it * 10 + 9]);
                ++ng;
            }
        }
        span += (double)(e - q[0]);
        ++nsp;
    }
    printf("  workgroups 0..%d: start after the first %.2f us (mean), gap between units %.2f us, span %.2f us\n", nwg - 1,
           nsp ? st0 / nsp * 0.01 : 0.0, ng ? gap / ng * 0.01 : 0.0, nsp ? span / nsp * 0.01 : 0.0);
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

// U pieces, bf16 (returned as the float-sized buffer holding the bits). Points 0..23: [slot 0..10][xi][piece][co][16 K]
// (32x32x16 B operands); slots 5c + ks (chunk c = 0, 1; ks = 0..4): K index k -> sub-kernel 2 ks + (k >> 3) (zero past
// 8), channel 8c + (k & 7); slot 10: K index k -> sub-kernel k (zero past 8), channel 16. Point 24 (16x16x32 B
// operands): [slot24 0..6][piece][co half][16 co][32 K]; slots 3c + ks (ks = 0..2): K index k -> sub-kernel 4 ks +
// (k >> 3) (zero past 8), channel 8c + (k & 7); slot 6: K index k -> sub-kernel k, channel 16. U = G g_ab G^T in f64
// (fixed operation order), rounded once to f32, split into three bf16 pieces with round-to-nearest-even at each step.
// Channels >= cin are zero.
std::vector<float> wino9f3_pack_weights(const float* kern, int cin) {
#pragma clang fp contract(off)
    static const double G[5][3] = {{0.5, 0, 0}, {0.5, 0.5, 0.5}, {1.0 / 6, -1.0 / 6, 1.0 / 6},
                                   {1.0 / 6, 1.0 / 3, 2.0 / 3}, {0, 0, 1}};
    const size_t n16 = (size_t)U_BYTES / 2;
    std::vector<uint16_t> U(n16, 0);
    // the three pieces of U[xi] of sub-kernel ab, input channel ci, output channel co
    auto pieces = [&](int ab, int ci, int co, int xi, uint16_t pc[3]) {
        const int sa = ab / 3, sb = ab % 3, p = xi / 5, q = xi % 5;
        double gg[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) gg[i][j] = kern[(((size_t)(3 * sa + i) * 9 + (3 * sb + j)) * cin + ci) * NCO + co];
        double u = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) u += G[p][i] * gg[i][j] * G[q][j];
        const float uf = (float)u;
        pc[0] = bf16_rne_host(uf);
        const float r = uf - bf16_val_host(pc[0]);
        pc[1] = bf16_rne_host(r);
        pc[2] = bf16_rne_host(r - bf16_val_host(pc[1]));
    };
    auto put = [&](int slot, int k, int ab, int ci) {   // points 0..23
        if (ab > 8 || ci >= cin) return;
        for (int xi = 0; xi < NXM; ++xi)
            for (int co = 0; co < NCO; ++co) {
                uint16_t pc[3];
                pieces(ab, ci, co, xi, pc);
                for (int pi = 0; pi < 3; ++pi) U[((((size_t)slot * NXM + xi) * 3 + pi) * NCO + co) * 16 + k] = pc[pi];
            }
    };
    auto put24 = [&](int slot24, int k, int ab, int ci) {   // point 24
        if (ab > 8 || ci >= cin) return;
        for (int co = 0; co < NCO; ++co) {
            uint16_t pc[3];
            pieces(ab, ci, co, 24, pc);
            for (int pi = 0; pi < 3; ++pi)
                U[U24_OFF / 2 + ((((size_t)slot24 * 3 + pi) * 2 + (co >> 4)) * 16 + (co & 15)) * 32 + k] = pc[pi];
        }
    };
    for (int c = 0; c < 2; ++c) {
        for (int ks = 0; ks < 5; ++ks)
            for (int k = 0; k < 16; ++k) put(5 * c + ks, k, 2 * ks + (k >> 3), 8 * c + (k & 7));
        for (int ks = 0; ks < 3; ++ks)
            for (int k = 0; k < 32; ++k) put24(3 * c + ks, k, 4 * ks + (k >> 3), 8 * c + (k & 7));
    }
    for (int k = 0; k < 16; ++k) put(10, k, k, 16);
    for (int k = 0; k < 32; ++k) put24(6, k, k, 16);
    std::vector<float> out(n16 / 2);
    std::memcpy(out.data(), U.data(), n16 * 2);
    return out;
}

hipError_t wino9f3_prepare() {
    hipError_t e = hipFuncSetAttribute((const void*)wino9f3_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)wino9f3_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)wino9f3_fused_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    return e;
}

int wino9f3_tiles_y(int H) { return (H + FT - 1) / FT; }
int wino9f3_tiles_x(int W) { return (W + FT - 1) / FT; }

hipError_t wino9f3_launch(const Wino9Args& a, hipStream_t st) {
    if (a.cin > 17 || a.cin <= 0 || a.tiles_y != (a.H + FT - 1) / FT || a.tiles_x != (a.W + FT - 1) / FT ||
        a.part != nullptr || a.bn_ab == nullptr)
        return hipErrorInvalidValue;   // inference only: folded BN affine
    if ((size_t)a.batch * a.H * a.W * a.cin * 4 >= (size_t)0x7FFFFFF0 || (size_t)a.batch * a.H * a.W * NCO * 4 >= (size_t)0x7FFFFFF0)
        return hipErrorInvalidValue;   // 32-bit buffer offsets; the idle offset must stay out of range
    const int n_blocks = a.batch * a.tiles_y * a.tiles_x;
    static int n_cu = 0;   // queried once (graph capture replays the recorded arguments)
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    const unsigned grid = (unsigned)(n_blocks < n_cu ? n_blocks : n_cu);
    // a last round that fills at most half the grid runs as a second launch of half-block units (one M block each):
    // 800 blocks on 256 CUs are 3 rounds and 32 blocks, i.e. 3.5 unit times instead of 4
    const int tail = n_blocks % (int)grid;
    const int n_full = (tail > 0 && 2 * tail <= (int)grid) ? n_blocks - tail : n_blocks;
    static const bool fused = [] {   // RST_F3_FUSED_TAIL=0: the tail as a second launch (A/B runs)
        const char* v = getenv("RST_F3_FUSED_TAIL");
        return !(v != nullptr && v[0] == '0');
    }();
    if (n_full < n_blocks && fused) {
        hipLaunchKernelGGL(wino9f3_fused_kernel, dim3(grid + (unsigned)(2 * tail)), dim3(NTHR), LDS_BYTES, st, a, n_full,
                           (int)grid);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(wino9f3_kernel<false>, dim3(grid), dim3(NTHR), LDS_BYTES, st, a, n_full, 0);
    if (n_full < n_blocks) {
        Wino9Args b = a;
        b.zero = nullptr;   // (cleared by the first launch)
        b.w_next = nullptr;
        hipLaunchKernelGGL(wino9f3_kernel<true>, dim3((unsigned)(2 * tail)), dim3(NTHR), LDS_BYTES, st, b, 2 * tail, n_full);
    }
    return hipGetLastError();
}

}  // namespace rst
