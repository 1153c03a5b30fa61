// wino_x6.hip — the residual-block convolutions (3x3, stride 1, SAME, 128 output channels;
// realtime_style_transfer/models/styleTransfer.py:144-185) as fused Winograd F(2x2, 3x3) whose
// transform-domain products run on the bf16 MFMA pipe with fp32-level accuracy
// (v_mfma_f32_32x32x16_bf16, 16x the f32-MFMA rate).
//
// Same algorithm as wino.hip: Y = A^T [ (G g G^T) (.) (B^T d B) ] A per 2x2 output tile. Every fp32
// operand of the 16 batched GEMMs (V = B^T d B and U = G g G^T) is split exactly into three bf16 pieces
// x = x0 + x1 + x2 (round-to-nearest-even at each step; the remainders are exact in fp32, so the three
// pieces hold all 24 significant bits), and a product becomes the six terms with i + j <= 2:
//     a b = a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0  (+ dropped terms <= 2^-25 |a b|),
// each term exact in the fp32 accumulator's input (bf16 x bf16), accumulated in fp32 — the products
// carry fp32 precision at 6/16 of the f32-MFMA cost. U is formed on the host in f64, rounded once to
// f32 (as wino.hip) and split on the host; V is split by the input-transform threads as they write it.
//
// Workgroup = 8 waves (two per SIMD), output tile 8 x 16 pixels = 32 Winograd tiles (one 32-row MFMA M
// tile) x 128 output channels. Wave (g, h) owns channels [32g, 32g+32) and the transform points of rows
// p = 2h, 2h+1 (points 8h .. 8h+7: 8 accumulators, 128 registers), so the two waves of a SIMD interleave
// and one wave's transform VALU issues while the other's MFMAs run (a single-wave-per-SIMD form holding
// all 16 points, 256 accumulator registers, left that VALU in the gaps of its own dependent MFMA chain:
// 34.8 vs 32.4 us at B=1). Input channels go in chunks of 16 = the MFMA K: per chunk and point the six
// terms are six MFMAs whose A operands are the V pieces (LDS, [piece][xi][tile][16 ch] bf16, one
// ds_read_b128 per lane per piece) and B operands the U pieces (L2, packed on the host in MFMA B-operand
// order, one 16-B load per lane per piece, a 2-point register ring). Per chunk c one software-pipelined
// step with one barrier: the 48 MFMAs of each wave on V(c) interleave with the input transform + split of
// chunk c+1 (thread = (half h, tile, channel pair): rows 2h, 2h+1 of B^T d from three patch rows, 12
// ds_read_b64, 32 adds, 3 v_cvt_pk_bf16_f32 per channel pair and point, 24 ds_write_b32), the staging of
// chunk c+2 (CIN affine [+ ReLU | + residual] prologue, materialised block output) and the loads of c+3.
// The loop is bound by the U stream (196 KB per workgroup and chunk from L2: 72-80 GB/s per CU, the
// L2-served rate MI355X_MICROARCH.md measures for shared rows); without the U reloads it runs 27 us.
// Epilogue: each half forms its partial output transform (Y = A^T M A is linear in the points) into an
// LDS image [pixel][channel]; all 512 threads add the halves, apply bias + ReLU, store whole pixels'
// channel quads (1 KB per wave instruction) and reduce the per-(workgroup, channel) two-pass {sum, M2, n}
// for the conditional instance norm that follows.
#include <hip/hip_ext.h>
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
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int XTH = 8, XTW = 16;                  // output pixels per workgroup
constexpr int XPH = XTH + 2, XPW = XTW + 2;       // input patch 10 x 18
constexpr int XNP = XPH * XPW;                    // 180 patch pixels
constexpr int XCK = 16;                           // input channels per chunk (= MFMA K)
constexpr int XPS = 24;                           // patch pixel stride (floats): 4 tiles' 64-B reads hit disjoint banks
constexpr int XN = 128;                           // output channels (4 waves x 32)
constexpr int XXI = 16;                           // transform points
constexpr int XPF4 = XNP * XCK / 4;               // 720 float4 per chunk patch
constexpr int XMAX_CIN = 256;
constexpr int XPATCH_FL = XNP * XPS;              // one patch buffer (floats)
constexpr int XVROW = 32;                         // bytes per (piece, xi, tile) row: 16 bf16
constexpr int XV_BYTES = 3 * XXI * 32 * XVROW;    // one V buffer: 48 KB
constexpr size_t XLDS_BYTES = (size_t)2 * XPATCH_FL * 4 + 2 * XV_BYTES + XMAX_CIN * sizeof(float2);   // loop

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

// two styles (styleTransfer.py:36-44): the per-pixel blend of the two CIN affines, as conv_mfma.hip's prologue
__device__ __forceinline__ float pro_apply_blend(int mode, float x, float2 ab, float2 ab1, float w, float r) {
    float y = style_blend(w, fmaf(ab.x, x, ab.y), fmaf(ab1.x, x, ab1.y));
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}

}  // namespace

// (The knock-out measurements quoted in DESIGN.md §3 — no U reloads, no transform, no staging, no barrier, no
// materialised stores — were built from this file as of commit 94f9b44; the product kernel carries no such switches.)
// In the chunk loop a store issued before a U load makes that load's vmcnt wait include the store (vmcnt retires in
// order): X6_MAT_LATE issues a chunk's materialised-output stores after the chunk's last U and staging loads.
#ifndef X6_MAT_LATE
#define X6_MAT_LATE 1
#endif
#ifdef X6_PROF
// timeline per (workgroup, wave < 8) on the constant 100 MHz clock: 0 start, 8 first loads issued, 4 affine formed,
// 5 chunk 0 staged, 1 pipeline filled, 2 chunk loop done, 6 epilogue image written, 7 outputs stored, 3 end
__device__ unsigned long long x6_tl[X6_PROF][8][12];
#ifndef X6_PROF_PRO
#define X6_PROF_PRO -1   // -1: every launch stamps; else only the launches of that prologue form
#endif
#define XTL(k) \
    if ((X6_PROF_PRO < 0 || PRO == X6_PROF_PRO) && blockIdx.x < X6_PROF && lane == 0) \
        x6_tl[blockIdx.x][wave][(k)] = __builtin_amdgcn_s_memrealtime()
#else
#define XTL(k)
#endif

#ifdef X6_PROF
// timeline summary of the most recent launch (tools/wino_x6_bench)
void x6_timeline_print(int nwg, int nwave) {
    std::vector<unsigned long long> tl((size_t)X6_PROF * 96);
    if (hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(x6_tl), tl.size() * 8) != hipSuccess) return;
    if (nwg > X6_PROF) nwg = X6_PROF;
    unsigned long long t0 = ~0ull, tend = 0, slast = 0;
    // phases in time order: 0 -> 8 -> 4 -> 5 -> 1 -> 2 -> 6 -> 7 -> 3
    const int ord[9] = {0, 8, 4, 5, 1, 2, 6, 7, 3};
    double ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pre[3] = {0, 0, 0};
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < nwave; ++w) {
            const unsigned long long* q = &tl[((size_t)g * 8 + w) * 12];
            pre[0] += (double)(q[9] - q[0]);
            pre[1] += (double)(q[10] - q[9]);
            pre[2] += (double)(q[11] - q[10]);
            t0 = q[0] < t0 ? q[0] : t0;
            tend = q[3] > tend ? q[3] : tend;
            slast = q[0] > slast ? q[0] : slast;
            for (int k = 0; k < 8; ++k) ph[k] += (double)(q[ord[k + 1]] - q[ord[k]]);
        }
    const double nw = nwg * (double)nwave * 100.0;
    printf("  timeline (us): first start -> last end %.2f, last start +%.2f; per wave: issue %.2f, affine %.2f, "
           "stage0 %.2f, transform0+stage1 %.2f, loop %.2f, epilogue image %.2f, stores %.2f, statistics %.2f\n",
           (tend - t0) * 0.01, (slast - t0) * 0.01, ph[0] / nw, ph[1] / nw, ph[2] / nw, ph[3] / nw, ph[4] / nw,
           ph[5] / nw, ph[6] / nw, ph[7] / nw);
    printf("  issue split (us): descriptors %.2f, accumulator loads issued %.2f, staging loads issued %.2f\n", pre[0] / nw,
           pre[1] / nw, pre[2] / nw);
}
// profiling builds of the library only (tools/build_prof_lib.sh): the timeline of the frame's last residual conv
extern "C" void rst_debug_x6_timeline(int nwg, int nwave) { x6_timeline_print(nwg, nwave); }
#endif

#ifndef X6W_RING
#define X6W_RING 2
#endif

constexpr int YT = 512;                             // threads per workgroup (8 waves)
constexpr int YPT = 8;                              // transform points per wave
constexpr int YST = (XPF4 + YT - 1) / YT;           // 2 staging float4 per thread
constexpr int YRING = X6W_RING;                     // U register ring (points in flight), divides 8
constexpr int YSTR = 132;                           // epilogue image row stride (floats): lh halves 32 banks apart
constexpr size_t YIMG_BYTES = (size_t)2 * 128 * YSTR * 4;       // epilogue: two halves' partial Y [pixel][channel]
constexpr size_t YRED_BYTES = (size_t)2 * 8 * 32 * 16;          // statistics reduction [2][8 waves][32] float4
constexpr size_t YEPI_BYTES = YIMG_BYTES + YRED_BYTES + 8 * XN * 8;   // + [8 waves][128] f64 (accumulator path)
constexpr size_t YLDS_BYTES = XLDS_BYTES > YEPI_BYTES ? XLDS_BYTES : YEPI_BYTES;
constexpr size_t YLDS_BLEND_BYTES = YLDS_BYTES + XMAX_CIN * sizeof(float2);   // + the second style's affine
static_assert(YLDS_BLEND_BYTES <= 160 * 1024, "LDS");
static_assert(8 % YRING == 0, "ring must divide the points per wave");

// Input prefetch by the workgroups past the tiles (wino_x6_launch adds them at B = 1, where 225 tiles leave 31 of the 256
// CUs idle). In the chunk loop the staging loads of chunk c + 3 and the U ring's L2 loads share the in-order vmcnt
// counter, so the U loads issued after a staging load wait out its HBM latency when they are consumed two points later.
// With the input already in the XCD's L2 that wait is an L2 latency. A prefetch workgroup with blockIdx % 8 = r (one XCD
// under the round-robin dispatch, speed only) reads one dword of every 128-B line of the input patches of the tiles
// xcd_tile_order gives the compute workgroups of residue r (and of the residual source), chunk pairs 1.. in order
// (chunks 0 and 1 the compute workgroups load at their start), split over the prefetch workgroups of residue r.
__device__ __forceinline__ unsigned x6_prefetch_input(const WinoArgs& a, int n_units, bool res) {
    const int r = (int)(blockIdx.x & 7);
    const int nk = (n_units - r + 7) >> 3;   // compute workgroups (tiles) of residue r
    if (nk <= 0) return 0u;
    const int base = n_units >> 3, rem = n_units & 7;
    const int t0 = r * base + min(r, rem);   // xcd_tile_order: their tiles are t0 .. t0 + nk - 1
    const int first = n_units + ((r - (n_units & 7)) & 7);   // first prefetch workgroup of residue r
    const int np = ((int)gridDim.x - first + 7) >> 3, j = ((int)blockIdx.x - first) >> 3;
    const int nq = a.cin >> 5;               // 128-B lines (32 channels) per pixel
    if (np <= 0 || nq < 2) return 0u;
    const int H = a.H, W = a.W;
    const int per_line = nk * XNP;           // lines of one chunk pair over the XCD's tiles
    const int n_items = (nq - 1) * per_line;
    const __amdgpu_buffer_rsrc_t isrd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.in), 0, (int)((size_t)a.batch * H * W * a.cin * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsrd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(res ? a.res : a.in), 0, (int)((size_t)a.batch * H * W * a.cin * 4), 0x00020000);
    unsigned f = 0u;
    for (int it = j * YT + (int)threadIdx.x; it < n_items; it += np * YT) {
        const int q = 1 + it / per_line, rr = it - (q - 1) * per_line;
        const int tl = rr / XNP, px = rr - tl * XNP;
        int t = t0 + tl;
        const int tx = t % a.tiles_x;
        t /= a.tiles_x;
        const int ty = t % a.tiles_y, b = t / a.tiles_y;
        const int iy = min(max(ty * XTH - 1 + px / XPW, 0), H - 1), ix = min(max(tx * XTW - 1 + px % XPW, 0), W - 1);
        const int off = (int)((((size_t)b * H + iy) * W + ix) * a.cin * 4) + q * 128;
        f ^= __builtin_amdgcn_raw_buffer_load_b32(isrd, off, 0, 0);
        if (res) f ^= __builtin_amdgcn_raw_buffer_load_b32(rsrd, off, 0, 0);
    }
    return f;   // (l2_touch_keep keeps the loads)
}

// BLEND: two styles — the prologue blends the two CIN affines per pixel (pro_ab1, pro_w)
template <int PRO, bool BLEND = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_x6_kernel(WinoArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* const patch = smem;                                            // [2][180][24] f32
    unsigned char* const vbytes = reinterpret_cast<unsigned char*>(smem + 2 * XPATCH_FL);   // [2][3][16][32][32 B]
    float2* const pab = reinterpret_cast<float2*>(vbytes + 2 * XV_BYTES);
    float2* const pab1 = reinterpret_cast<float2*>(reinterpret_cast<unsigned char*>(smem) + YLDS_BYTES);

    // wave-uniform by construction: the U loads' buffer offsets (from h) are then scalar operands; with a per-lane
    // wave index hipcc wrapped each of the 24 U loads per chunk in a readfirstlane waterfall loop
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 31, lh = lane >> 5;
    const int g = wave & 3, h = wave >> 2;   // output channel group, transform-point half
    XTL(0);
    const int n_units = a.batch * a.tiles_y * a.tiles_x;
    if ((int)blockIdx.x >= n_units) {   // a CU the tiles leave idle (B = 1): this XCD's later input chunks into its L2
        const unsigned f = x6_prefetch_input(a, n_units, PRO == PRO_AFF_RES);
        const l2_touch_t u = l2_touch_xcd_slice<YT, 2>(a.u_next, a.u_next_bytes);
        l2_touch_keep(l2_touch_t{f ^ u.x, u.y}, a.batch < 0, smem);
        tl_stamp_end(a.tl);
        return;
    }
    int bid = xcd_tile_order(blockIdx.x, n_units);
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * XTH, x0 = tx * XTW;
    const int H = a.H, W = a.W, Cin = a.cin;
    constexpr int pro = PRO;
    const size_t img = (size_t)b * H * W;
    const float* res_src = pro == PRO_AFF_RES ? a.res : a.in;
    const int nchunks = Cin / XCK;

    // the prologue affine into LDS (pab / pab1): given, or formed from the producer's fixed-point accumulators. The
    // accumulator loads are issued first (aff.issue, below) and merged after the first patch and U loads are issued
    // (aff.finish): vmcnt retires in order, so their wait does not include the later loads' HBM latency
    const bool split_aff = pro != PRO_NONE && a.pro_stat.acc != nullptr;   // wino_x6_launch: nslot <= 8
    CinAffineSplit<YT, 2> aff;
    auto load_affine = [&]() __attribute__((always_inline)) {
        if constexpr (pro != PRO_NONE) {
            if (a.pro_stat.acc != nullptr) {
                const bool store = tx == 0 && ty == 0;   // one workgroup per image keeps the host-visible copy
                const CinSrc& ps = a.pro_stat;
                aff.finish(ps, pab, BLEND ? pab1 : nullptr, store && ps.ab_out ? ps.ab_out + (size_t)b * Cin : nullptr,
                           store && ps.ab1_out ? ps.ab1_out + (size_t)b * Cin : nullptr);
            } else {
                for (int c = tid; c < Cin; c += YT) pab[c] = a.pro_ab[(size_t)b * Cin + c];
                if constexpr (BLEND)
                    for (int c = tid; c < Cin; c += YT) pab1[c] = a.pro_ab1[(size_t)b * Cin + c];
            }
        }
    };
    static_assert(!BLEND || PRO != PRO_NONE, "the blend is a prologue");

    // ---- staging descriptors (item k = float4 tid + 512k of a chunk's 720-float4 patch), as above --------
    int sg_goff[YST], sg_lf[YST], sg_moff[YST];
#pragma unroll
    for (int k = 0; k < YST; ++k) {
        const int it = tid + k * YT, itc = min(it, XPF4 - 1);
        const int px = itc >> 2, q = itc & 3;
        const int iy = y0 - 1 + px / XPW, ix = x0 - 1 + px % XPW;
        const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
        sg_goff[k] = (int)((img + (size_t)cy * W + cx) * Cin) + 4 * q;
        const bool inside = iy >= 0 && iy < H && ix >= 0 && ix < W;
        const int loff = it < XPF4 ? px * XPS + 4 * q : ((it - XPF4) >> 2) * XPS + XCK + 4 * (q & 1);
        sg_lf[k] = loff | (inside ? 1 << 16 : 0);
        const bool interior = it < XPF4 && inside && iy >= y0 && iy < y0 + XTH && ix >= x0 && ix < x0 + XTW;
        sg_moff[k] = interior ? (int)(((img + (size_t)iy * W + ix) * Cin + 4 * q) * 4) : 0x7F000000;
    }
    XTL(9);
    const __amdgpu_buffer_rsrc_t msrd = __builtin_amdgcn_make_buffer_rsrc(
        a.mat, 0, a.mat != nullptr ? (int)((size_t)a.batch * H * W * Cin * 4) : 0, 0x00020000);
    f32x4 xr[YST], rr[YST];
    float wr[YST];   // BLEND: the second style's weight at each staged pixel (loaded once: it has no channels)
#pragma unroll
    for (int k = 0; k < YST; ++k) {
        rr[k] = xr[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        wr[k] = 0.f;
        if constexpr (BLEND) wr[k] = a.pro_w[(sg_goff[k] - 4 * (tid & 3)) / Cin];
    }
    auto gload = [&](int k, int chunk) __attribute__((always_inline)) {
        const int gi = sg_goff[k] + chunk * XCK;
        xr[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
        if constexpr (pro == PRO_AFF_RES) rr[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
    };
    // chunk 1's staging loads, issued with chunk 0's at the start (registers that are free before the loop), so the
    // staging of chunk 1 does not wait for a load issued after chunk 0's staging
    f32x4 xr1[YST], rr1[YST];
    auto gload1 = [&](int k) __attribute__((always_inline)) {
        const int gi = sg_goff[k] + XCK;
        xr1[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
        if constexpr (pro == PRO_AFF_RES) rr1[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
    };
    // the materialised block output of staging item k of a chunk
    auto mat_store = [&](int k, int chunk, f32x4 v) __attribute__((always_inline)) {
        if (a.mat != nullptr) {
            if (a.wt_stores & 2)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), msrd, sg_moff[k] + chunk * XCK * 4, 0, 16);
            else
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), msrd, sg_moff[k] + chunk * XCK * 4, 0, 0);
        }
    };
    // prologue of the staged value (affine [+ ReLU | + residual]) and (store) the materialised block output
    auto stage_math = [&](int k, int chunk, f32x4 p01, f32x4 p23, bool store = true) __attribute__((always_inline)) {
        f32x4 v = xr[k];
        if constexpr (pro != PRO_NONE) {
            const f32x4 r = rr[k];
            if constexpr (BLEND) {
                const f32x4 q01 = *reinterpret_cast<const f32x4*>(pab1 + chunk * XCK + 4 * (tid & 3));
                const f32x4 q23 = *reinterpret_cast<const f32x4*>(pab1 + chunk * XCK + 4 * (tid & 3) + 2);
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
            if (store) mat_store(k, chunk, v);
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
    const int cq4 = 4 * (tid & 3);   // channel quad of every staging item of this thread
    auto stage_all = [&](int chunk, float* pbuf) __attribute__((always_inline)) {
        sfor<0, YST>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            f32x4 p01 = f32x4{0.f, 0.f, 0.f, 0.f}, p23 = p01;
            if constexpr (pro != PRO_NONE) {
                p01 = *reinterpret_cast<const f32x4*>(pab + chunk * XCK + cq4);
                p23 = *reinterpret_cast<const f32x4*>(pab + chunk * XCK + cq4 + 2);
            }
            stage_write(k, pbuf, stage_math(k, chunk, p01, p23));
        });
    };

    // ---- U pieces: lane (li, lh) of wave (g, h) reads U[chunk][8h + x][piece][32g + li][8lh .. 8lh+7] ------
    const __amdgpu_buffer_rsrc_t usrd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.U), 0, nchunks * XXI * 3 * XN * XVROW, 0x00020000);
    const int uvoff = (g * 32 + li) * XVROW + 16 * lh;
    short8 ur[YRING][3];
    auto load_u1 = [&](int chunk, int x, int s, int p) __attribute__((always_inline)) {
        ur[s][p] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(
                                                 usrd, uvoff, ((chunk * XXI + 8 * h + x) * 3 + p) * (XN * XVROW), 0));
    };

    // ---- input transform + split: thread = (half h, tile tt, channel pair cp) --------------------------
    // Rows 2h, 2h+1 of B^T d from patch rows f0, f1, f2 = (d0, d2, d1) for h = 0, (d2, d1, d3) for h = 1:
    // row 2h = f0 - f1, row 2h+1 = f1 + sgn f2 (sgn = +1 / -1; an fma with a +-1 factor rounds as the add).
    const int tt = (tid >> 3) & 31, cp = tid & 7;
    const int twy = tt >> 3, twx = tt & 7;
    const int rd0 = ((2 * twy) * XPW + 2 * twx) * XPS + 2 * cp;
    const int rofs0 = (2 * h) * XPW * XPS, rofs1 = (2 - h) * XPW * XPS, rofs2 = (1 + 2 * h) * XPW * XPS;
    const float sgn = h ? -1.f : 1.f;
    const int vwoff = tt * XVROW + 16 * ((cp >> 2) ^ ((tt >> 3) & 1)) + 4 * (cp & 3) + 8 * h * 32 * XVROW;
    float fx[3][4], fy[3][4];
    auto tr_read_col = [&](const float* pbuf, int c) __attribute__((always_inline)) {
        const f32x2 v0 = *reinterpret_cast<const f32x2*>(pbuf + rd0 + rofs0 + c * XPS);
        const f32x2 v1 = *reinterpret_cast<const f32x2*>(pbuf + rd0 + rofs1 + c * XPS);
        const f32x2 v2 = *reinterpret_cast<const f32x2*>(pbuf + rd0 + rofs2 + c * XPS);
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
    auto piece = [&](float& x, float& y, unsigned& p) __attribute__((always_inline)) { p = bf16_piece(x, y); };
    auto last_piece = [&](float x, float y) __attribute__((always_inline)) {
        return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
    };
    auto vwrite = [&](unsigned char* vbuf, int lx, unsigned p0, unsigned p1, unsigned p2) __attribute__((always_inline)) {
        *reinterpret_cast<unsigned*>(vbuf + ((0 * XXI + lx) * 32) * XVROW + vwoff) = p0;
        *reinterpret_cast<unsigned*>(vbuf + ((1 * XXI + lx) * 32) * XVROW + vwoff) = p1;
        *reinterpret_cast<unsigned*>(vbuf + ((2 * XXI + lx) * 32) * XVROW + vwoff) = p2;
    };
    // (B^T d) B of row rs (0: f0, 1: f2), points q0, q0 + 1 (local points lx = 4 rs + q0, + 1)
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

    floatx16 acc[YPT];
#pragma unroll
    for (int x = 0; x < YPT; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

    // ---- pipeline fill: V(0) in V[0], patch(1) in patch[1], patch(2) loads and U(0, 0..R-1) in flight ----
    if (split_aff) aff.issue(a.pro_stat, b, BLEND);
    XTL(10);
    sfor<0, YST>([&](auto K) __attribute__((always_inline)) { gload(decltype(K)::value, 0); });
    if (nchunks > 1) sfor<0, YST>([&](auto K) __attribute__((always_inline)) { gload1(decltype(K)::value); });
    XTL(11);
    sfor<0, YRING>([&](auto X) __attribute__((always_inline)) {
        sfor<0, 3>([&](auto Pc) __attribute__((always_inline)) {
            load_u1(0, decltype(X)::value, decltype(X)::value, decltype(Pc)::value);
        });
    });
    XTL(8);
    load_affine();
    XTL(4);
    if constexpr (pro != PRO_NONE) lds_barrier();   // pab visible before the first staging
    stage_all(0, patch);
    lds_barrier();
    XTL(5);
    transform_all(patch, vbytes);
    if (nchunks > 1) {
#pragma unroll
        for (int k = 0; k < YST; ++k) {
            xr[k] = xr1[k];
            rr[k] = rr1[k];
        }
        stage_all(1, patch + XPATCH_FL);
        if (nchunks > 2) sfor<0, YST>([&](auto K) __attribute__((always_inline)) { gload(decltype(K)::value, 2); });
    }
    lds_barrier();

    XTL(1);
    const int varow = li * XVROW + 16 * (lh ^ ((li >> 3) & 1)) + 8 * h * 32 * XVROW;
    unsigned qa0 = 0, qa1 = 0, qb0 = 0, qb1 = 0;
    f32x4 sp01 = f32x4{0.f, 0.f, 0.f, 0.f}, sp23 = sp01, sv = sp01, sv0 = sp01;
    static_assert(YST == 2, "the late materialised stores hold the chunk's two staging items");

    for (int c = 0; c < nchunks; ++c) {
        const int P = c & 1;
        const int c1 = min(c + 1, nchunks - 1), c2 = min(c + 2, nchunks - 1), c3 = min(c + 3, nchunks - 1);
        const unsigned char* va = vbytes + P * XV_BYTES + varow;
        unsigned char* const vnext = vbytes + (1 - P) * XV_BYTES;
        const float* const pnext = patch + (1 - P) * XPATCH_FL;
        float* const pstage = patch + P * XPATCH_FL;
        short8 av[2][3];
        sfor<0, 3>([&](auto Pc) __attribute__((always_inline)) {
            constexpr int p = decltype(Pc)::value;
            av[0][p] = *reinterpret_cast<const short8*>(va + (p * XXI) * 32 * XVROW);
        });
        __builtin_amdgcn_sched_barrier(0);
        sfor<0, YPT>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            constexpr int s = x % YRING;
            sfor<0, 6>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                constexpr int ap = k == 2 || k == 4 ? 1 : (k == 5 ? 2 : 0);
                constexpr int bp = k == 1 || k == 4 ? 1 : (k == 3 ? 2 : 0);
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[x & 1][ap], ur[s][bp], acc[x], 0, 0, 0);
                if constexpr (k == 0 && x + 1 < YPT) {
                    sfor<0, 3>([&](auto Pc) __attribute__((always_inline)) {
                        constexpr int p = decltype(Pc)::value;
                        av[(x + 1) & 1][p] = *reinterpret_cast<const short8*>(va + (p * XXI + x + 1) * 32 * XVROW);
                    });
                }
                if constexpr (k >= 3) {   // U ring refill (B2, B1, B0 last read by MFMAs 3, 4, 5)
                    constexpr int xn = (x + YRING) % YPT;
                    load_u1(x + YRING < YPT ? c : c1, xn, s, 5 - k);
                }
                // transform + split of chunk c+1 into V[1-P]
                if constexpr (x == 0 && k < 4) tr_read_col(pnext, k);
                if constexpr (x == 1 && k < 4) tr_rows_col(k);
                if constexpr (x >= 2 && x < 6) {
                    constexpr int rs = (x - 2) >> 1, q0 = ((x - 2) & 1) * 2, lx0 = 4 * rs + q0;
                    if constexpr (k == 0) cols(rs, q0);
                    if constexpr (k == 1) piece(w0x, w0y, qa0);
                    if constexpr (k == 2) piece(w0x, w0y, qa1);
                    if constexpr (k == 3) {
                        vwrite(vnext, lx0, qa0, qa1, last_piece(w0x, w0y));
                        piece(w1x, w1y, qb0);
                    }
                    if constexpr (k == 4) piece(w1x, w1y, qb1);
                    if constexpr (k == 5) vwrite(vnext, lx0 + 1, qb0, qb1, last_piece(w1x, w1y));
                }
                // staging of chunk c+2 into patch[P], then the loads of chunk c+3 into the freed registers
                if constexpr (x >= 6) {
                    constexpr int ks = x - 6;
                    if constexpr (k == 0 && pro != PRO_NONE) {
                        sp01 = *reinterpret_cast<const f32x4*>(pab + c2 * XCK + cq4);
                        sp23 = *reinterpret_cast<const f32x4*>(pab + c2 * XCK + cq4 + 2);
                    }
                    if constexpr (k == 2) sv = stage_math(ks, c2, sp01, sp23, !X6_MAT_LATE);
                    if constexpr (k == 4) stage_write(ks, pstage, sv);
                    if constexpr (X6_MAT_LATE && k == 4 && ks == 0) sv0 = sv;
                    if constexpr (k == 5) gload(ks, c3);
                    // X6_MAT_LATE: the chunk's materialised stores after all of its U and staging loads (below)
                    if constexpr (X6_MAT_LATE && pro != PRO_NONE && k == 5 && ks == YST - 1) {
                        mat_store(0, c2, sv0);
                        mat_store(1, c2, sv);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            });
        });
        lds_barrier();
    }

    XTL(2);
    // ---- the next layer's weights into this XCD's L2 (speed only), landing while the epilogue runs
    const l2_touch_t upf = l2_touch_xcd_slice<YT, 2>(a.u_next, a.u_next_bytes);
    // ---- epilogue: partial output transform per half -> LDS image, then sum + bias + ReLU + store + stats --
    float* const yimg = smem + h * (128 * YSTR);
    {
        const int co = g * 32 + li;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = (j & 3) + 8 * (j >> 2) + 4 * lh;   // Winograd tile of this accumulator row
            const int wy = row >> 3, wx = row & 7;
            float t0[4], t1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {   // T = A^T M over this half's two rows of M
                const float ma = acc[q][j], mb = acc[4 + q][j];
                t0[q] = h == 0 ? ma + mb : ma;
                t1[q] = h == 0 ? mb : -ma - mb;
            }
            const float yy[4] = {t0[0] + t0[1] + t0[2], t0[1] - t0[2] - t0[3], t1[0] + t1[1] + t1[2],
                                 t1[1] - t1[2] - t1[3]};
#pragma unroll
            for (int q = 0; q < 4; ++q) yimg[((2 * wy + (q >> 1)) * XTW + 2 * wx + (q & 1)) * YSTR + co] = yy[q];
        }
    }
    lds_barrier();
    XTL(6);
    // thread = (pixel column pr, channel quad cq); rows 0..7 of the tile
    const int cq = tid & 31, pr = tid >> 5;
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bias + 4 * cq);
    const __amdgpu_buffer_rsrc_t osrd =
        __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)((size_t)a.batch * H * W * XN * 4), 0x00020000);
    const bool col_ok = x0 + pr < W;
    f32x4 yv[XTH];
    f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < XTH; ++i) {
        const int off = (i * XTW + pr) * YSTR + 4 * cq;
        f32x4 v = *reinterpret_cast<const f32x4*>(smem + off) + *reinterpret_cast<const f32x4*>(smem + 128 * YSTR + off) + b4;
        if (!a.linear) {
            v.x = fmaxf(v.x, 0.f);
            v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f);
            v.w = fmaxf(v.w, 0.f);
        }
        const bool ok = col_ok && y0 + i < H;
        if (ok) {
            float* const po = a.out + (img + (size_t)(y0 + i) * W + x0 + pr) * XN + 4 * cq;
            if (a.wt_stores & 1)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), osrd,
                                                       (int)((po - a.out) * 4), 0, 16);
            else
                *reinterpret_cast<f32x4*>(po) = v;
        }
        yv[i] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        s4 += yv[i];
    }
    XTL(7);
    auto xsum = [&](f32x4 v) __attribute__((always_inline)) {
        v.x = lane_xor_sum<32>(v.x);
        v.y = lane_xor_sum<32>(v.y);
        v.z = lane_xor_sum<32>(v.z);
        v.w = lane_xor_sum<32>(v.w);
        return v;
    };
    f32x4* const red = reinterpret_cast<f32x4*>(reinterpret_cast<unsigned char*>(smem) + YIMG_BYTES);   // [2][8][32]
    if (a.stat.acc != nullptr) {
        // accumulator path: {S, M2 + S^2 / n} (finalize_kernel's merge quantity, a sum of squares formed around a
        // local mean) is additive over any partition of the tile, so each wave forms it over its own two pixel
        // columns (two-pass around the wave's mean, in registers) and the eight waves meet in LDS once, in f64 and
        // a fixed order: one barrier instead of the tile mean's two
        s4 = xsum(s4);
        const int vc = (x0 + 2 * wave < W ? 1 : 0) + (x0 + 2 * wave + 1 < W ? 1 : 0);
        const float nw = (float)(vc * min(XTH, H - y0));
        const f32x4 mw = nw > 0.f ? s4 / nw : f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 m2 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < XTH; ++i) {
            const bool ok = col_ok && y0 + i < H;
            const f32x4 d = yv[i] - mw;
            if (ok) m2 += d * d;
        }
        m2 = xsum(m2);
        float* const sf = reinterpret_cast<float*>(red);                                                  // [8][128]
        double* const qd = reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(smem) + YIMG_BYTES + YRED_BYTES);
        if (lh == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double dS = (double)s4[k];
                sf[wave * XN + 4 * cq + k] = s4[k];
                qd[wave * XN + 4 * cq + k] = nw > 0.f ? (double)m2[k] + dS * dS / (double)nw : 0.0;
            }
        }
        lds_barrier();
        if (tid < XN) {
            double S = 0.0, Q = 0.0;
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                S += (double)sf[w * XN + tid];
                Q += qd[w * XN + tid];
            }
            const int slot = (int)blockIdx.x % a.stat.nslot;
            cin_acc_add_value(a.stat, a.batch, XN, b, tid, slot, 0, S);
            cin_acc_add_value(a.stat, a.batch, XN, b, tid, slot, 1, Q);
        }
    } else if (a.part != nullptr) {
        const float cnt = (float)(min(XTH, H - y0) * min(XTW, W - x0));
        s4 = xsum(s4);
        if (lh == 0) red[wave * 32 + cq] = s4;
        lds_barrier();
        f32x4 S = red[cq];
#pragma unroll
        for (int w = 1; w < 8; ++w) S += red[w * 32 + cq];
        const f32x4 mean = S / cnt;
        f32x4 m2 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < XTH; ++i) {
            const bool ok = col_ok && y0 + i < H;
            const f32x4 d = yv[i] - mean;
            if (ok) m2 += d * d;
        }
        m2 = xsum(m2);
        if (lh == 0) red[256 + wave * 32 + cq] = m2;
        lds_barrier();
        if (tid < 32) {
            f32x4 M = red[256 + cq];
#pragma unroll
            for (int w = 1; w < 8; ++w) M += red[256 + w * 32 + cq];
            const int n_part = a.tiles_y * a.tiles_x;
            float4* const dst = a.part + ((size_t)b * XN + 4 * cq) * n_part + ty * a.tiles_x + tx;
            dst[0] = make_float4(S.x, M.x, cnt, 0.f);
            dst[n_part] = make_float4(S.y, M.y, cnt, 0.f);
            dst[2 * n_part] = make_float4(S.z, M.z, cnt, 0.f);
            dst[3 * n_part] = make_float4(S.w, M.w, cnt, 0.f);
        }
    }
    XTL(3);
    l2_touch_keep(upf, a.batch < 0, smem);
    tl_stamp_end(a.tl);
}

bool wino_x6_supported(int kh, int stride, int cin, int cout) {
    return kh == 3 && stride == 1 && cout == XN && cin % XCK == 0 && cin <= XMAX_CIN;
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

// U pieces [chunk][xi][piece][co][16] bf16 (returned as the float-sized buffer holding the bits):
// U = G g G^T in f64 rounded to f32 (bitwise wino_pack_weights' value), then split into three bf16 pieces
// with round-to-nearest-even at each step (the device split of V does the same with v_cvt_pk_bf16_f32)
std::vector<float> wino_x6_pack_weights(const float* kern, int cin) {
#pragma clang fp contract(off)
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    const size_t n16 = (size_t)cin / XCK * XXI * 3 * XN * XCK;
    std::vector<uint16_t> U(n16);
    for (int ci = 0; ci < cin; ++ci)
        for (int co = 0; co < XN; ++co) {
            double g[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) g[i][j] = kern[(((size_t)i * 3 + j) * cin + ci) * XN + co];
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
                    const int chunk = ci / XCK, c = ci % XCK, xi = p * 4 + q;
                    for (int k = 0; k < 3; ++k)
                        U[((((size_t)chunk * XXI + xi) * 3 + k) * XN + co) * XCK + c] = pc[k];
                }
        }
    std::vector<float> out((n16 + 1) / 2);
    std::memcpy(out.data(), U.data(), n16 * 2);
    return out;
}

// Device form of wino_x6_pack_weights (training re-packs after every optimizer step): one thread per
// (ci, co), U = G g G^T in float64 with the host's operation order and no contraction, rounded to f32,
// then split into three bf16 pieces with round-to-nearest-even at each step — bitwise the host image.
__device__ __forceinline__ void x6_transform_one(const float* __restrict__ kern, int cin, unsigned short* __restrict__ U,
                                                 int idx) {
#pragma clang fp contract(off)
    if (idx >= cin * XN) return;
    const int ci = idx / XN, co = idx - (idx / XN) * XN;
    const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    double g[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[i][j] = kern[(((size_t)i * 3 + j) * cin + ci) * XN + co];
    const int chunk = ci / XCK, c = ci % XCK;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double u = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) u = u + G[p][i] * g[i][j] * G[q][j];
            const float uf = (float)u;
            // pieces as the host computes them: RNE to bf16, remainder exact in f32
            const unsigned b0 = __builtin_bit_cast(unsigned short, (__bf16)uf);
            const float r = uf - __uint_as_float(b0 << 16);
            const unsigned b1 = __builtin_bit_cast(unsigned short, (__bf16)r);
            const unsigned b2 = __builtin_bit_cast(unsigned short, (__bf16)(r - __uint_as_float(b1 << 16)));
            const size_t base = ((size_t)chunk * XXI + p * 4 + q) * 3;
            U[((base + 0) * XN + co) * XCK + c] = (unsigned short)b0;
            U[((base + 1) * XN + co) * XCK + c] = (unsigned short)b1;
            U[((base + 2) * XN + co) * XCK + c] = (unsigned short)b2;
        }
}

__global__ __launch_bounds__(256) void wino_x6_transform_kernel(const float* __restrict__ kern, int cin,
                                                                unsigned short* __restrict__ U) {
    x6_transform_one(kern, cin, U, blockIdx.x * 256 + threadIdx.x);
}

// batched form: job = blockIdx.x / blocks_per_job (jobs with a smaller cin leave their last blocks idle)
__global__ __launch_bounds__(256) void wino_x6_transform_batch_kernel(X6TransformJobs jobs, int blocks_per_job) {
    const int job = blockIdx.x / blocks_per_job, blk = blockIdx.x - job * blocks_per_job;
    if (job >= jobs.n) return;
    x6_transform_one(jobs.kern[job], jobs.cin[job], reinterpret_cast<unsigned short*>(jobs.U[job]),
                     blk * 256 + threadIdx.x);
}

hipError_t wino_x6_transform_batch_launch(const X6TransformJobs& jobs, hipStream_t st) {
    if (jobs.n <= 0) return hipSuccess;
    if (jobs.n > X6_MAX_JOBS) return hipErrorInvalidValue;
    int max_cin = 0;
    for (int k = 0; k < jobs.n; ++k) {
        if (jobs.cin[k] % XCK != 0 || jobs.cin[k] > XMAX_CIN) return hipErrorInvalidValue;
        max_cin = jobs.cin[k] > max_cin ? jobs.cin[k] : max_cin;
    }
    const int bpj = (max_cin * XN + 255) / 256;
    hipLaunchKernelGGL(wino_x6_transform_batch_kernel, dim3((unsigned)(bpj * jobs.n)), dim3(256), 0, st, jobs, bpj);
    return hipGetLastError();
}

hipError_t wino_x6_transform_launch(const float* kern, int cin, float* U, hipStream_t st) {
    if (cin % XCK != 0 || cin > XMAX_CIN) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wino_x6_transform_kernel, dim3((unsigned)((cin * XN + 255) / 256)), dim3(256), 0, st, kern, cin,
                       reinterpret_cast<unsigned short*>(U));
    return hipGetLastError();
}

hipError_t wino_x6_prepare() {
    for (const void* k : {(const void*)wino_x6_kernel<PRO_NONE>, (const void*)wino_x6_kernel<PRO_AFF_RELU>,
                          (const void*)wino_x6_kernel<PRO_AFF>, (const void*)wino_x6_kernel<PRO_AFF_RES>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)YLDS_BYTES);
        if (e != hipSuccess) return e;
    }
    for (const void* k : {(const void*)wino_x6_kernel<PRO_AFF_RELU, true>, (const void*)wino_x6_kernel<PRO_AFF, true>,
                          (const void*)wino_x6_kernel<PRO_AFF_RES, true>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)YLDS_BLEND_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Optional kernel-execution timestamps for the next launch (rst_profile: the dominant kernel's duration
// measured by the dispatch itself, as rocprofv3 does, instead of marker events around the launch)
static thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
void wino_x6_set_timing_events(hipEvent_t start, hipEvent_t stop) {
    g_ev_start = start;
    g_ev_stop = stop;
}

hipError_t wino_x6_launch(const WinoArgs& a, hipStream_t st) {
    // the timing events belong to this launch only, also when it is refused below
    const hipEvent_t e0 = g_ev_start, e1 = g_ev_stop;
    g_ev_start = g_ev_stop = nullptr;
    if (a.cin % XCK != 0 || a.cin > XMAX_CIN || a.tiles_y != (a.H + XTH - 1) / XTH ||
        a.tiles_x != (a.W + XTW - 1) / XTW || (size_t)a.batch * a.H * a.W * a.cin * 4 >= (size_t)0x7F000000)
        return hipErrorInvalidValue;   // 32-bit staging offsets; the out-of-range store offset must stay out of range
    if (a.stat.acc != nullptr && (a.stat.nslot < 1 || a.stat.nslot > CIN_ACC_MAX_SLOTS))
        return hipErrorInvalidValue;
    const bool src_acc = a.pro_stat.acc != nullptr;
    // (nslot <= 8 and C <= 128: the kernel's split affine form, CinAffineSplit<512, 2>, covers the accumulators)
    if (src_acc && (a.pro_stat.nslot < 1 || a.pro_stat.nslot > 8 || a.pro_stat.C != a.cin || a.cin > XN ||
                    a.pro_stat.batch != a.batch || a.pro_stat.style == nullptr || a.pro_mode == PRO_NONE))
        return hipErrorInvalidValue;
    unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    {   // B = 1: the CUs the tiles leave idle prefetch the later input chunks into their XCD's L2 (x6_prefetch_input)
        static int n_cu = 0, pf = -1;
        if (pf < 0) {
            const char* e = getenv("RST_X6_PREFETCH");
            pf = e != nullptr ? atoi(e) : 1;
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                n_cu = 0;
        }
        if (pf && a.cin >= 64 && (int)grid < n_cu && (int)grid + 8 <= n_cu) grid = (unsigned)n_cu;
    }
    if (a.pro_w != nullptr) {   // two styles: the affines from pro_ab/pro_ab1, or both formed from pro_stat
        if (src_acc ? a.pro_stat.style1_offset < 0 : (a.pro_ab1 == nullptr || a.pro_ab == nullptr))
            return hipErrorInvalidValue;
        switch (a.pro_mode) {
            case PRO_AFF_RELU: hipExtLaunchKernelGGL((wino_x6_kernel<PRO_AFF_RELU, true>), dim3(grid), dim3(YT), YLDS_BLEND_BYTES, st, e0, e1, 0, a); break;
            case PRO_AFF: hipExtLaunchKernelGGL((wino_x6_kernel<PRO_AFF, true>), dim3(grid), dim3(YT), YLDS_BLEND_BYTES, st, e0, e1, 0, a); break;
            case PRO_AFF_RES: hipExtLaunchKernelGGL((wino_x6_kernel<PRO_AFF_RES, true>), dim3(grid), dim3(YT), YLDS_BLEND_BYTES, st, e0, e1, 0, a); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (a.pro_mode) {
        case PRO_NONE: hipExtLaunchKernelGGL(wino_x6_kernel<PRO_NONE>, dim3(grid), dim3(YT), YLDS_BYTES, st, e0, e1, 0, a); break;
        case PRO_AFF_RELU: hipExtLaunchKernelGGL(wino_x6_kernel<PRO_AFF_RELU>, dim3(grid), dim3(YT), YLDS_BYTES, st, e0, e1, 0, a); break;
        case PRO_AFF: hipExtLaunchKernelGGL(wino_x6_kernel<PRO_AFF>, dim3(grid), dim3(YT), YLDS_BYTES, st, e0, e1, 0, a); break;
        case PRO_AFF_RES: hipExtLaunchKernelGGL(wino_x6_kernel<PRO_AFF_RES>, dim3(grid), dim3(YT), YLDS_BYTES, st, e0, e1, 0, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rst
