// conv_last.hip — the final 9x9 Conv2DTranspose (16 -> 3 channels, SAME, stride 1) of the transfer
// network (realtime_style_transfer/models/styleTransfer.py:269-276, "expand_last") on the bf16 MFMA
// pipe with exact split-bf16 products (the RST_PRECISION_WINOGRAD_BF16X6 headline mode).
//
// A SAME 9x9 s1 transposed conv is the 9x9 correlation with the flipped kernel wf and pad 4. With
// three output channels an MFMA tile over (pixel, co) would idle 29 of 32 columns, so the kernel's
// column axis joins into N instead:
//   P[y][x'][(kx, co)] = sum_{ky, ci} in[y + ky - 4][x'][ci] . wf[ky][kx][ci][co]      (GEMM: M = x',
//                                                        K = (ky, ci) = 9 x 16, N = 9 x 3 = 27 of 32)
//   out[y][x][co]      = sum_kx P[y][x + kx - 4][(kx, co)]                          (diagonal sum)
// One v_mfma_f32_32x32x16_bf16 is one kernel row ky (K = the 16 input channels); each f32 operand is
// split exactly into three bf16 pieces (x = x0 + x1 + x2, all 24 significant bits) and the six product
// terms a0b0 a0b1 a1b0 a0b2 a1b1 a2b0 are accumulated in f32 (the dropped terms are <= 2^-25 of each
// product): fp32-level results, 6 bf16 MFMAs instead of 8 f32 ones per kernel row.
//
// Workgroup = 4 waves = 4 output rows x 120 output columns; x' spans the 128 input columns x0-4 ..
// x0+123 (4 MFMA tiles of 32). The 12 input rows of the tile (all 16 channels, CIN-apply + ReLU of
// expand_1 fused into the staging) sit in LDS as f32 with a 20-float pixel stride (odd 16-B slots:
// conflict-free A reads); the A fragment of each (tile, ky) is read as 2 x ds_read_b128 and split by
// the wave while the previous fragment's six MFMAs run (explicit slot interleave). The split weights
// (27 of 32 columns, 3 pieces) stay in 108 VGPRs. P goes through wave-private LDS for the diagonal
// sum; the epilogue adds the bias, stores the raw conv output and the tile's {sum, M2, n} per channel
// for the final CIN (finalize + sigmoid, norm.hip).
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>
#include <vector>

#include "kernels.h"

#ifdef LAST_PROF
// s_memrealtime (100 MHz) per (workgroup < 256, wave): start, staged, MFMAs done, end
__device__ unsigned long long last_tl[256][4][4];
__device__ unsigned long long last_st[256][4][8];
#define LSTL(k) \
    if (blockIdx.x < 256 && lane == 0) last_tl[blockIdx.x][wave][(k)] = __builtin_amdgcn_s_memrealtime()
#define LSST(kk, p) \
    if (blockIdx.x < 256 && lane == 0 && (kk) == 2) last_st[blockIdx.x][wave][(p)] = __builtin_amdgcn_s_memrealtime()
#else
#define LSTL(k)
#define LSST(kk, p)
#endif

namespace rst {

namespace lastx6 {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int CIN = 16, K = 9, PAD = 4;
constexpr int NT = 3, XW = 32 * NT;         // x' tiles of 32 per strip; x' columns per strip
constexpr int TWO = XW - (K - 1);           // 88 output columns per strip
constexpr int RB = 24;                      // output rows per workgroup (6 steps of 4: one row per wave)
constexpr int NS = RB / 4;
constexpr int RING = 12;                    // input row slots: rows 4k .. 4k + 11 of step k
constexpr int SLOT_B = 3 * 2 * XW * 16;     // bytes per row slot: [piece][k half][x'][8 bf16]
constexpr int RING_B = RING * SLOT_B;       // 110592
constexpr int PCOL = XW + 4;                // transposed P buffer [28 columns n][x'] row stride (floats):
                                            // 25 16-B slots, odd: conflict-free b128 writes
constexpr int P_B = 4 * 28 * PCOL * 4;      // 44800
constexpr int ROW_F4 = XW * CIN / 4;        // 384 float4 per staged input row
constexpr int PF = 4 * ROW_F4 / 256;        // 6 prefetch float4 per thread (4 rows)
constexpr size_t LDS_BYTES = (size_t)RING_B + P_B + 2 * 16 * 4 * 4 + 2 * CIN * 8;   // + prologue affine table
static_assert((4 * ROW_F4) % 256 == 0, "staging map");

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

// (x, y) -> three packed bf16 pairs, x = x0 + x1 + x2 exactly (round-to-nearest-even at each step)
__device__ __forceinline__ void split3(float x, float y, unsigned& p0, unsigned& p1, unsigned& p2) {
    p0 = bf16_piece(x, y);
    p1 = bf16_piece(x, y);
    p2 = bf16_last_piece(x, y);
}
// Sum over the 64 lanes of a wave, the same value in every lane, fixed order (deterministic): DPP
// butterflies inside each row of 16 (quad xor 1, xor 2, half-row mirror, row mirror), then the four row
// sums read out of lanes 0/16/32/48 — VALU only, no LDS round trips (ds_bpermute-based __shfl_xor
// chains cost ~1 us per step here).
__device__ __forceinline__ float wave_sum(float x) {
    auto dpp = [](float v, auto CTRL) __attribute__((always_inline)) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), decltype(CTRL)::value, 0xF, 0xF, true));
    };
    x += dpp(x, std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
    x += dpp(x, std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]
    x += dpp(x, std::integral_constant<int, 0x141>{});   // row_half_mirror
    x += dpp(x, std::integral_constant<int, 0x140>{});   // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
    return (r0 + r1) + (r2 + r3);
}
}  // namespace lastx6

// PROF: PRO_NONE / PRO_AFF_RELU, | 8 for two styles (the per-pixel blend of the two CIN affines)
template <int PROF>
__global__ __launch_bounds__(256, 1) void last_x6_kernel(LastArgs a) {
    using namespace lastx6;
    constexpr int PRO = PROF & 7;
    constexpr bool BLEND = (PROF & 8) != 0;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    unsigned char* const ring = reinterpret_cast<unsigned char*>(smem);        // [RING][3][2][XW][16 B]
    float* const pbuf = reinterpret_cast<float*>(ring + RING_B);               // [4 waves][28][PCOL] P^T
    float* const red = pbuf + P_B / 4;                                         // [2 steps][4 waves][4][4] stats

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    LSTL(0);
    int bid = xcd_tile_order(blockIdx.x, gridDim.x);
    const int sx = bid % a.tiles_x;                 // column strip
    bid /= a.tiles_x;
    const int n_rb = (a.H + RB - 1) / RB;
    const int rb = bid % n_rb;                      // row block
    const int b = bid / n_rb;
    const int y0 = rb * RB, x0 = sx * TWO;
    const int H = a.H, W = a.W;

    // the prologue affine's accumulator loads first (CinAffineSplit): merged after the weight and first row loads are
    // issued, so its wait does not include their latency (vmcnt retires in issue order)
    const bool split_aff = PRO != PRO_NONE && a.pro_stat.acc != nullptr;   // last_x6_launch: nslot <= 8
    CinAffineSplit<256, 2> aff;
    if (split_aff) aff.issue(a.pro_stat, b, BLEND);
    // ---- weights: lane (n = lane & 31, k half) holds B[ky][piece] = 8 bf16 of column n, 108 VGPRs -------
    short8 bw[K][3];
    {
        const u32x4* wp = reinterpret_cast<const u32x4*>(a.w);
        sfor<0, K>([&](auto KY) __attribute__((always_inline)) {
            constexpr int ky = decltype(KY)::value;
            sfor<0, 3>([&](auto P) __attribute__((always_inline)) {
                constexpr int p = decltype(P)::value;
                bw[ky][p] = __builtin_bit_cast(short8, wp[((ky * 3 + p) * 32 + (lane & 31)) * 2 + (lane >> 5)]);
            });
        });
    }
    const float bias0 = a.bias[0], bias1 = a.bias[1], bias2 = a.bias[2];

    // ---- staging of 4 input rows (relative rows r0 .. r0 + 3, relative row 0 = y0 - 4): item
    // it = tid + 256 k -> (row, x', channel quad q = tid & 3); CIN-apply + ReLU of expand_1 fused; each
    // value split into three bf16 pieces and written to the ring in the MFMA operand layout ----------------
    const int q = tid & 3;
    f32x4 pa01 = {1.f, 0.f, 1.f, 0.f}, pa23 = {1.f, 0.f, 1.f, 0.f}, pb01 = pa01, pb23 = pa23;
    // the prologue affine (given, or formed from the producer's fixed-point accumulators), after the first rows' loads
    // are issued so its latency overlaps theirs
    auto load_affine = [&]() __attribute__((always_inline)) {
    if constexpr (PRO != PRO_NONE) {
        const float2* ab = a.pro_ab + (size_t)b * CIN;
        const float2* ab1 = BLEND ? a.pro_ab1 + (size_t)b * CIN : nullptr;
        if (a.pro_stat.acc != nullptr) {   // formed from the producer's fixed-point accumulators (no finalize ran)
            float2* const ltab = reinterpret_cast<float2*>(red + 128);   // [2][16]
            const CinSrc& ps = a.pro_stat;
            const bool store = rb == 0 && sx == 0;   // one workgroup per image keeps the host-visible copy
            aff.finish(ps, ltab, BLEND ? ltab + CIN : nullptr, store && ps.ab_out ? ps.ab_out + (size_t)b * CIN : nullptr,
                       store && ps.ab1_out ? ps.ab1_out + (size_t)b * CIN : nullptr);
            lds_barrier();
            ab = ltab;
            ab1 = ltab + CIN;
        }
        const f32x4* pa = reinterpret_cast<const f32x4*>(ab + 4 * q);
        pa01 = pa[0];
        pa23 = pa[1];
        if constexpr (BLEND) {
            const f32x4* pb = reinterpret_cast<const f32x4*>(ab1 + 4 * q);
            pb01 = pb[0];
            pb23 = pb[1];
        }
    }
    };
    f32x4 pre[PF], pre2[PF];
    float prw[PF], prw2[PF];   // BLEND: the second style's weight at each staged pixel
    auto load_rows = [&](int r0, f32x4 (&pre)[PF], float (&prw)[PF]) __attribute__((always_inline)) {
        sfor<0, PF>([&](auto Kk) __attribute__((always_inline)) {
            constexpr int k = decltype(Kk)::value;
            const int it = tid + 256 * k, r = it / ROW_F4, xp = (it % ROW_F4) >> 2;
            const int iy = min(max(y0 - PAD + r0 + r, 0), H - 1), ix = min(max(x0 - PAD + xp, 0), W - 1);
            pre[k] = *reinterpret_cast<const f32x4*>(a.in + (((size_t)b * H + iy) * W + ix) * CIN + 4 * q);
            if constexpr (BLEND) prw[k] = a.pro_w[((size_t)b * H + iy) * W + ix];
        });
    };
    auto store_rows = [&](int r0, const f32x4 (&pre)[PF], const float (&prw)[PF]) __attribute__((always_inline)) {
        sfor<0, PF>([&](auto Kk) __attribute__((always_inline)) {
            constexpr int k = decltype(Kk)::value;
            const int it = tid + 256 * k, r = it / ROW_F4, xp = (it % ROW_F4) >> 2;
            const int iy = y0 - PAD + r0 + r, ix = x0 - PAD + xp;
            f32x4 t = pre[k];
            if constexpr (BLEND) {   // styleTransfer.py:36-44 (conv_mfma.hip's blend prologue)
                const float w = prw[k];
                t.x = fmaxf(style_blend(w, fmaf(pa01.x, t.x, pa01.y), fmaf(pb01.x, t.x, pb01.y)), 0.f);
                t.y = fmaxf(style_blend(w, fmaf(pa01.z, t.y, pa01.w), fmaf(pb01.z, t.y, pb01.w)), 0.f);
                t.z = fmaxf(style_blend(w, fmaf(pa23.x, t.z, pa23.y), fmaf(pb23.x, t.z, pb23.y)), 0.f);
                t.w = fmaxf(style_blend(w, fmaf(pa23.z, t.w, pa23.w), fmaf(pb23.z, t.w, pb23.w)), 0.f);
            } else if constexpr (PRO != PRO_NONE) {
                t.x = fmaxf(fmaf(pa01.x, t.x, pa01.y), 0.f);
                t.y = fmaxf(fmaf(pa01.z, t.y, pa01.w), 0.f);
                t.z = fmaxf(fmaf(pa23.x, t.z, pa23.y), 0.f);
                t.w = fmaxf(fmaf(pa23.z, t.w, pa23.w), 0.f);
            }
            if (!(iy >= 0 && iy < H && ix >= 0 && ix < W)) t = f32x4{0.f, 0.f, 0.f, 0.f};
            unsigned p0[2], p1[2], p2[2];
            split3(t.x, t.y, p0[0], p1[0], p2[0]);
            split3(t.z, t.w, p0[1], p1[1], p2[1]);
            // channels 4q .. 4q+3 = k half q >> 1, bf16 slots 4 (q & 1) .. +3 of the lane's 8
            unsigned char* dst = ring + ((r0 + r) % RING) * SLOT_B + ((q >> 1) * XW + xp) * 16 + (q & 1) * 8;
            *reinterpret_cast<uint2*>(dst) = make_uint2(p0[0], p0[1]);
            *reinterpret_cast<uint2*>(dst + 2 * XW * 16) = make_uint2(p1[0], p1[1]);
            *reinterpret_cast<uint2*>(dst + 4 * XW * 16) = make_uint2(p2[0], p2[1]);
        });
    };
    load_rows(0, pre, prw);
    load_rows(4, pre2, prw2);
    load_affine();
    store_rows(0, pre, prw);
    load_rows(8, pre, prw);
    store_rows(4, pre2, prw2);
    store_rows(8, pre, prw);
    lds_barrier();
    LSTL(1);

    // ---- steps: 4 output rows (one per wave); the input rows of step k+1 were loaded two steps earlier
    // (two register buffers: the HBM latency under load exceeds one step's MFMAs) -------------------------
    const unsigned char* const abase = ring + ((lane >> 5) * XW + (lane & 31)) * 16;   // + slot + piece + tile
    float* const pw = pbuf + wave * (28 * PCOL);
    const int n = lane & 31;
    const int n_tiles4 = (H + 3) / 4;
    // the output CIN's statistics into fixed-point accumulators (a.stat): lanes tid < 3 sum this workgroup's tiles
    // ({S, M2 + S^2/n}, finalize_kernel's merge quantity) and add them once at the end
    const bool to_acc = a.stat.acc != nullptr;
    double accS = 0.0, accQ = 0.0;
    auto step = [&](int k) __attribute__((always_inline)) {
        LSST(k, 0);
        f32x16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;
        // MFMA step s = (tile t, ky): A pieces of input row 4k + wave + ky, read one step ahead
        auto read = [&](int s, short8 (&A)[3]) __attribute__((always_inline)) {
            const unsigned char* p = abase + ((4 * k + wave + s % K) % RING) * SLOT_B + 32 * (s / K) * 16;
            A[0] = *reinterpret_cast<const short8*>(p);
            A[1] = *reinterpret_cast<const short8*>(p + 2 * XW * 16);
            A[2] = *reinterpret_cast<const short8*>(p + 4 * XW * 16);
        };
        short8 A0[3], A1[3];
        read(0, A0);
        sfor<0, NT * K>([&](auto S) __attribute__((always_inline)) {
            constexpr int s = decltype(S)::value, t = s / K, ky = s % K;
            if constexpr (s + 1 < NT * K) {
                if constexpr ((s & 1) == 0) read(s + 1, A1);
                else read(s + 1, A0);
            }
            __builtin_amdgcn_sched_barrier(0);
            constexpr int ap[6] = {0, 0, 1, 0, 1, 2}, bp[6] = {0, 1, 0, 2, 1, 0};
            sfor<0, 6>([&](auto M) __attribute__((always_inline)) {
                constexpr int mm = decltype(M)::value;
                if constexpr ((s & 1) == 0)
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0[ap[mm]], bw[ky][bp[mm]], acc[t], 0, 0, 0);
                else
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1[ap[mm]], bw[ky][bp[mm]], acc[t], 0, 0, 0);
            });
            __builtin_amdgcn_sched_barrier(0);
        });

        LSST(k, 1);
        // ---- diagonal sum over kx through the wave's transposed P buffer [28 n][x'] -----------------------
        if (n < 28)
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)   // accumulator rows 8 g4 + 4 (lane >> 5) + 0..3 = 4 consecutive x'
                    *reinterpret_cast<f32x4*>(pw + n * PCOL + 32 * t + 8 * g4 + 4 * (lane >> 5)) =
                        f32x4{acc[t][4 * g4], acc[t][4 * g4 + 1], acc[t][4 * g4 + 2], acc[t][4 * g4 + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        LSST(k, 2);
        const int y = y0 + 4 * k + wave;
        float o[2][3];
        bool ok[2];
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, cnt = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int xr = lane + 64 * h, xs = min(xr, TWO - 1);
            float v0 = bias0, v1 = bias1, v2 = bias2;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const float* pr = pw + 3 * kx * PCOL + xs + kx;
                v0 += pr[0];
                v1 += pr[PCOL];
                v2 += pr[2 * PCOL];
            }
            o[h][0] = v0;
            o[h][1] = v1;
            o[h][2] = v2;
            ok[h] = xr < TWO && y < H && x0 + xr < W;
            if (ok[h]) {
                float* dst = a.out + (((size_t)b * H + y) * W + x0 + xr) * 3;
                dst[0] = v0;
                dst[1] = v1;
                dst[2] = v2;
                s0 += v0;
                s1 += v1;
                s2 += v2;
                cnt += 1.f;
            }
        }
        LSST(k, 3);
        // ---- statistics of the 4-row x 88-column tile per channel: two-pass per wave (its row), the four
        // rows merged (Chan, fixed order) after the step's barrier ------------------------------------------
        s0 = wave_sum(s0);
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        cnt = wave_sum(cnt);
        const float mw[3] = {cnt > 0.f ? s0 / cnt : 0.f, cnt > 0.f ? s1 / cnt : 0.f, cnt > 0.f ? s2 / cnt : 0.f};
        float m2[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (ok[h])
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float d = o[h][c] - mw[c];
                    m2[c] = fmaf(d, d, m2[c]);
                }
#pragma unroll
        for (int c = 0; c < 3; ++c) m2[c] = wave_sum(m2[c]);
        float* const rs = red + (k & 1) * 64;   // [wave][channel][sum, M2], [wave][12] = n
        if (lane == 0) {
            rs[wave * 16 + 0] = s0; rs[wave * 16 + 1] = m2[0];
            rs[wave * 16 + 4] = s1; rs[wave * 16 + 5] = m2[1];
            rs[wave * 16 + 8] = s2; rs[wave * 16 + 9] = m2[2];
            rs[wave * 16 + 12] = cnt;
        }
        LSST(k, 4);
        lds_barrier();   // every wave is done reading ring rows 4k .. 4k + 3; the rows' statistics visible
        LSST(k, 5);
        const int ty4 = (y0 >> 2) + k;
        if (tid < 3 && ty4 < n_tiles4) {
            float S = 0.f, N = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                S += rs[w * 16 + 4 * tid];
                N += rs[w * 16 + 12];
            }
            const float mean = N > 0.f ? S / N : 0.f;
            float M2 = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const float nw = rs[w * 16 + 12];
                const float d = nw > 0.f ? rs[w * 16 + 4 * tid] / nw - mean : 0.f;
                M2 += rs[w * 16 + 4 * tid + 1] + nw * d * d;
            }
            if (to_acc) {
                const double dS = (double)S;
                accS += dS;
                if (N > 0.f) accQ += (double)M2 + dS * dS / (double)N;
            } else {
                const int n_part = a.tiles_y * a.tiles_x;
                a.part[((size_t)b * 3 + tid) * n_part + ty4 * a.tiles_x + sx] = make_float4(S, M2, N, 0.f);
            }
        }
    };
    // rows of step j (j >= 1) are 4 j + 8 .. 4 j + 11; they live in register buffer pre (j odd) / pre2 (j even)
    if (NS > 1) load_rows(RING, pre, prw);
    if (NS > 2) load_rows(RING + 4, pre2, prw2);
    for (int k = 0; k < NS; k += 2) {
        step(k);
        if (k + 1 < NS) {
            store_rows(4 * k + RING, pre, prw);                       // step k+1's rows into rows 4k .. 4k+3's slots
            lds_barrier();
            if (k + 3 < NS) load_rows(4 * k + 8 + RING, pre, prw);    // step k+3
            step(k + 1);
            if (k + 2 < NS) {
                LSST(k + 1, 6);
                store_rows(4 * k + 4 + RING, pre2, prw2);              // step k+2
                lds_barrier();
                LSST(k + 1, 7);
                if (k + 4 < NS) load_rows(4 * k + 12 + RING, pre2, prw2);   // step k+4
            }
        }
    }
    if (to_acc && tid < 3) cin_acc_add(a.stat, a.batch, 3, b, tid, (int)blockIdx.x % a.stat.nslot, accS, accQ);
    LSTL(3);
}

int last_x6_tiles_y(int H) { return (H + 3) / 4; }
int last_x6_tiles_x(int W) { return (W + lastx6::TWO - 1) / lastx6::TWO; }

#ifdef LAST_PROF
void last_timeline_print(int nwg) {
    std::vector<unsigned long long> tl((size_t)256 * 16);
    if (hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(last_tl), tl.size() * 8) != hipSuccess) return;
    if (nwg > 256) nwg = 256;
    double fill = 0, steps = 0;
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 4; ++w) {
            const unsigned long long* q = &tl[(g * 4 + w) * 4];
            fill += (double)(q[1] - q[0]);
            steps += (double)(q[3] - q[1]);
        }
    printf("    per wave (us): fill %.2f, per step %.2f\n", fill / (4 * nwg) * 0.01,
           steps / (4 * nwg) * 0.01 / lastx6::NS);
    std::vector<unsigned long long> st((size_t)256 * 32);
    if (hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(last_st), st.size() * 8) != hipSuccess) return;
    double d[7] = {0};
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 4; ++w)
            for (int p = 0; p < 7; ++p) d[p] += (double)(st[(g * 4 + w) * 8 + p + 1] - st[(g * 4 + w) * 8 + p]);
    printf("    step 2 (us): MFMA %.2f, P write %.2f, diag+store %.2f, stats %.2f, barrier %.2f, merge %.2f, "
           "refill+barrier %.2f\n", d[0] / (4 * nwg) * 0.01, d[1] / (4 * nwg) * 0.01, d[2] / (4 * nwg) * 0.01,
           d[3] / (4 * nwg) * 0.01, d[4] / (4 * nwg) * 0.01, d[5] / (4 * nwg) * 0.01, d[6] / (4 * nwg) * 0.01);
}
#endif


static uint16_t last_bf16_rne(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static float last_bf16_val(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// Keras Conv2DTranspose kernel (9, 9, 3, cin) [ky][kx][co][ci] -> flipped correlation kernel
// wf[ky][kx][ci][co] = kern[8-ky][8-kx][co][ci] -> B[ky][piece][n = 3 kx + co (27 of 32)][16 ci] bf16
std::vector<float> last_x6_pack_weights(const float* kern, int cin) {
    using namespace lastx6;
    std::vector<uint16_t> Bv((size_t)K * 3 * 32 * CIN, 0);
    for (int ky = 0; ky < K; ++ky)
        for (int kx = 0; kx < K; ++kx)
            for (int co = 0; co < 3; ++co)
                for (int ci = 0; ci < cin; ++ci) {
                    const float v = kern[(((size_t)(8 - ky) * 9 + (8 - kx)) * 3 + co) * cin + ci];
                    uint16_t p[3];
                    p[0] = last_bf16_rne(v);
                    const float r = v - last_bf16_val(p[0]);
                    p[1] = last_bf16_rne(r);
                    p[2] = last_bf16_rne(r - last_bf16_val(p[1]));
                    const int n = 3 * kx + co;
                    for (int k = 0; k < 3; ++k) Bv[(((size_t)ky * 3 + k) * 32 + n) * CIN + ci] = p[k];
                }
    std::vector<float> out(Bv.size() / 2);
    std::memcpy(out.data(), Bv.data(), Bv.size() * 2);
    return out;
}

hipError_t last_x6_prepare() {
    for (const void* k : {(const void*)last_x6_kernel<PRO_NONE>, (const void*)last_x6_kernel<PRO_AFF_RELU>,
                          (const void*)last_x6_kernel<PRO_AFF_RELU | 8>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lastx6::LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t last_x6_launch(const LastArgs& a, hipStream_t st) {
    if (a.cin != lastx6::CIN || a.tiles_y != last_x6_tiles_y(a.H) || a.tiles_x != last_x6_tiles_x(a.W) ||
        (a.part == nullptr) == (a.stat.acc == nullptr))
        return hipErrorInvalidValue;   // statistics: partials or accumulators
    if (a.stat.acc != nullptr && (a.stat.nslot < 1 || a.stat.nslot > CIN_ACC_MAX_SLOTS)) return hipErrorInvalidValue;
    const bool src_acc = a.pro_stat.acc != nullptr;
    // (nslot <= 8: the kernel's split affine form, CinAffineSplit<256, 2>, covers the accumulators)
    if (src_acc && (a.pro_stat.nslot < 1 || a.pro_stat.nslot > 8 || a.pro_stat.C != lastx6::CIN ||
                    a.pro_stat.batch != a.batch || a.pro_stat.style == nullptr))
        return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * ((a.H + lastx6::RB - 1) / lastx6::RB) * a.tiles_x);
    if (a.pro_w != nullptr) {   // two styles
        if (src_acc ? a.pro_stat.style1_offset < 0 : (a.pro_ab == nullptr || a.pro_ab1 == nullptr))
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(last_x6_kernel<PRO_AFF_RELU | 8>, dim3(grid), dim3(256), lastx6::LDS_BYTES, st, a);
    } else if (a.pro_ab != nullptr || src_acc)
        hipLaunchKernelGGL(last_x6_kernel<PRO_AFF_RELU>, dim3(grid), dim3(256), lastx6::LDS_BYTES, st, a);
    else
        hipLaunchKernelGGL(last_x6_kernel<PRO_NONE>, dim3(grid), dim3(256), lastx6::LDS_BYTES, st, a);
    return hipGetLastError();
}

}  // namespace rst
