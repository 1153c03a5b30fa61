// conv_bf3.hip — implicit-GEMM convolution with fp32-accurate split-bf16 products on gfx950
// (v_mfma_f32_32x32x16_bf16, 16x the f32-MFMA rate).
//
// Every fp32 operand x is split into hi = bf16(x) and lo = bf16(x - hi) (round-to-nearest-even),
// and each product block is accumulated in fp32 as  A_hi*B_hi + A_hi*B_lo + A_lo*B_hi  — three
// bf16 MFMAs ("bf16x3"). The representation keeps 16 significant bits per operand; the dropped
// A_lo*B_lo term is 2^-16 relative. That is ~30x more accurate than TF32 (10-bit mantissa), which
// TensorFlow uses by default for "fp32" convolutions on NVIDIA Ampere-class GPUs, at 3/16 of the
// f32-MFMA cost. This is an opt-in precision mode (RST_PRECISION_BF16X3); the exact-f32 kernel
// (conv_mfma.hip) stays the default. One plane (RST_PRECISION_BF16) is plain bf16 operands with fp32
// accumulation — the arithmetic of a Keras mixed_bfloat16 policy — at 1/16 of the f32-MFMA cost.
//
// Structure mirrors conv_mfma_kernel (same ConvArgs, prologue and epilogue semantics): output tile
// TH x TW pixels x NT channels per 4-wave workgroup, stage = (Cin chunk, tap group), weights of the
// next stage prefetched in registers, LDS images:
//   halo  [pixel][CK + 8] bf16, hi and lo planes (80-B pixel stride for CK = 32: 5 16-B slots,
//         conflict-free ds_read_b128 across a 16-lane group)
//   wts   [tap][kstep][hi/lo][lane half][n][8] bf16 (one ds_read_b128 per B fragment)
// The prologue (CIN affine / ReLU / residual add / two-style blend / materialise) runs in fp32 and
// the split happens as the value is written to LDS.
#include <hip/hip_runtime.h>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace rst {

namespace {
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef unsigned short ushort4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned short bf16_rne(float x) {
    const unsigned u = __float_as_uint(x);
    return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_val(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
// x = p0 [+ p1 [+ p2]]: each remainder is exact in fp32, every piece rounds to the nearest bf16
template <int NP>
__device__ __forceinline__ void split_bf16(float x, unsigned short* p) {
    p[0] = bf16_rne(x);
    if constexpr (NP >= 2) {
        const float r = x - bf16_val(p[0]);
        p[1] = bf16_rne(r);
        if constexpr (NP == 3) p[2] = bf16_rne(r - bf16_val(p[1]));
    }
}

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}
}  // namespace

#define RST_BP int KH, int KW, int S, int CK, int NT, int TH, int TW, int WM, int WN, int TPS, int NP, int PF
#define RST_BA KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF

template <RST_BP>
struct Bf3Cfg {
    static constexpr int KS = CK / 16;
    static constexpr int CSB = CK + 8;
    static constexpr int HH = (TH - 1) * S + KH;
    static constexpr int HWD = (TW - 1) * S + KW;
    static constexpr int HP = HH * HWD;
    static constexpr int MT = TH * TW / 32;
    static constexpr int MW = MT / WM;
    static constexpr int NTILES = NT / 32;
    static constexpr int NW = NTILES / WN;
    static constexpr int NTAPS = KH * KW;
    static constexpr int NGROUPS = NTAPS / TPS;
    static constexpr int WSTEP = 2 * NT * 8;                  // bf16 per (tap, kstep, plane)
    static constexpr int WSTAGE = TPS * KS * NP * WSTEP;      // bf16 per stage
    static constexpr int WCOPY = WSTAGE / 8;                  // 16-B units per stage
    static constexpr int HALO = ((HP * CSB + 7) / 8) * 8;     // bf16 per plane
    static constexpr int MAX_CIN = 256;
    static constexpr size_t LDS_BYTES = (size_t)(NP * HALO + 2 * WSTAGE) * 2 + 2 * MAX_CIN * 8;
    static_assert(NP >= 1 && NP <= 3, "one (bf16), two (bf16x3) or three (bf16x6) planes");
    static_assert(CK % 16 == 0, "bf16 k-steps of 16 channels");
    static_assert(WM * WN == 4 && MT % WM == 0 && NTILES % WN == 0, "4-wave tiling");
    static_assert(NTAPS % TPS == 0, "taps per stage");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

template <int WCOPY>
struct Bf3WeightRegs {
    static constexpr int N = (WCOPY + 255) / 256;
    f32x4 r[N];
    __device__ __forceinline__ void load(const unsigned short* __restrict__ src, int tid) {
        sfor<0, N>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int idx = k * 256 + tid;
            if (WCOPY % 256 == 0 || (k + 1) * 256 <= WCOPY || idx < WCOPY)
                r[k] = reinterpret_cast<const f32x4*>(src)[idx];
        });
    }
    __device__ __forceinline__ void store(unsigned short* dst, int tid) const {
        sfor<0, N>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int idx = k * 256 + tid;
            if (WCOPY % 256 == 0 || (k + 1) * 256 <= WCOPY || idx < WCOPY)
                reinterpret_cast<f32x4*>(dst)[idx] = r[k];
        });
    }
};

__device__ __forceinline__ float bf3_pro(int mode, float x, float2 ab, float r) {
    float y = fmaf(ab.x, x, ab.y);
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}
__device__ __forceinline__ float bf3_pro_blend(int mode, float x, float2 ab, float2 ab1, float w, float r) {
    const float y0 = fmaf(ab.x, x, ab.y), y1 = fmaf(ab1.x, x, ab1.y);
    float y = style_blend(w, y0, y1);
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}

template <RST_BP>
__global__ __launch_bounds__(256) void conv_bf3_kernel(ConvArgs a) {
    using C = Bf3Cfg<RST_BA>;
    constexpr int CSB = C::CSB, HWD = C::HWD, HP = C::HP, MW = C::MW, NW = C::NW, KS = C::KS;
    constexpr int HQ = CK / 4;   // float4 per halo pixel

    extern __shared__ __attribute__((aligned(16))) unsigned short smem_b[];
    unsigned short* halo = smem_b;   // NP planes of C::HALO
    unsigned short* wts0 = smem_b + NP * C::HALO;
    float2* pab = reinterpret_cast<float2*>(wts0 + 2 * C::WSTAGE);
    float2* pab1 = pab + C::MAX_CIN;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int li = lane & 31, lh = lane >> 5;

    int bid = blockIdx.x;
    const int nb = bid % a.n_blocks;
    bid /= a.n_blocks;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;
    const int iy0 = y0 * S - a.pad_t, ix0 = x0 * S - a.pad_l;
    const int Cin = a.cin;
    const int pro = a.pro_mode;
    const bool do_mat = (a.mat != nullptr) && nb == 0;
    const bool blend = a.pro_w != nullptr;
    const size_t img_base = (size_t)b * a.H * a.W;
    const unsigned short* wsrc = reinterpret_cast<const unsigned short*>(a.wpk) +
                                 (size_t)nb * a.nchunks * C::NGROUPS * C::WSTAGE;
    const int n_stages = a.nchunks * C::NGROUPS;

    int pixoff[MW];
#pragma unroll
    for (int m = 0; m < MW; ++m) {
        const int p = (wm * MW + m) * 32 + li;
        const int pr = p / TW, pc = p % TW;
        pixoff[m] = ((pr * S) * HWD + pc * S) * CSB + lh * 8;
    }
    int woff[NW];
#pragma unroll
    for (int n = 0; n < NW; ++n) woff[n] = (lh * NT + (wn * NW + n) * 32 + li) * 8;

    floatx16 acc[MW][NW];
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int n = 0; n < NW; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

    // Staging of one Cin chunk, in two halves so the global loads of chunk c+1 are issued at the start
    // of chunk c's MFMA stages and land in registers while they run: load_halo (fp32 input [+ ReLU-mask
    // / residual source]) and store_halo (prologue transform -> split into the planes -> LDS).
    constexpr int HITEMS = HP * HQ;
    constexpr int NPF = (HITEMS + 255) / 256;
    const bool need_r = pro == PRO_MASK || pro == PRO_AFF_RES;
    f32x4 pv[NPF], pr[NPF];
    auto halo_item = [&](int it, int chunk, int& hp, int& q, int& iy, int& ix, int& c) __attribute__((always_inline)) {
        hp = it / HQ;
        q = it - hp * HQ;
        const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
        iy = iy0 + hy;
        ix = ix0 + hx;
        c = chunk * CK + q * 4;
        return iy >= 0 && iy < a.H && ix >= 0 && ix < a.W && c < Cin;
    };
    // bf16 activations into one plane without a prologue (the plain-bf16 VGG16 forward): items of 8 channels (16-B
    // loads), stored to the halo image as they are (the bf16 bits are the operand), half the items of the f32 form
    constexpr int HQ8 = CK / 8, HITEMS8 = HP * HQ8;
    // (PF bit 3: the same for a bf16 gradient under a bf16 ReLU mask, PRO_MASK — the plain-bf16 VGG16's input-gradient
    // convs: both 16-B items loaded, the mask applied on the bits)
    constexpr bool in16 = (PF & 12) != 0;   // (conv_bf3_select(..., in_bf16 / mask_bf16): configs 144-147; launch-checked)
    constexpr bool mask16 = (PF & 8) != 0;
    auto load_halo = [&](int chunk) __attribute__((always_inline)) {
        if constexpr (in16) {
            sfor<0, NPF>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                const int it = k * 256 + tid;
                if constexpr (k * 256 >= HITEMS8) return;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                const int hp = it / HQ8, q = it - hp * HQ8;
                const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD, iy = iy0 + hy, ix = ix0 + hx, c = chunk * CK + q * 8;
                f32x4 r = {0.f, 0.f, 0.f, 0.f};
                if (it < HITEMS8 && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W && c < Cin) {
                    const size_t gi = (img_base + (size_t)iy * a.W + ix) * Cin + c;
                    v = __builtin_bit_cast(f32x4, *reinterpret_cast<const u32x4*>(
                                                      reinterpret_cast<const unsigned short*>(a.in) + gi));
                    if constexpr (mask16)
                        r = __builtin_bit_cast(f32x4, *reinterpret_cast<const u32x4*>(
                                                          reinterpret_cast<const unsigned short*>(a.res) + gi));
                }
                pv[k] = v;
                if constexpr (mask16) pr[k] = r;
            });
            return;
        }
        sfor<0, NPF>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = k * 256 + tid;
            int hp, q, iy, ix, c;
            f32x4 v = {0.f, 0.f, 0.f, 0.f}, r = {0.f, 0.f, 0.f, 0.f};
            if ((HITEMS % 256 == 0 || it < HITEMS) && halo_item(it, chunk, hp, q, iy, ix, c)) {
                const size_t gi = (img_base + (size_t)iy * a.W + ix) * Cin + c;
                if (a.act_bf16 & 1) {   // bf16 activations (8-B loads; the NP = 1 split below is then exact)
                    const float4 u = ld_bf16x4(a.in, gi);
                    v = f32x4{u.x, u.y, u.z, u.w};
                } else {
                    v = *reinterpret_cast<const f32x4*>(a.in + gi);
                }
                if (need_r) {
                    if (a.act_bf16 & 4) {
                        const float4 u = ld_bf16x4(a.res, gi);
                        r = f32x4{u.x, u.y, u.z, u.w};
                    } else {
                        r = *reinterpret_cast<const f32x4*>(a.res + gi);
                    }
                }
            }
            pv[k] = v;
            pr[k] = r;
        });
    };
    auto store_halo = [&](int chunk) __attribute__((always_inline)) {
        if constexpr (in16) {
            sfor<0, NPF>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                const int it = k * 256 + tid;
                if constexpr (k * 256 >= HITEMS8) return;
                if (it >= HITEMS8) return;
                const int hp = it / HQ8, q = it - hp * HQ8;
                u32x4 g = __builtin_bit_cast(u32x4, pv[k]);
                if constexpr (mask16) {   // ReLU backward: keep a gradient where the forward output is > 0, i.e. its bf16
                    const u32x4 m = __builtin_bit_cast(u32x4, pr[k]);   // bits are in [0x0001, 0x7FFF]
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const unsigned lo = m[w] & 0xFFFFu, hi = m[w] >> 16;
                        g[w] &= (lo - 1u < 0x7FFFu ? 0x0000FFFFu : 0u) | (hi - 1u < 0x7FFFu ? 0xFFFF0000u : 0u);
                    }
                }
                *reinterpret_cast<u32x4*>(halo + hp * CSB + q * 8) = g;
            });
            return;
        }
        sfor<0, NPF>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int it = k * 256 + tid;
            if (HITEMS % 256 != 0 && it >= HITEMS) return;
            int hp, q, iy, ix, c;
            float4 v = make_float4(pv[k][0], pv[k][1], pv[k][2], pv[k][3]);
            if (halo_item(it, chunk, hp, q, iy, ix, c) && pro != PRO_NONE) {
                const float4 r = make_float4(pr[k][0], pr[k][1], pr[k][2], pr[k][3]);
                if (pro == PRO_MASK) {   // ReLU backward: gradient masked by the forward output
                    v.x = r.x > 0.f ? v.x : 0.f;
                    v.y = r.y > 0.f ? v.y : 0.f;
                    v.z = r.z > 0.f ? v.z : 0.f;
                    v.w = r.w > 0.f ? v.w : 0.f;
                } else {
                    const size_t pix = img_base + (size_t)iy * a.W + ix;
                    if (blend) {
                        const float wpx = a.pro_w[pix];
                        v.x = bf3_pro_blend(pro, v.x, pab[c + 0], pab1[c + 0], wpx, r.x);
                        v.y = bf3_pro_blend(pro, v.y, pab[c + 1], pab1[c + 1], wpx, r.y);
                        v.z = bf3_pro_blend(pro, v.z, pab[c + 2], pab1[c + 2], wpx, r.z);
                        v.w = bf3_pro_blend(pro, v.w, pab[c + 3], pab1[c + 3], wpx, r.w);
                    } else {
                        v.x = bf3_pro(pro, v.x, pab[c + 0], r.x);
                        v.y = bf3_pro(pro, v.y, pab[c + 1], r.y);
                        v.z = bf3_pro(pro, v.z, pab[c + 2], r.z);
                        v.w = bf3_pro(pro, v.w, pab[c + 3], r.w);
                    }
                    if (do_mat && iy >= y0 * S && iy < (y0 + TH) * S && ix >= x0 * S && ix < (x0 + TW) * S)
                        *reinterpret_cast<float4*>(a.mat + pix * Cin + c) = v;
                }
            }
            unsigned short px[4][3];
            split_bf16<NP>(v.x, px[0]);
            split_bf16<NP>(v.y, px[1]);
            split_bf16<NP>(v.z, px[2]);
            split_bf16<NP>(v.w, px[3]);
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) {
                const ushort4v p4 = {px[0][pl], px[1][pl], px[2][pl], px[3][pl]};
                *reinterpret_cast<ushort4v*>(halo + pl * C::HALO + hp * CSB + q * 4) = p4;
            }
        });
    };

    if (pro != PRO_NONE && a.pro_ab != nullptr) {
        for (int c = tid; c < Cin; c += 256) pab[c] = a.pro_ab[b * Cin + c];
        if (blend)
            for (int c = tid; c < Cin; c += 256) pab1[c] = a.pro_ab1[b * Cin + c];
        __syncthreads();
    }
    {
        Bf3WeightRegs<C::WCOPY> w0;
        w0.load(wsrc, tid);
        load_halo(0);
        store_halo(0);
        w0.store(wts0, tid);
    }
    __syncthreads();

    // PF bit 0: the next Cin chunk's halo prefetched into registers during the chunk's first stage.
    // PF bit 1: the weights of stage s + 2 loaded during stage s (two register sets, so a stage's load has two
    // stages of MFMAs to land instead of one); stage s stores stage s + 1's set, loaded during stage s - 1.
    constexpr bool HPF = (PF & 1) != 0, WP2 = (PF & 2) != 0;
    Bf3WeightRegs<C::WCOPY> wA, wB;
    if constexpr (WP2) wA.load(wsrc + (size_t)(n_stages > 1 ? 1 : 0) * C::WSTAGE, tid);
    auto stage = [&](int s, auto& wcur, auto& wnxt) __attribute__((always_inline)) {
        const int chunk = s / C::NGROUPS;
        const int g = s - chunk * C::NGROUPS;
        const unsigned short* wts = wts0 + (s & 1) * C::WSTAGE;
        if constexpr (WP2) {
            const int s2 = s + 2 < n_stages ? s + 2 : n_stages - 1;
            wnxt.load(wsrc + (size_t)s2 * C::WSTAGE, tid);
        } else {
            const int s_next = (s + 1 < n_stages) ? s + 1 : s;
            wcur.load(wsrc + (size_t)s_next * C::WSTAGE, tid);
        }
        if (HPF && g == 0 && chunk + 1 < a.nchunks) load_halo(chunk + 1);
        {
            constexpr int U = TPS * KS;
            short8 af[2][NP][MW], bf[2][NP][NW];
            auto read_step = [&](int u, int slot) __attribute__((always_inline)) {
                const int t = u / KS, ks = u - (u / KS) * KS;
                const int tap = g * TPS + t;
                const int ky = tap / KW, kx = tap - (tap / KW) * KW;
                const int off = (ky * HWD + kx) * CSB + ks * 16;
                const unsigned short* wb = wts + (t * KS + ks) * NP * C::WSTEP;
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) {
#pragma unroll
                    for (int m = 0; m < MW; ++m)
                        af[slot][pl][m] = *reinterpret_cast<const short8*>(halo + pl * C::HALO + pixoff[m] + off);
#pragma unroll
                    for (int n = 0; n < NW; ++n)
                        bf[slot][pl][n] = *reinterpret_cast<const short8*>(wb + pl * C::WSTEP + woff[n]);
                }
            };
            read_step(0, 0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u + 1 < U) read_step(u + 1, (u + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
                const int sl = u & 1;
#pragma unroll
                for (int m = 0; m < MW; ++m)
#pragma unroll
                    for (int n = 0; n < NW; ++n) {
                        // small terms first: 2^-16 (NP == 3), then 2^-8, then 2^0
                        if constexpr (NP == 3) {
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][0][m], bf[sl][2][n], acc[m][n], 0, 0, 0);
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][1][m], bf[sl][1][n], acc[m][n], 0, 0, 0);
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][2][m], bf[sl][0][n], acc[m][n], 0, 0, 0);
                        }
                        if constexpr (NP >= 2) {
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][0][m], bf[sl][1][n], acc[m][n], 0, 0, 0);
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][1][m], bf[sl][0][n], acc[m][n], 0, 0, 0);
                        }
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][0][m], bf[sl][0][n], acc[m][n], 0, 0, 0);
                    }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        wcur.store(wts0 + ((s + 1) & 1) * C::WSTAGE, tid);
        __syncthreads();
        if (g == C::NGROUPS - 1 && chunk + 1 < a.nchunks) {
            if (!HPF) load_halo(chunk + 1);
            store_halo(chunk + 1);
            __syncthreads();
        }
    };
    if constexpr (WP2) {
        for (int s = 0; s < n_stages; s += 2) {
            stage(s, wA, wB);
            if (s + 1 < n_stages) stage(s + 1, wB, wA);
        }
    } else {
        for (int s = 0; s < n_stages; ++s) stage(s, wA, wA);
    }

    // ---------------- epilogue (as conv_mfma_kernel) ------------------------------------------
    const int epi = a.epi_mode;
    // VGG16 (no statistics, no shuffle, bias [+ ReLU]) with 64 channels per wave: through a wave-private LDS
    // image [32 px][64 ch] per M tile, stored as channel quads — four whole 256-B pixel rows per wave
    // instruction instead of two 128-B pieces (the accumulator column is one channel of 16 pixels). The
    // last stage's barrier has retired every operand read, so the halo image is free.
    if constexpr (NW == 2 && C::LDS_BYTES >= (size_t)4 * 32 * 64 * 4) {   // four 8-KB wave images fit
        if (a.part == nullptr && !a.shuffle && (epi == EPI_RELU_STATS || epi == EPI_NONE) &&
            a.ntot % NT == 0) {
            float* const ep = reinterpret_cast<float*>(smem_b) + wave * (32 * 64);
            const int ngb = nb * NT + wn * 64;
            const float bs0 = a.bias[ngb + li], bs1 = a.bias[ngb + 32 + li];
            const bool relu = epi == EPI_RELU_STATS;
            const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
            const __amdgpu_buffer_rsrc_t psrd = __builtin_amdgcn_make_buffer_rsrc(a.pool, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
            for (int m = 0; m < MW; ++m) {
                const int mt = wm * MW + m;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int px = (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const float v0 = acc[m][0][r] + bs0, v1 = acc[m][1][r] + bs1;
                    ep[px * 64 + li] = relu ? fmaxf(v0, 0.f) : v0;
                    ep[px * 64 + 32 + li] = relu ? fmaxf(v1, 0.f) : v1;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int px = 4 * it + (lane >> 4), c4 = 4 * (lane & 15), p = mt * 32 + px;
                    const int oy = y0 + p / TW, ox = x0 + p % TW;
                    const float4 v = *reinterpret_cast<const float4*>(ep + px * 64 + c4);
                    if (oy < a.Ho && ox < a.Wo) {
                        const size_t oi = (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.ntot + ngb + c4;
                        if (a.act_bf16 & 2) {   // bf16 layer output (mixed_bfloat16): 8 B per lane, 512 B per wave
                            *reinterpret_cast<uint2*>(reinterpret_cast<unsigned short*>(a.out) + oi) =
                                pack_bf16x4(v.x, v.y, v.z, v.w);
                        } else if (a.wt_stores) {   // write-through (sc1): no dirty lines left for the end-of-kernel write-back
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), osrd, (int)(oi * 4), 0, 16);
                        } else {
                            *reinterpret_cast<float4*>(a.out + oi) = v;
                        }
                    }
                }
                if constexpr (TW == 16 && TH % 2 == 0) {
                    // fused 2x2 / 2 max pool (VGG16 block ends; maxpool2_kernel's arithmetic): this M tile is two
                    // whole 16-pixel rows starting at an even row, so its eight windows are in the wave's image
                    if (a.pool != nullptr) {
                        const int Hp = a.Ho >> 1, Wp = a.Wo >> 1;
#pragma unroll
                        for (int it = 0; it < 2; ++it) {
                            const int j = 4 * it + (lane >> 4), c4 = 4 * (lane & 15);
                            const float* e0 = ep + (2 * j) * 64 + c4;
                            const f32x4 a0 = *reinterpret_cast<const f32x4*>(e0);
                            const f32x4 a1 = *reinterpret_cast<const f32x4*>(e0 + 64);
                            const f32x4 a2 = *reinterpret_cast<const f32x4*>(e0 + 16 * 64);
                            const f32x4 a3 = *reinterpret_cast<const f32x4*>(e0 + 17 * 64);
                            float4 m;
                            m.x = fmaxf(fmaxf(a0.x, a1.x), fmaxf(a2.x, a3.x));
                            m.y = fmaxf(fmaxf(a0.y, a1.y), fmaxf(a2.y, a3.y));
                            m.z = fmaxf(fmaxf(a0.z, a1.z), fmaxf(a2.z, a3.z));
                            m.w = fmaxf(fmaxf(a0.w, a1.w), fmaxf(a2.w, a3.w));
                            const int py = (y0 >> 1) + mt, qx = (x0 >> 1) + j;
                            if (py < Hp && qx < Wp) {
                                const size_t pi = (((size_t)b * Hp + py) * Wp + qx) * a.ntot + ngb + c4;
                                if (a.act_bf16 & 2)   // max of the rounded values = the rounded max (RNE is monotone)
                                    *reinterpret_cast<uint2*>(reinterpret_cast<unsigned short*>(a.pool) + pi) =
                                        pack_bf16x4(m.x, m.y, m.z, m.w);
                                else if (a.wt_stores)
                                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, m), psrd, (int)(pi * 4),
                                                                           0, 16);
                                else
                                    *reinterpret_cast<float4*>(a.pool + pi) = m;
                            }
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            }
            return;
        }
    }
    const int n_mtiles = a.tiles_y * a.tiles_x * C::MT;
    const __amdgpu_buffer_rsrc_t gsrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int n = 0; n < NW; ++n) {
        const int ng = nb * NT + (wn * NW + n) * 32 + li;
        const bool nvalid = ng < a.ntot;
        const float bias = nvalid ? a.bias[ng] : 0.f;
        float2 bn = make_float2(1.f, 0.f);
        if (epi == EPI_RELU_BN && nvalid) bn = a.bn_ab[ng];
        int co = ng, py = 0, px = 0;
        if (a.shuffle) {
            const int ph = ng / a.cout;
            co = ng - ph * a.cout;
            py = ph >> 1;
            px = ph & 1;
        }
#pragma unroll
        for (int m = 0; m < MW; ++m) {
            const int mt = wm * MW + m;
            float s = 0.f, cnt = 0.f;
            float vals[16];
            bool ok[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int p = mt * 32 + row;
                const int oy = y0 + p / TW, ox = x0 + p % TW;
                const bool valid = nvalid && oy < a.Ho && ox < a.Wo;
                float v = acc[m][n][r] + bias;
                if (epi == EPI_RELU_BN) {
                    v = fmaxf(v, 0.f);
                    v = fmaxf(fmaf(bn.x, v, bn.y), 0.f);
                } else if (epi == EPI_RELU_STATS) {
                    v = fmaxf(v, 0.f);
                }
                vals[r] = v;
                ok[r] = valid;
                if (valid) {
                    size_t oi;
                    if (a.shuffle)
                        oi = (((size_t)b * (2 * a.Ho) + 2 * oy + py) * (2 * a.Wo) + 2 * ox + px) * a.cout + co;
                    else
                        oi = (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.ntot + ng;
                    if (a.wt_stores)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), gsrd, (int)(oi * 4), 0, 16);
                    else
                        a.out[oi] = v;
                    s += v;
                    cnt += 1.f;
                }
            }
            if (a.part != nullptr) {
                s = lane_xor_sum<32>(s);
                cnt = lane_xor_sum<32>(cnt);
                const float mean = cnt > 0.f ? s / cnt : 0.f;
                float m2 = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float d = vals[r] - mean;
                    if (ok[r]) m2 = fmaf(d, d, m2);
                }
                m2 = lane_xor_sum<32>(m2);
                if (lh == 0 && nvalid) {
                    const int mtg = (ty * a.tiles_x + tx) * C::MT + mt;
                    a.part[((size_t)b * a.ntot + ng) * n_mtiles + mtg] = make_float4(s, m2, cnt, 0.f);
                }
            }
        }
    }
}

// ---- host side ---------------------------------------------------------------------------------
template <RST_BP>
static ConvTile bf3_tile_of() {
    using C = Bf3Cfg<RST_BA>;
    ConvTile t{};
    t.kh = KH; t.kw = KW; t.stride = S; t.ck = CK; t.nt = NT; t.th = TH; t.tw = TW; t.tps = TPS; t.hb = 1;
    t.vec = 8; t.mt = C::MT; t.ngroups = C::NGROUPS; t.wstage = C::WSTAGE; t.lds_bytes = (int)C::LDS_BYTES;
    t.bf3 = NP;
    return t;
}

// (ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF)
#define RST_BF3_CONFIGS(X)                               \
    X(101, 3, 3, 1, 32, 128, 4, 16, 2, 2, 1, 2, 0)       \
    X(102, 3, 3, 1, 32, 64, 4, 16, 2, 2, 1, 2, 0)        \
    X(104, 3, 3, 1, 32, 128, 8, 16, 2, 2, 1, 2, 0)       \
    X(111, 3, 3, 1, 32, 128, 4, 16, 2, 2, 1, 3, 0)       \
    X(112, 3, 3, 1, 32, 64, 4, 16, 2, 2, 1, 3, 0)        \
    X(113, 3, 3, 1, 32, 64, 8, 16, 2, 2, 1, 3, 0)        \
    X(134, 3, 3, 1, 32, 64, 8, 16, 4, 1, 3, 1, 0)        \
    X(135, 3, 3, 1, 32, 128, 8, 16, 2, 2, 3, 1, 0)       \
    X(136, 3, 3, 1, 32, 128, 8, 16, 2, 2, 3, 1, 2)       \
    X(144, 3, 3, 1, 32, 64, 8, 16, 4, 1, 3, 1, 4)        \
    X(145, 3, 3, 1, 32, 128, 8, 16, 2, 2, 3, 1, 4)       \
    X(146, 3, 3, 1, 32, 64, 8, 16, 4, 1, 3, 1, 8)        \
    X(147, 3, 3, 1, 32, 128, 8, 16, 2, 2, 3, 1, 8)       \
    X(140, 1, 1, 1, 32, 64, 8, 16, 4, 1, 1, 1, 0)        \
    X(141, 1, 1, 1, 32, 128, 8, 16, 2, 2, 1, 1, 0)

bool conv_bf3_select(int kh, int stride, int cin, int ntot, int planes, long long pixels, ConvTile* out, bool in_bf16,
                     bool mask_bf16) {
    if ((kh != 3 && kh != 1) || stride != 1 || cin % 32 != 0 || ntot % 64 != 0 || planes < 1 || planes > 3) return false;
    if (kh == 1 && planes != 1) return false;   // 1x1: the plain-bf16 Gram backward only
    // measured (tools/conv_bench, residual conv of rst-960-120-128-17): bf16x3 NT64 4x16 42.8 us at B=1;
    // bf16x6 NT64 8x16 62.8 us at B=1 / 437 us at B=8 (exact-f32 MFMA kernel: 92.5 / 611 us).
    // Plain bf16 (one plane, one MFMA per product block; tools/conv_bench vgg, VGG16 at 480x960, B=4):
    // three taps per stage (one barrier + weight-stage swap per 24 MFMAs instead of 8) on an 8x16 x 64
    // tile with the four waves stacked along M: block1_conv2 422 -> 312 us, block2_conv2 335 -> 231,
    // block3_conv2 254 -> 188, block5_conv2 101 -> 57 (previous 4x16 x 64 / 8x16 x 128 one-tap tiles).
    // Register prefetch of the next Cin chunk's halo (PF) only pays on the 512-channel layers with a
    // 128-wide tile while that still fills the chip (block4_conv2 188 -> 174 us); elsewhere its
    // registers cost more occupancy than it hides (bf16x3 residual: 43.8 -> 57.6 us).
    // Round 3 (tools/conv_bench 4 vgg, profiles/r03/conv_bench_vgg_tiles*.log): the 128-wide tile without the halo
    // register prefetch (config 135, 2 x 2 waves) beats 134 wherever it still gives >= ~900 workgroups
    // (b2c2 239 -> 227 us, b3c2 189 -> 182, b4c2 187 -> 170) and 132 everywhere; 134 keeps block 1 (Cout 64)
    // and block 5 (225 workgroups at 128 wide: 58 vs 66 us). Prefetching the weights two stages ahead (two
    // register sets, PF bit 1) costs the 64-wide tile a wave per SIMD of occupancy (25-70 % slower), but the
    // 128-wide tile is held to two workgroups per CU by its LDS anyway (200 -> 240 VGPRs, no occupancy lost):
    // config 136 = 135 + two-stage weights, standalone b2c1 134 -> 129 us, b2c2 216 -> 197, b3c2 176 -> 164,
    // b4c2 167 -> 162 (profiles/r03/conv_bench_vgg_z.log; with the halo prefetch as well, PF 3, 40-60 % slower) —
    // but the same within noise in the training step (three alternating same-box pairs 25.30 vs 25.12 ms,
    // profiles/r03/vgg_wp2_ab.log), so 135 stays selected.
    int want;
    if (kh == 1) want = ntot % 128 == 0 ? 141 : 140;
    else if (planes == 2) want = 102;
    else if (planes == 3) want = 113;
    else if (ntot % 128 == 0 && (pixels / 128) * (ntot / 128) >= 896) want = 135;
    else want = 134;
    // bf16 activations without a prologue (the plain-bf16 VGG16 forward): the same tiles staging 8-channel 16-B items
    // straight into the halo image (PF bit 2)
    if (in_bf16 && kh == 3 && planes == 1 && cin % 8 == 0) want = want == 135 ? 145 : 144;
    else if (mask_bf16 && kh == 3 && planes == 1 && cin % 8 == 0) want = want == 135 ? 147 : 146;
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF)                  \
    if (ID == want) {                                                           \
        *out = bf3_tile_of<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF>();   \
        out->id = ID;                                                           \
        return true;                                                            \
    }
    RST_BF3_CONFIGS(X)
#undef X
    return false;
}

hipError_t conv_bf3_launch(const ConvTile& t, const ConvArgs& a_in, hipStream_t st) {
    const ConvArgs a = conv_wt_checked(a_in);
    switch (t.id) {
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF)                                      \
    case ID: {                                                                                   \
        using C = Bf3Cfg<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF>;                            \
        if ((a.cin & 3) != 0) return hipErrorInvalidValue;                                       \
        if (a.pool != nullptr && !conv_bf3_fuses_pool(t, a)) return hipErrorInvalidValue;        \
        if ((a.act_bf16 & 2) && !conv_bf3_fuses_pool(t, a)) return hipErrorInvalidValue;        \
        if ((a.act_bf16 & 5) && NP != 1) return hipErrorInvalidValue;                             \
        if ((PF & 4) && (!(a.act_bf16 & 1) || a.pro_mode != PRO_NONE || (a.cin & 7) != 0))        \
            return hipErrorInvalidValue;                                                          \
        if ((PF & 8) && ((a.act_bf16 & 5) != 5 || a.pro_mode != PRO_MASK || (a.cin & 7) != 0))    \
            return hipErrorInvalidValue;                                                          \
        if (a.pro_w != nullptr && a.cin > C::MAX_CIN) return hipErrorInvalidValue;               \
        const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x * a.n_blocks);          \
        hipLaunchKernelGGL((conv_bf3_kernel<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF>), dim3(grid), \
                           dim3(256), C::LDS_BYTES, st, a);                                      \
        return hipGetLastError();                                                                \
    }
        RST_BF3_CONFIGS(X)
#undef X
        default:
            return hipErrorInvalidValue;
    }
}

bool conv_bf3_fuses_pool(const ConvTile& t, const ConvArgs& a) {
    // the wave-private epilogue (NW == 2 and its LDS images fit) with 16-pixel-wide, even-height tiles
    bool wave_epi = false;
    switch (t.id) {
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF)                                                    \
    case ID: {                                                                                                 \
        using C = Bf3Cfg<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF>;                                        \
        wave_epi = C::NW == 2 && C::LDS_BYTES >= (size_t)4 * 32 * 64 * 4 && TW == 16 && TH % 2 == 0 && S == 1; \
        break;                                                                                                 \
    }
        RST_BF3_CONFIGS(X)
#undef X
        default:
            return false;
    }
    return wave_epi && a.part == nullptr && !a.shuffle && (a.epi_mode == EPI_RELU_STATS || a.epi_mode == EPI_NONE) &&
           a.ntot % t.nt == 0 && a.Ho == a.H && a.Wo == a.W;
}

hipError_t conv_bf3_prepare(const ConvTile& t) {
    switch (t.id) {
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF)                                                   \
    case ID:                                                                                                  \
        return hipFuncSetAttribute((const void*)conv_bf3_kernel<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF>, \
                                   hipFuncAttributeMaxDynamicSharedMemorySize,                                 \
                                   (int)Bf3Cfg<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, NP, PF>::LDS_BYTES);
        RST_BF3_CONFIGS(X)
#undef X
        default:
            return hipErrorInvalidValue;
    }
}

// ---- VGG16 block1_conv1 on bf16 operands (the plain-bf16 loss) ----------------------------------------------
// 3 -> 64 channels, 3x3 SAME: K = 27 (tap, channel) pairs padded to 32 = two k-steps of v_mfma_f32_32x32x16_bf16.
// The conv_bf3 tiles need Cin % 32 == 0, and the f32 CK-4 kernel it replaces idled most of each f32 MFMA on the
// 4-channel K (200 us per B=4 forward, 2.4 TB/s of its 472 MB output). Workgroup = 8 x 32 output pixels, wave w
// rows 2w and 2w + 1 (one 32-pixel M tile each) x all 64 channels; the caffe preprocess (255 x - mean, BGR: the
// flip is in the weights) is applied as the 10 x 34 x 3 input patch is staged, rounded to bf16, into LDS; each
// lane gathers its A operand (8 consecutive (tap, channel) values of its pixel) from there; the B operand is
// pre-packed in lane order on the host (4 x 16 B per lane, loaded once). Epilogue: bias + ReLU, f32 NHWC store.
namespace vgg0 {
constexpr int TH = 8, TW = 32, PH = TH + 2, PW = TW + 2, PC = 4;   // patch [row][col][4] bf16 (channel 3 unused)
}
__global__ __launch_bounds__(256) void vgg_conv0_bf16_kernel(const float* __restrict__ img, const float2* __restrict__ pre,
                                                             const unsigned short* __restrict__ wpk,
                                                             const float* __restrict__ bias, float* __restrict__ out,
                                                             int H, int W, int tiles_x, int out_bf16) {
    using namespace vgg0;
    __shared__ __attribute__((aligned(16))) unsigned short patch[PH * PW * PC];
    __shared__ __attribute__((aligned(16))) float epi[4 * 32 * 64];   // per-wave epilogue images
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const int b = blockIdx.y, tyx = blockIdx.x;
    const int y0 = (tyx / tiles_x) * TH, x0 = (tyx % tiles_x) * TW;
    // B operand: wpk[(s * 2 + n) * 64 + lane] = 8 bf16 (k = 16 s + 8 lh + j, co = 32 n + li)
    short8 bw[2][2];
#pragma unroll
    for (int sn = 0; sn < 4; ++sn)
        bw[sn >> 1][sn & 1] = *reinterpret_cast<const short8*>(wpk + ((size_t)sn * 64 + lane) * 8);
    for (int i = tid; i < PH * PW * 3; i += 256) {
        const int c = i % 3, px = i / 3, r = px / PW, q = px % PW;
        const int gy = y0 - 1 + r, gx = x0 - 1 + q;
        float v = 0.f;   // SAME zero padding of the preprocessed image
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
            const float2 ab = pre[b * 3 + c];
            v = fmaf(ab.x, img[(((size_t)b * H + gy) * W + gx) * 3 + c], ab.y);
        }
        patch[px * PC + c] = bf16_rne(v);
    }
    __syncthreads();
    floatx16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int py = 2 * wave + m;   // output row within the tile; the lane's pixel is column li
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            unsigned short av[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 16 * s + 8 * lh + j;
                const int tap = k / 3, c = k - 3 * (k / 3), ky = tap / 3, kx = tap - 3 * (tap / 3);
                av[j] = k < 27 ? patch[((py + ky) * PW + li + kx) * PC + c] : (unsigned short)0;
            }
            short8 a8;
#pragma unroll
            for (int j = 0; j < 8; ++j) a8[j] = (short)av[j];
#pragma unroll
            for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, bw[s][n], acc[m][n], 0, 0, 0);
        }
    }
    // epilogue through a wave-private LDS image [32 px][64 ch] per output row: a lane's accumulator column is
    // one channel of 16 pixels, so direct stores wrote two 128-B pieces per wave instruction (2.8 TB/s on the
    // 472 MB output); read back as channel quads, a wave instruction stores four whole pixels, 1 KB contiguous.
    // Row stride 64 floats: the b32 writes and the b128 reads (lane groups of MI355X_MICROARCH.md) are
    // conflict-free.
    float* const ep = epi + wave * (32 * 64);
    const float bs0 = bias[li], bs1 = bias[32 + li];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int oy = y0 + 2 * wave + m;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int px = (r & 3) + 8 * (r >> 2) + 4 * lh;
            ep[px * 64 + li] = fmaxf(acc[m][0][r] + bs0, 0.f);
            ep[px * 64 + 32 + li] = fmaxf(acc[m][1][r] + bs1, 0.f);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int px = 4 * it + (lane >> 4), c4 = 4 * (lane & 15), ox = x0 + px;
            const float4 v = *reinterpret_cast<const float4*>(ep + px * 64 + c4);
            if (oy < H && ox < W) {
                const size_t oi = (((size_t)b * H + oy) * W + ox) * 64 + c4;
                if (out_bf16)   // bf16 layer output (mixed_bfloat16)
                    *reinterpret_cast<uint2*>(reinterpret_cast<unsigned short*>(out) + oi) = pack_bf16x4(v.x, v.y, v.z, v.w);
                else
                    *reinterpret_cast<float4*>(out + oi) = v;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
}

// Keras HWIO [3][3][3][64] (already BGR-flipped by the caller) -> the lane-order bf16 B image (4 x 64 x 8)
std::vector<unsigned short> vgg_conv0_bf16_pack(const float* wflip) {
    std::vector<unsigned short> out(4 * 64 * 8, 0);
    for (int sn = 0; sn < 4; ++sn)
        for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) {
                const int s = sn >> 1, n = sn & 1, li = lane & 31, lh = lane >> 5;
                const int k = 16 * s + 8 * lh + j, co = 32 * n + li;
                if (k < 27) {
                    const float v = wflip[(size_t)k * 64 + co];   // k = tap * 3 + c = (ky * 3 + kx) * 3 + c
                    unsigned u;
                    std::memcpy(&u, &v, 4);
                    out[((size_t)sn * 64 + lane) * 8 + j] = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
                }
            }
    return out;
}

hipError_t vgg_conv0_bf16_launch(const float* img, const float2* pre, const unsigned short* wpk, const float* bias,
                                 float* out, int batch, int H, int W, hipStream_t st, bool out_bf16) {
    using namespace vgg0;
    const int tiles_y = (H + TH - 1) / TH, tiles_x = (W + TW - 1) / TW;
    hipLaunchKernelGGL(vgg_conv0_bf16_kernel, dim3((unsigned)(tiles_y * tiles_x), (unsigned)batch), dim3(256), 0, st,
                       img, pre, wpk, bias, out, H, W, tiles_x, out_bf16 ? 1 : 0);
    return hipGetLastError();
}

}  // namespace rst
