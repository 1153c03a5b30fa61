// conv_mfma.hip — implicit-GEMM convolution on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One kernel template serves every conv of the transfer network
// (realtime_style_transfer/models/styleTransfer.py:95-205):
//   * Conv2D 'same' (contract 9x9 s1, 3x3 s2; residual 3x3 s1)       styleTransfer.py:170,194
//   * Conv2DTranspose 3x3 s2 'same' rewritten as a 2x2 stride-1 conv with N = 4 phases x Cout
//     and a pixel-shuffle store (no zero insertion)                    styleTransfer.py:115-119
// with the neighbouring element-wise work fused:
//   prologue (applied while the input halo is staged to LDS):
//     PRO_AFF_RELU  y = relu(a[c]*x + b[c])          CIN-apply + ReLU   (:173-182)
//     PRO_AFF       y = a[c]*x + b[c]                CIN-apply (block output of residual_block 0)
//     PRO_AFF_RES   y = r + a[c]*x + b[c]            CIN-apply + residual Add (:184)
//     (PRO_AFF / PRO_AFF_RES can also materialise y for the next skip connection)
//   epilogue:
//     EPI_RELU_BN    relu -> BatchNorm(inference) -> relu              contract (:194-203)
//     EPI_RELU_STATS relu, store, per-(tile, channel) {sum, M2, n}      residual conv (:170)
//     EPI_STATS      store, {sum, M2, n}                               expand conv (no act, :118)
//
// Numerics: exact f32 — every product is a single-rounding fmaf in the MFMA (no xf32 on
// gfx950), accumulation f32, tile statistics by two-pass (mean, M2) merged in f64 later.
//
// Data layout: activations NHWC fp32 in HBM. Per workgroup: an output tile of TH x TW
// pixels x NT channels. Input halo for one Cin chunk (CK channels) is staged in LDS as
// [halo pixel][CS] (CS = CK + pad, odd 16-B slot count -> conflict-free b128 column reads);
// the weight stage (TPS taps x CK x NT) is pre-packed on the host in exactly the LDS image
// order [tap][k-group][lane-half][n][VEC] so staging is a lane-linear copy.
//
// Pipeline (one barrier per stage): weights of stage s+1 are issued as global_load_lds
// (LDS-DMA, no VGPRs) into the other half of a double-buffered weight image while stage s
// computes; with HB = 2 the next Cin chunk's halo is prefetched into registers during the
// last stage of a chunk and written (CIN-apply fused) into the other halo buffer after it.
// K order inside a tap pairs channel s (lane half 0) with channel s + CK/2 (lane half 1),
// so one ds_read_b128 feeds 4 consecutive MFMA k-steps for both operands.
#include <hip/hip_runtime.h>
#include <type_traits>

#include "kernels.h"

namespace rst {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));   // native vector (HIP float4 is a struct)

template <int VEC>
struct vec_t;
template <>
struct vec_t<1> { typedef float type; };
template <>
struct vec_t<4> { typedef float4 type; };

__device__ __forceinline__ float vget(float v, int) { return v; }
__device__ __forceinline__ float vget(const float4& v, int q) {
    return q == 0 ? v.x : (q == 1 ? v.y : (q == 2 ? v.z : v.w));
}

// two-style blending (num_styles == 2, styleTransfer.py:36-44): the per-pixel affine is
// w0*(a0 x + b0) + w1*(a1 x + b1) with w0 = 1 - w1, i.e. y0 + w1*(y1 - y0)
__device__ __forceinline__ float apply_pro_blend(int mode, float x, float2 ab, float2 ab1, float w, float r) {
    const float y0 = fmaf(ab.x, x, ab.y), y1 = fmaf(ab1.x, x, ab1.y);
    float y = style_blend(w, y0, y1);
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}

__device__ __forceinline__ float apply_pro(int mode, float x, float2 ab, float r) {
    if (mode == PRO_MASK) return r > 0.f ? x : 0.f;   // ReLU backward: gradient masked by the forward output
    float y = fmaf(ab.x, x, ab.y);
    if (mode == PRO_AFF_RELU) y = fmaxf(y, 0.f);
    else if (mode == PRO_AFF_RES) y = r + y;
    return y;
}

#define RST_TP int KH, int KW, int S, int CK, int NT, int TH, int TW, int WM, int WN, int TPS, int HB
#define RST_TA KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB

template <RST_TP>
struct ConvCfg {
    static constexpr int VEC = ((CK / 2) % 4 == 0) ? 4 : 1;
    static constexpr int CS = (VEC == 4) ? (CK + 4) : (((CK + 1) & 1) ? CK + 1 : CK + 2);  // odd for VEC=1
    static constexpr int HH = (TH - 1) * S + KH;
    static constexpr int HWD = (TW - 1) * S + KW;
    static constexpr int HP = HH * HWD;
    static constexpr int MT = TH * TW / 32;
    static constexpr int MW = MT / WM;
    static constexpr int NTILES = NT / 32;
    static constexpr int NW = NTILES / WN;
    static constexpr int KSTEPS = CK / 2;
    static constexpr int SG = KSTEPS / VEC;
    static constexpr int WSTAGE = TPS * CK * NT;
    static constexpr int NTAPS = KH * KW;
    static constexpr int NGROUPS = NTAPS / TPS;
    static constexpr int HALO_FLOATS = ((HP * CS + 3) / 4) * 4;
    static constexpr int MAX_CIN = 256;
    static constexpr int HQ = CK / 4;                         // float4 per halo pixel (vector path)
    static constexpr int HREG = (HP * HQ + 255) / 256;        // halo prefetch registers (float4) per thread
    static constexpr int WCOPY = WSTAGE / 4;                  // float4 per weight stage
    static constexpr size_t LDS_BYTES = (size_t)(HB * HALO_FLOATS + 2 * WSTAGE) * 4 + MAX_CIN * 8;
    static_assert(WM * WN == 4, "4 waves per workgroup");
    static_assert(MT % WM == 0 && NTILES % WN == 0, "wave tiling");
    static_assert((TH * TW) % 32 == 0, "M tile = 32 pixels");
    static_assert(NTAPS % TPS == 0, "taps per stage");
    static_assert(KSTEPS % VEC == 0, "vector k-steps");
    static_assert(WSTAGE % 4 == 0, "weight stage is a float4 copy");
    static_assert(HB == 1 || (CK % 4) == 0, "halo prefetch needs the float4 path");
    static_assert(LDS_BYTES + MAX_CIN * 8 <= 160 * 1024, "LDS budget (incl. the two-style blend table)");
};

// Weight stages are staged through registers: global_load_dwordx4 issued at the start of a
// stage, ds_write_b128 after its MFMAs. (LDS-DMA would need no VGPRs, but hipcc orders every
// ds_read behind all pending LDS-DMA with s_waitcnt vmcnt(0), which would drain the prefetch at
// the first operand read of the stage.)
// Compile-time loop: the index is a constant expression from the front end on, so arrays
// indexed by it are promoted to registers (a #pragma-unrolled runtime index left the weight
// prefetch registers in scratch).
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

template <int WCOPY>
struct WeightRegs {
    static constexpr int N = (WCOPY + 255) / 256;
    f32x4 r[N];
    __device__ __forceinline__ void load(const float* __restrict__ src, int tid) {
        static_for<0, N>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int idx = k * 256 + tid;
            if (WCOPY % 256 == 0 || (k + 1) * 256 <= WCOPY || idx < WCOPY)
                r[k] = reinterpret_cast<const f32x4*>(src)[idx];
        });
    }
    __device__ __forceinline__ void store(float* dst, int tid) const {
        static_for<0, N>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int idx = k * 256 + tid;
            if (WCOPY % 256 == 0 || (k + 1) * 256 <= WCOPY || idx < WCOPY)
                reinterpret_cast<f32x4*>(dst)[idx] = r[k];
        });
    }
};

// OPT: experiment bits for tools/conv_bench (production uses RST_CONV_OPT):
//   bit0  pin LDS read-ahead before the MFMAs with sched_barrier
#ifndef RST_CONV_OPT
#define RST_CONV_OPT 1
#endif
template <RST_TP, int OPT = RST_CONV_OPT>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
    using C = ConvCfg<RST_TA>;
    constexpr int VEC = C::VEC, CS = C::CS, HWD = C::HWD, HP = C::HP;
    constexpr int MW = C::MW, NW = C::NW, SG = C::SG, KSTEPS = C::KSTEPS, HQ = C::HQ;
    typedef typename vec_t<VEC>::type vT;

    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* halo0 = smem;
    float* wts0 = smem + HB * C::HALO_FLOATS;
    float2* pab = reinterpret_cast<float2*>(wts0 + 2 * C::WSTAGE);
    float2* pab1 = pab + C::MAX_CIN;   // only present when launched with the blend LDS extension

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
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
    const size_t img_base = (size_t)b * a.H * a.W;
    const bool vec_in = ((Cin & 3) == 0) && ((CK & 3) == 0);
    const bool blend = a.pro_w != nullptr;
    const float* wsrc = a.wpk + (size_t)nb * a.nchunks * C::NGROUPS * C::WSTAGE;
    const int n_stages = a.nchunks * C::NGROUPS;

    int pixoff[MW];
#pragma unroll
    for (int m = 0; m < MW; ++m) {
        const int p = (wm * MW + m) * 32 + li;
        const int pr = p / TW, pc = p % TW;
        pixoff[m] = ((pr * S) * HWD + pc * S) * CS + lh * KSTEPS;
    }
    int woff[NW];
#pragma unroll
    for (int n = 0; n < NW; ++n) woff[n] = (lh * NT + (wn * NW + n) * 32 + li) * VEC;

    floatx16 acc[MW][NW];
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int n = 0; n < NW; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

    // ---- halo helpers -------------------------------------------------------------------------
    auto pixel_of = [&](int hp, int& iy, int& ix) __attribute__((always_inline)) {
        const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
        iy = iy0 + hy;
        ix = ix0 + hx;
        return iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    };
    auto transform4 = [&](float4 v, float4 r, int c, size_t gi, int iy, int ix) __attribute__((always_inline)) {
        if (pro == PRO_MASK) {   // no affine table (Cin may exceed MAX_CIN here)
            v.x = r.x > 0.f ? v.x : 0.f;
            v.y = r.y > 0.f ? v.y : 0.f;
            v.z = r.z > 0.f ? v.z : 0.f;
            v.w = r.w > 0.f ? v.w : 0.f;
        } else if (pro != PRO_NONE) {
            if (blend) {
                const float wpx = a.pro_w[img_base + (size_t)iy * a.W + ix];
                v.x = apply_pro_blend(pro, v.x, pab[c + 0], pab1[c + 0], wpx, r.x);
                v.y = apply_pro_blend(pro, v.y, pab[c + 1], pab1[c + 1], wpx, r.y);
                v.z = apply_pro_blend(pro, v.z, pab[c + 2], pab1[c + 2], wpx, r.z);
                v.w = apply_pro_blend(pro, v.w, pab[c + 3], pab1[c + 3], wpx, r.w);
            } else {
                v.x = apply_pro(pro, v.x, pab[c + 0], r.x);
                v.y = apply_pro(pro, v.y, pab[c + 1], r.y);
                v.z = apply_pro(pro, v.z, pab[c + 2], r.z);
                v.w = apply_pro(pro, v.w, pab[c + 3], r.w);
            }
            if (do_mat && iy >= y0 * S && iy < (y0 + TH) * S && ix >= x0 * S && ix < (x0 + TW) * S)
                *reinterpret_cast<float4*>(a.mat + gi) = v;
        }
        return v;
    };
    auto write_halo4 = [&](float* hbuf, int hp, int q, float4 v) __attribute__((always_inline)) {
        float* dst = hbuf + hp * CS + q * 4;
        if constexpr (VEC == 4) {
            *reinterpret_cast<float4*>(dst) = v;
        } else {
            dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
        }
    };
    // synchronous staging of one Cin chunk (prologue, and chunk changes when HB == 1)
    auto stage_halo_sync = [&](int chunk, float* hbuf) __attribute__((always_inline)) {
        if (vec_in) {
            for (int it = tid; it < HP * HQ; it += 256) {
                const int hp = it / HQ, q = it - (it / HQ) * HQ;
                int iy, ix;
                const int c = chunk * CK + q * 4;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (pixel_of(hp, iy, ix) && c < Cin) {
                    const size_t gi = (img_base + (size_t)iy * a.W + ix) * Cin + c;
                    v = (a.act_bf16 & 1) ? ld_bf16x4(a.in, gi) : *reinterpret_cast<const float4*>(a.in + gi);
                    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (pro == PRO_MASK && (a.act_bf16 & 4)) r = ld_bf16x4(a.res, gi);   // bf16 forward activations
                    else if (pro == PRO_AFF_RES || pro == PRO_MASK) r = *reinterpret_cast<const float4*>(a.res + gi);
                    v = transform4(v, r, c, gi, iy, ix);
                }
                write_halo4(hbuf, hp, q, v);
            }
        } else {
            for (int it = tid; it < HP * CK; it += 256) {
                const int hp = it / CK, q = it - (it / CK) * CK;
                int iy, ix;
                const int c = chunk * CK + q;
                float v = 0.f;
                if (pixel_of(hp, iy, ix) && c < Cin) {
                    const size_t gi = (img_base + (size_t)iy * a.W + ix) * Cin + c;
                    v = (a.act_bf16 & 1) ? ld_bf16(a.in, gi) : a.in[gi];
                    if (pro == PRO_MASK) {
                        v = ((a.act_bf16 & 4) ? ld_bf16(a.res, gi) : a.res[gi]) > 0.f ? v : 0.f;
                    } else if (pro != PRO_NONE) {
                        const float r = pro == PRO_AFF_RES ? a.res[gi] : 0.f;
                        v = blend ? apply_pro_blend(pro, v, pab[c], pab1[c],
                                                    a.pro_w[img_base + (size_t)iy * a.W + ix], r)
                                  : apply_pro(pro, v, pab[c], r);
                        if (do_mat && iy >= y0 * S && iy < (y0 + TH) * S && ix >= x0 * S && ix < (x0 + TW) * S) a.mat[gi] = v;
                    }
                }
                hbuf[hp * CS + q] = v;
            }
        }
    };

    // ---- prologue -----------------------------------------------------------------------------
    if (pro != PRO_NONE && a.pro_ab != nullptr) {
        for (int c = tid; c < Cin; c += 256) pab[c] = a.pro_ab[b * Cin + c];
        if (blend)
            for (int c = tid; c < Cin; c += 256) pab1[c] = a.pro_ab1[b * Cin + c];
        __syncthreads();
    }
    {
        WeightRegs<C::WCOPY> w0;
        w0.load(wsrc, tid);
        stage_halo_sync(0, halo0);
        w0.store(wts0, tid);
    }
    __syncthreads();

    const float* res_src = (pro == PRO_AFF_RES || pro == PRO_MASK) ? a.res : a.in;

    // Uniform pipeline stage (one body, so the accumulators keep their registers): prefetch the
    // weights of stage s+1 and slice g of the next chunk's halo (HB == 2), MFMAs of stage s from
    // LDS, then write the prefetched data into the other LDS buffers. All prefetch loads are
    // unconditional (addresses clamped into the tensor, dummy re-reads on the last stage/chunk)
    // so no register copies of in-flight loads are generated; validity is applied at the write.
    constexpr int HIT = HP * HQ;                                    // halo items per chunk
    constexpr int HSL = (HIT + C::NGROUPS - 1) / C::NGROUPS;        // items per stage slice
    constexpr int HSR = (HSL + 255) / 256;                          // registers per thread
    for (int s = 0; s < n_stages; ++s) {
        const int chunk = s / C::NGROUPS;
        const int g = s - chunk * C::NGROUPS;
        const int s_next = (s + 1 < n_stages) ? s + 1 : s;
        const bool has_next_chunk = chunk + 1 < a.nchunks;
        const float* halo = halo0 + (HB == 2 ? (chunk & 1) * C::HALO_FLOATS : 0);
        const float* wts = wts0 + (s & 1) * C::WSTAGE;
        WeightRegs<C::WCOPY> wnext;
        wnext.load(wsrc + (size_t)s_next * C::WSTAGE, tid);
        f32x4 hreg[HB == 2 ? HSR : 1], rreg[HB == 2 ? HSR : 1];
        if constexpr (HB == 2) {
            const int cn = has_next_chunk ? chunk + 1 : chunk;
            static_for<0, HSR>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                int it = g * HSL + k * 256 + tid;
                it = it < HIT ? it : HIT - 1;
                const int hp = it / HQ, q = it - (it / HQ) * HQ;
                const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
                const int iy = min(max(iy0 + hy, 0), a.H - 1), ix = min(max(ix0 + hx, 0), a.W - 1);
                const int c = min(cn * CK + q * 4, Cin - 4);
                const size_t gi = (img_base + (size_t)iy * a.W + ix) * Cin + c;
                hreg[k] = *reinterpret_cast<const f32x4*>(a.in + gi);
                rreg[k] = *reinterpret_cast<const f32x4*>(res_src + gi);
            });
        }
        // ---------------- MFMA main loop over the stage -------------------------------------
        // operand fragments for step u+1 are read from LDS before the MFMAs of step u
        {
            constexpr int U = TPS * SG;
            vT av[2][MW], bv[2][NW];
            auto read_step = [&](int u, vT* A, vT* Bv) __attribute__((always_inline)) {
                const int t = u / SG, sg = u - (u / SG) * SG;
                const int tap = g * TPS + t;
                const int ky = tap / KW, kx = tap - (tap / KW) * KW;
                const int off = (ky * HWD + kx) * CS + sg * VEC;
#pragma unroll
                for (int m = 0; m < MW; ++m) A[m] = *reinterpret_cast<const vT*>(halo + pixoff[m] + off);
#pragma unroll
                for (int n = 0; n < NW; ++n) Bv[n] = *reinterpret_cast<const vT*>(wts + u * 2 * NT * VEC + woff[n]);
            };
            read_step(0, av[0], bv[0]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u + 1 < U) read_step(u + 1, av[(u + 1) & 1], bv[(u + 1) & 1]);
                if constexpr (OPT & 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < VEC; ++q)
#pragma unroll
                    for (int m = 0; m < MW; ++m)
#pragma unroll
                        for (int n = 0; n < NW; ++n)
                            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(vget(av[u & 1][m], q),
                                                                             vget(bv[u & 1][n], q), acc[m][n], 0, 0, 0);
                if constexpr (OPT & 1) __builtin_amdgcn_sched_barrier(0);
            }
        }
        wnext.store(wts0 + ((s + 1) & 1) * C::WSTAGE, tid);
        if constexpr (HB == 2) {
            if (has_next_chunk) {
                float* hn = halo0 + ((chunk + 1) & 1) * C::HALO_FLOATS;
                static_for<0, HSR>([&](auto K) __attribute__((always_inline)) {
                    constexpr int k = decltype(K)::value;
                    const int it = g * HSL + k * 256 + tid;
                    if ((k * 256 < HSL) && (k * 256 + tid < HSL) && it < HIT) {
                        const int hp = it / HQ, q = it - (it / HQ) * HQ;
                        int iy, ix;
                        const int c = (chunk + 1) * CK + q * 4;
                        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (pixel_of(hp, iy, ix) && c < Cin) {
                            const size_t gi = (img_base + (size_t)iy * a.W + ix) * Cin + c;
                            const f32x4 h4 = hreg[k], r4 = rreg[k];
                            v = transform4(make_float4(h4.x, h4.y, h4.z, h4.w), make_float4(r4.x, r4.y, r4.z, r4.w),
                                           c, gi, iy, ix);
                        }
                        write_halo4(hn, hp, q, v);
                    }
                });
            }
        }
        __syncthreads();   // next weight stage / halo slice visible; this stage's buffers free
        if constexpr (HB == 1) {
            if (g == C::NGROUPS - 1 && has_next_chunk) {
                stage_halo_sync(chunk + 1, halo0);
                __syncthreads();
            }
        }
    }

    // ---------------- epilogue ---------------------------------------------------------------
    const int epi = a.epi_mode;
    const int n_mtiles = a.tiles_y * a.tiles_x * C::MT;
    const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
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
                    if (a.wt_stores)   // write-through (sc1): no dirty lines left for the end-of-kernel write-back
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), osrd, (int)(oi * 4), 0, 16);
                    else
                        a.out[oi] = v;
                    s += v;
                    cnt += 1.f;
                }
            }
            if (a.part != nullptr) {
                // two-pass tile statistics: lanes l and l^32 hold the two row halves of column ng
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

// ------------------------------------------------------------------------------------------
// host-side dispatch over the instantiated configurations
// ------------------------------------------------------------------------------------------
template <RST_TP>
static hipError_t launch_cfg(const ConvArgs& a, hipStream_t st) {
    using C = ConvCfg<RST_TA>;
    auto kern = conv_mfma_kernel<RST_TA>;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x * a.n_blocks);
    if (a.pro_w != nullptr && a.cin > C::MAX_CIN) return hipErrorInvalidValue;
    const size_t lds = C::LDS_BYTES + (a.pro_w != nullptr ? C::MAX_CIN * sizeof(float2) : 0);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, a);
    return hipGetLastError();
}

template <RST_TP>
static hipError_t prepare_cfg() {
    using C = ConvCfg<RST_TA>;
    auto kern = conv_mfma_kernel<RST_TA>;
    return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(C::LDS_BYTES + C::MAX_CIN * sizeof(float2)));
}

template <RST_TP>
static ConvTile tile_of() {
    using C = ConvCfg<RST_TA>;
    ConvTile t{};
    t.kh = KH; t.kw = KW; t.stride = S; t.ck = CK; t.nt = NT; t.th = TH; t.tw = TW; t.tps = TPS; t.hb = HB;
    t.vec = C::VEC; t.mt = C::MT; t.ngroups = C::NGROUPS; t.wstage = C::WSTAGE;
    t.lds_bytes = (int)C::LDS_BYTES;
    t.id = 0;
    return t;
}

// The configuration table. Each row: (ID, KH,KW,S,CK,NT,TH,TW,WM,WN,TPS,HB).
#define RST_CONV_CONFIGS(X)                       \
    X(1, 9, 9, 1, 18, 32, 8, 16, 4, 1, 3, 1)         \
    X(2, 9, 9, 1, 4, 32, 8, 16, 4, 1, 3, 1)          \
    X(3, 3, 3, 2, 16, 32, 8, 16, 4, 1, 3, 1)         \
    X(4, 3, 3, 2, 8, 32, 8, 16, 4, 1, 3, 1)          \
    X(5, 3, 3, 1, 32, 128, 4, 16, 2, 2, 1, 1)        \
    X(6, 3, 3, 1, 32, 32, 8, 16, 4, 1, 3, 1)         \
    X(7, 3, 3, 1, 8, 32, 8, 16, 4, 1, 9, 1)          \
    X(8, 2, 2, 1, 32, 128, 4, 16, 2, 2, 1, 1)        \
    X(9, 2, 2, 1, 32, 64, 8, 16, 2, 2, 1, 1)         \
    X(10, 2, 2, 1, 32, 32, 8, 16, 4, 1, 4, 1)        \
    X(11, 2, 2, 1, 16, 32, 8, 16, 4, 1, 4, 1)        \
    X(12, 2, 2, 1, 8, 32, 8, 16, 4, 1, 4, 1)         \
    X(13, 3, 3, 1, 16, 32, 8, 16, 4, 1, 9, 1)        \
    X(14, 3, 3, 2, 4, 32, 8, 16, 4, 1, 9, 1)         \
    X(15, 3, 3, 1, 4, 32, 8, 16, 4, 1, 9, 1)         \
    X(16, 2, 2, 1, 4, 32, 8, 16, 4, 1, 4, 1)         \
    X(17, 3, 3, 1, 32, 64, 8, 16, 2, 2, 1, 1)         \
    X(18, 1, 1, 1, 32, 64, 8, 16, 2, 2, 1, 1)         \
    X(19, 1, 1, 1, 32, 128, 4, 16, 2, 2, 1, 1)        \
    X(20, 1, 1, 1, 32, 32, 8, 16, 4, 1, 1, 1)

bool conv_select(int kh, int stride, int cin, int ntot, ConvTile* out) {
    // pick CK (Cin chunk) and NT (output columns per workgroup)
    int ck;
    if (cin <= 4) ck = 4;
    else if (cin <= 8) ck = 8;
    else if (cin <= 16) ck = 16;
    else if (cin <= 18) ck = 18;
    else if (cin % 32 == 0) ck = 32;
    else return false;
    if (kh == 3 && stride == 2 && ck == 32) ck = 16;   // keep the stride-2 halo within LDS budget
    int nt = ntot > 64 ? 128 : (ntot > 32 ? 64 : 32);
    if (ntot > 128 && ntot % 128 != 0) return false;
    if (kh == 9 || (kh == 3 && stride == 2)) nt = 32;  // these variants exist only with NT=32
    if (kh == 1 && ck != 32) return false;             // 1x1 (Gram backward GEMM): Cin multiple of 32
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB)                       \
    if (kh == KH && stride == S && ck == CK && nt == NT) {                   \
        *out = tile_of<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB>();           \
        out->id = ID;                                                        \
        return true;                                                         \
    }
    RST_CONV_CONFIGS(X)
#undef X
    // fall back to NT=32 variants (more N blocks)
    if (nt != 32) {
        nt = 32;
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB)                       \
    if (kh == KH && stride == S && ck == CK && nt == NT) {                   \
        *out = tile_of<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB>();           \
        out->id = ID;                                                        \
        return true;                                                         \
    }
        RST_CONV_CONFIGS(X)
#undef X
    }
    return false;
}

hipError_t conv_launch(const ConvTile& t, const ConvArgs& a_in, hipStream_t st) {
    if (t.bf3) return conv_bf3_launch(t, a_in, st);
    // bf16 activations on the f32 kernel: only the input and the ReLU-mask source of a synchronously staged ReLU-mask
    // halo (the VGG16 conv0 input gradient's 1x1 conv in the plain-bf16 loss); the output stays f32
    if ((a_in.act_bf16 & 2) || ((a_in.act_bf16 & 5) && (a_in.pro_mode != PRO_MASK || t.hb != 1)))
        return hipErrorInvalidValue;
    const ConvArgs a = conv_wt_checked(a_in);
    switch (t.id) {
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB) \
    case ID:                                          \
        return launch_cfg<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB>(a, st);
        RST_CONV_CONFIGS(X)
#undef X
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t conv_prepare(const ConvTile& t) {
    if (t.bf3) return conv_bf3_prepare(t);
    switch (t.id) {
#define X(ID, KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB) \
    case ID:                                          \
        return prepare_cfg<KH, KW, S, CK, NT, TH, TW, WM, WN, TPS, HB>();
        RST_CONV_CONFIGS(X)
#undef X
        default:
            return hipErrorInvalidValue;
    }
}

}  // namespace rst
