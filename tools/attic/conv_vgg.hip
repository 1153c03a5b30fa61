// RECORD ONLY (not built): the 8-wave 16x16-tile VGG16 conv measured in round 5 (profiles/r05/vgg/vgg_bench_r05z.log)
// against conv_bf3.hip's production tiles: equal or slower on every layer (block1 -18 %, block3/4 +5-8 %), so not adopted.
// conv_vgg.hip — the VGG16 3x3 convolutions of the style loss (realtime_style_transfer/models/styleLoss.py:69-109:
// keras VGG16 trunk, 3x3 s1 SAME + bias + ReLU, block-end 2x2 max pools) and their input gradients (the same conv with
// the flipped kernel, the gradient masked by the forward ReLU output) in plain bf16: bf16 operands, fp32 accumulation —
// the arithmetic of the Keras mixed_bfloat16 policy the bench's training line runs (conv_bf3.hip's one-plane mode,
// whose weight image this kernel reads unchanged).
//
// Why a second kernel: conv_bf3's 4-wave 8x16 x 128 tile ran these layers at 0.19-0.29 of the bf16 pipe in the
// training step (profiles/r04/sq_train_r25.txt): one wave per SIMD, the halo staged at every 32-channel chunk boundary
// behind a barrier, and the whole 3x3 weight set re-staged through LDS for only 128 pixels. Here:
//   * workgroup = 8 waves (two per SIMD), output tile 16 x 16 pixels x NT (128 or 64) channels; wave (wm, wn) owns
//     pixel rows 4 wm .. 4 wm + 3 (two 32-pixel M tiles) x NT / 2 channels (NT / 64 N tiles): 4 (2) accumulators;
//   * one stage = 16 input channels x all nine taps: halo 18 x 18 pixels x 16 channels bf16 (10 KB) + weights
//     9 x 2 x NT x 8 bf16 (36 KB at NT 128), double-buffered in LDS; the next stage's global loads are issued at the
//     top of a stage, converted (ReLU mask, f32 -> bf16) and written to the other buffer after its 36 MFMAs per wave:
//     one barrier per stage, no exposed staging;
//   * halo pixel = 32 B ([two 8-channel halves]), the half swapped on odd rows: every A read (ds_read_b128, all nine
//     tap shifts) and every staging write (ds_write_b64) is bank-conflict-free (exhaustive check over the lane groups);
//     the weight image's [tap][half][co][8] rows are conflict-free as they stand;
//   * epilogue from the accumulators: bias (+ ReLU), 128-B stores per 32-lane half, and the fused 2x2 max pool —
//     a 2x2 window is accumulator registers j, j + 1, j + 8, j + 9 of one lane, so it needs no data exchange.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kernels.h"

namespace rst {

namespace vggk {
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int TH = 16, TW = 16;              // output tile
constexpr int HH = TH + 2, HWD = TW + 2;     // halo 18 x 18
constexpr int HP = HH * HWD;                 // 324 halo pixels
constexpr int CK = 16;                       // input channels per stage (one MFMA K step per tap)
constexpr int HALO_B = HP * 32;              // 10368 bytes
constexpr int NTHR = 512;
constexpr int HITEMS = HP * 4;               // float4 halo items per stage
constexpr int NH = (HITEMS + NTHR - 1) / NTHR;

template <int NT>
struct Cfg {
    static constexpr int NW = NT / 64;                   // 32-channel N tiles per wave
    static constexpr int W_B = 9 * 2 * NT * 16;          // weight bytes per stage (conv_bf3 one-plane image)
    static constexpr int BUF_B = HALO_B + W_B;
    static constexpr int WITEMS = W_B / 16;
    static constexpr int NWI = (WITEMS + NTHR - 1) / NTHR;
    static constexpr size_t LDS_BYTES = 2 * (size_t)BUF_B;
    static_assert(NT == 64 || NT == 128, "tile width");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}
}  // namespace vggk

template <int NT>
__global__ __launch_bounds__(512) void vgg_conv_kernel(ConvArgs a) {
    using namespace vggk;
    using C = Cfg<NT>;
    constexpr int NW = C::NW;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 31, lh = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    int bid = blockIdx.x;
    const int nb = bid % a.n_blocks;
    bid /= a.n_blocks;
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;
    const int H = a.H, W = a.W, Cin = a.cin;
    const bool mask = a.pro_mode == PRO_MASK;
    const size_t img = (size_t)b * H * W;
    const int nst = a.nchunks;   // Cin / 16 stages
    const unsigned char* const wsrc = reinterpret_cast<const unsigned char*>(a.wpk) + (size_t)nb * nst * C::W_B;

    // ---- staging: halo item it = tid + 512 k -> (pixel hp = it / 4, channel quad q = it % 4); its global offset
    // (floats, stage 0) or -1 outside the image, and its LDS byte offset (half swapped on odd halo rows)
    int goff[NH], loff[NH];
#pragma unroll
    for (int k = 0; k < NH; ++k) {
        const int it = tid + k * NTHR, itc = it < HITEMS ? it : HITEMS - 1;
        const int hp = itc >> 2, q = itc & 3, hy = hp / HWD, hx = hp - hy * HWD;
        const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
        const bool in = it < HITEMS && iy >= 0 && iy < H && ix >= 0 && ix < W;
        goff[k] = in ? (int)(((img + (size_t)iy * W + ix) * Cin) + 4 * q) : -1;
        loff[k] = it < HITEMS ? hp * 32 + 16 * (((q >> 1) ^ hy) & 1) + 8 * (q & 1) : -1;
    }
    // two register sets of staged loads: stage s + 2's global loads are issued at the top of stage s (set s & 1) and
    // written to LDS at the end of stage s + 1, so each load has two stages of MFMAs (~2 us) to land: one stage did
    // not cover the HBM / MALL latency under load
    f32x4 hv[2][NH], hm[2][NH];
    u32x4 wv[2][C::NWI];
    auto gload = [&](int s, auto SET) __attribute__((always_inline)) {
        constexpr int st = decltype(SET)::value;
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            hv[st][k] = hm[st][k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (goff[k] >= 0) {
                hv[st][k] = *reinterpret_cast<const f32x4*>(a.in + goff[k] + s * CK);
                if (mask) hm[st][k] = *reinterpret_cast<const f32x4*>(a.res + goff[k] + s * CK);
            }
        }
        const u32x4* const ws = reinterpret_cast<const u32x4*>(wsrc + (size_t)s * C::W_B);
#pragma unroll
        for (int k = 0; k < C::NWI; ++k) {
            const int it = tid + k * NTHR;
            if (C::WITEMS % NTHR == 0 || it < C::WITEMS) wv[st][k] = ws[it];
        }
    };
    auto lstore = [&](int buf, auto SET) __attribute__((always_inline)) {
        constexpr int st = decltype(SET)::value;
        unsigned char* const hb = lds + buf * C::BUF_B;
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            if (loff[k] < 0) continue;
            f32x4 v = hv[st][k];
            if (mask) {   // ReLU backward: the gradient masked by the forward output (conv_bf3's PRO_MASK)
                v.x = hm[st][k].x > 0.f ? v.x : 0.f;
                v.y = hm[st][k].y > 0.f ? v.y : 0.f;
                v.z = hm[st][k].z > 0.f ? v.z : 0.f;
                v.w = hm[st][k].w > 0.f ? v.w : 0.f;
            }
            const unsigned p01 = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){v.x, v.y}, bf16x2));
            const unsigned p23 = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){v.z, v.w}, bf16x2));
            *reinterpret_cast<u32x2*>(hb + loff[k]) = u32x2{p01, p23};
        }
#pragma unroll
        for (int k = 0; k < C::NWI; ++k) {
            const int it = tid + k * NTHR;
            if (C::WITEMS % NTHR == 0 || it < C::WITEMS) *reinterpret_cast<u32x4*>(hb + HALO_B + it * 16) = wv[st][k];
        }
    };

    // ---- operands: M tile 2 wm + m: lane pixel row 4 wm + 2 m + (li >> 4), column li & 15; tap (ky, kx) shifts the
    // halo pixel by (ky, kx), and the half select by the row parity ((li >> 4) + ky) & 1
    int abase[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) abase[m] = ((4 * wm + 2 * m + (li >> 4)) * HWD + (li & 15)) * 32;
    const int hsel0 = 16 * (lh ^ ((li >> 4) & 1)), hsel1 = 16 - hsel0;
    int bbase[NW];
#pragma unroll
    for (int n = 0; n < NW; ++n) bbase[n] = HALO_B + (lh * NT + (wn * NW + n) * 32 + li) * 16;

    floatx16 acc[2][NW];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < NW; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    gload(0, S0{});
    if (nst > 1) gload(1, S1{});
    lstore(0, S0{});
    __syncthreads();
    // stage s: loads of s + 2 into set s & 1 (free: its stage s was written to LDS at the end of stage s - 1), the
    // MFMAs on buffer s & 1, stage s + 1 (set (s + 1) & 1) into buffer (s + 1) & 1, one barrier
    auto stage = [&](int s, auto SET) __attribute__((always_inline)) {
        constexpr int P = decltype(SET)::value;
        const unsigned char* const cb = lds + P * C::BUF_B;
        if (s + 2 < nst) gload(s + 2, SET);
        short8 A[2][2], B[2][NW];
        auto read_tap = [&](auto T, int slot) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value, ky = t / 3, kx = t % 3;
            const int hs = (ky & 1) ? hsel1 : hsel0;
#pragma unroll
            for (int m = 0; m < 2; ++m)
                A[slot][m] = *reinterpret_cast<const short8*>(cb + abase[m] + (ky * HWD + kx) * 32 + hs);
#pragma unroll
            for (int n = 0; n < NW; ++n) B[slot][n] = *reinterpret_cast<const short8*>(cb + bbase[n] + t * 2 * NT * 16);
        };
        read_tap(std::integral_constant<int, 0>{}, 0);
        vggk::sfor<0, 9>([&](auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            if constexpr (t + 1 < 9) read_tap(std::integral_constant<int, t + 1>{}, (t + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < NW; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[t & 1][m], B[t & 1][n], acc[m][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        });
        if (s + 1 < nst) lstore(1 - P, std::integral_constant<int, 1 - P>{});
        __syncthreads();
    };
    for (int s = 0; s < nst; s += 2) {   // (conv_vgg_launch: nst even)
        stage(s, S0{});
        stage(s + 1, S1{});
    }

    // ---- epilogue: register j of lane (li, lh) is M-tile pixel (j & 3) + 8 (j >> 2) + 4 lh, channel li
    const int epi = a.epi_mode;
    const int ntot = a.ntot;
    const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t psrd =
        __builtin_amdgcn_make_buffer_rsrc(a.pool != nullptr ? a.pool : a.out, 0, 0x7FFFFFF0, 0x00020000);
    const int Hp = H >> 1, Wp = W >> 1;
#pragma unroll
    for (int n = 0; n < NW; ++n) {
        const int co = nb * NT + (wn * NW + n) * 32 + li;
        const float bias = a.bias[co];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int mt = 2 * wm + m;
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int p = (j & 3) + 8 * (j >> 2) + 4 * lh;
                const int oy = y0 + 2 * mt + (p >> 4), ox = x0 + (p & 15);
                float x = acc[m][n][j] + bias;
                if (epi == EPI_RELU_STATS) x = fmaxf(x, 0.f);
                v[j] = x;
                if (oy < H && ox < W) {
                    const int oi = (int)(((img + (size_t)oy * W + ox) * ntot + co) * 4);
                    if (a.wt_stores)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), osrd, oi, 0, 16);
                    else
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), osrd, oi, 0, 0);
                }
            }
            if (a.pool != nullptr) {   // 2x2 / 2 max pool (maxpool2_kernel's arithmetic): windows j, j+1, j+8, j+9
                const int py = (y0 >> 1) + mt;
#pragma unroll
                for (int jj = 0; jj < 8; jj += 2) {
                    const int p = (jj & 3) + 8 * (jj >> 2) + 4 * lh;
                    const int qx = (x0 + (p & 15)) >> 1;
                    const float mx = fmaxf(fmaxf(v[jj], v[jj + 1]), fmaxf(v[jj + 8], v[jj + 9]));
                    if (py < Hp && qx < Wp) {
                        const int pi = (int)(((((size_t)b * Hp + py) * Wp + qx) * ntot + co) * 4);
                        if (a.wt_stores)
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mx), psrd, pi, 0, 16);
                        else
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mx), psrd, pi, 0, 0);
                    }
                }
            }
        }
    }
}

// ---- host side ---------------------------------------------------------------------------------------------
template <int NT>
static ConvTile vgg_tile_of(int id) {
    ConvTile t{};
    t.id = id;
    t.kh = 3; t.kw = 3; t.stride = 1; t.ck = vggk::CK; t.nt = NT; t.th = vggk::TH; t.tw = vggk::TW; t.tps = 9;
    t.hb = 1; t.vec = 8; t.mt = vggk::TH * vggk::TW / 32; t.ngroups = 1;
    t.wstage = 9 * 2 * NT * 8;   // bf16 elements per stage: pack_conv_tiles_bf3's (tap, half, n, 8) image at ck 16
    t.lds_bytes = (int)vggk::Cfg<NT>::LDS_BYTES;
    t.bf3 = 1;
    return t;
}

bool conv_vgg_select(int cin, int ntot, int batch, int H, int W, ConvTile* out) {
    // RST_VGG_CONV: 0 conv_bf3's tiles only, 1 (default) this kernel where its grid fills the chip, 2 wherever the
    // shapes allow (the small-shape parity tests); read at each selection (model creation), not per launch
    const char* e = getenv("RST_VGG_CONV");
    const int on = e != nullptr ? atoi(e) : 1;
    if (!on || cin % (2 * vggk::CK) != 0 || ntot % 64 != 0) return false;   // (an even number of stages)
    const int NT = ntot % 128 == 0 ? 128 : 64;
    // the grid must fill the chip: (H / 16) (W / 16) B (ntot / NT) workgroups of one per CU
    const long long wgs = (long long)batch * ((H + 15) / 16) * ((W + 15) / 16) * (ntot / NT);
    if (on == 1 && wgs < 480) return false;
    *out = NT == 128 ? vgg_tile_of<128>(160) : vgg_tile_of<64>(161);
    return true;
}

bool conv_vgg_is(const ConvTile& t) { return t.id == 160 || t.id == 161; }

bool conv_vgg_fuses_pool(const ConvTile& t, const ConvArgs& a) {
    return conv_vgg_is(t) && a.part == nullptr && !a.shuffle && (a.epi_mode == EPI_RELU_STATS || a.epi_mode == EPI_NONE) &&
           a.ntot % t.nt == 0 && a.Ho == a.H && a.Wo == a.W && a.H % 2 == 0 && a.W % 2 == 0;
}

hipError_t conv_vgg_prepare(const ConvTile& t) {
    if (t.id == 160)
        return hipFuncSetAttribute((const void*)vgg_conv_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)vggk::Cfg<128>::LDS_BYTES);
    if (t.id == 161)
        return hipFuncSetAttribute((const void*)vgg_conv_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)vggk::Cfg<64>::LDS_BYTES);
    return hipErrorInvalidValue;
}

hipError_t conv_vgg_launch(const ConvTile& t, const ConvArgs& a, hipStream_t st) {
    // shapes the kernel and its grid assume (checked here: an out-of-range tile would fault)
    if (!conv_vgg_is(t) || a.cin % (2 * vggk::CK) != 0 || a.nchunks != a.cin / vggk::CK || a.ntot % t.nt != 0 ||
        a.n_blocks != a.ntot / t.nt || a.tiles_y != (a.H + vggk::TH - 1) / vggk::TH ||
        a.tiles_x != (a.W + vggk::TW - 1) / vggk::TW || a.Ho != a.H || a.Wo != a.W || a.shuffle || a.part != nullptr ||
        (a.pro_mode != PRO_NONE && a.pro_mode != PRO_MASK) || (a.pro_mode == PRO_MASK && a.res == nullptr) ||
        (a.epi_mode != EPI_RELU_STATS && a.epi_mode != EPI_NONE) || (a.pool != nullptr && !conv_vgg_fuses_pool(t, a)))
        return hipErrorInvalidValue;
    const size_t in_b = (size_t)a.batch * a.H * a.W * a.cin * 4, out_b = (size_t)a.batch * a.H * a.W * a.ntot * 4;
    if (in_b >= (size_t)0x7FFFFFF0 || out_b >= (size_t)0x7FFFFFF0) return hipErrorInvalidValue;   // 32-bit offsets
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x * a.n_blocks);
    if (t.id == 160)
        hipLaunchKernelGGL(vgg_conv_kernel<128>, dim3(grid), dim3(vggk::NTHR), vggk::Cfg<128>::LDS_BYTES, st, a);
    else
        hipLaunchKernelGGL(vgg_conv_kernel<64>, dim3(grid), dim3(vggk::NTHR), vggk::Cfg<64>::LDS_BYTES, st, a);
    return hipGetLastError();
}

}  // namespace rst
