// gram.hip — Gram matrices of VGG feature maps on f32 MFMA.
//
// gram_matrix (realtime_style_transfer/models/styleLoss.py:21-37):
//   G[b,c,d] = einsum('bijc,bijd->bcd', F, F) / (H*W)
// A tall-skinny Fᵀ·F: M = N = C (64..512), K = H*W (up to 460 800 px at 480x960). The K
// dimension is split across workgroups (split-K) so every CU has work even for C = 64;
// each workgroup stages 64 pixels x (64 + 64) channels of F in LDS and its 4 waves each own
// one 32x32 block of a 64x64 G tile (v_mfma_f32_32x32x2_f32: exact f32 products). Partial
// tiles go to a slab [b][split][C][C]; a second kernel sums the splits in fixed order
// (bitwise reproducible, no float atomics) and scales by 1/(H*W). G is symmetric: only the tiles
// ti <= tj are computed; an off-diagonal tile is written to the slab at (ti, tj) and transposed at
// (tj, ti) (C = 512: 36 of 64 tiles).
#include <hip/hip_runtime.h>
#include "kernels.h"

namespace rst {

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace gram {
constexpr int KP = 64;        // pixels per LDS stage
constexpr int TILE = 64;      // G tile edge per workgroup
constexpr int LS = TILE + 1;  // padded LDS row
}  // namespace gram

static int gram_splits(int batch, int hw, int channels) {
    const int nt = channels / gram::TILE, tiles = nt * (nt + 1) / 2;
    int ns = 2048 / (batch * tiles);
    const int max_ns = (hw + 255) / 256;
    if (ns > max_ns) ns = max_ns;
    if (ns < 1) ns = 1;
    return ns;
}

size_t gram_workspace_bytes(int batch, int hw, int channels) {
    return (size_t)batch * gram_splits(batch, hw, channels) * channels * channels * sizeof(float);
}

__global__ __launch_bounds__(256) void gram_partial_kernel(const float* __restrict__ feat, float* __restrict__ slab,
                                                           int hw, int C, int nsplit, int span) {
    using namespace gram;
    __shared__ float la[KP * LS];
    __shared__ float lb[KP * LS];
    const int ntile = C / TILE;
    int bid = blockIdx.x;
    const int split = bid % nsplit;
    bid /= nsplit;
    const int npairs = ntile * (ntile + 1) / 2;
    int pair = bid % npairs;
    const int b = bid / npairs;
    int ti = 0;   // pair -> (ti, tj), ti <= tj, row-major over the upper triangle
    while (pair >= ntile - ti) {
        pair -= ntile - ti;
        ++ti;
    }
    const int tj = ti + pair;
    const int c0 = ti * TILE, d0 = tj * TILE;
    const int p_begin = split * span;
    const int p_end = min(hw, p_begin + span);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave >> 1, wj = wave & 1;
    const int li = lane & 31, lh = lane >> 5;
    const float* fb = feat + (size_t)b * hw * C;

    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;

    for (int p0 = p_begin; p0 < p_end; p0 += KP) {
        __syncthreads();
        // stage KP pixels x 64 channels for both operands (float4 loads, 16 per pixel row)
        for (int it = tid; it < KP * (TILE / 4); it += 256) {
            const int pp = it / (TILE / 4), q = it % (TILE / 4);
            const int p = p0 + pp;
            float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
            if (p < p_end) {
                va = *reinterpret_cast<const float4*>(fb + (size_t)p * C + c0 + 4 * q);
                vb = *reinterpret_cast<const float4*>(fb + (size_t)p * C + d0 + 4 * q);
            }
            float* da = la + pp * LS + 4 * q;
            float* db = lb + pp * LS + 4 * q;
            da[0] = va.x; da[1] = va.y; da[2] = va.z; da[3] = va.w;
            db[0] = vb.x; db[1] = vb.y; db[2] = vb.z; db[3] = vb.w;
        }
        __syncthreads();
#pragma unroll 8
        for (int s = 0; s < KP / 2; ++s) {
            const int p = 2 * s + lh;
            const float av = la[p * LS + wi * 32 + li];
            const float bv = lb[p * LS + wj * 32 + li];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
    }
    float* out = slab + ((size_t)b * nsplit + split) * C * C;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
        out[(size_t)(c0 + wi * 32 + row) * C + d0 + wj * 32 + li] = acc[r];
        if (ti != tj) out[(size_t)(d0 + wj * 32 + li) * C + c0 + wi * 32 + row] = acc[r];
    }
}

// The same partial Gram tiles with the features rounded to bf16 (RNE) and v_mfma_f32_32x32x16_bf16 (fp32
// accumulation): the RST_PRECISION_BF16 loss, whose VGG16 convs already take bf16 operands — the
// mixed_bfloat16 compute dtype of the Keras einsum (styleLoss.py gram_matrix). Per KP-pixel chunk each
// thread loads 16 pixels of one channel of both 64-channel slices (a wave's loads are one pixel's 64
// consecutive channels: coalesced), rounds them and writes them transposed, [channel][pixel] bf16 with a
// 72-element row (144 B: the ds_read_b128 lane groups of the operand reads and the 8-lane groups of the
// stores are conflict-free), so an MFMA operand (8 consecutive pixels of one channel) is one ds_read_b128.
// At 16x the f32 MFMA rate the kernel is bound by the feature reads, not the products.
namespace gramb {
constexpr int KP = 64, TILE = 64, RS = KP + 8;   // pixels per chunk, channels per slice, LDS row (bf16)
}
// FEAT_BF16: the features are stored as bf16 bits (the plain-bf16 VGG16's layer outputs): 8-B loads of channel quads
// (staging map below) and no rounding (the packed pieces are the stored bits)
template <bool FEAT_BF16>
__global__ __launch_bounds__(256) void gram_partial_bf16_kernel(const float* __restrict__ feat, float* __restrict__ slab,
                                                                int hw, int C, int nsplit, int span) {
    using namespace gramb;
    typedef short short8 __attribute__((ext_vector_type(8)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    __shared__ __attribute__((aligned(16))) unsigned short la[TILE * RS];
    __shared__ __attribute__((aligned(16))) unsigned short lb[TILE * RS];
    const int ntile = C / TILE;
    int bid = blockIdx.x;
    const int split = bid % nsplit;
    bid /= nsplit;
    const int npairs = ntile * (ntile + 1) / 2;
    int pair = bid % npairs;
    const int b = bid / npairs;
    int ti = 0;   // pair -> (ti, tj), ti <= tj, row-major over the upper triangle
    while (pair >= ntile - ti) {
        pair -= ntile - ti;
        ++ti;
    }
    const int tj = ti + pair;
    const int c0 = ti * TILE, d0 = tj * TILE;
    const int p_begin = split * span;
    const int p_end = min(hw, p_begin + span);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave >> 1, wj = wave & 1;
    const int li = lane & 31, lh = lane >> 5;
    const float* fb = feat + (size_t)b * hw * C;
    const int sc = tid & 63, sg = tid >> 6;   // staging: channel sc, pixels 16 sg .. 16 sg + 15 of the chunk

    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    auto pack = [](float x, float y) __attribute__((always_inline)) {
        return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
    };
    // FEAT_BF16 staging: thread = (slice, channel quad q4, pixel octet pg8): eight 8-B loads (its quad of eight
    // consecutive pixels; a wave's loads of one pixel cover 16 quads = one 128-B row piece), transposed with v_perm
    // into four 16-B LDS stores (eight pixels of one channel). Lane bits: 0-1 q4 low, 2-3 pg8 low, 4-5 q4 high; wave
    // bit 0 pg8 high, bit 1 the slice. A 16-lane store group then covers q4 = 4 consecutive rows (4 rows x 144 B apart
    // = 64 B mod 256) x 4 octets (16 B apart): 16 distinct 16-B bank slots (the first form, lanes = 16 quads of 4 pixels
    // with 8-B stores, put 4 lanes on each slot: SQ lds_conflict 0.78). The next chunk's loads are issued before this
    // chunk's stores and MFMAs.
    const int l64 = tid & 63;
    const int q4 = (l64 & 3) | ((l64 >> 4) << 2), pg8 = ((l64 >> 2) & 3) | ((wave & 1) << 2);
    const bool slice_b = (wave >> 1) != 0;
    const unsigned short* fsrc =
        reinterpret_cast<const unsigned short*>(feat) + (size_t)b * hw * C + (slice_b ? d0 : c0) + 4 * q4;
    unsigned short* const ldst = (slice_b ? lb : la) + (4 * q4) * RS + 8 * pg8;
    uint2 u8[8];
    auto load8 = [&](int p0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = p0 + 8 * pg8 + j;
            u8[j] = p < p_end ? *reinterpret_cast<const uint2*>(fsrc + (size_t)p * C) : make_uint2(0u, 0u);
        }
    };
    if constexpr (FEAT_BF16) load8(p_begin);
    for (int p0 = p_begin; p0 < p_end; p0 += KP) {
        if constexpr (FEAT_BF16) {
            // channel 4 q4 + k of pixel j: half (k & 1) of word (k >> 1) of u8[j]; v_perm selectors pick the low /
            // high bf16 of two words
            uint4 rows[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const unsigned sel = (k & 1) ? 0x07060302u : 0x05040100u;
                unsigned w[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) w[j] = (k >> 1) ? u8[j].y : u8[j].x;
                rows[k] = make_uint4(__builtin_amdgcn_perm(w[1], w[0], sel), __builtin_amdgcn_perm(w[3], w[2], sel),
                                     __builtin_amdgcn_perm(w[5], w[4], sel), __builtin_amdgcn_perm(w[7], w[6], sel));
            }
            if (p0 + KP < p_end) load8(p0 + KP);
            __syncthreads();   // the previous chunk's operand reads are done
#pragma unroll
            for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(ldst + k * RS) = rows[k];
            __syncthreads();
#pragma unroll
            for (int s = 0; s < KP / 16; ++s) {   // K step: pixels 16 s + 8 lh .. + 7
                const short8 av = *reinterpret_cast<const short8*>(la + (wi * 32 + li) * RS + 16 * s + 8 * lh);
                const short8 bv = *reinterpret_cast<const short8*>(lb + (wj * 32 + li) * RS + 16 * s + 8 * lh);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
            }
            continue;
        }
        float va[16], vb[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int p = p0 + 16 * sg + j;
            const bool ok = p < p_end;
            va[j] = ok ? fb[(size_t)p * C + c0 + sc] : 0.f;
            vb[j] = ok ? fb[(size_t)p * C + d0 + sc] : 0.f;
        }
        __syncthreads();   // the previous chunk's operand reads are done
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint4 wa = make_uint4(pack(va[8 * h], va[8 * h + 1]), pack(va[8 * h + 2], va[8 * h + 3]),
                                        pack(va[8 * h + 4], va[8 * h + 5]), pack(va[8 * h + 6], va[8 * h + 7]));
            const uint4 wb = make_uint4(pack(vb[8 * h], vb[8 * h + 1]), pack(vb[8 * h + 2], vb[8 * h + 3]),
                                        pack(vb[8 * h + 4], vb[8 * h + 5]), pack(vb[8 * h + 6], vb[8 * h + 7]));
            *reinterpret_cast<uint4*>(la + sc * RS + 16 * sg + 8 * h) = wa;
            *reinterpret_cast<uint4*>(lb + sc * RS + 16 * sg + 8 * h) = wb;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < KP / 16; ++s) {   // K step: pixels 16 s + 8 lh .. + 7
            const short8 av = *reinterpret_cast<const short8*>(la + (wi * 32 + li) * RS + 16 * s + 8 * lh);
            const short8 bv = *reinterpret_cast<const short8*>(lb + (wj * 32 + li) * RS + 16 * s + 8 * lh);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
        }
    }
    float* out = slab + ((size_t)b * nsplit + split) * C * C;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
        out[(size_t)(c0 + wi * 32 + row) * C + d0 + wj * 32 + li] = acc[r];
        if (ti != tj) out[(size_t)(d0 + wj * 32 + li) * C + c0 + wi * 32 + row] = acc[r];
    }
}

// Sums the splits in a fixed order: a workgroup owns 64 float4 of G; its four waves sum contiguous
// quarters of the split range, wave 0 adds the quarters in order and scales.
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          int C, int nsplit, float inv_hw, int batch) {
    const size_t cc4 = (size_t)C * C / 4;
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const size_t i = (size_t)blockIdx.x * 64 + lane;
    __shared__ float4 part[3][64];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool ok = i < (size_t)batch * cc4;
    if (ok) {
        const size_t b = i / cc4, e = i - b * cc4;
        const float4* s = reinterpret_cast<const float4*>(slab) + b * nsplit * cc4 + e;
        const int k0 = (nsplit * q) / 4, k1 = (nsplit * (q + 1)) / 4;
#pragma unroll 8
        for (int k = k0; k < k1; ++k) {
            const float4 v = s[(size_t)k * cc4];
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
    }
    if (q > 0) part[q - 1][lane] = acc;
    __syncthreads();
    if (q == 0 && ok) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float4 v = part[j][lane];
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
        reinterpret_cast<float4*>(out)[i] = make_float4(acc.x * inv_hw, acc.y * inv_hw, acc.z * inv_hw, acc.w * inv_hw);
    }
}

hipError_t gram_launch(const float* feat, int batch, int hw, int channels, float* out, void* ws, hipStream_t st,
                       bool bf16, bool feat_bf16) {
    if (channels % gram::TILE != 0) return hipErrorInvalidValue;
    const int ns = gram_splits(batch, hw, channels);
    int span = (hw + ns - 1) / ns;
    span = ((span + gram::KP - 1) / gram::KP) * gram::KP;
    const int ntile = channels / gram::TILE;
    const unsigned grid = (unsigned)(batch * (ntile * (ntile + 1) / 2) * ns);
    float* slab = static_cast<float*>(ws);
    if (feat_bf16)
        hipLaunchKernelGGL(gram_partial_bf16_kernel<true>, dim3(grid), dim3(256), 0, st, feat, slab, hw, channels, ns, span);
    else if (bf16)
        hipLaunchKernelGGL(gram_partial_bf16_kernel<false>, dim3(grid), dim3(256), 0, st, feat, slab, hw, channels, ns,
                           span);
    else
        hipLaunchKernelGGL(gram_partial_kernel, dim3(grid), dim3(256), 0, st, feat, slab, hw, channels, ns, span);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if ((reinterpret_cast<uintptr_t>(out) & 15) != 0) return hipErrorInvalidValue;
    const size_t total4 = (size_t)batch * channels * channels / 4;
    hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((total4 + 63) / 64)), dim3(256), 0, st, slab, out, channels,
                       ns, 1.0f / (float)hw, batch);
    return hipGetLastError();
}

}  // namespace rst
