// wino9_x6.hip — the network's first layer ("contract_start": Conv2D 9x9 s1 SAME, 17 -> 32 channels,
// built-in ReLU, then BatchNormalization and ReLU; realtime_style_transfer/models/styleTransfer.py:
// 188-205, 225-226) as the composite Winograd F(2x2, 3x3) of wino9.hip (nine 3x3 sub-kernels g_ab
// sharing one accumulator per transform point) with the transform-domain products on the bf16 MFMA
// pipe at fp32-level accuracy: every operand of the 16 batched GEMMs (V_ab = B^T d_ab B and
// U_ab = G g_ab G^T) split exactly into three bf16 pieces, six product terms, fp32 accumulation
// (dropped terms <= 2^-25 of each product; the scheme of wino_x6.hip).
//
// Workgroup = 4 waves, output block 8 x 16 pixels = 32 Winograd tiles x 32 output channels; wave w owns
// the transform points 4w..4w+3 (= row p = w of the 4x4 point grid; 64 accumulator registers), two
// workgroups per CU (75 KB of LDS each), so one workgroup's VALU-heavy transform + split phase runs
// beside the other's MFMA phase and two waves share each SIMD's VALU issue.
// K per sub-kernel: channels 0..15 are one K-step of the 32x32x16 MFMA (6 terms); channel 16 of all
// nine sub-kernels is gathered into one more K-step (K index = ab, 9 of 16 used) at the end, its V values
// kept in registers by the lanes that feed them to the MFMA. Per sub-kernel:
//   transform (thread = tile x channel pair: 16 ds_read_b64, 64 adds, split, 48 ds_write_b32) -> barrier
//   -> 24 MFMAs per wave (A: V pieces from LDS, B: U pieces from L2, prefetched one sub-kernel ahead)
//   -> barrier.
// Epilogue (as wino9.hip): M -> LDS, output transform per (tile, channel), bias -> ReLU -> BN (folded)
// -> ReLU, or in training the raw ReLU output and per-tile {sum, M2, n}.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace rst {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int TH = 8, TW = 16;                 // output pixels per workgroup
constexpr int PH = TH + 8, PW = TW + 8;        // input patch (pad 4 each side)
constexpr int NPX = PH * PW;                   // 384 patch pixels
constexpr int PS = 18;                         // patch pixel stride (floats): 17 channels + 1
constexpr int NT = 32;                         // output channels
constexpr int NXI = 16;                        // transform points
constexpr int VROW = 32;                       // bytes per (piece, xi, tile) row: 16 bf16
constexpr int V_BYTES = 3 * NXI * 32 * VROW;   // 48 KB
constexpr int PATCH_BYTES = NPX * PS * 4;      // 27 KB
constexpr int MS = 33;                         // M exchange row stride (floats)
constexpr int LDS_BYTES = PATCH_BYTES + V_BYTES;
static_assert(NXI * 32 * MS * 4 <= LDS_BYTES, "M exchange fits in the patch + V space");
constexpr int UBLK = NT * VROW;                // bytes per (ab, xi, piece) U block: 32 co x 16 bf16

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

// (x, y) -> the bf16 pair nearest them; (x, y) -= its value (exact in fp32)
__device__ __forceinline__ unsigned piece(float& x, float& y) {
    const unsigned p = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
    x = x - __uint_as_float(p << 16);
    y = y - __uint_as_float(p & 0xFFFF0000u);
    return p;
}

}  // namespace

// Experiment knobs (tools/wino9_x6_bench only; never set in the library build): W9_SKIP bit0 = no U loads
// in the loop, bit1 = no transform / split, bit2 = no MFMAs
#ifndef W9_SKIP
#define W9_SKIP 0
#endif

template <int CINT>
__global__ __launch_bounds__(256, 2) void wino9_x6_kernel(Wino9Args a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ float red[2][4][NT];   // training statistics: per-wave partial sums
    float* const patch = smem;                                                           // [384][18] f32
    unsigned char* const vbytes = reinterpret_cast<unsigned char*>(smem) + PATCH_BYTES;  // [3][16][32][32 B]
    float* const ms = smem;                                                              // [16][32][33] after

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    int bid = xcd_tile_order(blockIdx.x, gridDim.x);   // XCD-contiguous tile runs (halo reuse in L2)
    const int tx = bid % a.tiles_x;
    bid /= a.tiles_x;
    const int ty = bid % a.tiles_y;
    const int b = bid / a.tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;
    const int H = a.H, W = a.W, Cin = CINT > 0 ? CINT : a.cin;
    const size_t img = (size_t)b * H * W;

    // ---- U pieces: lane (li, lh) of wave w reads U[ab][4w + q][piece][co = li][8lh .. 8lh+7] ------
    const __amdgpu_buffer_rsrc_t usrd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U), 0, (9 + 1) * NXI * 3 * UBLK, 0x00020000);
    const int uvoff = li * VROW + 16 * lh;
    short8 ub[2][4][3];
    auto load_u = [&](auto BUF, int ab) __attribute__((always_inline)) {   // ab == 9: the channel-16 K-step
        constexpr int buf = decltype(BUF)::value;
        sfor<0, 4>([&](auto Q) __attribute__((always_inline)) {
            constexpr int q = decltype(Q)::value;
            sfor<0, 3>([&](auto Pc) __attribute__((always_inline)) {
                constexpr int p = decltype(Pc)::value;
                ub[buf][q][p] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(
                                                               usrd, uvoff, ((ab * NXI + 4 * wave + q) * 3 + p) * UBLK, 0));
            });
        });
    };
    load_u(std::integral_constant<int, 0>{}, 0);

    // ---- input patch (rows y0-4 .. y0+11, cols x0-4 .. x0+19) -> LDS [pixel][ch], zeros outside ----
    if constexpr (CINT > 0) {
        // all loads in flight before the first LDS write; clamped addresses, zeroed after the load
        constexpr int ROW = PW * CINT, TOTAL = PH * ROW, NIT = (TOTAL + 255) / 256;
        float v[NIT];
        sfor<0, NIT>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int i = min(tid + k * 256, TOTAL - 1);
            const int r = i / ROW, rem = i - r * ROW;
            const int px = rem / CINT, c = rem - px * CINT;
            const int gy = min(max(y0 - 4 + r, 0), H - 1), gx = min(max(x0 - 4 + px, 0), W - 1);
            v[k] = a.in[(img + (size_t)gy * W + gx) * CINT + c];
        });
        sfor<0, NIT>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            const int i = tid + k * 256;
            if (TOTAL % 256 == 0 || (k + 1) * 256 <= TOTAL || i < TOTAL) {
                const int r = i / ROW, rem = i - r * ROW;
                const int px = rem / CINT, c = rem - px * CINT;
                const int gy = y0 - 4 + r, gx = x0 - 4 + px;
                const bool inside = gy >= 0 && gy < H && gx >= 0 && gx < W;
                patch[(r * PW + px) * PS + c] = inside ? v[k] : 0.f;
            }
        });
    } else {
        const int row_fl = PW * Cin, total = PH * row_fl;
        for (int i = tid; i < total; i += 256) {
            const int r = i / row_fl, rem = i - r * row_fl;
            const int px = rem / Cin, c = rem - px * Cin;
            const int gy = y0 - 4 + r, gx = x0 - 4 + px;
            float v = 0.f;
            if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = a.in[(img + (size_t)gy * W + gx) * Cin + c];
            patch[(r * PW + px) * PS + c] = v;
        }
    }
    for (int i = tid; i < NPX * (PS - Cin); i += 256) {   // channels cin..17 of every pixel: zero
        const int px = i / (PS - Cin), c = Cin + i % (PS - Cin);
        patch[px * PS + c] = 0.f;
    }

    floatx16 acc[4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

    // transform role: tile tt (0..31), channel pair cp (channels 2cp, 2cp+1 of 0..15)
    const int tt = tid >> 3, cp = tid & 7;
    const int twy = tt >> 3, twx = tt & 7;
    const int vwoff = tt * VROW + 16 * ((cp >> 2) ^ ((tt >> 3) & 1)) + 4 * (cp & 3);
    auto vwrite = [&](int xi, unsigned p0, unsigned p1, unsigned p2) __attribute__((always_inline)) {
        *reinterpret_cast<unsigned*>(vbytes + ((0 * NXI + xi) * 32) * VROW + vwoff) = p0;
        *reinterpret_cast<unsigned*>(vbytes + ((1 * NXI + xi) * 32) * VROW + vwoff) = p1;
        *reinterpret_cast<unsigned*>(vbytes + ((2 * NXI + xi) * 32) * VROW + vwoff) = p2;
    };
    auto transform = [&](int sa, int sb) __attribute__((always_inline)) {
        const float* src = patch + ((2 * twy + 3 * sa) * PW + 2 * twx + 3 * sb) * PS + 2 * cp;
        float dx[4][4], dy[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const f32x2 v = *reinterpret_cast<const f32x2*>(src + (r * PW + c) * PS);
                dx[r][c] = v.x;
                dy[r][c] = v.y;
            }
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // B^T d
            const float a0 = dx[0][c], a1 = dx[1][c], a2 = dx[2][c], a3 = dx[3][c];
            dx[0][c] = a0 - a2; dx[1][c] = a1 + a2; dx[2][c] = a2 - a1; dx[3][c] = a1 - a3;
            const float b0 = dy[0][c], b1 = dy[1][c], b2 = dy[2][c], b3 = dy[3][c];
            dy[0][c] = b0 - b2; dy[1][c] = b1 + b2; dy[2][c] = b2 - b1; dy[3][c] = b1 - b3;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // (B^T d) B, split, write
            float vx[4] = {dx[r][0] - dx[r][2], dx[r][1] + dx[r][2], dx[r][2] - dx[r][1], dx[r][1] - dx[r][3]};
            float vy[4] = {dy[r][0] - dy[r][2], dy[r][1] + dy[r][2], dy[r][2] - dy[r][1], dy[r][1] - dy[r][3]};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned p0 = piece(vx[q], vy[q]);
                const unsigned p1 = piece(vx[q], vy[q]);
                const unsigned p2 = piece(vx[q], vy[q]);
                vwrite(r * 4 + q, p0, p1, p2);
            }
        }
    };
    // channel 16: lane (li, lh) of wave w keeps V_ab[p = w][q][tile li][ch 16] for the K index ab = 8lh + j
    float v16[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) v16[q][j] = 0.f;
    const int lwy = li >> 3, lwx = li & 7;
    auto transform16 = [&](int ab, int sa, int sb) __attribute__((always_inline)) {
        const float* src = patch + ((2 * lwy + 3 * sa) * PW + 2 * lwx + 3 * sb) * PS + 16;
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // row p = wave of B^T d (wave-uniform branch)
            const float d0 = src[(0 * PW + c) * PS], d1 = src[(1 * PW + c) * PS];
            const float d2 = src[(2 * PW + c) * PS], d3 = src[(3 * PW + c) * PS];
            t[c] = wave == 0 ? d0 - d2 : (wave == 1 ? d1 + d2 : (wave == 2 ? d2 - d1 : d1 - d3));
        }
        const float v[4] = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
        const bool mine = (ab >> 3) == lh;
#pragma unroll
        for (int q = 0; q < 4; ++q) v16[q][ab & 7] = mine ? v[q] : v16[q][ab & 7];
    };

    // A operands of point 4w + q: the three pieces of this lane's tile row, 16-B half lh (swizzled)
    const int varow = li * VROW + 16 * (lh ^ ((li >> 3) & 1));
    auto mfma6 = [&](int q, const short8* A, const short8* B) __attribute__((always_inline)) {
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], acc[q], 0, 0, 0);   // a0 b0
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], acc[q], 0, 0, 0);   // a0 b1
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], acc[q], 0, 0, 0);   // a1 b0
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], acc[q], 0, 0, 0);   // a0 b2
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], acc[q], 0, 0, 0);   // a1 b1
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], acc[q], 0, 0, 0);   // a2 b0
    };

    __syncthreads();   // patch + zero pads visible
    // sub-kernel loop fully unrolled: the U double buffer is indexed at compile time (registers)
    sfor<0, 9>([&](auto AB) __attribute__((always_inline)) {
        constexpr int ab = decltype(AB)::value, cur = ab & 1, sa = ab / 3, sb = ab % 3;
        if constexpr (!(W9_SKIP & 2)) {
            transform(sa, sb);
            transform16(ab, sa, sb);
        }
        __syncthreads();   // V(ab) complete
        if constexpr (!(W9_SKIP & 1)) load_u(std::integral_constant<int, cur ^ 1>{}, ab + 1);   // ab + 1 == 9: channel 16
        sfor<0, 4>([&](auto Q) __attribute__((always_inline)) {
            constexpr int q = decltype(Q)::value;
            short8 A[3];
            sfor<0, 3>([&](auto Pc) __attribute__((always_inline)) {
                constexpr int p = decltype(Pc)::value;
                A[p] = *reinterpret_cast<const short8*>(vbytes + ((p * NXI + 4 * wave + q) * 32) * VROW + varow);
            });
            if constexpr (!(W9_SKIP & 4)) mfma6(q, A, ub[cur][q]);
            else acc[q][0] += __builtin_bit_cast(float, (int)A[0][0] + (int)ub[cur][q][0][0]);
        });
        __syncthreads();   // V free for the next sub-kernel's transform
    });
    // channel-16 K-step: lane (li, lh) supplies K = 8lh .. 8lh+7 (ab; 9..15 are zero)
    sfor<0, 4>([&](auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        unsigned pk[3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float x = v16[q][2 * j], y = v16[q][2 * j + 1];
            pk[0][j] = piece(x, y);
            pk[1][j] = piece(x, y);
            pk[2][j] = piece(x, y);
        }
        short8 A[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) A[p] = __builtin_bit_cast(short8, (u32x4){pk[p][0], pk[p][1], pk[p][2], pk[p][3]});
        mfma6(q, A, ub[1][q]);   // 9 sub-kernels: the last load_u (ab + 1 == 9) went to buffer 9 & 1 = 1
    });
    __syncthreads();   // V / patch reads done before M overwrites them

    // ---- M -> LDS [xi][tile][co]: accumulator j of lane (li, lh) is tile (j&3) + 8(j>>2) + 4lh, channel li
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = (j & 3) + 8 * (j >> 2) + 4 * lh;
            ms[((wave * 4 + x) * 32 + row) * MS + li] = acc[x][j];
        }
    __syncthreads();

    // ---- output transform + epilogue: thread = (channel co, tiles 4g..4g+3) ----------------------
    const int co = tid & 31, g = tid >> 5;
    const float bias = a.bias[co];
    const bool train = a.part != nullptr;
    const float2 bn = train ? make_float2(1.f, 0.f) : a.bn_ab[co];
    float yv[16];
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int tile = g * 4 + k;
        const int wy = tile >> 3, wx = tile & 7;
        float m[16];
#pragma unroll
        for (int x = 0; x < NXI; ++x) m[x] = ms[(x * 32 + tile) * MS + co];
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
            const bool ok = oy < H && ox < W;
            const float v = fmaxf(yy[q] + bias, 0.f);                 // Conv2D(..., activation='relu')
            yv[k * 4 + q] = ok ? v : 0.f;
            if (ok) {
                // inference: BN (folded moving statistics) -> ReLU; training: the raw ReLU output
                a.out[(img + (size_t)oy * W + ox) * NT + co] = train ? v : fmaxf(fmaf(bn.x, v, bn.y), 0.f);
                s += v;
                cnt += 1.f;
            }
        }
    }
    if (train) {   // per-tile {sum, M2, n} of channel co over the 128 pixels (two-pass, fixed order)
        s += __shfl_xor(s, 32);
        cnt += __shfl_xor(cnt, 32);
        if (lane < 32) {
            red[0][wave][co] = s;
            red[1][wave][co] = cnt;
        }
        __syncthreads();
        const float S = (red[0][0][co] + red[0][1][co]) + (red[0][2][co] + red[0][3][co]);
        const float N = (red[1][0][co] + red[1][1][co]) + (red[1][2][co] + red[1][3][co]);
        const float mean = N > 0.f ? S / N : 0.f;
        float m2 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int tile = g * 4 + k;
                const int oy = y0 + 2 * (tile >> 3) + (q >> 1), ox = x0 + 2 * (tile & 7) + (q & 1);
                const float d = yv[k * 4 + q] - mean;
                if (oy < H && ox < W) m2 = fmaf(d, d, m2);
            }
        m2 += __shfl_xor(m2, 32);
        __syncthreads();
        if (lane < 32) red[0][wave][co] = m2;
        __syncthreads();
        if (tid < 32) {
            const float M2 = (red[0][0][co] + red[0][1][co]) + (red[0][2][co] + red[0][3][co]);
            const int n_part = a.tiles_y * a.tiles_x;
            a.part[((size_t)b * NT + co) * n_part + ty * a.tiles_x + tx] = make_float4(S, M2, N, 0.f);
        }
    }
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

hipError_t wino9_x6_prepare() {
    for (const void* k : {(const void*)wino9_x6_kernel<17>, (const void*)wino9_x6_kernel<0>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t wino9_x6_launch(const Wino9Args& a, hipStream_t st) {
    if (a.cin > 17 || a.cin <= 0 || a.tiles_y != (a.H + TH - 1) / TH || a.tiles_x != (a.W + TW - 1) / TW)
        return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    if (a.cin == 17)
        hipLaunchKernelGGL(wino9_x6_kernel<17>, dim3(grid), dim3(256), LDS_BYTES, st, a);
    else
        hipLaunchKernelGGL(wino9_x6_kernel<0>, dim3(grid), dim3(256), LDS_BYTES, st, a);
    return hipGetLastError();
}

}  // namespace rst
