// wino9.hip — the network's first layer ("contract_start": Conv2D 9x9 s1 SAME, 17 -> 32 channels,
// built-in ReLU, then BatchNormalization and ReLU; realtime_style_transfer/models/styleTransfer.py:
// 188-205, 225-226) as a composite Winograd F(2x2, 3x3) implicit GEMM on f32 MFMA.
//
// A 9x9 kernel is the sum of nine 3x3 sub-kernels g_ab[i][j] = w[3a+i][3b+j] (a, b in 0..2) applied to
// the input shifted by (3a, 3b). Each sub-conv is a Winograd F(2x2,3x3); the nine share one
// accumulator per transform point, so per 2x2 output tile the GEMM is
//     M[xi][co] = sum_{a,b} sum_ci V_ab[xi][ci] U_ab[xi][ci][co],   V_ab = B^T d_ab B,  U_ab = G g_ab G^T
// with one output transform Y = A^T M A at the end: 16 x 9 x 17 multiplies per tile and channel
// instead of 4 x 81 x 17 (2.25x fewer MFMA operations). The input tile of sub-kernel (a, b) starts at
// (2ty + 3a, 2tx + 3b) in the padded patch, so the transforms are recomputed per sub-kernel (cheap
// adds; the MFMAs dominate). Numerics: fp32 throughout, transforms exact ({0, +-1} adds), U formed
// on the host in f64 and rounded once — the same scheme as the residual-conv Winograd (wino.hip).
//
// Workgroup = 4 waves, output block 8 x 16 pixels = 4 x 8 = 32 Winograd tiles (one 32-row MFMA M
// tile) x 32 output channels (one 32-column N tile). Wave w owns the transform points 4w..4w+3:
// 4 accumulators (64 registers), so two workgroups fit per CU (LDS 70 KB each) and one workgroup's
// transforms and barriers hide behind the other's MFMAs. K per transform point = 9 sub-kernels x 18
// channels (17 + one zero), 9 MFMA k-steps (32x32x2) per sub-kernel:
//   k-steps 0..3: channel kk + 4*lh, 4..7: 8 + (kk-4) + 4*lh, 8: 16 + lh   (lh = lane half)
// so each lane reads its A operands as two ds_read_b128 + one ds_read_b32 per transform point, and
// its B operands (U, packed on the host in exactly this order) as three 16-B loads from L2.
// Epilogue: M -> LDS, output transform per (tile, channel), bias -> ReLU -> BN (folded) -> ReLU.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace rst {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TH = 8, TW = 16;                 // output pixels per workgroup
constexpr int PH = TH + 8, PW = TW + 8;        // input patch (pad 4 each side)
constexpr int NPX = PH * PW;                   // 384 patch pixels
constexpr int PS = 19;                         // patch pixel stride (floats): conflict-free transform reads
constexpr int VS = 20;                         // V row stride (floats): 5 x 16 B (odd), b128-aligned reads
constexpr int NT = 32;                         // output channels
constexpr int NXI = 16;                        // transform points
constexpr int USTR = 12;                       // U floats per (ab, xi, lane): 9 k-steps + 3 pad
constexpr int PATCH_FL = NPX * PS;             // 7296
constexpr int V_FL = NXI * 32 * VS;            // 10240
constexpr int MS = 33;                         // M exchange row stride
constexpr int M_FL = NXI * 32 * MS;            // 16896 (aliases patch + V after the main loop)
constexpr int LDS_FL = PATCH_FL + V_FL;        // 17536 floats = 70,144 B
static_assert(M_FL <= LDS_FL, "M exchange fits in the patch + V space");

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, N>(f);
    }
}

}  // namespace

// CINT > 0: the input channel count as a compile-time constant (the patch staging's index math
// divides by it); CINT == 0: any cin <= 17 at run time
template <int CINT>
__global__ __launch_bounds__(256, 2) void wino9_conv_kernel(Wino9Args a) {
    __shared__ __attribute__((aligned(16))) float smem[LDS_FL];
    __shared__ float red[2][4][NT];   // training statistics: per-wave partial sums
    float* const patch = smem;              // [384][19]
    float* const vs = smem + PATCH_FL;      // [16][32][20]
    float* const ms = smem;                 // [16][32][33] after the main loop

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

    // ---- U(ab) operands: lane (li, lh) of wave w, points 4w..4w+3, three 16-B loads each --------
    const f32x4* ug = reinterpret_cast<const f32x4*>(a.U) + ((size_t)(wave * 4) * 64 + lane) * (USTR / 4);
    f32x4 ur[2][4][3];
    auto load_u = [&](int buf, int ab) __attribute__((always_inline)) {
        const f32x4* p = ug + (size_t)ab * (NXI * 64 * (USTR / 4));
        sfor<0, 4>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            sfor<0, 3>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                ur[buf][x][q] = p[x * 64 * (USTR / 4) + q];
            });
        });
    };
    load_u(0, 0);

    // ---- input patch (rows y0-4 .. y0+11, cols x0-4 .. x0+19) -> LDS [pixel][ch], zeros outside ----
    // a patch row is PW*Cin contiguous floats in HBM (Cin = 17: not 16-B aligned, so 4-B loads)
    if constexpr (CINT > 0) {
        // all loads in flight before the first LDS write (a load-store loop serialises on vmcnt(0));
        // clamped addresses, zeroed after the load (branch-free)
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
    {
        for (int i = tid; i < NPX * (PS - Cin); i += 256) {   // channels cin..18 of every pixel: zero
            const int px = i / (PS - Cin), c = Cin + i % (PS - Cin);
            patch[px * PS + c] = 0.f;
        }
        for (int i = tid; i < NXI * 32 * (VS - 17); i += 256) {   // V channels 17..19 stay zero
            const int row = i / (VS - 17);
            vs[row * VS + 17 + i % (VS - 17)] = 0.f;
        }
    }

    floatx16 acc[4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

    // transform role: tile tt (0..31), channels tc, tc + 8 (and 16 for tc == 0)
    const int tt = tid & 31, tc = tid >> 5;
    const int twy = tt >> 3, twx = tt & 7;
    auto transform = [&](int ab, int c) __attribute__((always_inline)) {
        const int sa = ab / 3, sb = ab - 3 * (ab / 3);
        const float* src = patch + ((2 * twy + 3 * sa) * PW + 2 * twx + 3 * sb) * PS + c;
        float d[4][4], t[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) d[r][q] = src[(r * PW + q) * PS];
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // B^T d
            t[0][q] = d[0][q] - d[2][q];
            t[1][q] = d[1][q] + d[2][q];
            t[2][q] = d[2][q] - d[1][q];
            t[3][q] = d[1][q] - d[3][q];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // (B^T d) B
            float* dst = vs + ((r * 4) * 32 + tt) * VS + c;
            dst[0 * 32 * VS] = t[r][0] - t[r][2];
            dst[1 * 32 * VS] = t[r][1] + t[r][2];
            dst[2 * 32 * VS] = t[r][2] - t[r][1];
            dst[3 * 32 * VS] = t[r][1] - t[r][3];
        }
    };

    __syncthreads();   // patch + zero pads visible
    // sub-kernel loop fully unrolled: the U double buffer is indexed at compile time (registers)
    sfor<0, 9>([&](auto AB) __attribute__((always_inline)) {
        constexpr int ab = decltype(AB)::value, cur = ab & 1;
        transform(ab, tc);
        transform(ab, tc + 8);
        if (tc == 0) transform(ab, 16);
        __syncthreads();   // V(ab) complete
        if constexpr (ab + 1 < 9) load_u(cur ^ 1, ab + 1);
        sfor<0, 4>([&](auto X) __attribute__((always_inline)) {
            constexpr int x = decltype(X)::value;
            const float* va = vs + ((wave * 4 + x) * 32 + li) * VS;
            const f32x4 a0 = *reinterpret_cast<const f32x4*>(va + 4 * lh);
            const f32x4 a1 = *reinterpret_cast<const f32x4*>(va + 8 + 4 * lh);
            const float a2 = va[16 + lh];
            const f32x4 u0 = ur[cur][x][0], u1 = ur[cur][x][1], u2 = ur[cur][x][2];
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, u0.x, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, u0.y, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, u0.z, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, u0.w, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, u1.x, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, u1.y, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, u1.z, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, u1.w, acc[x], 0, 0, 0);
            acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2, u2.x, acc[x], 0, 0, 0);
        });
        __syncthreads();   // V free for the next sub-kernel's transform
    });

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
                // inference: BN (folded moving statistics) -> ReLU; training: the raw ReLU output, the
                // consumer's prologue applies the batch-statistics BN + ReLU
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

bool wino9_supported(int kh, int stride, int cin, int cout) { return kh == 9 && stride == 1 && cout == NT && cin <= 17; }
int wino9_tiles_y(int H) { return (H + TH - 1) / TH; }
int wino9_tiles_x(int W) { return (W + TW - 1) / TW; }

// U[ab][xi][lh][li][12]: k-step kk of lane (li, lh) = (G g_ab G^T)[xi] for input channel
// ch(kk, lh) (kk 0..3: kk + 4lh; 4..7: 8 + (kk-4) + 4lh; 8: 16 + lh) and output channel li;
// g_ab[i][j] = Keras HWIO kernel (9, 9, cin, 32) at tap (3a + i, 3b + j); channels >= cin are zero.
std::vector<float> wino9_pack_weights(const float* kern, int cin) {
#pragma clang fp contract(off)   // same operation order as wino9_transform_kernel
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    std::vector<float> U((size_t)9 * NXI * 64 * USTR, 0.f);
    for (int ab = 0; ab < 9; ++ab) {
        const int sa = ab / 3, sb = ab % 3;
        for (int lh = 0; lh < 2; ++lh)
            for (int kk = 0; kk < 9; ++kk) {
                const int ci = kk < 4 ? kk + 4 * lh : (kk < 8 ? 8 + (kk - 4) + 4 * lh : 16 + lh);
                if (ci >= cin) continue;
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
                            const int xi = p * 4 + q;
                            U[((((size_t)ab * NXI + xi) * 2 + lh) * 32 + co) * USTR + kk] = (float)u;
                        }
                }
            }
    }
    return U;
}

// Device form of wino9_pack_weights (training re-packs after every optimizer step): one thread per
// (ab, lh, kk, co); f64 with the host's operation order and no contraction (bitwise the host image).
// Entries for channels >= cin and the 3 pad slots are never written (U is zero-initialised).
__global__ __launch_bounds__(256) void wino9_transform_kernel(const float* __restrict__ kern, int cin,
                                                              float* __restrict__ U) {
#pragma clang fp contract(off)
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= 9 * 2 * 9 * NT) return;
    const int co = idx % NT, kk = (idx / NT) % 9, lh = (idx / (NT * 9)) % 2, ab = idx / (NT * 9 * 2);
    const int ci = kk < 4 ? kk + 4 * lh : (kk < 8 ? 8 + (kk - 4) + 4 * lh : 16 + lh);
    if (ci >= cin) return;
    const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    const int sa = ab / 3, sb = ab % 3;
    double gg[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) gg[i][j] = kern[(((size_t)(3 * sa + i) * 9 + (3 * sb + j)) * cin + ci) * NT + co];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double u = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) u = u + G[p][i] * gg[i][j] * G[q][j];
            U[((((size_t)ab * NXI + p * 4 + q) * 2 + lh) * 32 + co) * USTR + kk] = (float)u;
        }
}

hipError_t wino9_transform_launch(const float* kern, int cin, float* U, hipStream_t st) {
    if (cin > 17 || cin <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wino9_transform_kernel, dim3((9 * 2 * 9 * NT + 255) / 256), dim3(256), 0, st, kern, cin, U);
    return hipGetLastError();
}

hipError_t wino9_launch(const Wino9Args& a, hipStream_t st) {
    if (a.cin > 17 || a.cin <= 0) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)(a.batch * a.tiles_y * a.tiles_x);
    if (a.cin == 17)
        hipLaunchKernelGGL(wino9_conv_kernel<17>, dim3(grid), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(wino9_conv_kernel<0>, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace rst
