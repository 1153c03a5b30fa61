// wgrad.hip — weight gradients of the transfer network's convs on f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// dW[r][c] = sum_q S(q, r) * U(q, c), a GEMM with M = rows r = (tap, channel of the shifted operand),
// N = columns c, K = pixels q (all images):
//   conv  (styleTransfer.py:170,194):  S = X at q*s + tap - pad  (r = (tap, ci)),  U = dZ at q
//   convT (styleTransfer.py:115-119):  S = dZ at q*s + tap - pad (r = (tap, co)),  U = X at q
// Both land directly in the canonical Keras kernel layout ((kh,kw,in,out) resp. (kh,kw,out,in)).
//
// Workgroup = 4 waves, output tile TR x TC, K split over pixel ranges (split-K) so every layer
// fills the chip; per-split slabs are reduced in a fixed order (bitwise reproducible, no atomics).
// Per stage KP = 32 pixels: each thread owns a fixed row vector of S (its tap / channel decode is
// done once per kernel) and a fixed column vector of U (U is linear in q: no decode at all); the
// next stage's loads are issued into registers before this stage's MFMAs (register prefetch),
// then written to LDS behind one barrier. LDS reads are ds_read_b32 with 32 consecutive rows per
// lane half: conflict-free (banks (a/4)%32 per 32-lane half).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.h"
#include "train.h"

namespace rst {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace wg {
constexpr int KP = 32;   // pixels per stage
}

struct WgradGeom {
    int Cs, Cu, R, SH, SW;
    const float* S;
    const float* U;
};

__device__ __forceinline__ WgradGeom wgrad_geom(const WgradArgs& a) {
    WgradGeom g;
    const bool tr = a.transposed != 0;
    g.Cs = tr ? a.C2 : a.C1;
    g.Cu = tr ? a.C1 : a.C2;
    g.R = a.kh * a.kw * g.Cs;
    g.SH = tr ? a.DH : a.XH;
    g.SW = tr ? a.DW : a.XW;
    g.S = tr ? a.D : a.X;
    g.U = tr ? a.X : a.D;
    return g;
}

template <int TR, int TC, int WR, int WC, bool VS>
__global__ __launch_bounds__(256) void wgrad_mfma_kernel(WgradArgs a) {
    using wg::KP;
    constexpr int MR = TR / WR / 32, MC = TC / WC / 32;
    constexpr int AV = VS ? 4 : 1;
    constexpr int RA = TR / AV;          // S vectors per pixel
    constexpr int PSA = 256 / RA;        // pixel step of one thread's S loads
    constexpr int NA = KP / PSA;         // S loads per thread per stage
    constexpr int CB = TC / 4;           // U float4 per pixel
    constexpr int PSB = 256 / CB;
    constexpr int NB = KP / PSB;
    static_assert(WR * WC == 4 && MR >= 1 && MC >= 1, "4 waves");
    static_assert(256 % RA == 0 && KP % PSA == 0 && 256 % CB == 0 && KP % PSB == 0, "load mapping");
    typedef typename std::conditional<VS, f32x4, float>::type sT;

    __shared__ float la[KP * TR];
    __shared__ float lb[KP * TC];

    const WgradGeom g = wgrad_geom(a);
    const int nr = (g.R + TR - 1) / TR, nc = (g.Cu + TC - 1) / TC;
    int bid = blockIdx.x;
    const int split = bid % a.nsplit;
    bid /= a.nsplit;
    const int tc = bid % nc;
    const int trw = bid / nc;
    const int r0 = trw * TR, c0 = tc * TC;
    const long qhw = (long)a.Qh * a.Qw;
    const long total = (long)a.batch * qhw;
    const long q_begin = (long)split * a.span;
    const long q_end = min(total, q_begin + a.span);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WC, wc = wave % WC;
    const int li = lane & 31, lh = lane >> 5;

    // fixed S row vector of this thread: rows r .. r+AV-1 share one tap (Cs % AV == 0)
    const int ra = tid % RA, pa0 = tid / RA;
    const int r = r0 + ra * AV;
    const bool rvalid = r < g.R;
    const int tap = rvalid ? r / g.Cs : 0;
    const int ch = rvalid ? r - tap * g.Cs : 0;
    const int ky = tap / a.kw, kx = tap - (tap / a.kw) * a.kw;
    const int dy = ky - a.pad_t, dx = kx - a.pad_l;
    // fixed U column vector
    const int cb = tid % CB, pb0 = tid / CB;
    const int c = c0 + cb * 4;
    const bool cvalid = c < g.Cu;

    sT sreg[NA];
    f32x4 ureg[NB];
    auto load_stage = [&](long q0) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const long q = q0 + pa0 + k * PSA;
            sT v = sT(0.f);
            if (rvalid && q < q_end) {
                const int b = (int)(q / qhw);
                const int rem = (int)(q - (long)b * qhw);
                const int qy = rem / a.Qw, qx = rem - (rem / a.Qw) * a.Qw;
                const int sy = qy * a.stride + dy, sx = qx * a.stride + dx;
                if (sy >= 0 && sy < g.SH && sx >= 0 && sx < g.SW)
                    v = *reinterpret_cast<const sT*>(g.S + (((size_t)b * g.SH + sy) * g.SW + sx) * g.Cs + ch);
            }
            sreg[k] = v;
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const long q = q0 + pb0 + k * PSB;
            f32x4 v = f32x4(0.f);
            if (cvalid && q < q_end) v = *reinterpret_cast<const f32x4*>(g.U + (size_t)q * g.Cu + c);
            ureg[k] = v;
        }
    };
    auto store_stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NA; ++k) *reinterpret_cast<sT*>(&la[(pa0 + k * PSA) * TR + ra * AV]) = sreg[k];
#pragma unroll
        for (int k = 0; k < NB; ++k) *reinterpret_cast<f32x4*>(&lb[(pb0 + k * PSB) * TC + cb * 4]) = ureg[k];
    };

    floatx16 acc[MR][MC];
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < MC; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

    const int arow = wr * (TR / WR) + li, bcol = wc * (TC / WC) + li;
    if (q_begin < q_end) {
        load_stage(q_begin);
        store_stage();
        __syncthreads();
        for (long q0 = q_begin; q0 < q_end; q0 += KP) {
            const bool more = q0 + KP < q_end;
            if (more) load_stage(q0 + KP);
#pragma unroll 4
            for (int s = 0; s < KP / 2; ++s) {
                const int p = 2 * s + lh;
                float av[MR], bv[MC];
#pragma unroll
                for (int m = 0; m < MR; ++m) av[m] = la[p * TR + arow + m * 32];
#pragma unroll
                for (int n = 0; n < MC; ++n) bv[n] = lb[p * TC + bcol + n * 32];
#pragma unroll
                for (int m = 0; m < MR; ++m)
#pragma unroll
                    for (int n = 0; n < MC; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m], bv[n], acc[m][n], 0, 0, 0);
            }
            __syncthreads();
            if (more) {
                store_stage();
                __syncthreads();
            }
        }
    }
    const int Rp = nr * TR, Cp = nc * TC;
    float* out = a.slab + (size_t)split * Rp * Cp;
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < MC; ++n)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * lh;
                out[(size_t)(r0 + wr * (TR / WR) + m * 32 + row) * Cp + c0 + wc * (TC / WC) + n * 32 + li] =
                    acc[m][n][i];
            }
}

// dW[r][c] = sum over splits (fixed order)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(WgradArgs a, int Rp, int Cp) {
    const WgradGeom g = wgrad_geom(a);
    const size_t total = (size_t)g.R * g.Cu;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const size_t r = i / g.Cu, c = i % g.Cu;
        float s = 0.f;
        for (int k = 0; k < a.nsplit; ++k) s += a.slab[((size_t)k * Rp + r) * Cp + c];
        a.dW[i] = s;
    }
}

// ---- host side -------------------------------------------------------------------------------
namespace {
struct WTile {
    int tr, tc;
};

WTile wgrad_tile(const WgradArgs& a) {
    const int Cu = a.transposed ? a.C1 : a.C2;
    return Cu > 32 ? WTile{128, 128} : WTile{256, 32};
}

void wgrad_dims(const WgradArgs& a, int& R, int& Cu, int& Cs) {
    Cs = a.transposed ? a.C2 : a.C1;
    Cu = a.transposed ? a.C1 : a.C2;
    R = a.kh * a.kw * Cs;
}
}  // namespace

int wgrad_choose_splits(const WgradArgs& a) {
    int R, Cu, Cs;
    wgrad_dims(a, R, Cu, Cs);
    const WTile t = wgrad_tile(a);
    const long tiles = (long)((R + t.tr - 1) / t.tr) * ((Cu + t.tc - 1) / t.tc);
    const long total = (long)a.batch * a.Qh * a.Qw;
    long ns = 1024 / tiles;                      // ~4 workgroups per CU
    const long max_ns = (total + 8 * wg::KP - 1) / (8 * wg::KP);   // >= 8 stages per split
    if (ns > max_ns) ns = max_ns;
    return (int)(ns < 1 ? 1 : ns);
}

size_t wgrad_slab_bytes(const WgradArgs& a) {
    int R, Cu, Cs;
    wgrad_dims(a, R, Cu, Cs);
    const WTile t = wgrad_tile(a);
    const size_t Rp = (size_t)((R + t.tr - 1) / t.tr) * t.tr, Cp = (size_t)((Cu + t.tc - 1) / t.tc) * t.tc;
    return (size_t)a.nsplit * Rp * Cp * sizeof(float);
}

hipError_t wgrad_launch(WgradArgs a, hipStream_t st) {
    int R, Cu, Cs;
    wgrad_dims(a, R, Cu, Cs);
    if (Cu % 4 != 0) return hipErrorInvalidValue;
    const WTile t = wgrad_tile(a);
    const long total = (long)a.batch * a.Qh * a.Qw;
    long span = (total + a.nsplit - 1) / a.nsplit;
    span = ((span + wg::KP - 1) / wg::KP) * wg::KP;
    a.span = span;
    const int nr = (R + t.tr - 1) / t.tr, nc = (Cu + t.tc - 1) / t.tc;
    const dim3 grid((unsigned)(nr * nc * a.nsplit));
    const bool vs = Cs % 4 == 0;
    if (t.tr == 128) {
        if (vs) hipLaunchKernelGGL((wgrad_mfma_kernel<128, 128, 2, 2, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((wgrad_mfma_kernel<128, 128, 2, 2, false>), grid, dim3(256), 0, st, a);
    } else {
        if (vs) hipLaunchKernelGGL((wgrad_mfma_kernel<256, 32, 4, 1, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((wgrad_mfma_kernel<256, 32, 4, 1, false>), grid, dim3(256), 0, st, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t n = (size_t)R * Cu;
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, a, nr * t.tr, nc * t.tc);
    return hipGetLastError();
}

}  // namespace rst
