// kernels.h — internal kernel interfaces of librst (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <type_traits>
#include <vector>

namespace rst {

enum ProMode { PRO_NONE = 0, PRO_AFF_RELU = 1, PRO_AFF = 2, PRO_AFF_RES = 3, PRO_MASK = 4 };
enum EpiMode { EPI_NONE = 0, EPI_RELU_BN = 1, EPI_RELU_STATS = 2, EPI_STATS = 3 };

// Workgroup barrier that orders LDS only: __syncthreads() is a workgroup-scope fence on all memory, which
// on gfx950 waits for every outstanding global load and store of the wave (s_waitcnt vmcnt(0)) — the
// prefetched operands still in flight and the epilogue's stores. Kernels whose global traffic is not
// exchanged through the barrier use this one (s_waitcnt lgkmcnt(0); s_barrier).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Two-style blending (num_styles == 2, styleTransfer.py:36-44 with the weights completed as
// [1 - w1, w1] at :297-302): w0*v0 + w1*v1 = v0 + w1*(v1 - v0). The one formula every blend site
// uses (conv prologues, the standalone affine kernel, rst_style_param_map).
__device__ __forceinline__ float style_blend(float w1, float v0, float v1) { return fmaf(w1, v1 - v0, v0); }

// Exact three-piece bf16 split (the split-bf16 x6 kernels): (x, y) -> the packed bf16 pair nearest them (RNE),
// then (x, y) -= its value; the remainder is exact in fp32 (x's own low bits). The subtraction must be an IEEE
// f32 subtract: v_dot2c_f32_bf16 (x + (-1)·piece in one instruction) was measured NOT to reproduce it —
// tools/dot2_split_check: 16.5 M of 16.8 M random pairs differ in some piece (round 4) — so the piece is widened
// with a shift / mask and subtracted.
typedef float rst_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 rst_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned bf16_piece(float& x, float& y) {
    const unsigned p = __builtin_bit_cast(unsigned, __builtin_convertvector((rst_f32x2){x, y}, rst_bf16x2));
    x = x - __uint_as_float(p << 16);
    y = y - __uint_as_float(p & 0xFFFF0000u);
    return p;
}
__device__ __forceinline__ unsigned bf16_last_piece(float x, float y) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector((rst_f32x2){x, y}, rst_bf16x2));
}

// bf16 activation storage (the plain-bf16 VGG16: Keras mixed_bfloat16 layer outputs are bf16). Four consecutive
// bf16 values at element index i of `base` widened to f32 (exact), and four f32 values rounded to bf16 (RNE, as
// every bf16 operand rounding here) and packed for one 8-byte store.
__device__ __forceinline__ float4 ld_bf16x4(const void* base, size_t i) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const unsigned short*>(base) + i);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xFFFF0000u));
}
__device__ __forceinline__ float ld_bf16(const void* base, size_t i) {
    return __uint_as_float((unsigned)reinterpret_cast<const unsigned short*>(base)[i] << 16);
}
__device__ __forceinline__ uint2 pack_bf16x4(float x, float y, float z, float w) {
    return make_uint2(bf16_last_piece(x, y), bf16_last_piece(z, w));
}

// In-graph kernel timeline (rst_timeline_begin / rst_timeline_read): every wave of a launch stores the 100-MHz
// realtime counter as it ends into its slot of the layer's buffer (TL_SLOTS entries); the host takes the latest
// stamp per layer, so end(k) - end(k - 1) is layer k's share of a graph replay. Measurement only: a null tl (the
// default) stores nothing. The store is a vector store (global_store_dwordx2 from lane 0).
constexpr int TL_SLOTS = 16384;   // >= waves of any stamped launch (wino_x6 at B = 8: 1800 x 8)
__device__ __forceinline__ void tl_stamp_end(unsigned long long* tl) {
    if (tl != nullptr && (threadIdx.x & 63) == 0) {
        const unsigned idx = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (idx < (unsigned)TL_SLOTS) tl[idx] = __builtin_amdgcn_s_memrealtime();
    }
}

// x + x[lane ^ O] for O = 16 / 32 on the VALU (v_permlane16/32_swap, gfx950) instead of ds_bpermute (__shfl_xor,
// an LDS round trip per value): the swap hands each lane the partner's value, the add is commutative, so the result
// is bitwise __shfl_xor's
template <int O>
__device__ __forceinline__ float lane_xor_sum(float x) {
    static_assert(O == 16 || O == 32, "permlane swaps cover xor 16 / 32");
    const unsigned u = __float_as_uint(x);
    if constexpr (O == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else {
        const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
}

// XCD-aware block order: the dispatcher deals workgroup ids round-robin over the 8 XCDs (each with
// its own L2), so consecutive ids (neighbouring tiles, whose halos overlap) land on different L2s.
// Remap so XCD x processes one contiguous run of the tile order: a bijection on [0, n).
__device__ __forceinline__ int xcd_tile_order(int bid, int n) {
    constexpr int NXCD = 8;
    const int x = bid % NXCD, k = bid / NXCD;
    const int base = n / NXCD, rem = n % NXCD;
    return x * base + min(x, rem) + k;
}

// ---- next-layer weights into L2 (inference; speed only) -----------------------------------------------
// Every workgroup of a launch reads one slice of the next layer's weight image, one dword per 128-B line, all its
// loads issued at once: the workgroups with the same blockIdx % 8 (one XCD under the round-robin dispatch) cover the
// whole image, so the next kernel's first weight loads hit its XCD's L2 instead of all missing together. The caller
// passes the loaded words to l2_touch_keep at its end (keeps the loads). Measured on the residual convs: cold U cost
// 6-9 us per launch in the frame.
// The loaded words are returned unfolded: their first use (l2_touch_keep, at the kernel's end) is where the compiler
// waits for them, so a touch issued inside a branch does not drain the caller's outstanding loads there.
typedef unsigned l2_touch_t __attribute__((ext_vector_type(2)));
template <int NT, int NLD>
__device__ __forceinline__ l2_touch_t l2_touch_xcd_slice(const void* p, int bytes) {
    static_assert(NLD == 1 || NLD == 2, "one or two lines per thread");
    l2_touch_t f = {0u, 0u};
    if (p == nullptr || bytes <= 0) return f;
    const int xr = (int)(blockIdx.x & 7), k = (int)(blockIdx.x >> 3);
    const int nk = ((int)gridDim.x - xr + 7) >> 3;   // workgroups with this XCD residue
    const int nl = bytes >> 7, per = (nl + nk - 1) / nk;
    const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
    const int beg = k * per, end = min(beg + per, nl);
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
        const int i = beg + (int)threadIdx.x + j * NT;
        f[j] = __builtin_amdgcn_raw_buffer_load_b32(srd, i < end ? i * 128 : 0x7FFFFFF0, 0, 0);
    }
    return f;
}
__device__ __forceinline__ void l2_touch_keep(l2_touch_t f, bool never, float* sink) {
    if ((f.x ^ f.y) == 0x9E3779B9u && never) *sink = 0.f;   // never true: only keeps the loads
}

// ---- CIN statistics through fixed-point accumulators (inference) ---------------------------------------
// The producer of a conditional-instance-normalised layer adds, per workgroup and channel, its
// {sum, sum of squares} (f64, formed in a fixed order) into one of nslot accumulator copies (no-return atomics,
// executed at the memory side; the copies bound the adders per address); the consumer's workgroups merge the
// copies and form the affine themselves (cin_affine: the finalize_kernel arithmetic), so no finalize kernel runs
// between the two. Per workgroup the sum of squares is M2 + S^2/n of its two-pass tile statistics — the
// quantity finalize_kernel merges.
// The adds are exact integer adds, so the merged sums do not depend on the order the atomics land in: each f64
// addend is cut (magnitude truncated at 2^-48, sign applied to every limb) into CIN_LIMBS signed 64-bit limbs of
// weights 2^-48, 2^-8 and 2^32 (payloads 40, 40 and up to 52 bits; |addend| < 2^84), added limb by limb; the
// consumer sums the limbs as integers, carries, and converts once. Bitwise-deterministic CIN statistics
// (SURVEY §7), at least as accurate as the f64 sums (the merge itself is exact; the truncation is below 2^-48
// absolute per workgroup, i.e. far below the 1e-5 epsilon the variance is used with).
constexpr int CIN_ACC_MAX_SLOTS = 64;
constexpr int CIN_LIMBS = 3;
typedef long long cin_word;
struct CinAcc {              // producer side (null acc: the per-tile partials path)
    cin_word* acc;           // [nslot][B][2][CIN_LIMBS][C]: sums, then sums of squares; zeroed before the producer
    int nslot;
};
struct CinSrc {              // consumer side: the producer's accumulators and its CIN parameters
    const cin_word* acc;     // [nslot][B][2][CIN_LIMBS][C] (null: the prologue reads pro_ab as before)
    int nslot, C, batch;
    double n;                // values per (image, channel): the producer's Ho * Wo
    const float* style;      // style parameters: image b's scale at style[b*style_stride + style_offset + c],
    int style_stride;        // its bias C further; the second style (two styles) style1_offset further
    int style_offset;
    int style1_offset;
    float eps;
    float2* ab_out;          // stored by workgroup 0 (rst_copy_activation and the host read them); may be null
    float2* ab1_out;
};

// v -> limbs (l0, l1, l2) with v ~= l2 * 2^32 + l1 * 2^-8 + l0 * 2^-48 (every step exact on |v|: the remainders
// are v's own low bits; bits below 2^-48 dropped)
__device__ __forceinline__ void cin_fixed_split(double v, cin_word& l0, cin_word& l1, cin_word& l2) {
    const double a = fabs(v);
    const double h = floor(a * 0x1p-32);
    const double r = a - h * 0x1p32;          // [0, 2^32)
    const double m = floor(r * 0x1p8);
    const double r2 = r - m * 0x1p-8;         // [0, 2^-8)
    const cin_word k0 = (cin_word)floor(r2 * 0x1p48), k1 = (cin_word)m, k2 = (cin_word)h;
    const bool neg = v < 0.0;
    l0 = neg ? -k0 : k0;
    l1 = neg ? -k1 : k1;
    l2 = neg ? -k2 : k2;
}

// summed limbs -> the value: the magnitude's limbs are carried into canonical form (lower limbs in [0, 2^40)) and
// converted as a sum of non-negative terms (no cancellation), then the sign is applied; deterministic
__device__ __forceinline__ double cin_fixed_value(cin_word l0, cin_word l1, cin_word l2) {
    auto carry = [](cin_word& a0, cin_word& a1, cin_word& a2) __attribute__((always_inline)) {
        cin_word c = a0 >> 40;
        a0 -= c << 40;
        a1 += c;
        c = a1 >> 40;
        a1 -= c << 40;
        a2 += c;
    };
    cin_word m0 = l0, m1 = l1, m2 = l2;
    carry(m0, m1, m2);
    const bool neg = m2 < 0;                  // the value is l2 * 2^32 + [0, 2^32)
    if (neg) {
        m0 = -l0;
        m1 = -l1;
        m2 = -l2;
        carry(m0, m1, m2);
    }
    const double v = (double)m2 * 0x1p32 + ((double)m1 * 0x1p-8 + (double)m0 * 0x1p-48);
    return neg ? -v : v;
}

__device__ __forceinline__ void cin_word_add(cin_word* p, cin_word v) {
    if (v != 0) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one value (which = 0: sum, 1: sum of squares) of image b, channel c into copy `slot`
__device__ __forceinline__ void cin_acc_add_value(const CinAcc& a, int batch, int C, int b, int c, int slot,
                                                  int which, double v) {
    cin_word* const p = a.acc + ((size_t)((slot * batch + b) * 2 + which) * CIN_LIMBS) * C + c;
    cin_word l0, l1, l2;
    cin_fixed_split(v, l0, l1, l2);
    cin_word_add(p, l0);
    cin_word_add(p + C, l1);
    cin_word_add(p + 2 * C, l2);
}

__device__ __forceinline__ void cin_acc_add(const CinAcc& a, int batch, int C, int b, int c, int slot, double S,
                                            double Q) {
    cin_acc_add_value(a, batch, C, b, c, slot, 0, S);
    cin_acc_add_value(a, batch, C, b, c, slot, 1, Q);
}

// One pass structure of cin_affine_table with R copies per lane (compile time): every lane issues its R x 2 x CIN_LIMBS
// accumulator loads and its style-parameter loads unconditionally (clamped to a valid address, masked after), so they
// are all in flight together and the lane waits once. (The round-4 form guarded each load by its copy / item test:
// hipcc then waited for every load before issuing the next — 6 R serialized L2 round trips after a full drain of the
// caller's staging loads, 4.2 us of a 31 us residual conv at the frame's 8 copies.)
template <int NT, int R>
__device__ __forceinline__ void cin_affine_pass(const CinSrc& s, int b0, int n, int L, float2* tab, float2* tab1,
                                                float2* out, float2* out1) {
    auto pass = [&](int base) __attribute__((always_inline)) {
        const int i = base + (int)threadIdx.x;
        const bool live = i < n;
        const int ic = live ? i : n - 1;
        const int it = ic / L, l = ic & (L - 1);
        const int j = it / s.C, c = it - j * s.C, b = b0 + j;
        const bool head = live && l == 0;
        const float* const sp = s.style + (size_t)b * s.style_stride + s.style_offset;
        const float g0 = sp[c], be0 = sp[s.C + c];   // independent of the accumulators: in flight with them
        float g1 = 0.f, be1 = 0.f;
        if (tab1 != nullptr) {   // uniform
            g1 = sp[s.style1_offset + c];
            be1 = sp[s.style1_offset + s.C + c];
        }
        cin_word v[R][2 * CIN_LIMBS];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int k = l + L * r;
            const int kc = k < s.nslot ? k : 0;
            const cin_word* const p = s.acc + ((size_t)(kc * s.batch + b) * 2 * CIN_LIMBS) * s.C + c;
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) v[r][q] = p[q * s.C];
        }
        cin_word w[2 * CIN_LIMBS] = {};
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const cin_word m = l + L * r < s.nslot ? ~(cin_word)0 : (cin_word)0;   // copies past nslot add nothing
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += v[r][q] & m;
        }
        // the L lanes of an item are consecutive: within a quad (L <= 4) the partner words move by DPP (VALU) instead
        // of ds_bpermute round trips; integer adds, so the merged words do not depend on the order
        auto dpp64 = [](cin_word x, auto CTRL) __attribute__((always_inline)) {
            constexpr int ctrl = decltype(CTRL)::value;
            const unsigned lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)x, ctrl, 0xF, 0xF, true);
            const unsigned hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)((unsigned long long)x >> 32), ctrl, 0xF,
                                                            0xF, true);
            return (cin_word)(((unsigned long long)hi << 32) | lo);
        };
        if (L >= 2) {
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += dpp64(w[q], std::integral_constant<int, 0xB1>{});   // xor 1
        }
        if (L >= 4) {
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += dpp64(w[q], std::integral_constant<int, 0x4E>{});   // xor 2
        }
        for (int o = 4; o < L; o <<= 1) {
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += __shfl_xor(w[q], o);
        }
        if (head) {
            const double S = cin_fixed_value(w[0], w[1], w[2]), Q = cin_fixed_value(w[3], w[4], w[5]);
            const double N = s.n, mean = S / N, var = fmax(Q - S * mean, 0.0) / N;
            const float rstd = (float)(1.0 / sqrt(var + (double)s.eps));
            const float aa = g0 * rstd;
            const float2 vv = make_float2(aa, be0 - (float)mean * aa);
            tab[it] = vv;
            if (out != nullptr) out[it] = vv;
            if (tab1 != nullptr) {
                const float a1 = g1 * rstd;
                const float2 v1 = make_float2(a1, be1 - (float)mean * a1);
                tab1[it] = v1;
                if (out1 != nullptr) out1[it] = v1;
            }
        }
    };
    // the first pass outside the loop: a loop's back edge makes hipcc wait for the previous iteration's loads at the
    // loop top (register reuse), which at the first entry drains every load the caller has in flight
    pass(0);
    for (int base = NT; base < n; base += NT) pass(base);
}

// Every thread of an NT-thread workgroup calls this: the affine of images b0 .. b0 + nb - 1, channels [0, C)
// (finalize_kernel's arithmetic on the merged sums) into tab[j * C + c] for image b0 + j (and the second
// style's into tab1[j * C + c] when tab1 is given; LDS or global), also into out / out1 when given (the
// host-visible copies, same indexing). L lanes per (image, channel) (a power of two, L * nb * C <= NT where
// possible) each read K / L of the K = nslot (rounded up to a power of two) accumulator copies, all loads
// issued together with the style-parameter loads, and reduce by DPP / xor shuffles: one memory latency per pass.
template <int NT, int RMAX = 8>
__device__ __forceinline__ void cin_affine_table(const CinSrc& s, int b0, int nb, float2* tab, float2* tab1,
                                                 float2* out, float2* out1) {
    // RMAX: copies per lane (each 2 x CIN_LIMBS words in flight). Every instantiated pass width is register-allocated
    // for the whole kernel, so a register-tight caller passes RMAX = 1 (one copy per lane, more lanes per item)
    static_assert(RMAX == 1 || RMAX == 2 || RMAX == 4 || RMAX == 8, "RMAX");
    int K = 1;
    while (K < s.nslot) K <<= 1;
    const int items = nb * s.C;
    int L = K / RMAX > 1 ? K / RMAX : 1;                   // at most RMAX copies per lane
    // more lanes while one pass still covers every item, up to a quad (the lanes of an item merge by DPP: VALU only)
    while (L < K && L < 4 && 2 * L * items <= NT) L <<= 1;
    const int R = K / L, n = items * L;
    if (RMAX == 1 || R == 1) cin_affine_pass<NT, 1>(s, b0, n, L, tab, tab1, out, out1);   // R is uniform
    else if constexpr (RMAX >= 2) {
        if (R == 2) cin_affine_pass<NT, 2>(s, b0, n, L, tab, tab1, out, out1);
        else if constexpr (RMAX >= 4) {
            if (R == 4) cin_affine_pass<NT, 4>(s, b0, n, L, tab, tab1, out, out1);
            else if constexpr (RMAX >= 8) cin_affine_pass<NT, 8>(s, b0, n, L, tab, tab1, out, out1);
        }
    }
}

// Split form of cin_affine_table for one image (nb = 1) whose whole table is one pass (C * L <= NT) and whose copies
// per lane fit RS: issue() sends the accumulator and style-parameter loads, finish() (after the caller has issued its
// own first loads) merges them and writes the table. vmcnt retires loads in issue order, so the accumulator loads
// issued first are waited for without waiting for the caller's later (HBM) loads — the two latencies overlap instead
// of adding. usable() says whether the split form applies (uniform); otherwise call cin_affine_table.
template <int NT, int RS>
struct CinAffineSplit {
    cin_word v[RS][2 * CIN_LIMBS];
    float g0, be0, g1, be1;
    int it, l, L;
    bool head;
    static __device__ __forceinline__ int lanes(const CinSrc& s, int& K) {
        K = 1;
        while (K < s.nslot) K <<= 1;
        int L = K / 8 > 1 ? K / 8 : 1;
        while (L < K && L < 4 && 2 * L * s.C <= NT) L <<= 1;
        return L;
    }
    static __device__ __forceinline__ bool usable(const CinSrc& s) {
        int K;
        const int L = lanes(s, K);
        return K / L <= RS && s.C * L <= NT;
    }
    __device__ __forceinline__ void issue(const CinSrc& s, int b, bool two_styles) {
        int K;
        L = lanes(s, K);
        const int n = s.C * L;
        const int i = (int)threadIdx.x, ic = i < n ? i : n - 1;
        it = ic / L;
        l = ic & (L - 1);
        head = i < n && l == 0;
        const float* const sp = s.style + (size_t)b * s.style_stride + s.style_offset;
        g0 = sp[it];
        be0 = sp[s.C + it];
        g1 = be1 = 0.f;
        if (two_styles) {
            g1 = sp[s.style1_offset + it];
            be1 = sp[s.style1_offset + s.C + it];
        }
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const int k = l + L * r;
            const int kc = k < s.nslot ? k : 0;
            const cin_word* const p = s.acc + ((size_t)(kc * s.batch + b) * 2 * CIN_LIMBS) * s.C + it;
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) v[r][q] = p[q * s.C];
        }
    }
    __device__ __forceinline__ void finish(const CinSrc& s, float2* tab, float2* tab1, float2* out, float2* out1) {
        cin_word w[2 * CIN_LIMBS] = {};
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const cin_word m = l + L * r < s.nslot ? ~(cin_word)0 : (cin_word)0;
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += v[r][q] & m;
        }
        auto dpp64 = [](cin_word x, auto CTRL) __attribute__((always_inline)) {
            constexpr int ctrl = decltype(CTRL)::value;
            const unsigned lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)x, ctrl, 0xF, 0xF, true);
            const unsigned hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)((unsigned long long)x >> 32), ctrl, 0xF,
                                                            0xF, true);
            return (cin_word)(((unsigned long long)hi << 32) | lo);
        };
        if (L >= 2) {
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += dpp64(w[q], std::integral_constant<int, 0xB1>{});
        }
        if (L >= 4) {
#pragma unroll
            for (int q = 0; q < 2 * CIN_LIMBS; ++q) w[q] += dpp64(w[q], std::integral_constant<int, 0x4E>{});
        }
        if (head) {
            const double S = cin_fixed_value(w[0], w[1], w[2]), Q = cin_fixed_value(w[3], w[4], w[5]);
            const double N = s.n, mean = S / N, var = fmax(Q - S * mean, 0.0) / N;
            const float rstd = (float)(1.0 / sqrt(var + (double)s.eps));
            const float aa = g0 * rstd;
            const float2 vv = make_float2(aa, be0 - (float)mean * aa);
            tab[it] = vv;
            if (out != nullptr) out[it] = vv;
            if (tab1 != nullptr) {
                const float a1 = g1 * rstd;
                const float2 v1 = make_float2(a1, be1 - (float)mean * a1);
                tab1[it] = v1;
                if (out1 != nullptr) out1[it] = v1;
            }
        }
    }
};

// Arguments of the implicit-GEMM MFMA conv kernel (conv_mfma.hip).
struct ConvArgs {
    const float* in;        // NHWC [B][H][W][cin] raw producer output
    const float* res;       // residual source (PRO_AFF_RES), same shape as in
    float* mat;             // materialise transformed input here (or null)
    const float2* pro_ab;   // [B][cin] prologue affine (a, b)
    const float2* pro_ab1;  // [B][cin] second style's affine (two-style blending) or null
    const float* pro_w;     // [B][H][W] per-pixel weight of the second style (with pro_ab1)
    const float* wpk;       // packed weights [n_blocks][nchunks][ngroups][wstage]
    const float* bias;      // [ntot]
    const float2* bn_ab;    // [ntot] BatchNorm affine (EPI_RELU_BN)
    float* out;             // NHWC output
    float4* part;           // [B][ntot][n_mtiles] {sum, M2, n} or null
    int batch, H, W, cin;
    int Ho, Wo;             // GEMM-space output dims (convT: input dims, shuffle doubles them)
    int ntot;               // GEMM N
    int cout;               // stored channels (convT: per phase)
    int pad_t, pad_l;
    int tiles_y, tiles_x, n_blocks, nchunks;
    int pro_mode, epi_mode, shuffle;
    CinAcc stat;            // conv_lite inference: CIN statistics into f64 accumulators instead of part
    CinSrc pro_stat;        // conv_lite inference: the prologue affine formed from the producer's accumulators
    float* pool;            // conv_bf3 VGG16 epilogue (conv_bf3_fuses_pool): also the 2x2 / 2 max-pooled output
                            // [B][Ho/2][Wo/2][ntot] (VALID, as maxpool2_launch), or null
    const void* w_next;     // conv_lite inference: the next layer's weight image into L2 (l2_touch_xcd_slice)
    int w_next_bytes;
    int wt_stores;          // nonzero: output stored write-through (sc1), as WinoArgs::wt_stores
    unsigned long long* tl; // conv_lite: in-graph timeline stamps (tl_stamp_end) or null
    int act_bf16;           // conv_bf3 / conv_mfma, the plain-bf16 VGG16 (Keras mixed_bfloat16 layer outputs): bit 0 `in`,
                            // bit 1 `out` and `pool`, bit 2 `res` (PRO_MASK) hold bf16 bits (unsigned short), not f32
};

// Write-through stores address the output with 32-bit buffer offsets: the byte extent of what the kernel indexes
// (pixel-shuffled 2Ho x 2Wo x cout for transposed convs, Ho x Wo x ntot otherwise; the fused pool is smaller) must fit,
// or the launch falls back to plain stores (conv_launch, conv_bf3_launch)
inline ConvArgs conv_wt_checked(const ConvArgs& a) {
    const size_t px = a.shuffle ? (size_t)a.batch * (2 * (size_t)a.Ho) * (2 * (size_t)a.Wo) * a.cout
                                : (size_t)a.batch * a.Ho * a.Wo * a.ntot;
    ConvArgs b = a;
    if (px * 4 >= (size_t)0x7FFFFFF0) b.wt_stores = 0;
    return b;
}

// A compiled tile configuration of conv_mfma_kernel.
struct ConvTile {
    int id;
    int kh, kw, stride, ck, nt, th, tw, tps, hb, vec, mt, ngroups, wstage, lds_bytes;
    int bf3;                // split-bf16 kernel (conv_bf3.hip): number of bf16 planes (2: bf16x3, 3: bf16x6), 0: f32
};

bool conv_select(int kh, int stride, int cin, int ntot, ConvTile* out);
hipError_t conv_launch(const ConvTile& t, const ConvArgs& a, hipStream_t st);
// one-time per-configuration setup (dynamic LDS > 64 KB); call outside graph capture
hipError_t conv_prepare(const ConvTile& t);
// split-bf16 variant (conv_bf3.hip): 3x3 s1, Cin % 32 == 0; conv_launch/conv_prepare dispatch on t.bf3
// in_bf16: the input is bf16 activations and the conv has no prologue (the plain-bf16 VGG16 forward after conv 0);
// mask_bf16: a bf16 gradient under a bf16 ReLU mask (PRO_MASK: the plain-bf16 VGG16's input-gradient convs)
bool conv_bf3_select(int kh, int stride, int cin, int ntot, int planes, long long pixels, ConvTile* out,
                     bool in_bf16 = false, bool mask_bf16 = false);
hipError_t conv_bf3_launch(const ConvTile& t, const ConvArgs& a, hipStream_t st);
hipError_t conv_bf3_prepare(const ConvTile& t);
// whether conv_bf3_launch can also write the 2x2 max-pooled output (ConvArgs.pool) for these arguments: the VGG16
// epilogue (wave-private image of whole pixel rows, 16-pixel-wide tiles, even row/column origins)
bool conv_bf3_fuses_pool(const ConvTile& t, const ConvArgs& a);
// VGG16 block1_conv1 (3 -> 64, preprocess fused) on bf16 operands: the plain-bf16 loss (conv_bf3.hip)
std::vector<unsigned short> vgg_conv0_bf16_pack(const float* wflip);
// out_bf16: the output is stored as bf16 bits (the plain-bf16 VGG16's layer outputs)
hipError_t vgg_conv0_bf16_launch(const float* img, const float2* pre, const unsigned short* wpk, const float* bias,
                                 float* out, int batch, int H, int W, hipStream_t st, bool out_bf16 = false);

// Residual-block conv (3x3 s1 SAME, 128 output channels) as fused Winograd F(2x2,3x3) on f32 MFMA
// (wino.hip). Epilogue: bias + ReLU + store + per-(workgroup, channel) {sum, M2, n}, n_part =
// tiles_y * tiles_x per image.
struct WinoArgs {
    const float* in;        // NHWC [B][H][W][cin] raw producer output
    const float* res;       // residual source (PRO_AFF_RES)
    float* mat;             // materialise the transformed input here (or null)
    const float2* pro_ab;   // [B][cin] prologue affine
    const float* U;         // transformed weights [cin/8][16][128][8]
    const float* bias;      // [128]
    float* out;             // NHWC [B][H][W][128]
    float4* part;           // [B][128][tiles_y*tiles_x] or null
    int batch, H, W, cin, tiles_y, tiles_x, pro_mode;
    int linear;             // 0: out = ReLU(conv + bias) (the residual convs); 1: conv + bias (input gradient)
    const float2* pro_ab1;  // two styles (wino_x6 only): [B][cin] the second style's affine, or null
    const float* pro_w;     // with pro_ab1: [B][H][W] per-pixel weight of the second style (style_blend)
    CinAcc stat;            // wino_x6 inference: CIN statistics into f64 accumulators instead of part
    CinSrc pro_stat;        // wino_x6 inference: the prologue affine formed from the producer's accumulators
    const void* u_next;     // wino_x6: the next layer's weight image, read into each XCD's L2 during the
    int u_next_bytes;       // epilogue (l2_touch_xcd_slice: its first loads then hit L2), or null
    int wt_stores;          // wino_x6: bit0 output, bit1 materialised input stored write-through (sc1): no dirty
                            // lines left in L2 for the end-of-kernel write-back
    unsigned long long* tl; // wino_x6: in-graph timeline stamps (tl_stamp_end) or null
};
bool wino_supported(int kh, int stride, int cin, int cout);

// First layer (Conv2D 9x9 s1 SAME, cin <= 17 -> 32, ReLU -> BN(inference) -> ReLU) as composite
// Winograd F(2x2,3x3) over nine 3x3 sub-kernels (wino9.hip).
struct Wino9Args {
    const float* in;        // NHWC [B][H][W][cin] network input
    const float* U;         // transformed weights [9][16][2][32][12]
    const float* bias;      // [32]
    const float2* bn_ab;    // [32] BatchNorm affine (folded moving statistics); inference only
    float* out;             // NHWC [B][H][W][32]
    float4* part;           // training: out = ReLU(conv + bias) and per-tile {sum, M2, n} at
                            // [B][32][n_part] for the batch-statistics BatchNorm; null: inference.
                            // n_part = tiles_y*tiles_x (wino9.hip), 2*tiles_y*tiles_x (wino9_x6.hip:
                            // one entry per 16 x 8 M block)
    int batch, H, W, cin, tiles_y, tiles_x;
    cin_word* zero;         // wino9_x6 inference: zero [zero_n2] 16-B words first (the frame's CIN accumulators,
    long zero_n2;           // kernels.h CinAcc, written by later layers only) or null
    const void* w_next;     // wino9_x6 inference: the next layer's weight image into L2 (l2_touch_xcd_slice)
    int w_next_bytes;
    int wt_stores;          // nonzero: output stored write-through (sc1), as WinoArgs::wt_stores
    unsigned* queue;        // inference: [2] work-queue counters (zero at the first launch, reset by the last workgroup
                            // of each launch), or null: the static unit order
};
bool wino9_supported(int kh, int stride, int cin, int cout);

// G-buffer ingest (ingest.hip): channel planes -> TF bilinear (half-pixel) resize -> center crop/pad
constexpr int GBUFFER_MAX_PLANES = 32;
struct GbufferArgs {
    const float* planes[GBUFFER_MAX_PLANES];   // plane k: element (y, x) at planes[k][y*row_stride + x*pixel_stride]
    int num_planes, src_h, src_w;
    long row_stride, pixel_stride;
    float* dst;                                 // NHWC [dst_h][dst_w][num_planes]
    int dst_h, dst_w;
    int new_h, new_w;                           // resized size (before the crop)
    int off_y, off_x;                           // resized coordinate of dst (0, 0): crop offset - pad offset
    float scale_y, scale_x;                     // float(src) / new
};
hipError_t gbuffer_resize_crop_launch(const GbufferArgs& a, hipStream_t st);
int wino9_tiles_y(int H);
int wino9_tiles_x(int W);
std::vector<float> wino9_pack_weights(const float* kern, int cin);
// wino9_pack_weights on the device (kern: HWIO [9][9][cin][32] on the device; U zero-initialised)
hipError_t wino9_transform_launch(const float* kern, int cin, float* U, hipStream_t st);
hipError_t wino9_launch(const Wino9Args& a, hipStream_t st);
// The same layer with the transform-domain products as exact 3-piece split-bf16 MFMA terms (wino9_x6.hip);
// U = wino9_x6_pack_weights (bf16 pieces [10][16][3][32][16]).
std::vector<float> wino9_x6_pack_weights(const float* kern, int cin);
hipError_t wino9_x6_prepare();
// device form of wino9_x6_pack_weights (bitwise the host image; training re-packs after every step)
hipError_t wino9_x6_transform_launch(const float* kern, int cin, float* U, hipStream_t st);
size_t wino9_x6_weight_floats();
int wino9_x6_tiles_y(int H);   // 16 x 16-pixel workgroup blocks
int wino9_x6_tiles_x(int W);
hipError_t wino9_x6_launch(const Wino9Args& a, hipStream_t st);
// The same layer for inference as nine 3x3 sub-kernels on Winograd F(3x3, 3x3) tiles sharing one input-transform grid
// (wino9f3.hip; 24 x 24-pixel blocks, exact split-bf16 x6 products); U = wino9f3_pack_weights.
std::vector<float> wino9f3_pack_weights(const float* kern, int cin);
hipError_t wino9f3_prepare();
int wino9f3_tiles_y(int H);
int wino9f3_tiles_x(int W);
hipError_t wino9f3_launch(const Wino9Args& a, hipStream_t st);
int wino_tiles_y(int H);
int wino_tiles_x(int W);
std::vector<float> wino_pack_weights(const float* kern, int cin);
hipError_t wino_prepare();
// wino_pack_weights on the device (kern: HWIO [3][3][cin][128] float32 on the device)
hipError_t wino_transform_launch(const float* kern, int cin, float* U, hipStream_t st);
hipError_t wino_launch(const WinoArgs& a, hipStream_t st);
// Residual convs as Winograd F(2x2,3x3) with the transform-domain products as exact 3-piece split-bf16
// MFMA terms (wino_x6.hip); same WinoArgs, U = wino_x6_pack_weights (bf16 pieces [cin/16][16][3][128][16]).
bool wino_x6_supported(int kh, int stride, int cin, int cout);
std::vector<float> wino_x6_pack_weights(const float* kern, int cin);
// wino_x6_pack_weights on the device (kern: HWIO [3][3][cin][128] on the device; bitwise the host image)
hipError_t wino_x6_transform_launch(const float* kern, int cin, float* U, hipStream_t st);
// Several layers' x6 transforms in one launch (training re-pack after every optimizer step): job k maps
// kern[k] (HWIO, cin[k] -> 128) to U[k]; at most X6_MAX_JOBS jobs per call.
constexpr int X6_MAX_JOBS = 24;
struct X6TransformJobs {
    const float* kern[X6_MAX_JOBS];
    float* U[X6_MAX_JOBS];
    int cin[X6_MAX_JOBS];
    int n;
};
hipError_t wino_x6_transform_batch_launch(const X6TransformJobs& jobs, hipStream_t st);
hipError_t wino_x6_prepare();
hipError_t wino_x6_launch(const WinoArgs& a, hipStream_t st);
// kernel-execution timestamps (hipExtLaunchKernel events) for the next wino_x6_launch on this thread
void wino_x6_set_timing_events(hipEvent_t start, hipEvent_t stop);

// Final 9x9 transposed conv with Cout = 3 on the VALU (conv_small.hip).
struct SmallConvArgs {
    const float* in;        // [B][H][W][cin]
    const float2* pro_ab;   // [B][cin] prologue affine + ReLU (or null: identity)
    const float* w;         // packed [ky][ci][28] ([kx][3] + 1 pad)
    const float* bias;      // [3]
    float* out;             // [B][H][W][3] raw conv output
    float4* part;           // [B][3][n_tiles]
    int batch, H, W, cin;
    int tiles_y, tiles_x;
};
hipError_t small_conv_launch(const SmallConvArgs& a, hipStream_t st);
int small_conv_tiles_y(int H);
int small_conv_tiles_x(int W);
int small_conv_weight_stride();

// Narrow-channel 3x3 stride-2 convs (contract_0/1) and 3x3 s2 transposed convs (expand_0/1) on f32
// MFMA with no idle columns and no zero-tap products (conv_lite.hip). Reuses ConvArgs: Ho/Wo are the
// GEMM grid (conv: output dims; transposed: input dims), cout the stored channels, pro_mode/part as
// for conv_mfma; the transposed form writes one {sum, M2, n} per (tile, channel), phases merged.
struct LiteTile {
    int id, mode, cin, nc, ckc, th, tw, lds_bytes;
    int x6;                 // 1: split-bf16 x6 operands on the bf16 MFMA pipe (fp32-level products)
};
bool conv_lite_select(int keras_kind, int k, int stride, int cin, int cout, bool x6, LiteTile* t);
constexpr int LITE_MAX_BATCH = 16;   // the prologue affine table [batch][cin] lives in LDS
std::vector<float> conv_lite_pack_weights(const LiteTile& t, const float* kern);
hipError_t conv_lite_launch(const LiteTile& t, const ConvArgs& a, hipStream_t st);
hipError_t conv_lite_prepare(const LiteTile& t);

// Final 9x9 Conv2DTranspose (16 -> 3) on the bf16 MFMA pipe with exact split-bf16 products (conv_last.hip)
struct LastArgs {
    const float* in;        // [B][H][W][16] raw expand output
    const float2* pro_ab;   // [B][16] CIN affine of the input (+ ReLU), or null (input already applied)
    const float* w;         // last_x6_pack_weights image
    const float* bias;      // [3]
    float* out;             // [B][H][W][3] raw conv output
    float4* part;           // [B][3][tiles_y * tiles_x] {sum, M2, n}
    int batch, H, W, cin, tiles_y, tiles_x;
    const float2* pro_ab1;  // two styles: [B][16] the second style's affine, or null
    const float* pro_w;     // with pro_ab1: [B][H][W] per-pixel weight of the second style (style_blend)
    CinAcc stat;            // inference: the output CIN's statistics into f64 accumulators instead of part
    CinSrc pro_stat;        // inference: the prologue affine formed from the producer's accumulators
};
std::vector<float> last_x6_pack_weights(const float* kern, int cin);
int last_x6_tiles_y(int H);
int last_x6_tiles_x(int W);
hipError_t last_x6_prepare();
hipError_t last_x6_launch(const LastArgs& a, hipStream_t st);

// CIN statistics finalize: merge per-tile {sum, M2, n} (Chan, f64) -> per-(b,c) affine.
struct FinalizeArgs {
    const float4* part;      // [B][ntot][n_part]
    const float* style;      // style params base (B, S, P) or null (then scale=1, bias=0)
    const float* scale;      // alternative explicit scale [B][C] (or null)
    const float* bias;       // alternative explicit bias [B][C] (or null)
    float2* ab;              // out [B][C]
    float2* ab1;             // optional out [B][C]: the second style's affine (num_styles == 2)
    int style1_offset;       // offset of the second style's parameter vector (P)
    float2* mr;              // optional out [B][C] (mean, rstd) for the backward pass
    int affine_bstride;      // image stride of scale/bias (C per image; 0 = per-channel, BatchNorm)
    int merge_images;        // BatchNorm (training): statistics over the whole batch
    float* moving_mean;      // optional BatchNorm moving statistics update (Keras momentum)
    float* moving_var;
    float momentum;
    int batch, C, ntot, n_part, phases;
    int style_stride;        // S*P
    int style_offset;        // offset of scale in the style vector; bias at +C
    float eps;
};
hipError_t finalize_launch(const FinalizeArgs& a, hipStream_t st);
// The network output: the last layer's CIN affine (3 channels, num_styles = 1; from its f64 accumulators) fused
// with the affine + sigmoid over the (B, hw, 3) raw output; also stores s.ab_out
hipError_t fin_sigmoid3_launch(const CinSrc& s, const float* x, float* y, long hw, int batch, hipStream_t st);

// y = act(a*x + b [+ res]) element-wise, act: 0 none, 1 relu, 2 sigmoid.  x,res,y [B][HW][C]
hipError_t affine_act_launch(const float* x, const float2* ab, const float* res, float* y, int batch, long hw, int C,
                             int act, hipStream_t st);
// two-style blend: t = a0*x + b0 + w[pixel] * ((a1*x + b1) - (a0*x + b0)), then [+ res], act
hipError_t style_param_map_launch(const float* w1, const float* params, float* out, int batch, long hw, int n,
                                  hipStream_t st);
hipError_t affine_act_blend_launch(const float* x, const float2* ab, const float2* ab1, const float* w,
                                   const float* res, float* y, int batch, long hw, int C, int act, hipStream_t st);
// TF AvgPool2D(2) (valid) of a one-channel map [B][H][W] -> [B][H/2][W/2]
hipError_t avgpool2_1ch_launch(const float* x, float* y, int batch, int H, int W, hipStream_t st);

// Per-tile statistics of an NHWC tensor (standalone instance norm).
hipError_t tile_stats_launch(const float* x, float4* part, int batch, long hw, int C, int tile, hipStream_t st);

// Gram matrices (gram.hip)
size_t gram_workspace_bytes(int batch, int hw, int channels);
// bf16: features rounded to bf16, bf16 MFMA (RST_PRECISION_BF16 loss; the mixed_bfloat16 einsum)
// feat_bf16: the features are stored as bf16 bits (the plain-bf16 VGG16's layer outputs; implies bf16)
hipError_t gram_launch(const float* feat, int batch, int hw, int channels, float* out, void* ws, hipStream_t st,
                       bool bf16 = false, bool feat_bf16 = false);

// Loss kernels (loss.hip)
hipError_t maxpool2_launch(const float* x, float* y, int B, int H, int W, int C, hipStream_t st);
int loss_partial_blocks(long n);
// in_bf16: a and c hold bf16 bits (the plain-bf16 VGG16's block5_conv3 features)
hipError_t sqdiff_loss_launch(const float* a, const float* c, int B, long n, float* partial, double scale, float* out,
                              int out_stride, int out_col, int accumulate, hipStream_t st, bool in_bf16 = false);
// bf16 bits -> f32 (rst_loss_copy_feature of the plain-bf16 VGG16's stored layer outputs)
hipError_t bf16_to_f32_launch(const void* x, float* y, size_t n, hipStream_t st);
hipError_t tv_loss_launch(const float* x, int B, int H, int W, int C, float* partial, double scale, float* out,
                          int out_stride, int out_col, hipStream_t st);
hipError_t loss_combine_launch(float* table, int B, hipStream_t st);

}  // namespace rst
