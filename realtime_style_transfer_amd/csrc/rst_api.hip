// rst_api.hip — host side of the librst C ABI (include/rst.h).
//
// rst_create restates create_style_transfer_model's block derivation
// (realtime_style_transfer/models/styleTransfer.py:213-332), uploads the Keras-ordered weights
// into the device layouts the kernels stage from, and allocates every activation / statistics
// buffer once (sized for max_batch; HBM is plentiful — 288 GB — so every layer keeps its own
// output buffer and nothing is allocated or freed in the hot path).
//
// rst_forward launches, in order, one kernel per conv (+ one CIN-finalize per normalised conv)
// on the caller's stream. Fusion across the layer boundary:
//   contract:  conv + bias + ReLU + BN + ReLU in one epilogue                 (:194-203)
//   residual:  conv + ReLU + tile stats;  CIN-apply (+ReLU | +skip Add) is done by the NEXT
//              conv while it stages its input halo, which also materialises the block output
//              needed by the next skip connection                              (:144-185)
//   expand:    2x2 phase conv (pixel-shuffle store) + tile stats; CIN-apply + ReLU in the
//              next conv's prologue                                            (:95-141)
//   last:      VALU 9x9 conv (CIN-apply+ReLU prologue) + stats -> finalize -> sigmoid(CIN) (:269-276)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "kernels.h"
#include "net.h"

using namespace rst;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail(RST_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

}  // namespace

namespace rst {
size_t layer_weight_count(const LayerSpec& s) {
    size_t n = (size_t)s.k * s.k * s.cin * s.cout + s.cout;
    if (s.norm == N_BN) n += 4 * (size_t)s.cout;
    return n;
}

int build_plan(const rst_shape* sh, std::vector<LayerSpec>& L, int* P) {
    if (sh->in_h <= 0 || sh->in_w <= 0 || sh->in_c <= 0 || sh->out_h <= 0 || sh->out_w <= 0 ||
        sh->bottleneck_res_y <= 0 || sh->bottleneck_num_filters <= 0 || sh->num_styles <= 0)
        return fail(RST_ERR_INVALID, "rst_shape: all dimensions must be positive");
    const int n_c = (int)std::ceil(std::log2((double)sh->in_h) - std::log2((double)sh->bottleneck_res_y));
    if (n_c < 0 || n_c > 4) return fail(RST_ERR_UNSUPPORTED, "number of contract blocks must be in [0, 4]");
    int H = sh->in_h, W = sh->in_w, cin = sh->in_c;
    L.clear();
    L.push_back({"contract_start", 0, 9, 1, cin, 32, H, W, H, W, N_BN, P_RELU, true, -1, -1, -1});
    cin = 32;
    for (int i = 0; i < n_c; ++i) {
        const int f = CONTRACT_FILTERS[i];
        const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
        L.push_back({"contract_" + std::to_string(i), 0, 3, 2, cin, f, H, W, Ho, Wo, N_BN, P_RELU, true, -1, -1, -1});
        H = Ho; W = Wo; cin = f;
    }
    const int F = sh->bottleneck_num_filters;
    int off = 0;
    for (int r = 0; r < 5; ++r)
        for (int j = 0; j < 2; ++j) {
            L.push_back({"residual_block_" + std::to_string(r) + "_conv" + std::to_string(j), 0, 3, 1, cin, F, H, W, H,
                         W, N_CIN, j == 0 ? P_RELU : P_NONE, true, off, r, j});
            off += 2 * F;
            cin = F;
        }
    const int n_e = (int)std::ceil(std::log2((double)sh->out_h) - std::log2((double)H));
    if (n_e < 0 || n_e > 8) return fail(RST_ERR_UNSUPPORTED, "number of expand blocks must be in [0, 8]");
    for (int i = 0; i < n_e; ++i) {
        const int f = EXPAND_FILTERS[i];
        L.push_back({"expand_" + std::to_string(i), 1, 3, 2, cin, f, H, W, 2 * H, 2 * W, N_CIN, P_RELU, false, off,
                     -1, -1});
        off += 2 * f;
        H *= 2; W *= 2; cin = f;
    }
    L.push_back({"expand_last", 1, 9, 1, cin, 3, H, W, H, W, N_CIN, P_SIGMOID, false, off, -1, -1});
    off += 6;
    if (H != sh->out_h || W != sh->out_w)
        return fail(RST_ERR_INVALID, "plan output " + std::to_string(H) + "x" + std::to_string(W) +
                                         " does not match out_h x out_w");
    *P = off;
    return RST_OK;
}

std::vector<float> pack_tiles(const std::vector<float>& Wg, int taps, int cin, int ntot, const ConvTile& t) {
    return pack_conv_tiles(Wg, taps, cin, ntot, t);
}

int set_error(int code, const std::string& msg) { return fail(code, msg); }

namespace {
struct GuardRec {
    char* base;
    size_t bytes;
};
std::vector<GuardRec> g_guards;   // live guarded allocations (diagnostic runs only)
const unsigned char GUARD_BYTE = 0xA5;
}  // namespace

size_t guard_pad() {
    static const size_t pad = [] {
        const char* v = getenv("RST_ALLOC_PAD");
        return v != nullptr ? (size_t)(strtoull(v, nullptr, 0) + 255) / 256 * 256 : (size_t)0;
    }();
    return pad;
}

hipError_t guard_malloc(void** p, size_t bytes) {
    const size_t pad = guard_pad();
    if (pad == 0) return hipMalloc(p, bytes);
    char* base = nullptr;
    hipError_t e = hipMalloc((void**)&base, bytes + 2 * pad);
    if (e != hipSuccess) return e;
    if ((e = hipMemset(base, GUARD_BYTE, pad)) != hipSuccess ||
        (e = hipMemset(base + pad + bytes, GUARD_BYTE, pad)) != hipSuccess) {
        (void)hipFree(base);
        return e;
    }
    g_guards.push_back({base, bytes});
    *p = base + pad;
    return hipSuccess;
}

void guard_free(void* p) {
    const size_t pad = guard_pad();
    if (pad == 0) {
        (void)hipFree(p);
        return;
    }
    for (size_t i = 0; i < g_guards.size(); ++i)
        if (g_guards[i].base + pad == p) {
            (void)hipFree(g_guards[i].base);
            g_guards.erase(g_guards.begin() + i);
            return;
        }
    (void)hipFree(p);
}

int guard_check(const char* when) {
    const size_t pad = guard_pad();
    if (pad == 0) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    int bad = 0;
    std::vector<unsigned char> h(pad);
    for (size_t i = 0; i < g_guards.size(); ++i)
        for (int side = 0; side < 2; ++side) {
            const char* band = g_guards[i].base + (side ? pad + g_guards[i].bytes : 0);
            if (hipMemcpy(h.data(), band, pad, hipMemcpyDeviceToHost) != hipSuccess) return -1;
            size_t first = pad, last = 0, n = 0;
            for (size_t k = 0; k < pad; ++k)
                if (h[k] != GUARD_BYTE) {
                    first = std::min(first, k);
                    last = k;
                    ++n;
                }
            if (n == 0) continue;
            ++bad;
            fprintf(stderr, "RST_ALLOC_PAD %s: allocation %zu (%zu bytes at %p): %zu bytes written in the %s band, "
                            "offsets %lld .. %lld from the buffer start\n",
                    when, i, g_guards[i].bytes, (void*)(g_guards[i].base + pad), n, side ? "trailing" : "leading",
                    side ? (long long)(g_guards[i].bytes + first) : -(long long)(pad - first),
                    side ? (long long)(g_guards[i].bytes + last) : -(long long)(pad - last));
            (void)hipMemset((void*)band, GUARD_BYTE, pad);   // re-armed: the next check reports new writes only
        }
    return bad;
}

std::vector<float> pack_conv_tiles(const std::vector<float>& Wg, int taps, int cin, int ntot, const ConvTile& t) {
    const int ck = t.ck, nt = t.nt, tps = t.tps, vec = t.vec;
    const int ksteps = ck / 2, sg_n = ksteps / vec;
    const int nchunks = (cin + ck - 1) / ck, nblocks = (ntot + nt - 1) / nt, ngroups = taps / tps;
    std::vector<float> out((size_t)nblocks * nchunks * ngroups * t.wstage, 0.f);
    size_t idx = 0;
    for (int nb = 0; nb < nblocks; ++nb)
        for (int c = 0; c < nchunks; ++c)
            for (int g = 0; g < ngroups; ++g)
                for (int tt = 0; tt < tps; ++tt)
                    for (int sg = 0; sg < sg_n; ++sg)
                        for (int h = 0; h < 2; ++h)
                            for (int n = 0; n < nt; ++n)
                                for (int v = 0; v < vec; ++v) {
                                    const int tap = g * tps + tt;
                                    const int ci = c * ck + h * ksteps + sg * vec + v;
                                    const int ng = nb * nt + n;
                                    float val = 0.f;
                                    if (ci < cin && ng < ntot) val = Wg[((size_t)tap * cin + ci) * ntot + ng];
                                    out[idx++] = val;
                                }
    return out;
}
static unsigned short host_bf16_rne(float x) {
    unsigned u;
    std::memcpy(&u, &x, 4);
    return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

std::vector<float> pack_conv_tiles_bf3(const std::vector<float>& Wg, int taps, int cin, int ntot, const ConvTile& t) {
    const int ck = t.ck, nt = t.nt, tps = t.tps, ks_n = ck / 16, np_ = t.bf3;
    const int nchunks = (cin + ck - 1) / ck, nblocks = (ntot + nt - 1) / nt, ngroups = taps / tps;
    std::vector<unsigned short> out((size_t)nblocks * nchunks * ngroups * t.wstage, 0);
    auto val = [](unsigned short h) {
        unsigned u = (unsigned)h << 16;
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    };
    size_t idx = 0;
    for (int nb = 0; nb < nblocks; ++nb)
        for (int c = 0; c < nchunks; ++c)
            for (int g = 0; g < ngroups; ++g)
                for (int tt = 0; tt < tps; ++tt)
                    for (int ks = 0; ks < ks_n; ++ks)
                        for (int pl = 0; pl < np_; ++pl)
                            for (int h = 0; h < 2; ++h)
                                for (int n = 0; n < nt; ++n)
                                    for (int j = 0; j < 8; ++j) {
                                        const int tap = g * tps + tt;
                                        const int ci = c * ck + ks * 16 + h * 8 + j;
                                        const int ng = nb * nt + n;
                                        float v = 0.f;
                                        if (ci < cin && ng < ntot) v = Wg[((size_t)tap * cin + ci) * ntot + ng];
                                        unsigned short p[3];
                                        p[0] = host_bf16_rne(v);
                                        const float r = v - val(p[0]);
                                        p[1] = host_bf16_rne(r);
                                        p[2] = host_bf16_rne(r - val(p[1]));
                                        out[idx++] = p[pl];
                                    }
    std::vector<float> packed((out.size() + 1) / 2, 0.f);
    std::memcpy(packed.data(), out.data(), out.size() * 2);
    return packed;
}

// The bf16-element positions of pack_conv_tiles_bf3's one-plane image: the index of each element's source
// in Wg ([tap][cin][ntot]), -1 for padding (a gather map for weights re-packed on the device every step)
std::vector<int> pack_conv_tiles_bf3_index(int taps, int cin, int ntot, const ConvTile& t) {
    const int ck = t.ck, nt = t.nt, tps = t.tps, ks_n = ck / 16;
    const int nchunks = (cin + ck - 1) / ck, nblocks = (ntot + nt - 1) / nt, ngroups = taps / tps;
    std::vector<int> out((size_t)nblocks * nchunks * ngroups * t.wstage, -1);
    size_t idx = 0;
    for (int nb = 0; nb < nblocks; ++nb)
        for (int c = 0; c < nchunks; ++c)
            for (int g = 0; g < ngroups; ++g)
                for (int tt = 0; tt < tps; ++tt)
                    for (int ks = 0; ks < ks_n; ++ks)
                        for (int h = 0; h < 2; ++h)
                            for (int n = 0; n < nt; ++n)
                                for (int j = 0; j < 8; ++j) {
                                    const int tap = g * tps + tt;
                                    const int ci = c * ck + ks * 16 + h * 8 + j;
                                    const int ng = nb * nt + n;
                                    out[idx++] = (ci < cin && ng < ntot) ? (int)(((size_t)tap * cin + ci) * ntot + ng) : -1;
                                }
    return out;
}
}  // namespace rst

namespace rst {
// Geometry, kernel choice and device weight image of one layer (no device work). `kern`/`bias`
// point at the layer's Keras weights; passing an array of (index + 1) values instead yields the
// gather map from canonical weights to the packed image (training re-packs after each update).
int prepare_layer(LayerExec& e, const LayerSpec& s, const float* kern, const float* bias, std::vector<float>& packed,
                  std::vector<float>& bias_n, int precision, bool allow_lite, bool inference) {
    const size_t kcount = (size_t)s.k * s.k * s.cin * s.cout;
    (void)kcount;
    if (s.keras_kind == 1 && s.k == 9 && s.stride == 1) {
        // ---- final 9x9 transposed conv: flip -> correlation, pack [ky][ci][kx][co]
        if (s.cout != 3) return fail(RST_ERR_UNSUPPORTED, "last layer must have 3 channels");
        if (allow_lite && precision == RST_PRECISION_WINOGRAD_BF16X6 && s.cin == 16) {
            // bf16 MFMA with exact split products (conv_last.hip)
            e.kind = K_LASTX6;
            packed = last_x6_pack_weights(kern, s.cin);
            bias_n.assign(bias, bias + 3);
            e.ntot = 3;
            e.tiles_y = last_x6_tiles_y(s.Ho);
            e.tiles_x = last_x6_tiles_x(s.Wo);
            e.n_part = e.tiles_y * e.tiles_x;
            return RST_OK;
        }
        e.kind = K_SMALL;
        const int ws = small_conv_weight_stride();
        std::vector<float> w((size_t)9 * s.cin * ws, 0.f);
        for (int ky = 0; ky < 9; ++ky)
            for (int kx = 0; kx < 9; ++kx)
                for (int ci = 0; ci < s.cin; ++ci)
                    for (int co = 0; co < 3; ++co)
                        w[((size_t)ky * s.cin + ci) * ws + kx * 3 + co] =
                            kern[(((size_t)(8 - ky) * 9 + (8 - kx)) * 3 + co) * s.cin + ci];
        packed.swap(w);
        bias_n.assign(bias, bias + 3);
        e.ntot = 3;
        e.tiles_y = small_conv_tiles_y(s.Ho);
        e.tiles_x = small_conv_tiles_x(s.Wo);
        e.n_part = e.tiles_y * e.tiles_x;
    } else if ((precision == RST_PRECISION_FP32_WINOGRAD || precision == RST_PRECISION_WINOGRAD_BF16X6) &&
               s.keras_kind == 0 && wino9_supported(s.k, s.stride, s.cin, s.cout) && s.norm == N_BN && s.conv_relu) {
        // ---- first layer (9x9 conv + ReLU + BN + ReLU) as composite Winograd: f32 MFMA (wino9.hip) or
        // exact split-bf16 MFMA products (wino9_x6.hip)
        const bool x6 = precision == RST_PRECISION_WINOGRAD_BF16X6;
        // inference: the F(3x3, 3x3) form (wino9f3.hip; RST_START_F3=0 keeps wino9_x6 for A/B runs)
        static const bool f3_on = [] { const char* v = getenv("RST_START_F3"); return !(v != nullptr && v[0] == '0'); }();
        const bool f3 = x6 && inference && f3_on;
        e.kind = f3 ? K_WINO9F3 : x6 ? K_WINO9X6 : K_WINO9;
        packed = f3 ? wino9f3_pack_weights(kern, s.cin) : x6 ? wino9_x6_pack_weights(kern, s.cin) : wino9_pack_weights(kern, s.cin);
        bias_n.assign(bias, bias + s.cout);
        e.ntot = s.cout;
        e.pad_t = e.pad_l = 4;
        e.gHo = s.Ho;
        e.gWo = s.Wo;
        e.tiles_y = f3 ? wino9f3_tiles_y(s.Ho) : x6 ? wino9_x6_tiles_y(s.Ho) : wino9_tiles_y(s.Ho);
        e.tiles_x = f3 ? wino9f3_tiles_x(s.Wo) : x6 ? wino9_x6_tiles_x(s.Wo) : wino9_tiles_x(s.Wo);
        e.n_part = 0;
    } else if ((precision == RST_PRECISION_FP32_WINOGRAD && wino_supported(s.k, s.stride, s.cin, s.cout) ||
                precision == RST_PRECISION_WINOGRAD_BF16X6 && wino_x6_supported(s.k, s.stride, s.cin, s.cout)) &&
               s.keras_kind == 0 && s.res_block >= 0) {
        // ---- residual conv as fused Winograd F(2x2,3x3): f32 MFMA (wino.hip) or exact split-bf16 MFMA
        // products (wino_x6.hip)
        const bool x6 = precision == RST_PRECISION_WINOGRAD_BF16X6;
        e.kind = x6 ? K_WINOX6 : K_WINO;
        packed = x6 ? wino_x6_pack_weights(kern, s.cin) : wino_pack_weights(kern, s.cin);
        bias_n.assign(bias, bias + s.cout);
        e.ntot = s.cout;
        e.pad_t = e.pad_l = 1;
        e.gHo = s.Ho;
        e.gWo = s.Wo;
        e.tiles_y = wino_tiles_y(s.Ho);
        e.tiles_x = wino_tiles_x(s.Wo);
        e.n_part = e.tiles_y * e.tiles_x;
    } else if (allow_lite && conv_lite_select(s.keras_kind, s.k, s.stride, s.cin, s.cout,
                                              precision == RST_PRECISION_WINOGRAD_BF16X6, &e.lite) &&
               (s.keras_kind == 0 ? (s.norm == N_BN && s.conv_relu) : (s.norm == N_CIN && !s.conv_relu))) {
        // ---- narrow 3x3 s2 conv / transposed conv: exact f32 MFMA, no idle columns, no zero taps
        e.kind = K_LITE;
        packed = conv_lite_pack_weights(e.lite, kern);
        bias_n.assign(bias, bias + s.cout);
        e.ntot = s.cout;
        if (s.keras_kind == 0) {
            const int pt = std::max((s.Ho - 1) * 2 + 3 - s.H, 0), pl = std::max((s.Wo - 1) * 2 + 3 - s.W, 0);
            e.pad_t = pt / 2;
            e.pad_l = pl / 2;
            e.gHo = s.Ho;
            e.gWo = s.Wo;
        } else {
            e.gHo = s.H;
            e.gWo = s.W;
        }
        e.tiles_y = (e.gHo + e.lite.th - 1) / e.lite.th;
        e.tiles_x = (e.gWo + e.lite.tw - 1) / e.lite.tw;
        e.n_part = e.tiles_y * e.tiles_x;
    } else {
        int taps, ntot, kh;
        std::vector<float> Wg;
        if (s.keras_kind == 0) {
            kh = s.k;
            taps = s.k * s.k;
            ntot = s.cout;
            Wg.assign(kern, kern + kcount);   // HWIO already == [tap][ci][co]
            e.kind = K_CONV;
            const int pt = std::max((s.Ho - 1) * s.stride + s.k - s.H, 0);
            const int pl = std::max((s.Wo - 1) * s.stride + s.k - s.W, 0);
            e.pad_t = pt / 2;
            e.pad_l = pl / 2;
            e.gHo = s.Ho;
            e.gWo = s.Wo;
            bias_n.assign(bias, bias + s.cout);
        } else {
            if (!(s.k == 3 && s.stride == 2))
                return fail(RST_ERR_UNSUPPORTED, "Conv2DTranspose other than 3x3/s2 and 9x9/s1");
            // 3x3 s2 SAME transposed conv == 2x2 conv (pad 1) with 4 output phases:
            // out[2p+py][2q+px][co] = sum_{ty,tx} in[p+ty-1][q+tx-1] . w[py+2(1-ty)][px+2(1-tx)][co]
            kh = 2;
            taps = 4;
            ntot = 4 * s.cout;
            e.kind = K_CONVT2;
            Wg.assign((size_t)4 * s.cin * ntot, 0.f);
            for (int ty = 0; ty < 2; ++ty)
                for (int tx = 0; tx < 2; ++tx)
                    for (int py = 0; py < 2; ++py)
                        for (int px = 0; px < 2; ++px) {
                            const int ky = py + 2 * (1 - ty), kx = px + 2 * (1 - tx);
                            if (ky > 2 || kx > 2) continue;
                            for (int ci = 0; ci < s.cin; ++ci)
                                for (int co = 0; co < s.cout; ++co)
                                    Wg[((size_t)(ty * 2 + tx) * s.cin + ci) * ntot + (py * 2 + px) * s.cout + co] =
                                        kern[(((size_t)ky * 3 + kx) * s.cout + co) * s.cin + ci];
                        }
            e.pad_t = e.pad_l = 1;
            e.gHo = s.H;
            e.gWo = s.W;
            for (int n = 0; n < ntot; ++n) bias_n.push_back(bias[n % s.cout]);
        }
        const int gs = s.keras_kind == 0 ? s.stride : 1;
        const int planes = bf16_planes(precision);
        const bool bf3 = planes > 0 && conv_bf3_select(kh, gs, s.cin, ntot, planes, (long long)e.gHo * e.gWo, &e.tile);
        if (!bf3 && !conv_select(kh, gs, s.cin, ntot, &e.tile))
            return fail(RST_ERR_UNSUPPORTED, "no conv tile configuration for layer " + s.name);
        e.ntot = ntot;
        e.tiles_y = (e.gHo + e.tile.th - 1) / e.tile.th;
        e.tiles_x = (e.gWo + e.tile.tw - 1) / e.tile.tw;
        e.n_blocks = (ntot + e.tile.nt - 1) / e.tile.nt;
        e.nchunks = (s.cin + e.tile.ck - 1) / e.tile.ck;
        e.n_part = e.tiles_y * e.tiles_x * e.tile.mt;
        packed = e.tile.bf3 ? pack_conv_tiles_bf3(Wg, taps, s.cin, ntot, e.tile)
                            : pack_tiles(Wg, taps, s.cin, ntot, e.tile);
    }
    return RST_OK;
}
}  // namespace rst

extern "C" {

const char* rst_last_error(void) { return g_last_error.c_str(); }
const char* rst_version(void) { return "rst-mi355x 0.1 (gfx950, f32 MFMA)"; }

size_t rst_num_weights_for_shape(const rst_shape* shape) {
    std::vector<LayerSpec> L;
    int P = 0;
    if (shape == nullptr || build_plan(shape, L, &P) != RST_OK) return 0;
    size_t n = 0;
    for (auto& s : L) n += layer_weight_count(s);
    return n;
}

int rst_num_style_params(const rst_handle* h) { return h ? h->P : -1; }
int rst_num_layers(const rst_handle* h) { return h ? (int)h->layers.size() : -1; }

int rst_create(const rst_shape* shape, const float* weights_host, size_t num_weights, rst_handle** out) {
    return rst_create_ex(shape, weights_host, num_weights, RST_PRECISION_FP32, out);
}

int rst_create_ex(const rst_shape* shape, const float* weights_host, size_t num_weights, int precision,
                  rst_handle** out) {
    if (shape == nullptr || out == nullptr || weights_host == nullptr)
        return fail(RST_ERR_INVALID, "rst_create: null argument");
    if (precision != RST_PRECISION_FP32 && precision != RST_PRECISION_BF16X3 && precision != RST_PRECISION_BF16X6 &&
        precision != RST_PRECISION_FP32_WINOGRAD && precision != RST_PRECISION_BF16 &&
        precision != RST_PRECISION_WINOGRAD_BF16X6)
        return fail(RST_ERR_INVALID, "rst_create_ex: unknown precision mode");
    *out = nullptr;
    if (shape->num_styles > 2)
        return fail(RST_ERR_UNSUPPORTED, "rst_create: num_styles > 2: the reference blends style parameters only for "
                                         "two styles (styleTransfer.py:38-44; for more it returns them unblended, "
                                         "which does not broadcast against the feature map)");
    if (shape->max_batch <= 0) return fail(RST_ERR_INVALID, "rst_create: max_batch must be positive");
    std::vector<LayerSpec> specs;
    int P = 0;
    int st = build_plan(shape, specs, &P);
    if (st != RST_OK) return st;
    size_t expect = 0;
    for (auto& s : specs) expect += layer_weight_count(s);
    if (expect != num_weights)
        return fail(RST_ERR_INVALID, "rst_create: expected " + std::to_string(expect) + " weights, got " +
                                         std::to_string(num_weights));

    rst_handle* h = new rst_handle();
    h->shape = *shape;
    h->P = P;
    h->precision = precision;
    {
        const char* nup = getenv("RST_NO_U_PREFETCH");
        h->no_u_prefetch = nup != nullptr && nup[0] == '1';
        const char* wts = getenv("RST_WT_STORES");
        // default: every output and the residual convs' materialised input (round 4: 15 vs round 3's 13 +0.6 % frames,
        // 7 same-box pairs, profiles/r04/ab_wt_stores.log)
        h->wt_stores = wts != nullptr ? atoi(wts) : 15;
    }
    const int B = shape->max_batch;
    const float* wp = weights_host;
    h->layers.resize(specs.size());
    for (size_t li = 0; li < specs.size(); ++li) {
        LayerExec& e = h->layers[li];
        const LayerSpec& s = specs[li];
        e.s = s;
        const size_t kcount = (size_t)s.k * s.k * s.cin * s.cout;
        const float* kern = wp;
        const float* bias = wp + kcount;
        wp += kcount + s.cout;
        std::vector<float> bias_n, packed;
        // two styles: a layer whose input is a conditional-instance-normalised output blends the two styles' CIN
        // affines per pixel in its prologue. The split-bf16 residual kernel (wino_x6), the narrow-conv kernel
        // (conv_lite), the final 9x9 kernel (last_x6) and the direct kernel have that blend; the f32 Winograd kernel
        // does not (its layers keep the direct kernel)
        const bool blend_in = shape->num_styles == 2 && li > 0 && specs[li - 1].norm == N_CIN;
        const int lp = (blend_in && precision == RST_PRECISION_FP32_WINOGRAD) ? RST_PRECISION_FP32 : precision;
        if ((st = prepare_layer(e, s, kern, bias, packed, bias_n, lp, shape->max_batch <= LITE_MAX_BATCH, true)) != RST_OK) {
            delete h;
            return st;
        }
        if ((st = h->alloc(&e.d_w, packed.size() * 4, packed.data())) != RST_OK) { delete h; return st; }
        e.w_bytes = packed.size() * 4;
        if ((st = h->alloc(&e.d_bias, bias_n.size() * 4, bias_n.data())) != RST_OK) { delete h; return st; }
        if (s.norm == N_BN) {
            const float* gamma = wp;
            const float* beta = wp + s.cout;
            const float* mm = wp + 2 * s.cout;
            const float* mv = wp + 3 * s.cout;
            wp += 4 * s.cout;
            std::vector<float2> ab(s.cout);
            for (int c = 0; c < s.cout; ++c) {
                const double inv = (double)gamma[c] / std::sqrt((double)mv[c] + 1e-3);
                ab[c] = make_float2((float)inv, (float)((double)beta[c] - (double)mm[c] * inv));
            }
            if ((st = h->alloc(&e.d_bn, ab.size() * sizeof(float2), ab.data())) != RST_OK) { delete h; return st; }
        } else {
            if ((st = h->alloc(&e.d_part, (size_t)B * e.ntot * e.n_part * sizeof(float4))) != RST_OK) { delete h; return st; }
            if ((st = h->alloc(&e.d_ab, (size_t)B * s.cout * sizeof(float2))) != RST_OK) { delete h; return st; }
            if (shape->num_styles == 2 &&
                (st = h->alloc(&e.d_ab1, (size_t)B * s.cout * sizeof(float2))) != RST_OK) { delete h; return st; }
        }
        if ((st = h->alloc(&e.d_out, (size_t)B * s.Ho * s.Wo * s.cout * 4)) != RST_OK) { delete h; return st; }
    }

    // ---- wire prologues: how each layer consumes its predecessor (see file header)
    const float* block_input = nullptr;   // materialised input of the current residual block
    for (size_t li = 0; li < h->layers.size(); ++li) {
        LayerExec& e = h->layers[li];
        if (li == 0) { e.pro = PRO_NONE; e.pro_src = -1; continue; }
        LayerExec& p = h->layers[li - 1];
        e.pro_src = (int)li - 1;
        if (p.s.norm == N_BN) {
            e.pro = PRO_NONE;
        } else if (p.s.post == P_RELU) {
            e.pro = PRO_AFF_RELU;
        } else {
            // predecessor is the second conv of residual block r: block output = [x_r +] CIN(h)
            const bool first = p.s.res_block == 0;
            e.pro = first ? PRO_AFF : PRO_AFF_RES;
            e.pro_res = first ? nullptr : block_input;
            p.emit_res = e.pro_res;
            if (e.s.res_block > 0 && e.s.res_conv == 0) {
                // this conv opens residual block r>0: materialise its input for the skip add
                if ((st = h->alloc(&e.d_mat, (size_t)B * e.s.H * e.s.W * e.s.cin * 4)) != RST_OK) { delete h; return st; }
            }
        }
        if (e.s.res_block >= 1 && e.s.res_conv == 0) block_input = e.d_mat;
    }
    // CIN statistics through fixed-point accumulators (kernels.h CinAcc / CinSrc) where the producer adds them and
    // the consumer forms its affine from them: no finalize kernel between the two. The copies keep the
    // adders per address near 16-28: a residual conv has 225 workgroups at B = 1 (8 copies), the persistent
    // transposed convs up to a few per CU (32), the last layer ~900 (64).
    {
        size_t n_acc = 0;
        auto takes_acc = [](int kind) { return kind == K_WINOX6 || kind == K_LITE || kind == K_LASTX6; };
        const LayerExec& last = h->layers.back();
        const bool fused_out = shape->num_styles == 1 && last.kind == K_LASTX6 && last.s.cout == 3 &&
                               last.s.norm == N_CIN && ((long)last.s.Ho * last.s.Wo * 3) % 4 == 0;
        for (size_t li = 0; li < h->layers.size(); ++li) {
            LayerExec& e = h->layers[li];
            if (e.s.norm != N_CIN || !takes_acc(e.kind)) continue;
            const bool consumer_ok = li + 1 < h->layers.size()
                                         ? h->layers[li + 1].pro_src == (int)li && takes_acc(h->layers[li + 1].kind)
                                         : fused_out;
            if (!consumer_ok) continue;
            // accumulator copies (<= 8: the consumers' split affine form, kernels.h CinAffineSplit). The consumers' merge reads
            // scale with the count while the producers' no-return atomics run at one rate for 1 to 32 adders per
            // address (MI355X_MICROARCH.md). Same-box frame A/Bs (profiles/r04/ab_nslot.log): narrow / last layers 8
            // copies +1.4 % over 32; residual convs 4 copies +2.8 % over 8, 2 equal, 1 -3 %.
            // RST_ACC_NSLOT / RST_ACC_NSLOT_X6 override (A/B knobs).
            auto env_slots = [](const char* name, int def) { const char* v = getenv(name); const int n = v ? atoi(v) : 0;
                                                             return n >= 1 && n <= 8 ? n : def; };
            static const int nslot_lite = env_slots("RST_ACC_NSLOT", 8), nslot_x6 = env_slots("RST_ACC_NSLOT_X6", 4);
            e.nslot = e.kind == K_WINOX6 ? nslot_x6 : nslot_lite;
            e.acc_off = (long)n_acc;                   // per image: the layer's block scales with the batch
            n_acc += (size_t)e.nslot * 2 * CIN_LIMBS * e.s.cout;
        }
        if (n_acc > 0) {
            h->acc_per_image = n_acc;
            if ((st = h->alloc(&h->d_acc_all, n_acc * B * sizeof(cin_word))) != RST_OK) { delete h; return st; }
        }
        const unsigned qz[2] = {0u, 0u};
        if ((st = h->alloc(&h->d_w9_queue, sizeof(qz), qz)) != RST_OK) { delete h; return st; }
        const char* wq = getenv("RST_W9_QUEUE");
        h->w9_queue = !(wq != nullptr && wq[0] == '0');
    }
    // two styles: the style-weight mip chain (AvgPool2 keyed by width, num_expand_blocks + 1 levels)
    if (shape->num_styles == 2) {
        int mh = shape->out_h, mw = shape->out_w;
        h->d_mip.push_back(nullptr);   // level 0: the caller's style_weights
        h->mip_h.push_back(mh);
        h->mip_w.push_back(mw);
        int n_e = 0;
        for (auto& s : specs)
            if (s.keras_kind == 1 && s.stride == 2) ++n_e;
        for (int k = 0; k < n_e + 1; ++k) {
            mh /= 2;
            mw /= 2;
            float* m = nullptr;
            if ((st = h->alloc(&m, (size_t)B * std::max(mh, 1) * std::max(mw, 1) * 4)) != RST_OK) { delete h; return st; }
            h->d_mip.push_back(m);
            h->mip_h.push_back(mh);
            h->mip_w.push_back(mw);
        }
        for (auto& e : h->layers) {
            if (e.s.norm != N_CIN) continue;
            for (size_t k = 0; k < h->mip_w.size(); ++k)
                if (h->mip_w[k] == e.s.Wo && h->mip_h[k] == e.s.Ho) e.out_mip = (int)k;
            if (e.out_mip < 0) {
                delete h;
                return fail(RST_ERR_UNSUPPORTED, "no style-weight mip matches layer " + e.s.name + " (" +
                                                     std::to_string(e.s.Ho) + "x" + std::to_string(e.s.Wo) + ")");
            }
        }
        const LayerExec& last = h->layers.back();
        if ((st = h->alloc(&h->d_xlast, (size_t)B * last.s.H * last.s.W * last.s.cin * 4)) != RST_OK) { delete h; return st; }
    }
    // kernels with > 64 KB of dynamic LDS need the attribute before any (graph-captured) launch
    for (auto& e : h->layers) {
        if (e.kind == K_SMALL || e.kind == K_WINO9) continue;
        if (e.kind == K_LASTX6) {
            const hipError_t pe = last_x6_prepare();
            if (pe != hipSuccess) {
                delete h;
                return fail(RST_ERR_HIP, std::string("last_x6_prepare: ") + hipGetErrorString(pe));
            }
            continue;
        }
        hipError_t pe = e.kind == K_WINO      ? wino_prepare()
                        : e.kind == K_WINOX6  ? wino_x6_prepare()
                        : e.kind == K_WINO9X6 ? wino9_x6_prepare()
                        : e.kind == K_WINO9F3 ? wino9f3_prepare()
                        : e.kind == K_LITE    ? conv_lite_prepare(e.lite)
                                              : conv_prepare(e.tile);
        if (pe != hipSuccess) {
            delete h;
            return fail(RST_ERR_HIP, std::string("conv_prepare: ") + hipGetErrorString(pe));
        }
    }
    *out = h;
    return RST_OK;
}

void rst_destroy(rst_handle* h) { delete h; }

static const float* mip_ptr(const rst_handle* h, int level, const float* style_weights) {
    if (level < 0) return nullptr;
    return level == 0 ? style_weights : h->d_mip[level];
}

// num_styles = 1 with last_x6: the last CIN's statistics go to fixed-point accumulators and the output kernel forms the
// affine itself (fin_sigmoid3_launch): no finalize, no separate activation pass
static bool output_finalize_fused(const rst_handle* h) { return h->layers.back().acc_off >= 0; }

// layer e's accumulators for a forward of B images (null: e uses partials + finalize)
static cin_word* acc_ptr(const rst_handle* h, const LayerExec& e, int B) {
    return e.acc_off >= 0 ? h->d_acc_all + (size_t)e.acc_off * B : nullptr;
}

// the consumer-side view of a producer's CIN accumulators (the FinalizeArgs fields of its finalize)
static CinSrc cin_src(const rst_handle* h, const LayerExec& p, const float* style, int B) {
    CinSrc c{};
    c.acc = acc_ptr(h, p, B);
    c.nslot = p.nslot;
    c.C = p.s.cout;
    c.batch = B;
    c.n = (double)p.s.Ho * p.s.Wo;
    c.style = style;
    c.style_stride = h->shape.num_styles * h->P;
    c.style_offset = p.s.style_offset;
    c.style1_offset = h->shape.num_styles == 2 ? h->P : -1;
    c.eps = 1e-5f;
    c.ab_out = p.d_ab;
    c.ab1_out = p.d_ab1;
    return c;
}

// The next layer's packed weights (what l2_touch_xcd_slice reads into L2 during layer li), unless disabled
static void next_weights(const rst_handle* h, size_t li, const void** p, int* bytes) {
    if (h->no_u_prefetch || li + 1 >= h->layers.size()) return;
    const LayerExec& n = h->layers[li + 1];
    if (n.d_w == nullptr || n.w_bytes >= (size_t)0x7FFFFFFF) return;
    *p = n.d_w;
    *bytes = (int)n.w_bytes;
}

// Write-through store bits of layer e (RST_WT_STORES & mask), when its output (and a wino_x6 materialised input of
// the same or fewer bytes) is addressable by the kernels' 32-bit buffer offsets
static int wt_bits(const rst_handle* h, const LayerExec& e, int B, int mask) {
    const size_t bytes = (size_t)B * e.s.Ho * e.s.Wo * (e.s.cout > e.s.cin ? e.s.cout : e.s.cin) * 4;
    return bytes < (size_t)0x7FFFFFF0 ? (h->wt_stores & mask) : 0;
}

static int launch_layer(rst_handle* h, size_t li, const float* content, const float* style, const float* sw, int B,
                        hipStream_t st) {
    LayerExec& e = h->layers[li];
    const bool two = h->shape.num_styles == 2;
    hipEvent_t* ev = nullptr;
    if (h->prof_on && h->prof_step < h->prof_max_steps)
        ev = &h->prof_events[((size_t)h->prof_step * h->layers.size() + li) * 3];
    // the split-bf16 residual conv (the dominant kernel) records its own execution interval into ev[0..1]
    const bool ext_ev = ev != nullptr && e.kind == K_WINOX6;
    if (ev && !ext_ev) HIP_TRY(hipEventRecord(ev[0], st));
    const float* in = (e.pro_src < 0) ? content : h->layers[e.pro_src].d_out;
    const float2* pro_ab = (e.pro_src >= 0 && e.pro != PRO_NONE) ? h->layers[e.pro_src].d_ab : nullptr;
    const bool blend = two && pro_ab != nullptr;
    const LayerExec* src = e.pro_src >= 0 ? &h->layers[e.pro_src] : nullptr;
    if (e.kind == K_LASTX6) {
        LastArgs a{};
        a.in = in;
        a.pro_ab = pro_ab;
        if (blend) {   // two styles: its blend prologue
            a.pro_ab1 = src->d_ab1;
            a.pro_w = mip_ptr(h, src->out_mip, sw);
        }
        if (e.pro != PRO_AFF_RELU && e.pro != PRO_NONE)
            return fail(RST_ERR_UNSUPPORTED, "last layer prologue must be CIN+ReLU");
        a.w = e.d_w;
        a.bias = e.d_bias;
        a.out = e.d_out;
        a.part = e.d_part;
        a.batch = B;
        a.H = e.s.H;
        a.W = e.s.W;
        a.cin = e.s.cin;
        a.tiles_y = e.tiles_y;
        a.tiles_x = e.tiles_x;
        if (e.acc_off >= 0) {   // the output CIN's statistics -> fixed-point accumulators (fin_sigmoid3 reads them)
            a.part = nullptr;
            a.stat.acc = acc_ptr(h, e, B);
            a.stat.nslot = e.nslot;
        }
        if (src != nullptr && src->acc_off >= 0 && pro_ab != nullptr) {
            a.pro_stat = cin_src(h, *src, style, B);
            a.pro_ab = a.pro_ab1 = nullptr;
        }
        HIP_TRY(last_x6_launch(a, st));
    } else if (e.kind == K_SMALL) {
        SmallConvArgs a{};
        a.in = in;
        a.pro_ab = pro_ab;
        if (blend) {   // the VALU kernel has no blend prologue: materialise its blended input first
            HIP_TRY(affine_act_blend_launch(in, pro_ab, src->d_ab1, mip_ptr(h, src->out_mip, sw), nullptr, h->d_xlast,
                                            B, (long)e.s.H * e.s.W, e.s.cin, 1, st));
            a.in = h->d_xlast;
            a.pro_ab = nullptr;
        }
        a.w = e.d_w;
        a.bias = e.d_bias;
        a.out = e.d_out;
        a.part = e.d_part;
        a.batch = B;
        a.H = e.s.H;
        a.W = e.s.W;
        a.cin = e.s.cin;
        a.tiles_y = e.tiles_y;
        a.tiles_x = e.tiles_x;
        if (e.pro != PRO_AFF_RELU && e.pro != PRO_NONE)
            return fail(RST_ERR_UNSUPPORTED, "last layer prologue must be CIN+ReLU");
        HIP_TRY(small_conv_launch(a, st));
    } else if (e.kind == K_WINO9 || e.kind == K_WINO9X6 || e.kind == K_WINO9F3) {
        if (e.pro != PRO_NONE) return fail(RST_ERR_UNSUPPORTED, "9x9 Winograd conv reads the network input only");
        Wino9Args a{};
        a.in = in;
        a.U = e.d_w;
        a.bias = e.d_bias;
        a.bn_ab = e.d_bn;
        a.out = e.d_out;
        a.batch = B;
        a.H = e.s.H;
        a.W = e.s.W;
        a.cin = e.s.cin;
        a.tiles_y = e.tiles_y;
        a.tiles_x = e.tiles_x;
        if ((e.kind == K_WINO9X6 || e.kind == K_WINO9F3) && li == 0 && h->d_acc_all != nullptr) {   // it zeroes the frame's accumulators
            a.zero = h->d_acc_all;
            a.zero_n2 = (long)(h->acc_per_image * B / 2);
        }
        if (e.kind == K_WINO9X6 || e.kind == K_WINO9F3) next_weights(h, li, &a.w_next, &a.w_next_bytes);
        if (e.kind == K_WINO9X6 && h->w9_queue) a.queue = h->d_w9_queue;
        a.wt_stores = wt_bits(h, e, B, 4);
        HIP_TRY(e.kind == K_WINO9F3 ? wino9f3_launch(a, st) : e.kind == K_WINO9X6 ? wino9_x6_launch(a, st) : wino9_launch(a, st));
    } else if (e.kind == K_WINO || e.kind == K_WINOX6) {
        WinoArgs a{};
        a.in = in;
        a.res = e.pro_res;
        a.mat = e.d_mat;
        a.pro_ab = pro_ab;
        a.U = e.d_w;
        a.bias = e.d_bias;
        a.out = e.d_out;
        a.part = e.d_part;
        a.batch = B;
        a.H = e.s.H;
        a.W = e.s.W;
        a.cin = e.s.cin;
        a.tiles_y = e.tiles_y;
        a.tiles_x = e.tiles_x;
        a.pro_mode = e.pro;
        a.linear = e.s.conv_relu ? 0 : 1;
        if (blend) {
            if (e.kind != K_WINOX6) return fail(RST_ERR_UNSUPPORTED, "f32 Winograd conv has no two-style blend prologue");
            a.pro_ab1 = src->d_ab1;
            a.pro_w = mip_ptr(h, src->out_mip, sw);
        }
        if (e.acc_off >= 0) {   // this layer's statistics -> fixed-point accumulators (its consumer forms the affine)
            a.part = nullptr;
            a.stat.acc = acc_ptr(h, e, B);
            a.stat.nslot = e.nslot;
        }
        if (src != nullptr && src->acc_off >= 0 && pro_ab != nullptr) {   // the affine from the producer's
            a.pro_stat = cin_src(h, *src, style, B);                            // accumulators (no finalize ran)
            a.pro_ab = a.pro_ab1 = nullptr;
        }
        if (e.kind == K_WINOX6) next_weights(h, li, &a.u_next, &a.u_next_bytes);   // into L2 during the epilogue
        a.wt_stores = wt_bits(h, e, B, 3);
        if (h->d_tl && e.kind == K_WINOX6) a.tl = h->d_tl + li * (size_t)TL_SLOTS;
        if (ext_ev) wino_x6_set_timing_events(ev[0], ev[1]);
        HIP_TRY(e.kind == K_WINOX6 ? wino_x6_launch(a, st) : wino_launch(a, st));
    } else {
        ConvArgs a{};
        a.in = in;
        a.res = e.pro_res;
        a.mat = e.d_mat;
        a.pro_ab = pro_ab;
        if (blend) {
            a.pro_ab1 = src->d_ab1;
            a.pro_w = mip_ptr(h, src->out_mip, sw);
        }
        a.wpk = e.d_w;
        a.bias = e.d_bias;
        a.bn_ab = e.d_bn;
        a.out = e.d_out;
        a.part = e.d_part;
        a.batch = B;
        a.H = e.s.H;
        a.W = e.s.W;
        a.cin = e.s.cin;
        a.Ho = e.gHo;
        a.Wo = e.gWo;
        a.ntot = e.ntot;
        a.cout = e.s.cout;
        a.pad_t = e.pad_t;
        a.pad_l = e.pad_l;
        a.tiles_y = e.tiles_y;
        a.tiles_x = e.tiles_x;
        a.n_blocks = e.n_blocks;
        a.nchunks = e.nchunks;
        a.pro_mode = e.pro;
        a.epi_mode = e.s.norm == N_BN ? EPI_RELU_BN : (e.s.conv_relu ? EPI_RELU_STATS : EPI_STATS);
        a.shuffle = e.kind == K_CONVT2 ? 1 : 0;
        if (e.kind == K_LITE) {
            if (e.acc_off >= 0) {   // this layer's statistics -> fixed-point accumulators (its consumer forms the affine)
                a.part = nullptr;
                a.stat.acc = acc_ptr(h, e, B);
                a.stat.nslot = e.nslot;
            }
            if (src != nullptr && src->acc_off >= 0 && pro_ab != nullptr) {
                a.pro_stat = cin_src(h, *src, style, B);
                a.pro_ab = a.pro_ab1 = nullptr;
            }
            next_weights(h, li, &a.w_next, &a.w_next_bytes);
            a.wt_stores = wt_bits(h, e, B, 8);
            if (h->d_tl) a.tl = h->d_tl + li * (size_t)TL_SLOTS;
            HIP_TRY(conv_lite_launch(e.lite, a, st));   // two styles: its blend prologue (pro_ab1, pro_w)
        } else {
            HIP_TRY(conv_launch(e.tile, a, st));
        }
    }
    if (ev && !ext_ev) HIP_TRY(hipEventRecord(ev[1], st));
    // the last layer's finalize (one style) is fused into the output kernel (fin_sigmoid3_launch, rst_forward)
    const bool fused_out_fin = li + 1 == h->layers.size() && output_finalize_fused(h);
    if (e.s.norm == N_CIN && !fused_out_fin && e.acc_off < 0) {
        FinalizeArgs f{};
        f.part = e.d_part;
        f.style = style;
        f.ab = e.d_ab;
        f.batch = B;
        f.C = e.s.cout;
        f.ntot = e.ntot;
        f.n_part = e.n_part;
        f.phases = e.kind == K_CONVT2 ? 4 : 1;
        f.style_stride = h->shape.num_styles * h->P;
        f.style_offset = e.s.style_offset;
        if (two) {
            f.ab1 = e.d_ab1;
            f.style1_offset = h->P;
        }
        f.eps = 1e-5f;
        static const bool dbg = std::getenv("RST_DEBUG_FINALIZE") != nullptr;
        if (dbg)
            std::fprintf(stderr, "finalize %s: C=%d ntot=%d n_part=%d phases=%d batch=%d\n", e.s.name.c_str(), f.C,
                         f.ntot, f.n_part, f.phases, f.batch);
        HIP_TRY(finalize_launch(f, st));
    }
    if (ev) HIP_TRY(hipEventRecord(ev[2], st));
    return RST_OK;
}

int rst_forward(rst_handle* h, const float* content, const float* style_params, const float* style_weights,
                float* out, int batch, void* stream) {
    if (h == nullptr || content == nullptr || style_params == nullptr || out == nullptr)
        return fail(RST_ERR_INVALID, "rst_forward: null argument");
    if (batch <= 0 || batch > h->shape.max_batch)
        return fail(RST_ERR_INVALID, "rst_forward: batch " + std::to_string(batch) + " outside [1, max_batch=" +
                                         std::to_string(h->shape.max_batch) + "]");
    if (style_weights != nullptr && h->shape.num_styles == 1)
        return fail(RST_ERR_INVALID, "rst_forward: style_weights given but num_styles == 1");
    if (style_weights == nullptr && h->shape.num_styles == 2)
        return fail(RST_ERR_INVALID, "rst_forward: num_styles == 2 needs style_weights (B, out_h, out_w, 1)");
    hipStream_t st = static_cast<hipStream_t>(stream);
    // the CIN accumulators start at zero: cleared by the first layer's kernel when that is wino9_x6
    if (h->d_acc_all != nullptr && h->layers[0].kind != K_WINO9X6 && h->layers[0].kind != K_WINO9F3)
        HIP_TRY(hipMemsetAsync(h->d_acc_all, 0, h->acc_per_image * batch * sizeof(cin_word), st));
    for (size_t k = 1; k < h->d_mip.size(); ++k)
        HIP_TRY(avgpool2_1ch_launch(mip_ptr(h, (int)k - 1, style_weights), h->d_mip[k], batch, h->mip_h[k - 1],
                                    h->mip_w[k - 1], st));
    for (size_t li = 0; li < h->layers.size(); ++li) {
        int r = launch_layer(h, li, content, style_params, style_weights, batch, st);
        if (r != RST_OK) return r;
    }
    const LayerExec& last = h->layers.back();
    if (h->shape.num_styles == 2) {
        HIP_TRY(affine_act_blend_launch(last.d_out, last.d_ab, last.d_ab1, mip_ptr(h, last.out_mip, style_weights),
                                        nullptr, out, batch, (long)last.s.Ho * last.s.Wo, 3, 2, st));
    } else if (output_finalize_fused(h)) {   // the last CIN's affine (from its accumulators) + the output sigmoid
        HIP_TRY(fin_sigmoid3_launch(cin_src(h, last, style_params, batch), last.d_out, out,
                                    (long)last.s.Ho * last.s.Wo, batch, st));
    } else {
        HIP_TRY(affine_act_launch(last.d_out, last.d_ab, nullptr, out, batch, (long)last.s.Ho * last.s.Wo, 3, 2, st));
    }
    h->last_style_weights = style_weights;
    if (h->prof_on && h->prof_step < h->prof_max_steps) h->prof_step++;
    return RST_OK;
}

int rst_profile_begin(rst_handle* h, int max_steps) {
    if (h == nullptr || max_steps <= 0) return fail(RST_ERR_INVALID, "rst_profile_begin: bad argument");
    h->prof_free();
    h->prof_events.resize((size_t)max_steps * h->layers.size() * 3);
    for (auto& e : h->prof_events) HIP_TRY(hipEventCreate(&e));
    h->prof_max_steps = max_steps;
    h->prof_step = 0;
    h->prof_on = true;
    return RST_OK;
}

int rst_profile_end(rst_handle* h, float* conv_ms, float* layer_ms, int* steps) {
    if (h == nullptr || conv_ms == nullptr || layer_ms == nullptr || steps == nullptr)
        return fail(RST_ERR_INVALID, "rst_profile_end: bad argument");
    const size_t L = h->layers.size();
    for (size_t i = 0; i < L; ++i) conv_ms[i] = layer_ms[i] = 0.f;
    *steps = h->prof_step;
    if (h->prof_step > 0) HIP_TRY(hipEventSynchronize(h->prof_events[((size_t)(h->prof_step - 1) * L + L - 1) * 3 + 2]));
    for (int s = 0; s < h->prof_step; ++s)
        for (size_t i = 0; i < L; ++i) {
            hipEvent_t* ev = &h->prof_events[((size_t)s * L + i) * 3];
            float a = 0.f, b = 0.f;
            HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
            HIP_TRY(hipEventElapsedTime(&b, ev[0], ev[2]));
            conv_ms[i] += a;
            layer_ms[i] += b;
        }
    h->prof_free();
    return RST_OK;
}

int rst_timeline_begin(rst_handle* h) {
    if (h == nullptr) return fail(RST_ERR_INVALID, "rst_timeline_begin: null handle");
    h->tl_free();
    const size_t bytes = h->layers.size() * (size_t)TL_SLOTS * sizeof(unsigned long long);
    HIP_TRY(hipMalloc(&h->d_tl, bytes));
    HIP_TRY(hipMemset(h->d_tl, 0, bytes));
    HIP_TRY(hipDeviceSynchronize());
    return RST_OK;
}

int rst_timeline_read(rst_handle* h, double* end_us, int n) {
    if (h == nullptr || end_us == nullptr || n != (int)h->layers.size())
        return fail(RST_ERR_INVALID, "rst_timeline_read: bad argument");
    if (h->d_tl == nullptr) return fail(RST_ERR_INVALID, "rst_timeline_read: no rst_timeline_begin");
    std::vector<unsigned long long> tl((size_t)n * TL_SLOTS);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(tl.data(), h->d_tl, tl.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long t0 = 0;
    for (int i = 0; i < n; ++i) {
        unsigned long long m = 0;
        for (int k = 0; k < TL_SLOTS; ++k) m = std::max(m, tl[(size_t)i * TL_SLOTS + k]);
        end_us[i] = m ? (double)m : -1.0;
        if (m && !t0) t0 = m;
    }
    for (int i = 0; i < n; ++i)   // 100-MHz ticks -> us after the first stamped layer's end
        if (end_us[i] >= 0.0) end_us[i] = (end_us[i] - (double)t0) * 0.01;
    return RST_OK;
}

int rst_timeline_end(rst_handle* h) {
    if (h == nullptr) return fail(RST_ERR_INVALID, "rst_timeline_end: null handle");
    HIP_TRY(hipDeviceSynchronize());
    h->tl_free();
    return RST_OK;
}

int rst_precision(const rst_handle* h) { return h ? h->precision : -1; }

int rst_layer_kernel_id(const rst_handle* h, int idx) {
    if (h == nullptr || idx < 0 || idx >= (int)h->layers.size()) return -1;
    const LayerExec& e = h->layers[idx];
    switch (e.kind) {
        case K_SMALL: return 100;
        case K_WINO: return 200;
        case K_WINO9: return 201;
        case K_WINOX6: return 202;
        case K_WINO9X6: return 203;
        case K_WINO9F3: return 205;
        case K_LITE: return 300 + e.lite.id;   // 305: the x6 expand_0 form
        case K_LASTX6: return 204;
        default: return e.tile.id;
    }
}

int rst_layer_output_shape(const rst_handle* h, int idx, int batch, int* hwc3) {
    if (h == nullptr || idx < 0 || idx >= (int)h->layers.size() || hwc3 == nullptr)
        return fail(RST_ERR_INVALID, "rst_layer_output_shape: bad argument");
    const LayerSpec& s = h->layers[idx].s;
    hwc3[0] = s.Ho;
    hwc3[1] = s.Wo;
    hwc3[2] = s.cout;
    (void)batch;
    return RST_OK;
}

int rst_copy_activation(rst_handle* h, int idx, float* dst, size_t count, int batch, void* stream) {
    if (h == nullptr || idx < 0 || idx >= (int)h->layers.size() || dst == nullptr)
        return fail(RST_ERR_INVALID, "rst_copy_activation: bad argument");
    const LayerExec& e = h->layers[idx];
    const size_t n = (size_t)batch * e.s.Ho * e.s.Wo * e.s.cout;
    if (count != n) return fail(RST_ERR_INVALID, "rst_copy_activation: count mismatch, expected " + std::to_string(n));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (e.s.norm == N_BN) {
        HIP_TRY(hipMemcpyAsync(dst, e.d_out, n * 4, hipMemcpyDeviceToDevice, st));
    } else {
        const int act = e.s.post == P_RELU ? 1 : (e.s.post == P_SIGMOID ? 2 : 0);
        if (h->shape.num_styles == 2)
            HIP_TRY(affine_act_blend_launch(e.d_out, e.d_ab, e.d_ab1, mip_ptr(h, e.out_mip, h->last_style_weights),
                                            e.emit_res, dst, batch, (long)e.s.Ho * e.s.Wo, e.s.cout, act, st));
        else
            HIP_TRY(affine_act_launch(e.d_out, e.d_ab, e.emit_res, dst, batch, (long)e.s.Ho * e.s.Wo, e.s.cout, act,
                                      st));
    }
    return RST_OK;
}

size_t rst_gram_workspace_size(int batch, int hw, int channels) { return gram_workspace_bytes(batch, hw, channels); }

int rst_gram(const float* feat, int batch, int hw, int channels, float* out, void* workspace, void* stream) {
    if (feat == nullptr || out == nullptr || workspace == nullptr || batch <= 0 || hw <= 0 || channels <= 0)
        return fail(RST_ERR_INVALID, "rst_gram: bad argument");
    if (channels % 64 != 0) return fail(RST_ERR_UNSUPPORTED, "rst_gram: channels must be a multiple of 64");
    HIP_TRY(gram_launch(feat, batch, hw, channels, out, workspace, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

static const int IN_TILE = 256;

int rst_style_param_map(const float* style_weights, const float* style_params, int batch, int hw, int num_styles,
                        int n, float* out, void* stream) {
    if (style_weights == nullptr || style_params == nullptr || out == nullptr || batch <= 0 || hw <= 0 || n <= 0)
        return fail(RST_ERR_INVALID, "rst_style_param_map: null pointer or empty shape");
    if (num_styles != 2)
        return fail(RST_ERR_UNSUPPORTED, "rst_style_param_map: the per-pixel blend exists only for num_styles == 2 "
                                         "(styleTransfer.py:38-44 returns the params unblended otherwise)");
    HIP_TRY(style_param_map_launch(style_weights, style_params, out, batch, hw, n, (hipStream_t)stream));
    return RST_OK;
}

size_t rst_instance_norm_workspace_size(int batch, int hw, int channels) {
    const size_t n_tiles = (size_t)(hw + IN_TILE - 1) / IN_TILE;
    return (size_t)batch * channels * n_tiles * sizeof(float4) + (size_t)batch * channels * sizeof(float2);
}

int rst_instance_norm(const float* x, int batch, int hw, int channels, const float* scale, const float* bias,
                      float eps, int relu, float* y, void* workspace, void* stream) {
    if (x == nullptr || y == nullptr || workspace == nullptr || scale == nullptr || bias == nullptr || batch <= 0 ||
        hw <= 0 || channels <= 0)
        return fail(RST_ERR_INVALID, "rst_instance_norm: bad argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int n_tiles = (hw + IN_TILE - 1) / IN_TILE;
    float4* part = static_cast<float4*>(workspace);
    float2* ab = reinterpret_cast<float2*>(part + (size_t)batch * channels * n_tiles);
    HIP_TRY(tile_stats_launch(x, part, batch, hw, channels, IN_TILE, st));
    FinalizeArgs f{};
    f.part = part;
    f.scale = scale;
    f.bias = bias;
    f.ab = ab;
    f.batch = batch;
    f.C = channels;
    f.ntot = channels;
    f.n_part = n_tiles;
    f.phases = 1;
    f.affine_bstride = channels;
    f.eps = eps;
    HIP_TRY(finalize_launch(f, st));
    HIP_TRY(affine_act_launch(x, ab, nullptr, y, batch, hw, channels, relu ? 1 : 0, st));
    return RST_OK;
}

}  // extern "C"
