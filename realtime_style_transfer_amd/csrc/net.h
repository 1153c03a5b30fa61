// net.h — the transfer network's host-side description, shared by the inference (rst_api.hip)
// and training (train_api.hip) translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "kernels.h"

namespace rst {

const int CONTRACT_FILTERS[4] = {16, 32, 32, 32};                // styleTransfer.py:218-223
const int EXPAND_FILTERS[8] = {32, 16, 8, 4, 3, 3, 3, 3};        // styleTransfer.py:247-256

enum LayerKind { K_CONV = 0, K_CONVT2 = 1, K_SMALL = 2, K_WINO = 3, K_WINO9 = 4, K_WINOX6 = 5, K_WINO9X6 = 6, K_LITE = 7, K_LASTX6 = 8, K_WINO9F3 = 9 };
enum Norm { N_BN = 0, N_CIN = 1 };
enum Post { P_RELU = 0, P_NONE = 1, P_SIGMOID = 2 };

struct LayerSpec {
    std::string name;
    int keras_kind;      // 0 Conv2D, 1 Conv2DTranspose
    int k, stride, cin, cout;
    int H, W, Ho, Wo;    // input / output spatial dims
    int norm, post;
    bool conv_relu;
    int style_offset;
    int res_block;       // residual block index or -1
    int res_conv;        // 0/1 within the residual block
};

struct LayerExec {
    LayerSpec s;
    int kind = K_CONV;
    ConvTile tile{};
    LiteTile lite{};
    int ntot = 0, gHo = 0, gWo = 0, pad_t = 0, pad_l = 0;
    int tiles_y = 0, tiles_x = 0, n_blocks = 1, nchunks = 1;
    int n_part = 0;
    float* d_w = nullptr;
    size_t w_bytes = 0;           // bytes of the packed weight image d_w
    float* d_bias = nullptr;
    float2* d_bn = nullptr;
    float* d_out = nullptr;       // raw (CIN) or final (BN) output [max_batch][Ho][Wo][cout]
    float4* d_part = nullptr;
    float2* d_ab = nullptr;       // CIN affine of this layer's output [max_batch][cout]
    float2* d_ab1 = nullptr;      // second style's CIN affine (num_styles == 2)
    int out_mip = -1;             // style-weight mip level at this layer's output width (num_styles == 2)
    float* d_mat = nullptr;       // block input materialised by this layer's prologue (or null)
    long acc_off = -1;            // CIN statistics as fixed-point accumulators [nslot][batch][2][limb][cout] (kernels.h
    int nslot = 0;                // CinAcc) at d_acc_all + acc_off * batch, when producer and consumer both
                                  // take them (else d_part and a finalize kernel)
    // prologue (how this layer reads its input)
    int pro = PRO_NONE;
    int pro_src = -1;             // layer whose d_ab/d_out feed the prologue (-1: network input)
    const float* pro_res = nullptr;
    // debug "emitted" tensor of this layer = act(a*raw + b) [+ res]
    const float* emit_res = nullptr;
};

size_t layer_weight_count(const LayerSpec& s);
int build_plan(const rst_shape* sh, std::vector<LayerSpec>& L, int* P);
int prepare_layer(LayerExec& e, const LayerSpec& s, const float* kern, const float* bias, std::vector<float>& packed,
                  std::vector<float>& bias_n, int precision = RST_PRECISION_FP32,
                  bool allow_lite = false, bool inference = false);

template <typename T>
int upload(T** dst, const void* src, size_t bytes) {
    if (hipMalloc((void**)dst, bytes) != hipSuccess) return set_error(RST_ERR_ALLOC, "hipMalloc failed");
    if (src != nullptr && hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
        return set_error(RST_ERR_HIP, "hipMemcpy failed");
    return RST_OK;
}

}  // namespace rst

struct rst_handle {
    using LayerExec = rst::LayerExec;
    rst_shape shape;
    int P = 0;
    int precision = RST_PRECISION_FP32;
    std::vector<LayerExec> layers;
    // two-style blending: AvgPool2 mips of the second style's weight map, keyed by width
    // (styleTransfer.py:335-345); level 0 is the caller's style_weights (out_h x out_w)
    std::vector<float*> d_mip;
    std::vector<int> mip_h, mip_w;
    float* d_xlast = nullptr;     // blended input of the last (VALU) layer
    rst::cin_word* d_acc_all = nullptr;  // every layer's accumulators for max_batch (a forward of B images uses the
    size_t acc_per_image = 0;       // first acc_per_image * B words, zeroed at its start)
    unsigned* d_w9_queue = nullptr;   // the start conv's work-queue counters [2] (wino9_x6, self-resetting)
    bool w9_queue = true;             // RST_W9_QUEUE=0 at creation: static unit order (A/B runs)
    const float* last_style_weights = nullptr;   // for the debug copies of the most recent forward
    std::vector<void*> allocs;
    // optional per-layer timing: 3 events per layer per step (before conv, after conv, after finalize)
    std::vector<hipEvent_t> prof_events;
    int prof_max_steps = 0, prof_step = 0;
    bool prof_on = false;
    int wt_stores = 15;               // RST_WT_STORES at creation: write-through output stores (1 wino_x6 output, 2 its
                                      // materialised input, 4 wino9_x6 output, 8 conv_lite output)
    bool no_u_prefetch = false;       // RST_NO_U_PREFETCH=1 at creation: no next-layer U prefetch (A/B runs)
    unsigned long long* d_tl = nullptr;   // rst_timeline_begin: [layers][TL_SLOTS] wave end stamps (wino_x6, conv_lite)
    void tl_free() {
        if (d_tl) (void)hipFree(d_tl);
        d_tl = nullptr;
    }
    void prof_free() {
        for (hipEvent_t e : prof_events) (void)hipEventDestroy(e);
        prof_events.clear();
        prof_on = false;
        prof_max_steps = prof_step = 0;
    }
    ~rst_handle() {
        prof_free();
        tl_free();
        for (void* p : allocs) (void)hipFree(p);
    }
    template <typename T>
    int alloc(T** p, size_t bytes, const void* src = nullptr) {
        int st = rst::upload(p, src, bytes);
        if (*p) allocs.push_back((void*)*p);
        return st;
    }
};

