// train_api.hip — C ABI of the training step (include/rst.h, rst_trainer_*).
//
// One step of train_network.py:102-138 (Keras fit: StyleTransferTrainingModel.train_step,
// styleTransferTrainingModel.py:26-29, loss styleLoss.py:295-369, RMSprop OptimizerV2) for the
// transfer network, with the style parameters as an input (the predictor is a separate model):
//
//   forward (training mode)   every conv on conv_mfma_kernel / conv_small_kernel as in inference,
//                             but BatchNorm uses batch statistics (finalize merges all images,
//                             updates the moving statistics, momentum 0.99, styleTransfer.py:201),
//                             every conv input is materialised by the conv's own prologue (wgrad
//                             operand) and every normaliser keeps (mean, rstd) for its backward.
//   loss                      rst_loss_forward (VGG16 runs style, content, prediction — the
//                             prediction's activations stay resident for the backward).
//   VGG backward              content term cf/N (F5p - F5c); per style layer the Gram backward
//                             F (Gp - Gs) sf / (2 C^2 HW) as a per-image 1x1 MFMA conv; max-pool
//                             backward; dgrad of each 3x3 conv = conv with the flipped kernel whose
//                             prologue applies the ReLU mask (PRO_MASK); the preprocess (x 255,
//                             RGB->BGR) is folded into conv0's dgrad weights; TV sign gradient.
//   transfer backward         per layer: norm backward (CIN / BN) -> bias grad, split-K MFMA wgrad,
//                             dgrad on conv_mfma_kernel (residual: flipped kernel; stride-2 conv:
//                             4-phase transposed conv; transposed conv: stride-2 conv; last 9x9
//                             transposed conv: 9x9 conv), skip-connection gradient chain.
//   apply                     RMSprop on the canonical (Keras-order) weights, then a gather re-packs
//                             them into every kernel's weight image (forward and dgrad).
// Gradients are of the batch-summed loss (Keras minimises the (B,) loss vector's sum).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "kernels.h"
#include "lossnet.h"
#include "net.h"
#include "train.h"

// Geometry of a layer's weight-gradient GEMM (shared by the workspace sizing at create time and the
// launch, so the split count and slab size always agree).
static rst::WgradArgs wgrad_geometry(const rst::LayerSpec& s, const rst::LayerExec& e, int B) {
    rst::WgradArgs w{};
    w.batch = B;
    w.XH = s.H;
    w.XW = s.W;
    w.C1 = s.cin;
    w.DH = s.Ho;
    w.DW = s.Wo;
    w.C2 = s.cout;
    w.kh = w.kw = s.k;
    w.stride = s.stride;
    if (s.keras_kind == 0) {
        w.Qh = s.Ho;
        w.Qw = s.Wo;
        w.pad_t = e.pad_t;
        w.pad_l = e.pad_l;
        w.transposed = 0;
    } else {
        w.Qh = s.H;
        w.Qw = s.W;
        w.pad_t = w.pad_l = std::max(s.k - s.stride, 0) / 2;
        w.transposed = 1;
    }
    return w;
}

using namespace rst;

namespace {

struct TLayer {
    LayerExec e;                          // forward geometry; d_w / d_bias packed from the canonical weights
    size_t woff = 0, boff = 0, goff = 0;  // canonical offsets of kernel, bias, BN gamma (0: CIN layer)
    size_t kcount = 0;
    float2* d_mr = nullptr;               // (mean, rstd) per (image, channel)
    float* d_x = nullptr;                 // conv input as the kernel sees it (layer 0: the network input)
    float* d_g = nullptr;                 // gradient w.r.t. the post-activation output (before any skip add)
    int* d_map_w = nullptr;
    size_t n_w = 0;
    int* d_map_b = nullptr;
    size_t n_b = 0;
    bool has_dgrad = false;
    LayerExec dg;                         // input-gradient conv (its input is this layer's dz)
    float* d_wdg = nullptr;
    int* d_map_dg = nullptr;
    size_t n_dg = 0;
    int norm_tile = 0;
    // Winograd residual convs (precision FP32_WINOGRAD): the weight images are transforms, not gathers —
    // the forward image is computed from the canonical HWIO kernel, the input-gradient image from the
    // flipped kernel gathered into d_kflip (d_map_dg then maps canonical -> flipped HWIO)
    bool wino_fwd = false, wino_dg = false;
    float* d_kflip = nullptr;
};

struct ConvBwd {   // a backward conv with static weights (VGG dgrad, Gram 1x1)
    ConvTile tile{};
    int tiles_y = 0, tiles_x = 0, n_blocks = 0, nchunks = 0, n_packed = 0;
    float* d_w = nullptr;
    int* d_map = nullptr;
};

int norm_tile_for(long hw, int B) {
    long t = (hw * B + 1023) / 1024;
    t = ((t + 63) / 64) * 64;
    return (int)std::max<long>(t, 64);
}

std::vector<int> to_map(const std::vector<float>& packed) {
    std::vector<int> m(packed.size());
    for (size_t i = 0; i < packed.size(); ++i) m[i] = (int)std::lrint(packed[i]) - 1;
    return m;
}

ConvArgs conv_geometry(const LayerExec& e, int B) {
    ConvArgs a{};
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
    a.shuffle = e.kind == K_CONVT2 ? 1 : 0;
    return a;
}

}  // namespace

struct rst_trainer {
    rst_shape shape{};
    int P = 0;
    size_t nw = 0;
    std::vector<TLayer> L;
    rst_loss_handle* loss = nullptr;
    ConvBwd vgg[13];
    ConvBwd vgg0p;   // VGG conv0 input gradient as a 1x1 conv 64 -> (tap, c) columns + tap3_sum
    ConvBwd gram[4];
    std::vector<void*> allocs;
    float* d_wc = nullptr;        // canonical weights (Keras order)
    float* d_ms = nullptr;        // RMSprop slots
    float* d_zero = nullptr;      // zero bias of the backward convs
    float* d_dz = nullptr;        // norm-backward output of the current layer
    float* d_tmp = nullptr;       // skip-chain scratch
    float2* d_nb_part = nullptr;
    float2* d_nb_consts = nullptr;
    float* d_slab = nullptr;
    float* d_gstyle = nullptr;    // style-param gradient scratch (caller passed none)
    float* d_vg[2] = {nullptr, nullptr};
    float* d_vpool = nullptr;
    float* d_gram_packed = nullptr;
    float* d_vgg_dbg[13] = {};    // debug: d loss / d (VGG conv i output), when enabled
    int* d_stat_index = nullptr;  // canonical index of every BN moving_mean / moving_variance entry
    size_t n_stat = 0;
    // the loss targets (style Grams, content features) run on a side stream beside the predictor / transfer
    // forward: fork after the caller's stream, join before the prediction's VGG16 pass (same VGG16 buffers)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // recorded in backward() right after the last CIN layer's norm backward: from there on grad_style_params is final
    // and the rest of the backward (the contract layers, the start conv's weight gradient) no longer touches it, so the
    // style predictor's backward can run beside it (rst_trainer_wait_style_gradient)
    hipEvent_t ev_gstyle = nullptr;
    bool gstyle_recorded = false;
    bool targets_pending = false;
    bool serial_targets = false;  // RST_SERIAL_TARGETS=1 at creation: targets on the caller's stream (A/B runs)
    bool vgg_grad_f32 = false;    // RST_VGG_GRAD_F32=1 at creation: f32 VGG16 gradients beside bf16 activations (A/B)
    int wt_stores = 5;            // RST_TRAIN_WT at creation: bit0 Winograd conv outputs, bit1 the residual convs'
                                  // materialised inputs, bit2 the other transfer convs' outputs (forward and input
                                  // gradient), bit3 the VGG16 input gradients, stored write-through (sc1); default 5
    const float* pend_content = nullptr;
    const float* pend_style = nullptr;
    int pend_batch = 0;
    ~rst_trainer() {
        if (side) {
            (void)hipStreamSynchronize(side);
            (void)hipStreamDestroy(side);
        }
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (ev_gstyle) (void)hipEventDestroy(ev_gstyle);
        if (loss) rst_loss_destroy(loss);
        for (void* p : allocs) rst::guard_free(p);
    }
    template <typename T>
    int alloc(T** p, size_t bytes, const void* src = nullptr) {
        int st = RST_OK;
        if (rst::guard_malloc((void**)p, bytes ? bytes : 4) != hipSuccess) {
            *p = nullptr;
            st = rst::set_error(RST_ERR_ALLOC, "hipMalloc failed");
        } else if (src != nullptr && hipMemcpy(*p, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
            st = rst::set_error(RST_ERR_HIP, "hipMemcpy failed");
        }
        if (*p) allocs.push_back((void*)*p);
        if (st == RST_OK && src == nullptr && hipMemset(*p, 0, bytes ? bytes : 4) != hipSuccess)
            return set_error(RST_ERR_HIP, "hipMemset failed");
        return st;
    }
};

namespace {

int repack(rst_trainer* t, hipStream_t st) {
    // the x6 transforms of every layer go into batched launches after the gathers that feed them; the gathers go into
    // batched launches too (flushed before anything that reads their outputs)
    GatherJobs gj{};
    auto gather = [&](const int* map, float* dst, size_t n) -> hipError_t {
        if (gj.n == GATHER_MAX_JOBS) {
            const hipError_t e = gather_batch_launch(t->d_wc, gj, st);
            if (e != hipSuccess) return e;
        }
        gj.map[gj.n] = map;
        gj.dst[gj.n] = dst;
        gj.count[gj.n] = n;
        ++gj.n;
        return hipSuccess;
    };
    X6TransformJobs jobs{};
    auto add_job = [&](const float* kern, int cin, float* U) -> int {
        if (jobs.n == X6_MAX_JOBS) {
            RST_HIP_TRY(gather_batch_launch(t->d_wc, gj, st));   // (a job may read a gathered d_kflip)
            RST_HIP_TRY(wino_x6_transform_batch_launch(jobs, st));
            jobs.n = 0;
        }
        jobs.kern[jobs.n] = kern;
        jobs.cin[jobs.n] = cin;
        jobs.U[jobs.n] = U;
        ++jobs.n;
        return RST_OK;
    };
    for (TLayer& T : t->L) {
        int r = RST_OK;
        if (T.e.kind == K_WINO9) RST_HIP_TRY(wino9_transform_launch(t->d_wc + T.woff, T.e.s.cin, T.e.d_w, st));
        else if (T.e.kind == K_WINO9X6) RST_HIP_TRY(wino9_x6_transform_launch(t->d_wc + T.woff, T.e.s.cin, T.e.d_w, st));
        else if (T.e.kind == K_WINOX6) r = add_job(t->d_wc + T.woff, T.e.s.cin, T.e.d_w);
        else if (T.wino_fwd) RST_HIP_TRY(wino_transform_launch(t->d_wc + T.woff, T.e.s.cin, T.e.d_w, st));
        else RST_HIP_TRY(gather(T.d_map_w, T.e.d_w, T.n_w));
        if (r != RST_OK) return r;
        RST_HIP_TRY(gather(T.d_map_b, T.e.d_bias, T.n_b));
        if (T.has_dgrad && T.wino_dg) {
            RST_HIP_TRY(gather(T.d_map_dg, T.d_kflip, T.n_dg));
            if (T.dg.kind == K_WINOX6) {
                if ((r = add_job(T.d_kflip, T.dg.s.cin, T.d_wdg)) != RST_OK) return r;
            } else {
                RST_HIP_TRY(gather_batch_launch(t->d_wc, gj, st));
                RST_HIP_TRY(wino_transform_launch(T.d_kflip, T.dg.s.cin, T.d_wdg, st));
            }
        } else if (T.has_dgrad) {
            RST_HIP_TRY(gather(T.d_map_dg, T.d_wdg, T.n_dg));
        }
    }
    RST_HIP_TRY(gather_batch_launch(t->d_wc, gj, st));
    RST_HIP_TRY(wino_x6_transform_batch_launch(jobs, st));
    return RST_OK;
}

// Write-through output stores (RST_TRAIN_WT=1) where the outputs' byte offsets fit the kernels' 32-bit buffer offsets
static int train_wt(const rst_trainer* t, size_t elems, int mask = 1) {
    return elems * 4 < (size_t)0x7FFFFFF0 ? (t->wt_stores & mask) : 0;
}

// ---- forward (training mode) ------------------------------------------------------------------
int forward(rst_trainer* t, const float* content, const float* style, int B, float* prediction, hipStream_t st) {
    // The forward waits for the loss targets before its layer join_at (default 0: the targets never run beside the
    // transfer network's forward; they still run beside the style predictor's forward, train_step). With the plain-bf16
    // VGG16 targets running beside it, the forward's prediction was not repeatable (tools/pred_race_check.py: ~all
    // pixels, up to 7e-2, from call to call, profiles/r06/r06am): joining before any of layers 0-13 made it bitwise
    // repeatable, overlapping the targets with expand_0 .. expand_last did not. Traced to the last conv's packed-FMA
    // accumulate chains taking wrong sums when bf16-VGG16 waves shared its CU; that kernel now uses scalar
    // FMAs and is clean without the join, which stays as a second fence. RST_TARGETS_JOIN_AT=k moves it (-1: none).
    static const int join_at = [] {
        const char* v = getenv("RST_TARGETS_JOIN_AT");
        return v != nullptr ? atoi(v) : 0;
    }();
    // diagnostic: RST_LDS_POISON=<bits> fills every CU's LDS with that pattern before each kernel of layer
    // RST_LDS_POISON_LAYER (default -1: every layer; L.size(): the final sigmoid), so a read of LDS the kernel did not
    // write shows in the prediction
    static const long long poison_bits = [] {
        const char* v = getenv("RST_LDS_POISON");
        return v != nullptr ? (long long)strtoull(v, nullptr, 0) : -1LL;
    }();
    static const int poison_layer = [] {
        const char* v = getenv("RST_LDS_POISON_LAYER");
        return v != nullptr ? atoi(v) : -1;
    }();
    // diagnostic: RST_TARGETS_JOIN_KERNEL=k joins the loss targets before the forward's k-th kernel instead (counting
    // every conv, materialisation, finalize and the final sigmoid in launch order)
    static const int join_kernel = [] {
        const char* v = getenv("RST_TARGETS_JOIN_KERNEL");
        return v != nullptr ? atoi(v) : -1;
    }();
    // diagnostic: RST_FENCE_KERNEL=k puts a cross-stream dependency (an event recorded on an idle stream) before the
    // forward's k-th kernel: a barrier packet with its cache fences, without waiting for the targets
    static const int fence_kernel = [] {
        const char* v = getenv("RST_FENCE_KERNEL");
        return v != nullptr ? atoi(v) : -1;
    }();
    static hipStream_t fence_stream = nullptr;
    static hipEvent_t fence_event = nullptr;
    size_t li = 0;
    int kernel_idx = 0;
    auto poison = [&]() -> hipError_t {
        if (kernel_idx == fence_kernel) {
            hipError_t e = hipSuccess;
            if (fence_stream == nullptr) e = hipStreamCreateWithFlags(&fence_stream, hipStreamNonBlocking);
            if (e == hipSuccess && fence_event == nullptr) e = hipEventCreateWithFlags(&fence_event, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventRecord(fence_event, fence_stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(st, fence_event, 0);
            if (e != hipSuccess) return e;
        }
        if (kernel_idx++ == join_kernel && t->targets_pending) {
            const hipError_t e = hipStreamWaitEvent(st, t->ev_join, 0);
            if (e != hipSuccess) return e;
        }
        if (poison_bits < 0 || (poison_layer >= 0 && (size_t)poison_layer != li)) return hipSuccess;
        return lds_poison_launch((unsigned)poison_bits, st);
    };
    for (li = 0; li < t->L.size(); ++li) {
        if ((int)li == join_at && t->targets_pending) RST_HIP_TRY(hipStreamWaitEvent(st, t->ev_join, 0));
        RST_HIP_TRY(poison());
        TLayer& T = t->L[li];
        LayerExec& e = T.e;
        const TLayer* Pv = li ? &t->L[li - 1] : nullptr;
        if (e.kind == K_SMALL) {
            // its input (CIN + ReLU of the predecessor) is materialised for the wgrad anyway
            RST_HIP_TRY(affine_act_launch(Pv->e.d_out, Pv->e.d_ab, nullptr, T.d_x, B, (long)e.s.H * e.s.W, e.s.cin,
                                          1, st));
            SmallConvArgs a{};
            a.in = T.d_x;
            a.pro_ab = nullptr;
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
            RST_HIP_TRY(poison());
            RST_HIP_TRY(small_conv_launch(a, st));
        } else if (e.kind == K_WINO9 || e.kind == K_WINO9X6) {
            Wino9Args a{};
            a.in = content;
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
            a.wt_stores = train_wt(t, (size_t)B * e.s.H * e.s.W * e.s.cout);
            RST_HIP_TRY(e.kind == K_WINO9X6 ? wino9_x6_launch(a, st) : wino9_launch(a, st));
        } else if (e.kind == K_WINO || e.kind == K_WINOX6) {
            WinoArgs a{};
            a.in = Pv->e.d_out;
            a.res = e.pro_res;
            a.mat = T.d_x;
            a.pro_ab = Pv->e.d_ab;
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
            a.wt_stores = train_wt(t, (size_t)B * e.s.H * e.s.W * 128, 3);   // bit 1 (RST_TRAIN_WT=3): also mat
            RST_HIP_TRY(e.kind == K_WINOX6 ? wino_x6_launch(a, st) : wino_launch(a, st));
        } else {
            ConvArgs a = conv_geometry(e, B);
            a.in = Pv ? Pv->e.d_out : content;
            a.res = e.pro_res;
            a.mat = T.d_x;   // null for the first layer (its input is the content itself)
            a.pro_ab = Pv ? Pv->e.d_ab : nullptr;
            a.wpk = e.d_w;
            a.bias = e.d_bias;
            a.out = e.d_out;
            a.part = e.d_part;
            a.pro_mode = e.pro;
            a.epi_mode = e.s.conv_relu ? EPI_RELU_STATS : EPI_STATS;
            a.wt_stores = train_wt(t, (size_t)B * e.s.Ho * e.s.Wo * e.s.cout, 4);
            RST_HIP_TRY(conv_launch(e.tile, a, st));
        }
        FinalizeArgs f{};
        f.part = e.d_part;
        f.ab = e.d_ab;
        f.mr = T.d_mr;
        f.batch = B;
        f.C = e.s.cout;
        f.ntot = e.ntot;
        f.n_part = e.n_part;
        f.phases = e.kind == K_CONVT2 ? 4 : 1;
        if (e.s.norm == N_CIN) {
            f.style = style;
            f.style_stride = t->P;
            f.style_offset = e.s.style_offset;
            f.eps = 1e-5f;
        } else {
            f.scale = t->d_wc + T.goff;
            f.bias = t->d_wc + T.goff + e.s.cout;
            f.affine_bstride = 0;
            f.merge_images = 1;
            f.moving_mean = t->d_wc + T.goff + 2 * e.s.cout;
            f.moving_var = t->d_wc + T.goff + 3 * e.s.cout;
            f.momentum = 0.99f;
            f.eps = 1e-3f;
        }
        RST_HIP_TRY(poison());
        RST_HIP_TRY(finalize_launch(f, st));
    }
    const LayerExec& last = t->L.back().e;
    RST_HIP_TRY(poison());
    RST_HIP_TRY(affine_act_launch(last.d_out, last.d_ab, nullptr, prediction, B, (long)last.s.Ho * last.s.Wo, 3, 2, st));
    return RST_OK;
}

// ---- VGG16 backward: d(loss)/d(prediction) into gimg ------------------------------------------
int vgg_backward(rst_trainer* t, const float* prediction, int B, float* gimg, hipStream_t st) {
    rst_loss_handle* h = t->loss;
    const rst_loss_shape& ls = h->shape;
    const VggConv& c5 = h->convs[CONTENT_IDX];
    const size_t f5 = (size_t)c5.H * c5.W * c5.cout;
    int which = 0;
    float* g = t->d_vg[0];
    // act: the forward activations (ReLU masks, pool routing, features) are bf16 bits, and so are the gradients of the
    // VGG16 layer outputs (mixed_bfloat16: a bf16 layer's output gradient is bf16; every stored gradient is one rounding
    // of an f32 value, sums of two bf16 gradients rounded once); the gradient reaching the prediction stays f32
    const bool xa = h->act_bf16;                 // forward activations stored bf16
    const bool act = xa && !t->vgg_grad_f32;     // ... and the gradients (RST_VGG_GRAD_F32=1 at creation: f32, A/B runs)
    RST_HIP_TRY(scaled_diff_launch(c5.d_out, h->d_content_feat, (float)(ls.content_factor / (double)f5), g, B * f5, 0,
                                   st, xa, act));
    for (int i = CONTENT_IDX; i >= 0; --i) {
        const VggConv& c = h->convs[i];
        const ConvBwd& vb = t->vgg[i];
        if (t->d_vgg_dbg[i]) {
            if (act)
                RST_HIP_TRY(bf16_to_f32_launch(g, t->d_vgg_dbg[i], (size_t)B * c.H * c.W * c.cout, st));
            else
                RST_HIP_TRY(hipMemcpyAsync(t->d_vgg_dbg[i], g, (size_t)B * c.H * c.W * c.cout * 4, hipMemcpyDeviceToDevice,
                                           st));
        }
        const bool pooled = i > 0 && VGG_POOL[i - 1];
        if (i == 0) {   // 64 -> 3: 1x1 conv to the 27 (tap, c) columns (into the free gradient buffer), tap sum
            const ConvBwd& pb = t->vgg0p;
            float* pbuf = t->d_vg[which ^ 1];
            ConvArgs a{};
            a.in = g;
            a.res = c.d_out;              // ReLU mask from the forward output
            a.wpk = pb.d_w;
            a.bias = t->d_zero;
            a.out = pbuf;
            a.batch = B;
            a.H = c.H;
            a.W = c.W;
            a.cin = c.cout;
            a.Ho = c.H;
            a.Wo = c.W;
            a.ntot = 32;
            a.cout = 32;
            a.pad_t = a.pad_l = 0;
            a.tiles_y = pb.tiles_y;
            a.tiles_x = pb.tiles_x;
            a.n_blocks = pb.n_blocks;
            a.nchunks = pb.nchunks;
            a.pro_mode = PRO_MASK;
            a.epi_mode = EPI_NONE;
            a.act_bf16 = (act ? 1 : 0) | (xa ? 4 : 0);   // bf16 gradient / mask in, f32 out (the f32 prediction's gradient)
            RST_HIP_TRY(conv_launch(pb.tile, a, st));
            RST_HIP_TRY(tap3_sum_launch(pbuf, gimg, B, c.H, c.W, st));
            break;
        }
        float* dst = pooled ? t->d_vpool : t->d_vg[which ^ 1];
        ConvArgs a{};
        a.in = g;
        a.res = c.d_out;                  // ReLU mask from the forward output
        a.wpk = vb.d_w;
        a.bias = t->d_zero;
        a.out = dst;
        a.batch = B;
        a.H = c.H;
        a.W = c.W;
        a.cin = c.cout;
        a.Ho = c.H;
        a.Wo = c.W;
        a.ntot = c.cin;
        a.cout = c.cin;
        a.pad_t = a.pad_l = 1;
        a.tiles_y = vb.tiles_y;
        a.tiles_x = vb.tiles_x;
        a.n_blocks = vb.n_blocks;
        a.nchunks = vb.nchunks;
        a.pro_mode = PRO_MASK;
        a.epi_mode = EPI_NONE;
        a.wt_stores = train_wt(t, (size_t)B * c.H * c.W * c.cin, 8);
        a.act_bf16 = (act ? 1 | 2 : 0) | (xa ? 4 : 0);
        RST_HIP_TRY(conv_launch(vb.tile, a, st));
        if (i == 0) break;
        const int p = i - 1;
        const VggConv& cp = h->convs[p];
        float* gprev = t->d_vg[which ^ 1];
        int k = -1;
        for (int q = 0; q < 4; ++q)
            if (STYLE_IDX[q] == p) k = q;
        if (k >= 0) {
            if (!pooled) return set_error(RST_ERR_UNSUPPORTED, "style layer without a following pool");
            const ConvBwd& gb = t->gram[k];
            const int C = cp.cout;
            const long hw = (long)cp.H * cp.W;
            const float scale = (float)(ls.style_factor / (2.0 * C * C * (double)hw));
            const bool gbf16 = gb.tile.bf3 != 0;   // weights as conv_bf3's bf16 image (n_packed bf16 per image)
            if (gbf16)
                RST_HIP_TRY(gram_bwd_weights_bf16_launch(h->d_gram_pred[k], h->d_gram_style[k], gb.d_map, gb.n_packed, C,
                                                         scale, reinterpret_cast<unsigned short*>(t->d_gram_packed), B,
                                                         st));
            else
                RST_HIP_TRY(gram_bwd_weights_launch(h->d_gram_pred[k], h->d_gram_style[k], gb.d_map, gb.n_packed, C,
                                                    scale, t->d_gram_packed, B, st));
            for (int b = 0; b < B; ++b) {
                ConvArgs m{};
                m.in = xa ? reinterpret_cast<const float*>(reinterpret_cast<const unsigned short*>(cp.d_out) +
                                                           (size_t)b * hw * C)
                          : cp.d_out + (size_t)b * hw * C;
                m.act_bf16 = xa ? 1 : 0;
                m.wpk = gbf16 ? reinterpret_cast<const float*>(reinterpret_cast<const unsigned short*>(t->d_gram_packed) +
                                                               (size_t)b * gb.n_packed)
                              : t->d_gram_packed + (size_t)b * gb.n_packed;
                m.bias = t->d_zero;
                m.out = gprev + (size_t)b * hw * C;   // f32 (the bf16 sum with the pool's gradient is rounded once)
                m.batch = 1;
                m.H = cp.H;
                m.W = cp.W;
                m.cin = C;
                m.Ho = cp.H;
                m.Wo = cp.W;
                m.ntot = C;
                m.cout = C;
                m.tiles_y = gb.tiles_y;
                m.tiles_x = gb.tiles_x;
                m.n_blocks = gb.n_blocks;
                m.nchunks = gb.nchunks;
                m.pro_mode = PRO_NONE;
                m.epi_mode = EPI_NONE;
                RST_HIP_TRY(conv_launch(gb.tile, m, st));
            }
        }
        if (pooled && act && k >= 0) {
            // bf16 gradients at a style layer: bf16(Gram gradient (f32, in gprev) + routed pool gradient) into the buffer
            // of g (already consumed by the input-gradient conv above); `which` stays
            float* gsum = t->d_vg[which];
            RST_HIP_TRY(maxpool2_bwd_launch(cp.d_out, t->d_vpool, gsum, B, cp.H, cp.W, cp.cout, 0, st, xa, true, gprev));
            g = gsum;
            continue;
        }
        if (pooled)
            RST_HIP_TRY(maxpool2_bwd_launch(cp.d_out, t->d_vpool, gprev, B, cp.H, cp.W, cp.cout, k >= 0, st, xa, act));
        which ^= 1;
        g = gprev;
    }
    RST_HIP_TRY(tv_bwd_launch(prediction, ls.tv_factor, gimg, B, ls.h, ls.w, 3, st));
    return RST_OK;
}

// ---- transfer-network backward ------------------------------------------------------------
int backward(rst_trainer* t, const float* content, int B, float* grad, float* gstyle, hipStream_t st) {
    const int n = (int)t->L.size();
    int first_cin = -1;   // the last CIN layer the backward reaches
    for (int li = n - 1; li >= 0; --li)
        if (t->L[li].e.s.norm == N_CIN) first_cin = li;
    if (first_cin < 0) RST_HIP_TRY(hipEventRecord(t->ev_gstyle, st));
    for (int li = n - 1; li >= 0; --li) {
        TLayer& T = t->L[li];
        const LayerExec& e = T.e;
        const LayerSpec& s = e.s;
        const long hw = (long)s.Ho * s.Wo;
        NormBwdArgs nb{};
        nb.g = T.d_g;
        nb.z = e.d_out;
        nb.ab = e.d_ab;
        nb.mr = T.d_mr;
        nb.part = t->d_nb_part;
        nb.consts = t->d_nb_consts;
        if (s.norm == N_CIN) {
            nb.dscale = gstyle + s.style_offset;
            nb.dbias = gstyle + s.style_offset + s.cout;
            nb.dstride = t->P;
        } else {
            nb.dscale = grad + T.goff;
            nb.dbias = grad + T.goff + s.cout;
            nb.merge_images = 1;
        }
        nb.dz = t->d_dz;
        nb.batch = B;
        nb.hw = (int)hw;
        nb.C = s.cout;
        nb.tile = norm_tile_for(hw, B);
        nb.n_tiles = (int)((hw + nb.tile - 1) / nb.tile);
        nb.post = s.post;
        nb.conv_relu = s.conv_relu ? 1 : 0;
        nb.dconv_bias = grad + T.boff;
        RST_HIP_TRY(norm_bwd_launch(nb, st));
        if (li == first_cin) RST_HIP_TRY(hipEventRecord(t->ev_gstyle, st));   // grad_style_params final
        WgradArgs w = wgrad_geometry(s, e, B);
        w.X = li == 0 ? content : T.d_x;
        w.D = t->d_dz;
        w.slab = t->d_slab;
        w.dW = grad + T.woff;
        // WINOGRAD_BF16X6: the residual convs' weight gradient on the split-bf16 x6 kernel (fp32-level
        // products, wgrad.hip); the other layers and modes keep the f32-MFMA kernel
        w.x6 = T.e.kind == K_WINOX6 || T.e.kind == K_WINO9X6 ? 1 : 0;   // the split-bf16 trainer's convs
        w.nsplit = wgrad_choose_splits(w);
        RST_HIP_TRY(wgrad_launch(w, st));
        if (!T.has_dgrad) continue;
        // input gradient: to the predecessor's output gradient, or (conv0 of residual block r > 0)
        // through the skip chain g_r = dgrad + g_{r+1}
        TLayer& Pv = t->L[li - 1];
        const bool open_block = s.res_block > 0 && s.res_conv == 0;   // conv0 of residual block r > 0
        float* target = open_block ? t->d_tmp : Pv.d_g;
        if (T.wino_dg) {
            WinoArgs a{};
            a.in = t->d_dz;
            a.U = T.d_wdg;
            a.bias = t->d_zero;
            a.out = target;
            a.batch = B;
            a.H = T.dg.s.H;
            a.W = T.dg.s.W;
            a.cin = T.dg.s.cin;
            a.tiles_y = T.dg.tiles_y;
            a.tiles_x = T.dg.tiles_x;
            a.pro_mode = PRO_NONE;
            a.linear = 1;
            a.wt_stores = train_wt(t, (size_t)B * T.dg.s.H * T.dg.s.W * 128);
            RST_HIP_TRY(T.dg.kind == K_WINOX6 ? wino_x6_launch(a, st) : wino_launch(a, st));
        } else {
            ConvArgs a = conv_geometry(T.dg, B);
            a.in = t->d_dz;
            a.wpk = T.d_wdg;
            a.bias = t->d_zero;
            a.out = target;
            a.pro_mode = PRO_NONE;
            a.epi_mode = EPI_NONE;
            a.wt_stores = train_wt(t, (size_t)B * T.dg.s.Ho * T.dg.s.Wo * T.dg.s.cout, 4);
            RST_HIP_TRY(conv_launch(T.dg.tile, a, st));
        }
        if (open_block) {
            // g_r = (conv path) + g_{r+1}; g_{r+1} is the gradient of conv1 of block r (= T(li+1).d_g)
            const TLayer& c1 = t->L[li + 1];
            RST_HIP_TRY(add_launch(t->d_tmp, c1.d_g, Pv.d_g, (size_t)B * s.H * s.W * s.cin, st));
        }
    }
    return RST_OK;
}

int fail_delete(rst_trainer* t, int st) {
    delete t;
    return st;
}

}  // namespace

extern "C" {

int rst_trainer_create(const rst_shape* shape, const float* weights_host, size_t num_weights,
                       const rst_loss_shape* loss, const float* vgg_weights_host, size_t num_vgg_weights,
                       rst_trainer** out) {
    return rst_trainer_create_ex(shape, weights_host, num_weights, loss, vgg_weights_host, num_vgg_weights,
                                 RST_PRECISION_FP32, out);
}

int rst_trainer_create_ex(const rst_shape* shape, const float* weights_host, size_t num_weights,
                          const rst_loss_shape* loss, const float* vgg_weights_host, size_t num_vgg_weights,
                          int precision, rst_trainer** out) {
    if (!shape || !weights_host || !loss || !vgg_weights_host || !out)
        return set_error(RST_ERR_INVALID, "rst_trainer_create: null argument");
    *out = nullptr;
    if (precision != RST_PRECISION_FP32 && precision != RST_PRECISION_FP32_WINOGRAD &&
        precision != RST_PRECISION_WINOGRAD_BF16X6)
        return set_error(RST_ERR_INVALID, "rst_trainer_create_ex: transfer-network precision must be FP32, "
                                          "FP32_WINOGRAD or WINOGRAD_BF16X6");
    if (shape->num_styles != 1)
        return set_error(RST_ERR_UNSUPPORTED, "rst_trainer_create: num_styles must be 1 (train_network.py:55)");
    if (shape->max_batch <= 0) return set_error(RST_ERR_INVALID, "rst_trainer_create: max_batch must be positive");
    if (loss->h != shape->out_h || loss->w != shape->out_w || loss->max_batch != shape->max_batch)
        return set_error(RST_ERR_INVALID, "rst_trainer_create: loss shape must match out_h, out_w, max_batch");
    std::vector<LayerSpec> specs;
    int P = 0;
    int st = build_plan(shape, specs, &P);
    if (st != RST_OK) return st;
    size_t expect = 0;
    for (auto& s : specs) expect += layer_weight_count(s);
    if (expect != num_weights)
        return set_error(RST_ERR_INVALID, "rst_trainer_create: expected " + std::to_string(expect) + " weights, got " +
                                              std::to_string(num_weights));
    for (auto& s : specs)
        if (s.stride == 2 && (s.keras_kind == 0 ? (s.H % 2 || s.W % 2) : false))
            return set_error(RST_ERR_UNSUPPORTED, "rst_trainer_create: odd size at stride-2 layer " + s.name +
                                                      " (its input gradient needs the even-size phase split)");
    rst_trainer* t = new rst_trainer();
    // (A CU-masked targets stream that left 16 / 32 / 64 CUs to the caller's stream ran the config-4 step at 41.5 / 38.7 /
    // 38.9 ms against 20.7 ms unmasked, same box: profiles/r06/r06i. Not used.)
    const hipError_t se = hipStreamCreateWithFlags(&t->side, hipStreamNonBlocking);
    if (se != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&t->ev_gstyle, hipEventDisableTiming) != hipSuccess)
        return fail_delete(t, set_error(RST_ERR_HIP, "rst_trainer_create_ex: stream / event creation failed"));
    {
        const char* ser = getenv("RST_SERIAL_TARGETS");
        t->serial_targets = ser != nullptr && ser[0] == '1';
        const char* vg = getenv("RST_VGG_GRAD_F32");
        t->vgg_grad_f32 = vg != nullptr && vg[0] == '1';
        const char* twt = getenv("RST_TRAIN_WT");
        t->wt_stores = twt != nullptr ? atoi(twt) : 5;   // default: the transfer convs' outputs (-1.4 %, -0.4 % per step)
    }
    t->shape = *shape;
    t->P = P;
    t->nw = expect;
    if ((st = rst_loss_create(loss, vgg_weights_host, num_vgg_weights, &t->loss)) != RST_OK) return fail_delete(t, st);
    const int B = shape->max_batch;
    if ((st = t->alloc(&t->d_wc, expect * 4, weights_host)) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_ms, expect * 4)) != RST_OK) return fail_delete(t, st);

    size_t off = 0, max_out = 0, slab = 0;
    int max_ntot = 512;
    long max_nb = 0;
    t->L.resize(specs.size());
    for (size_t li = 0; li < specs.size(); ++li) {
        TLayer& T = t->L[li];
        const LayerSpec& s = specs[li];
        T.e.s = s;
        T.kcount = (size_t)s.k * s.k * s.cin * s.cout;
        T.woff = off;
        T.boff = off + T.kcount;
        off += T.kcount + s.cout;
        if (s.norm == N_BN) {
            T.goff = off;
            off += 4 * (size_t)s.cout;
        }
        // gather maps: pack (canonical index + 1) through the same packing code as inference
        std::vector<float> kidx(T.kcount), bidx(s.cout);
        for (size_t i = 0; i < T.kcount; ++i) kidx[i] = (float)(T.woff + i + 1);
        for (int c = 0; c < s.cout; ++c) bidx[c] = (float)(T.boff + c + 1);
        std::vector<float> packed, bias_n;
        // residual convs on Winograd when asked (their prologue always materialises the input for wgrad)
        // and the 9x9 start conv on the composite Winograd kernel (training mode: raw ReLU output + tile stats)
        // WINOGRAD_BF16X6: residual convs (forward, input gradient, weight gradient) and the start conv's
        // forward on the split-bf16 x6 kernels (wino9_x6.hip in its training mode)
        const bool wmode = precision == RST_PRECISION_FP32_WINOGRAD || precision == RST_PRECISION_WINOGRAD_BF16X6;
        const int lp = !wmode || (s.res_block < 0 && li != 0) ? RST_PRECISION_FP32 : precision;
        if ((st = prepare_layer(T.e, s, kidx.data(), bidx.data(), packed, bias_n, lp)) != RST_OK)
            return fail_delete(t, st);
        T.wino_fwd = T.e.kind == K_WINO || T.e.kind == K_WINOX6 || T.e.kind == K_WINO9 || T.e.kind == K_WINO9X6;
        if (T.e.kind == K_WINO9) T.e.n_part = T.e.tiles_y * T.e.tiles_x;   // batch statistics per tile
        if (T.e.kind == K_WINO9X6) T.e.n_part = 2 * T.e.tiles_y * T.e.tiles_x;   // per 16 x 8 M block
        std::vector<int> mw = T.wino_fwd ? std::vector<int>() : to_map(packed), mb = to_map(bias_n);
        T.n_w = packed.size();
        T.n_b = mb.size();
        if (!T.wino_fwd && (st = t->alloc(&T.d_map_w, mw.size() * 4, mw.data())) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&T.d_map_b, mb.size() * 4, mb.data())) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&T.e.d_w, T.n_w * 4)) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&T.e.d_bias, mb.size() * 4)) != RST_OK) return fail_delete(t, st);
        const size_t nout = (size_t)B * s.Ho * s.Wo * s.cout;
        if ((st = t->alloc(&T.e.d_out, nout * 4)) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&T.e.d_part, (size_t)B * T.e.ntot * T.e.n_part * sizeof(float4))) != RST_OK)
            return fail_delete(t, st);
        if ((st = t->alloc(&T.e.d_ab, (size_t)B * s.cout * sizeof(float2))) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&T.d_mr, (size_t)B * s.cout * sizeof(float2))) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&T.d_g, nout * 4)) != RST_OK) return fail_delete(t, st);
        if (li > 0 && (st = t->alloc(&T.d_x, (size_t)B * s.H * s.W * s.cin * 4)) != RST_OK) return fail_delete(t, st);
        max_out = std::max(max_out, nout);
        max_ntot = std::max(max_ntot, T.e.ntot);
        // norm-backward partials: B * n_tiles <= 1024 + B for every batch (norm_tile_for)
        max_nb = std::max(max_nb, (long)s.cout * (1024 + B + 64));
        // input-gradient conv (none for the first layer: the content needs no gradient)
        if (li > 0) {
            LayerSpec ds = s;
            ds.name = s.name + "_dgrad";
            ds.cin = s.cout;
            ds.cout = s.cin;
            ds.H = s.Ho;
            ds.W = s.Wo;
            ds.Ho = s.H;
            ds.Wo = s.W;
            std::vector<float> kd;
            if (s.keras_kind == 0 && s.stride == 1) {
                // dX = correlation of dZ with the spatially flipped kernel, channels swapped
                const int taps = s.k * s.k;
                kd.resize(T.kcount);
                for (int tp = 0; tp < taps; ++tp)
                    for (int co = 0; co < s.cout; ++co)
                        for (int ci = 0; ci < s.cin; ++ci)
                            kd[((size_t)tp * s.cout + co) * s.cin + ci] =
                                kidx[((size_t)(taps - 1 - tp) * s.cin + ci) * s.cout + co];
                ds.keras_kind = 0;
            } else if (s.keras_kind == 0) {
                // stride-2 conv: its input gradient is the transposed conv of dZ with the same array
                kd = kidx;
                ds.keras_kind = 1;
            } else {
                // transposed conv: its input gradient is a conv of dZ with the same array (HWIO, in = cout)
                kd = kidx;
                ds.keras_kind = 0;
            }
            std::vector<float> zb(ds.cout, 0.f), pdg, bdg;
            if ((st = prepare_layer(T.dg, ds, kd.data(), zb.data(), pdg, bdg, lp)) != RST_OK) return fail_delete(t, st);
            if (T.dg.kind == K_SMALL) return fail_delete(t, set_error(RST_ERR_UNSUPPORTED, "dgrad kind"));
            T.dg.s = ds;
            T.wino_dg = T.dg.kind == K_WINO || T.dg.kind == K_WINOX6;
            std::vector<int> md = to_map(T.wino_dg ? kd : pdg);   // Winograd: canonical -> flipped HWIO
            T.n_dg = md.size();
            if ((st = t->alloc(&T.d_map_dg, md.size() * 4, md.data())) != RST_OK) return fail_delete(t, st);
            if ((st = t->alloc(&T.d_wdg, pdg.size() * 4)) != RST_OK) return fail_delete(t, st);
            if (T.wino_dg && (st = t->alloc(&T.d_kflip, kd.size() * 4)) != RST_OK) return fail_delete(t, st);
            T.has_dgrad = true;
            max_ntot = std::max(max_ntot, T.dg.ntot);
            max_out = std::max(max_out, (size_t)B * s.H * s.W * s.cin);
        }
        // same geometry as the launch (the split count and slab size depend on every field)
        WgradArgs w = wgrad_geometry(s, T.e, B);
        w.x6 = T.e.kind == K_WINOX6 || T.e.kind == K_WINO9X6 ? 1 : 0;   // as backward() sets it before choosing
        w.nsplit = wgrad_choose_splits(w);
        slab = std::max(slab, wgrad_slab_bytes(w));
    }
    // prologue wiring of the training forward (BatchNorm is no longer folded into the epilogue)
    for (size_t li = 1; li < t->L.size(); ++li) {
        TLayer& T = t->L[li];
        const TLayer& Pv = t->L[li - 1];
        if (Pv.e.s.post == P_RELU) {
            T.e.pro = PRO_AFF_RELU;
        } else if (Pv.e.s.res_block == 0) {
            T.e.pro = PRO_AFF;
        } else {
            T.e.pro = PRO_AFF_RES;
            T.e.pro_res = t->L[li - 2].d_x;   // input of the block = input of its conv0
        }
        if (T.e.kind == K_SMALL && Pv.e.s.post != P_RELU)
            return fail_delete(t, set_error(RST_ERR_UNSUPPORTED, "last layer must follow a ReLU expand block"));
    }
    for (auto& T : t->L) {
        if (T.e.kind != K_SMALL) {
            hipError_t pe = T.e.kind == K_WINO9    ? hipSuccess
                            : T.e.kind == K_WINO9X6 ? wino9_x6_prepare()
                            : T.e.kind == K_WINOX6 ? wino_x6_prepare()
                            : T.wino_fwd           ? wino_prepare()
                                                   : conv_prepare(T.e.tile);
            if (pe != hipSuccess) return fail_delete(t, set_error(RST_ERR_HIP, hipGetErrorString(pe)));
        }
        if (T.has_dgrad) {
            hipError_t pe = T.dg.kind == K_WINOX6 ? wino_x6_prepare() : T.wino_dg ? wino_prepare() : conv_prepare(T.dg.tile);
            if (pe != hipSuccess) return fail_delete(t, set_error(RST_ERR_HIP, hipGetErrorString(pe)));
        }
    }
    // ---- VGG16 input-gradient convs (frozen weights, packed once) and Gram-backward 1x1 maps
    {
        const std::vector<float>& vw = t->loss->host_w;
        size_t vo = 0;
        int cin = 3;
        for (int i = 0; i < 13; ++i) {
            const int cout = VGG_CH[i];
            const VggConv& c = t->loss->convs[i];
            std::vector<float> wd((size_t)9 * cin * cout);
            for (int tp = 0; tp < 9; ++tp)
                for (int co = 0; co < cout; ++co)
                    for (int ci = 0; ci < cin; ++ci) {
                        // conv0: the forward reads RGB with BGR-flipped weights after x*255 - mean
                        const int cs = i == 0 ? 2 - ci : ci;
                        const float v = vw[vo + ((size_t)(8 - tp) * cin + cs) * cout + co];
                        wd[((size_t)tp * cout + co) * cin + ci] = i == 0 ? 255.f * v : v;
                    }
            vo += (size_t)9 * cin * cout + cout;
            ConvBwd& vb = t->vgg[i];
            const int lp = loss->precision;
            const int planes = bf16_planes(lp);
            // bf16 gradients under bf16 ReLU masks (vgg_backward's `act`): the 16-B staging tiles
            const bool gmask = t->loss->act_bf16 && !t->vgg_grad_f32 && i > 0;
            const bool bf3 = planes > 0 && conv_bf3_select(3, 1, cout, cin, planes, (long long)B * c.H * c.W, &vb.tile,
                                                           false, gmask);
            if (!bf3 && !conv_select(3, 1, cout, cin, &vb.tile))
                return fail_delete(t, set_error(RST_ERR_UNSUPPORTED, "no tile for VGG dgrad " + std::to_string(i)));
            vb.tiles_y = (c.H + vb.tile.th - 1) / vb.tile.th;
            vb.tiles_x = (c.W + vb.tile.tw - 1) / vb.tile.tw;
            vb.n_blocks = (cin + vb.tile.nt - 1) / vb.tile.nt;
            vb.nchunks = (cout + vb.tile.ck - 1) / vb.tile.ck;
            std::vector<float> pk = vb.tile.bf3 ? pack_conv_tiles_bf3(wd, 9, cout, cin, vb.tile)
                                                : pack_conv_tiles(wd, 9, cout, cin, vb.tile);
            if ((st = t->alloc(&vb.d_w, pk.size() * 4, pk.data())) != RST_OK) return fail_delete(t, st);
            hipError_t pe = conv_prepare(vb.tile);
            if (pe != hipSuccess) return fail_delete(t, set_error(RST_ERR_HIP, hipGetErrorString(pe)));
            if (i == 0) {   // the 1x1 form used by vgg_backward: W1[ci][(tap, c)] = wd[tap][ci][c], 27 of 32 columns
                ConvBwd& pb = t->vgg0p;
                if (cin != 3 || !conv_select(1, 1, cout, 32, &pb.tile))
                    return fail_delete(t, set_error(RST_ERR_UNSUPPORTED, "no 1x1 tile for the VGG conv0 input gradient"));
                std::vector<float> w1((size_t)cout * 32, 0.f);
                for (int tp = 0; tp < 9; ++tp)
                    for (int co = 0; co < cout; ++co)
                        for (int ci = 0; ci < 3; ++ci) w1[(size_t)co * 32 + tp * 3 + ci] = wd[((size_t)tp * cout + co) * 3 + ci];
                pb.tiles_y = (c.H + pb.tile.th - 1) / pb.tile.th;
                pb.tiles_x = (c.W + pb.tile.tw - 1) / pb.tile.tw;
                pb.n_blocks = (32 + pb.tile.nt - 1) / pb.tile.nt;
                pb.nchunks = (cout + pb.tile.ck - 1) / pb.tile.ck;
                std::vector<float> pk1 = pack_conv_tiles(w1, 1, cout, 32, pb.tile);
                if ((st = t->alloc(&pb.d_w, pk1.size() * 4, pk1.data())) != RST_OK) return fail_delete(t, st);
                pe = conv_prepare(pb.tile);
                if (pe != hipSuccess) return fail_delete(t, set_error(RST_ERR_HIP, hipGetErrorString(pe)));
            }
            cin = cout;
        }
        size_t max_packed = 0;
        for (int k = 0; k < 4; ++k) {
            const VggConv& c = t->loss->convs[STYLE_IDX[k]];
            const int C = c.cout;
            ConvBwd& gb = t->gram[k];
            // plain-bf16 loss: the Gram backward dF = F W on bf16 operands as well (conv_bf3 1x1, the weights
            // rounded to bf16 when packed), the gradient of the bf16 Gram forward
            const bool gbf16 = loss->precision == RST_PRECISION_BF16 &&
                               conv_bf3_select(1, 1, C, C, 1, (long long)B * c.H * c.W, &gb.tile);
            if (!gbf16 && !conv_select(1, 1, C, C, &gb.tile))
                return fail_delete(t, set_error(RST_ERR_UNSUPPORTED, "no 1x1 tile for the Gram backward"));
            gb.tiles_y = (c.H + gb.tile.th - 1) / gb.tile.th;
            gb.tiles_x = (c.W + gb.tile.tw - 1) / gb.tile.tw;
            gb.n_blocks = (C + gb.tile.nt - 1) / gb.tile.nt;
            gb.nchunks = (C + gb.tile.ck - 1) / gb.tile.ck;
            std::vector<int> m;
            if (gbf16) {
                m = pack_conv_tiles_bf3_index(1, C, C, gb.tile);   // bf16 elements: n_packed / 2 floats per image
            } else {
                std::vector<float> idx((size_t)C * C);
                for (size_t i = 0; i < idx.size(); ++i) idx[i] = (float)(i + 1);
                m = to_map(pack_conv_tiles(idx, 1, C, C, gb.tile));
            }
            gb.n_packed = (int)m.size();
            max_packed = std::max(max_packed, gbf16 ? (m.size() + 1) / 2 : m.size());
            if ((st = t->alloc(&gb.d_map, m.size() * 4, m.data())) != RST_OK) return fail_delete(t, st);
            hipError_t pe = conv_prepare(gb.tile);
            if (pe != hipSuccess) return fail_delete(t, set_error(RST_ERR_HIP, hipGetErrorString(pe)));
        }
        if ((st = t->alloc(&t->d_gram_packed, (size_t)B * max_packed * 4)) != RST_OK) return fail_delete(t, st);
        const size_t img = (size_t)B * shape->out_h * shape->out_w;
        if ((st = t->alloc(&t->d_vg[0], img * 64 * 4)) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&t->d_vg[1], img * 64 * 4)) != RST_OK) return fail_delete(t, st);
        if ((st = t->alloc(&t->d_vpool, img * 16 * 4)) != RST_OK) return fail_delete(t, st);
    }
    if ((st = t->alloc(&t->d_zero, (size_t)max_ntot * 4)) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_dz, max_out * 4)) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_tmp, max_out * 4)) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_nb_part, (size_t)max_nb * sizeof(float2))) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_nb_consts, (size_t)B * 256 * sizeof(float2))) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_slab, slab)) != RST_OK) return fail_delete(t, st);
    if ((st = t->alloc(&t->d_gstyle, (size_t)B * P * 4)) != RST_OK) return fail_delete(t, st);
    {   // BN moving statistics in get_weights() order: per BN layer moving_mean[cout], moving_variance[cout]
        std::vector<int> idx;
        for (const TLayer& T : t->L)
            if (T.goff)
                for (int i = 0; i < 2 * T.e.s.cout; ++i) idx.push_back((int)(T.goff + 2 * T.e.s.cout + i));
        t->n_stat = idx.size();
        if (!idx.empty() && (st = t->alloc(&t->d_stat_index, idx.size() * 4, idx.data())) != RST_OK)
            return fail_delete(t, st);
    }
    // the last layer's output gradient is d(loss)/d(prediction), written by the VGG backward
    if ((st = repack(t, nullptr)) != RST_OK) return fail_delete(t, st);
    if (hipDeviceSynchronize() != hipSuccess) return fail_delete(t, set_error(RST_ERR_HIP, "rst_trainer_create sync"));
    *out = t;
    return RST_OK;
}

void rst_trainer_destroy(rst_trainer* t) { delete t; }

int rst_trainer_num_style_params(const rst_trainer* t) { return t ? t->P : -1; }
rst_loss_handle* rst_trainer_loss(rst_trainer* t) { return t ? t->loss : nullptr; }
size_t rst_trainer_num_weights(const rst_trainer* t) { return t ? t->nw : 0; }

int rst_trainer_compute_targets(rst_trainer* t, const float* gt_content, const float* gt_style, int batch,
                                void* stream) {
    if (!t || !gt_content || !gt_style) return set_error(RST_ERR_INVALID, "rst_trainer_compute_targets: null argument");
    if (batch <= 0 || batch > t->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_trainer_compute_targets: batch outside [1, max_batch]");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (t->targets_pending) {
        // targets of a step that never reached compute_gradients (its caller failed in between): join the side
        // stream's work into the caller's stream and start over (the new targets overwrite the same buffers
        // after that join)
        t->targets_pending = false;
        RST_HIP_TRY(hipStreamWaitEvent(st, t->ev_join, 0));
    }
    hipStream_t ts = t->serial_targets ? st : t->side;
    if (ts != st) {
        RST_HIP_TRY(hipEventRecord(t->ev_fork, st));
        RST_HIP_TRY(hipStreamWaitEvent(ts, t->ev_fork, 0));
    }
    int r = loss_targets(t->loss, gt_content, gt_style, batch, ts);
    RST_HIP_TRY(hipEventRecord(t->ev_join, ts));   // recorded even after a failed launch: joins stay balanced
    if (r != RST_OK) {
        RST_HIP_TRY(hipStreamWaitEvent(st, t->ev_join, 0));
        return r;
    }
    t->targets_pending = true;
    t->pend_content = gt_content;
    t->pend_style = gt_style;
    t->pend_batch = batch;
    return RST_OK;
}

int rst_trainer_compute_gradients(rst_trainer* t, const float* content, const float* style_params,
                                  const float* gt_content, const float* gt_style, int batch, float* prediction,
                                  float* losses, float* grad, float* grad_style_params, void* stream) {
    if (!t || !content || !style_params || !gt_content || !gt_style || !prediction || !losses || !grad)
        return set_error(RST_ERR_INVALID, "rst_trainer_compute_gradients: null argument");
    t->gstyle_recorded = false;   // a failure on any path below leaves no stale event for wait_style_gradient
    if (rst::guard_pad() != 0) rst::guard_check("before compute_gradients");   // diagnostic runs only
    if (batch <= 0 || batch > t->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_trainer_compute_gradients: batch outside [1, max_batch]");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int B = batch;
    int r;
    if (t->targets_pending && (t->pend_content != gt_content || t->pend_style != gt_style || t->pend_batch != B)) {
        t->targets_pending = false;
        RST_HIP_TRY(hipStreamWaitEvent(st, t->ev_join, 0));   // the side stream's work is joined either way
        return set_error(RST_ERR_INVALID, "rst_trainer_compute_gradients: targets started for other inputs");
    }
    if (!t->targets_pending && (r = rst_trainer_compute_targets(t, gt_content, gt_style, B, stream)) != RST_OK) return r;
    r = forward(t, content, style_params, B, prediction, st);
    t->targets_pending = false;                            // joined on every path, failed forward included
    RST_HIP_TRY(hipStreamWaitEvent(st, t->ev_join, 0));
    // diagnostic (race bisection): RST_RACE_DUMP=<prefix> writes the last layer's raw output, its statistics partials
    // and its input to <prefix>_{out,part,in}_<call>.bin after every forward
    static const char* dump = getenv("RST_RACE_DUMP");
    static int dump_call = 0;
    if (dump != nullptr && r == RST_OK) {
        const TLayer& T = t->L.back();
        const LayerExec& e = T.e;
        const size_t n_out = (size_t)B * e.s.Ho * e.s.Wo * e.s.cout, n_in = (size_t)B * e.s.H * e.s.W * e.s.cin;
        const size_t n_part = (size_t)B * e.ntot * e.n_part * 4;
        RST_HIP_TRY(hipStreamSynchronize(st));
        const struct { const char* tag; const float* p; size_t n; } items[3] = {
            {"out", e.d_out, n_out}, {"part", reinterpret_cast<const float*>(e.d_part), n_part}, {"in", T.d_x, n_in}};
        for (const auto& it : items) {
            std::vector<float> h(it.n);
            RST_HIP_TRY(hipMemcpy(h.data(), it.p, it.n * 4, hipMemcpyDeviceToHost));
            const std::string fn = std::string(dump) + "_" + it.tag + "_" + std::to_string(dump_call) + ".bin";
            FILE* f = fopen(fn.c_str(), "wb");
            if (f != nullptr) {
                fwrite(h.data(), 4, h.size(), f);
                fclose(f);
            }
        }
        ++dump_call;
    }
    if (r != RST_OK) return r;
    if ((r = loss_prediction(t->loss, prediction, B, losses, st)) != RST_OK) return r;
    if ((r = vgg_backward(t, prediction, B, t->L.back().d_g, st)) != RST_OK) return r;
    RST_HIP_TRY(hipMemsetAsync(grad, 0, t->nw * 4, st));
    float* gs = grad_style_params ? grad_style_params : t->d_gstyle;
    RST_HIP_TRY(hipMemsetAsync(gs, 0, (size_t)B * t->P * 4, st));
    if ((r = backward(t, content, B, grad, gs, st)) != RST_OK) return r;
    t->gstyle_recorded = true;
    return RST_OK;
}

int rst_trainer_wait_style_gradient(rst_trainer* t, void* stream) {
    if (!t) return set_error(RST_ERR_INVALID, "rst_trainer_wait_style_gradient: null handle");
    if (!t->gstyle_recorded)
        return set_error(RST_ERR_INVALID, "rst_trainer_wait_style_gradient: no completed rst_trainer_compute_gradients");
    RST_HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(stream), t->ev_gstyle, 0));
    return RST_OK;
}

int rst_trainer_apply_gradients(rst_trainer* t, const float* grad, float learning_rate, float rho, float epsilon,
                                void* stream) {
    if (!t || !grad) return set_error(RST_ERR_INVALID, "rst_trainer_apply_gradients: null argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    RST_HIP_TRY(rmsprop_launch(t->d_wc, t->d_ms, grad, t->nw, learning_rate, rho, epsilon, st));
    return repack(t, st);
}

int rst_trainer_copy_weights(rst_trainer* t, float* dst, size_t count, void* stream) {
    if (!t || !dst || count != t->nw) return set_error(RST_ERR_INVALID, "rst_trainer_copy_weights: bad argument");
    RST_HIP_TRY(hipMemcpyAsync(dst, t->d_wc, count * 4, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

int rst_trainer_copy_slots(rst_trainer* t, float* dst, size_t count, void* stream) {
    if (!t || !dst || count != t->nw) return set_error(RST_ERR_INVALID, "rst_trainer_copy_slots: bad argument");
    RST_HIP_TRY(hipMemcpyAsync(dst, t->d_ms, count * 4, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

int rst_trainer_set_slots(rst_trainer* t, const float* src, size_t count, void* stream) {
    if (!t || !src || count != t->nw) return set_error(RST_ERR_INVALID, "rst_trainer_set_slots: bad argument");
    RST_HIP_TRY(hipMemcpyAsync(t->d_ms, src, count * 4, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

int rst_trainer_cancel_targets(rst_trainer* t, void* stream) {
    if (!t) return set_error(RST_ERR_INVALID, "rst_trainer_cancel_targets: null handle");
    if (t->targets_pending) {
        t->targets_pending = false;
        RST_HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(stream), t->ev_join, 0));
    }
    return RST_OK;
}

int rst_trainer_copy_output_gradient(rst_trainer* t, int layer, float* dst, size_t count, int batch, void* stream) {
    if (!t || !dst || layer < 0 || layer >= (int)t->L.size())
        return set_error(RST_ERR_INVALID, "rst_trainer_copy_output_gradient: bad argument");
    const LayerSpec& s = t->L[layer].e.s;
    const size_t n = (size_t)batch * s.Ho * s.Wo * s.cout;
    if (count != n) return set_error(RST_ERR_INVALID, "rst_trainer_copy_output_gradient: count mismatch");
    RST_HIP_TRY(hipMemcpyAsync(dst, t->L[layer].d_g, n * 4, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

int rst_trainer_debug_vgg_gradient(rst_trainer* t, int layer, float* dst, size_t count, int batch, void* stream) {
    if (!t || layer < 0 || layer > CONTENT_IDX) return set_error(RST_ERR_INVALID, "rst_trainer_debug_vgg_gradient");
    const VggConv& c = t->loss->convs[layer];
    const size_t full = (size_t)t->shape.max_batch * c.H * c.W * c.cout;
    if (!t->d_vgg_dbg[layer]) {   // first call only arms the tap (allocation: not for the hot path)
        int st = t->alloc(&t->d_vgg_dbg[layer], full * 4);
        return st;
    }
    const size_t n = (size_t)batch * c.H * c.W * c.cout;
    if (!dst || count != n) return set_error(RST_ERR_INVALID, "rst_trainer_debug_vgg_gradient: count mismatch");
    RST_HIP_TRY(hipMemcpyAsync(dst, t->d_vgg_dbg[layer], n * 4, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

size_t rst_trainer_num_moving_statistics(const rst_trainer* t) { return t ? t->n_stat : 0; }

int rst_trainer_get_moving_statistics(rst_trainer* t, float* dst, size_t count, void* stream) {
    if (!t || !dst || count != t->n_stat) return set_error(RST_ERR_INVALID, "rst_trainer_get_moving_statistics: bad argument");
    if (count) RST_HIP_TRY(gather_launch(t->d_wc, t->d_stat_index, dst, count, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

int rst_trainer_set_moving_statistics(rst_trainer* t, const float* src, size_t count, float divisor, void* stream) {
    if (!t || !src || count != t->n_stat || !(divisor > 0.f))
        return set_error(RST_ERR_INVALID, "rst_trainer_set_moving_statistics: bad argument");
    // no re-pack: no packed kernel image is derived from the moving statistics in training mode
    RST_HIP_TRY(scatter_div_launch(src, t->d_stat_index, t->d_wc, count, divisor, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

int rst_trainer_set_weights(rst_trainer* t, const float* src, size_t count, void* stream) {
    if (!t || !src || count != t->nw) return set_error(RST_ERR_INVALID, "rst_trainer_set_weights: bad argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    RST_HIP_TRY(hipMemcpyAsync(t->d_wc, src, count * 4, hipMemcpyDeviceToDevice, st));
    return repack(t, st);
}

}  // extern "C"
