// loss_api.hip — C ABI of the VGG16 / Gram style loss (include/rst.h, rst_loss_*).
//
// Restates StyleLossModelVGG (realtime_style_transfer/models/styleLoss.py:69-109) and
// make_style_loss_function (:295-369) without the MiDaS depth term (a remote TF-Hub model):
//   x*255 -> vgg16.preprocess_input ('caffe': RGB->BGR, minus [103.939, 116.779, 123.68])
//   -> keras VGG16 trunk (13 x Conv3x3 s1 SAME + ReLU, 4 x MaxPool2) up to block5_conv3;
//   feature_loss = mean_l2(F5(pred) - F5(gt_content)) * content_factor          (:324-328)
//   style_loss   = mean over block{1,2}_conv2, block{3,4}_conv3 of
//                  mean_l2(G(pred) - G(style)) * style_factor                    (:330-335)
//   tv_loss      = total_variation(pred) * tv_factor                             (:337-338)
//   loss         = feature + style + tv                                          (:344-346)
// mean_l2(t) = mean(0.5 t^2) per image (:290-292). The preprocess is folded into the first conv:
// its input channels are flipped (BGR) in the packed weights and the prologue applies
// y = 255 x - mean per channel, so SAME zero padding still applies to the preprocessed image.
// Every conv runs on conv_mfma_kernel (f32 MFMA) or, in a bf16 precision mode, conv_bf3 (block1_conv1 in the
// plain-bf16 mode: vgg_conv0_bf16); Gram matrices on gram.hip; reductions on loss.hip.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "kernels.h"
#include "lossnet.h"

using namespace rst;

namespace rst {
int vgg_run(rst_loss_handle* h, const float* img, int B, int last, hipStream_t st) {
    const float* in = img;
    for (int i = 0; i <= last; ++i) {
        VggConv& c = h->convs[i];
        if (c.d_w0bf != nullptr) {   // plain-bf16 loss: block1_conv1 on bf16 operands, preprocess fused
            RST_HIP_TRY(vgg_conv0_bf16_launch(in, h->d_pre, c.d_w0bf, c.d_b, c.d_out, B, c.H, c.W, st, h->act_bf16));
            in = c.d_out;
            continue;
        }
        ConvArgs a{};
        a.in = in;
        a.pro_ab = i == 0 ? h->d_pre : nullptr;
        a.wpk = c.d_w;
        a.bias = c.d_b;
        a.out = c.d_out;
        a.batch = B;
        a.H = c.H;
        a.W = c.W;
        a.cin = c.cin;
        a.Ho = c.H;
        a.Wo = c.W;
        a.ntot = c.cout;
        a.cout = c.cout;
        a.pad_t = a.pad_l = 1;
        a.tiles_y = c.tiles_y;
        a.tiles_x = c.tiles_x;
        a.n_blocks = c.n_blocks;
        a.nchunks = c.nchunks;
        a.pro_mode = i == 0 ? PRO_AFF : PRO_NONE;
        a.epi_mode = EPI_RELU_STATS;   // part == nullptr: bias + ReLU only
        a.shuffle = 0;
        // the block-end max pool inside the conv's epilogue where the tile allows it (one pass over the block's
        // output fewer), else its own launch
        const bool pool = c.pool_after && i < last;
        const bool fused = pool && c.tile.bf3 && conv_bf3_fuses_pool(c.tile, a);
        if (fused) a.pool = c.d_pool;
        // write-through output stores (sc1, the VGG epilogue of conv_bf3) where the offsets fit 32 bits
        a.wt_stores = h->wt_stores && c.tile.bf3 && (size_t)B * c.H * c.W * c.cout * 4 < (size_t)0x7FFFFFF0 ? 1 : 0;
        // bf16 layer outputs: this conv reads its input (the previous conv's or pool's bf16 output; conv 0 here only in
        // the f32 modes) and stores its output and fused pool as bf16
        if (h->act_bf16) a.act_bf16 = (i > 0 ? 1 : 0) | 2;
        RST_HIP_TRY(conv_launch(c.tile, a, st));
        in = c.d_out;
        if (pool) {
            if (!fused && h->act_bf16) return set_error(RST_ERR_UNSUPPORTED, "bf16 VGG16 activations need the fused pool");
            if (!fused) RST_HIP_TRY(maxpool2_launch(c.d_out, c.d_pool, B, c.H, c.W, c.cout, st));
            in = c.d_pool;
        }
    }
    return RST_OK;
}

int loss_targets(rst_loss_handle* h, const float* gt_content, const float* gt_style, int B, hipStream_t st) {
    // plain-bf16 loss: the Gram matrices on bf16-rounded features as well (mixed_bfloat16 compute dtype)
    const bool gram_bf16 = h->shape.precision == RST_PRECISION_BF16;
    int r;
    // diagnostic (race bisection): RST_TARGETS_PARTS bit 0 style VGG16, 1 its Grams, 2 content VGG16, 3 the content
    // copy (default all); the losses are meaningless without all four
    static const int parts = [] {
        const char* v = getenv("RST_TARGETS_PARTS");
        return v != nullptr ? atoi(v) : 15;
    }();
    // style image: grams of the four style layers
    if ((parts & 1) && (r = vgg_run(h, gt_style, B, STYLE_IDX[3], st)) != RST_OK) return r;
    for (int k = 0; k < 4 && (parts & 2); ++k) {
        const VggConv& c = h->convs[STYLE_IDX[k]];
        RST_HIP_TRY(gram_launch(c.d_out, B, c.H * c.W, c.cout, h->d_gram_style[k], h->d_gram_ws, st, gram_bf16,
                                h->act_bf16));
    }
    // ground-truth content: block5_conv3 features
    if ((parts & 4) && (r = vgg_run(h, gt_content, B, CONTENT_IDX, st)) != RST_OK) return r;
    const VggConv& c5 = h->convs[CONTENT_IDX];
    const size_t f5 = (size_t)c5.H * c5.W * c5.cout;
    if (parts & 8)
        RST_HIP_TRY(hipMemcpyAsync(h->d_content_feat, c5.d_out, (size_t)B * f5 * (h->act_bf16 ? 2 : 4),
                                   hipMemcpyDeviceToDevice, st));
    return RST_OK;
}

int loss_prediction(rst_loss_handle* h, const float* prediction, int B, float* losses, hipStream_t st) {
    const bool gram_bf16 = h->shape.precision == RST_PRECISION_BF16;
    int r;
    const VggConv& c5 = h->convs[CONTENT_IDX];
    const size_t f5 = (size_t)c5.H * c5.W * c5.cout;
    if ((r = vgg_run(h, prediction, B, CONTENT_IDX, st)) != RST_OK) return r;
    RST_HIP_TRY(sqdiff_loss_launch(c5.d_out, h->d_content_feat, B, (long)f5, h->d_partial,
                                   0.5 / (double)f5 * h->shape.content_factor, losses, 4, 1, 0, st, h->act_bf16));
    for (int k = 0; k < 4; ++k) {
        const VggConv& c = h->convs[STYLE_IDX[k]];
        RST_HIP_TRY(gram_launch(c.d_out, B, c.H * c.W, c.cout, h->d_gram_pred[k], h->d_gram_ws, st, gram_bf16,
                                h->act_bf16));
        const long n = (long)c.cout * c.cout;
        RST_HIP_TRY(sqdiff_loss_launch(h->d_gram_pred[k], h->d_gram_style[k], B, n, h->d_partial,
                                       0.5 / (double)n / 4.0 * h->shape.style_factor, losses, 4, 2, k > 0, st));
    }
    RST_HIP_TRY(tv_loss_launch(prediction, B, h->shape.h, h->shape.w, 3, h->d_partial, h->shape.tv_factor, losses, 4,
                               3, st));
    RST_HIP_TRY(loss_combine_launch(losses, B, st));
    return RST_OK;
}

}  // namespace rst

extern "C" {

size_t rst_loss_num_weights(void) {
    size_t n = 0;
    int cin = 3;
    for (int i = 0; i < 13; ++i) {
        n += (size_t)9 * cin * VGG_CH[i] + VGG_CH[i];
        cin = VGG_CH[i];
    }
    return n;
}

int rst_loss_create(const rst_loss_shape* shape, const float* vgg_weights_host, size_t num_weights,
                    rst_loss_handle** out) {
    if (!shape || !vgg_weights_host || !out) return set_error(RST_ERR_INVALID, "rst_loss_create: null argument");
    *out = nullptr;
    if (shape->h % 16 != 0 || shape->w % 16 != 0 || shape->h <= 0 || shape->w <= 0 || shape->max_batch <= 0)
        return set_error(RST_ERR_INVALID, "rst_loss_create: image H and W must be positive multiples of 16 "
                                          "(four 2x2 max-pools)");
    if (shape->precision < RST_PRECISION_FP32 || shape->precision > RST_PRECISION_BF16 ||
        shape->precision == RST_PRECISION_FP32_WINOGRAD)
        return set_error(RST_ERR_INVALID, "rst_loss_create: unknown precision mode");
    if (num_weights != rst_loss_num_weights())
        return set_error(RST_ERR_INVALID, "rst_loss_create: expected " + std::to_string(rst_loss_num_weights()) +
                                              " VGG16 weights, got " + std::to_string(num_weights));
    rst_loss_handle* h = new rst_loss_handle();
    {
        const char* wt = getenv("RST_LOSS_WT");
        h->wt_stores = wt != nullptr && wt[0] == '1' ? 1 : 0;
        const char* af = getenv("RST_VGG_ACT_F32");
        h->act_bf16 = shape->precision == RST_PRECISION_BF16 && !(af != nullptr && af[0] == '1');
    }
    const size_t es = h->act_bf16 ? 2 : 4;   // bytes per stored VGG16 activation
    h->shape = *shape;
    h->host_w.assign(vgg_weights_host, vgg_weights_host + num_weights);
    const int B = shape->max_batch;
    int H = shape->h, W = shape->w, cin = 3;
    const float* wp = vgg_weights_host;
    int st;
    for (int i = 0; i < 13; ++i) {
        VggConv c{};
        c.cin = cin;
        c.cout = VGG_CH[i];
        c.H = H;
        c.W = W;
        c.pool_after = VGG_POOL[i];
        const size_t kc = (size_t)9 * cin * c.cout;
        std::vector<float> Wg(wp, wp + kc);
        if (i == 0) {   // RGB -> BGR: preprocessed channel c' = 2 - c reads input channel c
            for (int tap = 0; tap < 9; ++tap)
                for (int ci = 0; ci < 3; ++ci)
                    for (int co = 0; co < c.cout; ++co)
                        Wg[((size_t)tap * 3 + ci) * c.cout + co] = wp[((size_t)tap * 3 + (2 - ci)) * c.cout + co];
        }
        const float* bias = wp + kc;
        wp += kc + c.cout;
        const int planes = bf16_planes(shape->precision);
        const bool bf3 = planes > 0 && conv_bf3_select(3, 1, cin, c.cout, planes, (long long)B * H * W, &c.tile,
                                                       h->act_bf16 && i > 0);
        if (!bf3 && !conv_select(3, 1, cin, c.cout, &c.tile)) {
            delete h;
            return set_error(RST_ERR_UNSUPPORTED, "no conv tile configuration for VGG layer " + std::to_string(i));
        }
        c.tiles_y = (H + c.tile.th - 1) / c.tile.th;
        c.tiles_x = (W + c.tile.tw - 1) / c.tile.tw;
        c.n_blocks = (c.cout + c.tile.nt - 1) / c.tile.nt;
        c.nchunks = (cin + c.tile.ck - 1) / c.tile.ck;
        std::vector<float> pk = c.tile.bf3 ? pack_conv_tiles_bf3(Wg, 9, cin, c.cout, c.tile)
                                           : pack_conv_tiles(Wg, 9, cin, c.cout, c.tile);
        if ((st = h->alloc(&c.d_w, pk.size() * 4, pk.data())) != RST_OK) { delete h; return st; }
        if (i == 0 && shape->precision == RST_PRECISION_BF16) {   // mixed_bfloat16: block1_conv1 in bf16 as well
            const std::vector<unsigned short> w0 = vgg_conv0_bf16_pack(Wg.data());
            if ((st = h->alloc(&c.d_w0bf, w0.size() * 2, w0.data())) != RST_OK) { delete h; return st; }
        }
        if ((st = h->alloc(&c.d_b, (size_t)c.cout * 4, bias)) != RST_OK) { delete h; return st; }
        if ((st = h->alloc(&c.d_out, (size_t)B * H * W * c.cout * es)) != RST_OK) { delete h; return st; }
        if (c.pool_after)
            if ((st = h->alloc(&c.d_pool, (size_t)B * (H / 2) * (W / 2) * c.cout * es)) != RST_OK) { delete h; return st; }
        hipError_t pe = conv_prepare(c.tile);
        if (pe != hipSuccess) { delete h; return set_error(RST_ERR_HIP, hipGetErrorString(pe)); }
        h->convs.push_back(c);
        if (c.pool_after) { H /= 2; W /= 2; }
        cin = c.cout;
    }
    // preprocess affine (per image, per input channel c: y = 255 x - mean_bgr[2 - c])
    std::vector<float2> pre((size_t)B * 3);
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < 3; ++c) pre[(size_t)b * 3 + c] = make_float2(255.f, (float)(-VGG_MEAN_BGR[2 - c]));
    if ((st = h->alloc(&h->d_pre, pre.size() * sizeof(float2), pre.data())) != RST_OK) { delete h; return st; }
    const VggConv& c5 = h->convs[CONTENT_IDX];
    if ((st = h->alloc(&h->d_content_feat, (size_t)B * c5.H * c5.W * c5.cout * es)) != RST_OK) { delete h; return st; }
    size_t ws = 0;
    for (int k = 0; k < 4; ++k) {
        const VggConv& c = h->convs[STYLE_IDX[k]];
        if ((st = h->alloc(&h->d_gram_style[k], (size_t)B * c.cout * c.cout * 4)) != RST_OK) { delete h; return st; }
        if ((st = h->alloc(&h->d_gram_pred[k], (size_t)B * c.cout * c.cout * 4)) != RST_OK) { delete h; return st; }
        ws = std::max(ws, gram_workspace_bytes(B, c.H * c.W, c.cout));
    }
    if ((st = h->alloc((char**)&h->d_gram_ws, ws)) != RST_OK) { delete h; return st; }
    h->gram_ws_bytes = ws;
    if ((st = h->alloc(&h->d_partial, (size_t)B * 1024 * 4)) != RST_OK) { delete h; return st; }
    *out = h;
    return RST_OK;
}

void rst_loss_destroy(rst_loss_handle* h) { delete h; }

int rst_loss_forward(rst_loss_handle* h, const float* prediction, const float* gt_content, const float* gt_style,
                     int batch, float* losses, void* stream) {
    if (!h || !prediction || !gt_content || !gt_style || !losses)
        return set_error(RST_ERR_INVALID, "rst_loss_forward: null argument");
    if (batch <= 0 || batch > h->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_loss_forward: batch outside [1, max_batch]");
    hipStream_t st = static_cast<hipStream_t>(stream);
    int r;
    if ((r = loss_targets(h, gt_content, gt_style, batch, st)) != RST_OK) return r;
    return loss_prediction(h, prediction, batch, losses, st);
}

int rst_loss_copy_feature(rst_loss_handle* h, int layer, float* dst, size_t count, int batch, void* stream) {
    if (!h || layer < 0 || layer >= 13 || !dst) return set_error(RST_ERR_INVALID, "rst_loss_copy_feature: bad argument");
    const VggConv& c = h->convs[layer];
    const size_t n = (size_t)batch * c.H * c.W * c.cout;
    if (count != n) return set_error(RST_ERR_INVALID, "rst_loss_copy_feature: count mismatch");
    if (h->act_bf16)   // the stored bf16 layer output, widened (exactly) to f32
        RST_HIP_TRY(bf16_to_f32_launch(c.d_out, dst, n, static_cast<hipStream_t>(stream)));
    else
        RST_HIP_TRY(hipMemcpyAsync(dst, c.d_out, n * 4, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
    return RST_OK;
}

}  // extern "C"
