// lossnet.h — VGG16 loss network internals shared by loss_api.hip and train_api.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "kernels.h"

namespace rst {
struct VggConv {
    int cin, cout, H, W;     // input dims (output H, W equal: SAME, stride 1)
    bool pool_after;
    ConvTile tile;
    int tiles_y, tiles_x, n_blocks, nchunks;
    float* d_w = nullptr;
    float* d_b = nullptr;
    float* d_out = nullptr;  // [B][H][W][cout]
    float* d_pool = nullptr; // [B][H/2][W/2][cout] when pool_after
    unsigned short* d_w0bf = nullptr;   // block1_conv1, plain-bf16 loss: vgg_conv0_bf16 B image (else null)
};

const int VGG_CH[13] = {64, 64, 128, 128, 256, 256, 256, 512, 512, 512, 512, 512, 512};
const bool VGG_POOL[13] = {false, true, false, true, false, false, true, false, false, true, false, false, false};
const int STYLE_IDX[4] = {1, 3, 6, 9};   // block1_conv2, block2_conv2, block3_conv3, block4_conv3
const int CONTENT_IDX = 12;              // block5_conv3
const double VGG_MEAN_BGR[3] = {103.939, 116.779, 123.68};

}  // namespace rst

struct rst_loss_handle {
    rst_loss_shape shape;
    std::vector<rst::VggConv> convs;
    std::vector<void*> allocs;
    float2* d_pre = nullptr;              // preprocess affine [max_batch][3]
    float* d_content_feat = nullptr;      // F5(gt_content)
    float* d_gram_style[4] = {nullptr, nullptr, nullptr, nullptr};
    float* d_gram_pred[4] = {nullptr, nullptr, nullptr, nullptr};
    void* d_gram_ws = nullptr;
    float* d_partial = nullptr;
    size_t gram_ws_bytes = 0;
    int wt_stores = 0;                    // RST_LOSS_WT at creation: VGG conv outputs stored write-through (sc1)
    bool act_bf16 = false;                // plain-bf16 loss: every VGG16 layer output (conv, pool, the content
                                          // target) stored as bf16 bits, as Keras mixed_bfloat16 layers emit them
                                          // (RST_VGG_ACT_F32=1 at creation: f32 storage, for A/B runs)
    std::vector<float> host_w;            // VGG16 weights as given (Keras order), for the backward packing
    ~rst_loss_handle() {
        for (void* p : allocs) rst::guard_free(p);
    }
    template <typename T>
    int alloc(T** p, size_t bytes, const void* src = nullptr) {
        if (rst::guard_malloc((void**)p, bytes) != hipSuccess) return rst::set_error(RST_ERR_ALLOC, "hipMalloc failed");
        allocs.push_back((void*)*p);
        if (src && hipMemcpy(*p, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
            return rst::set_error(RST_ERR_HIP, "hipMemcpy failed");
        return RST_OK;
    }
};

namespace rst {
// Run the VGG16 trunk on B images up to (and including) conv `last`; conv outputs land in convs[i].d_out.
int vgg_run(rst_loss_handle* h, const float* img, int B, int last, hipStream_t st);
// rst_loss_forward in two parts: the ground-truth targets (style-image Grams, content-image block5_conv3
// features; independent of the prediction) and the prediction's VGG16 pass + the loss terms. Both use the same
// per-layer VGG16 buffers: the targets must be complete before loss_prediction runs.
int loss_targets(rst_loss_handle* h, const float* gt_content, const float* gt_style, int B, hipStream_t st);
int loss_prediction(rst_loss_handle* h, const float* prediction, int B, float* losses, hipStream_t st);
}  // namespace rst

