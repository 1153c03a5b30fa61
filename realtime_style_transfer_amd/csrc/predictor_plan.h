// predictor_plan.h — layer plan of the style predictor, shared by inference (predictor_api.hip) and
// training (predictor_train_api.hip).
//
// create_style_prediction_model (realtime_style_transfer/models/stylePrediction.py:25-75) with the
// MobileNetV3Small trunk as Keras 2.9 builds it (keras/applications/mobilenet_v3.py; restated in
// oracle/predictor_ref.py): every conv unit (conv -> BatchNormalization -> activation) with its
// input/shortcut/SE wiring and the offsets of its weights in the Keras get_weights() order.
#pragma once
#include <algorithm>
#include <cstddef>
#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "predictor.h"

namespace rst {

enum PUnitKind { PU_STEM = 0, PU_PW = 1, PU_DW = 2, PU_DUMMY = 3 };

struct PUnit {
    int kind;
    int H = 0, W = 0, cin = 0, Ho = 0, Wo = 0, cout = 0, k = 1, stride = 1, pad_t = 0, pad_l = 0;
    int act = ACT_NONE;     // after BN
    size_t woff = 0;        // conv kernel (Keras layout == the kernels' layout: HWIO / [cin][cout] / [k][k][C])
    size_t goff = 0;        // BN gamma (beta +C, moving_mean +2C, moving_variance +3C); DUMMY: conv bias
    int in = -1;            // unit whose output feeds this conv (-1: network input)
    int se = -1;            // SE block scaling this conv's input (project convs), -1: none
    int res = -1;           // unit whose output is added after BN (shortcut), -1: none
    int block = -1;         // inverted-residual block index (stem: -1)
    bool stage = false;     // debug stage (stem, block outputs, features)
};

struct PSE {
    int C = 0, R = 0, Ho = 0, Wo = 0;
    int src = -1;           // depthwise unit whose activated output is squeezed and scaled
    size_t w1 = 0, b1 = 0, w2 = 0, b2 = 0;
};

struct PPlan {
    std::vector<PUnit> units;
    std::vector<PSE> ses;
    int feat_unit = -1, feat_c = 0, feat_hw = 0;
    size_t head_w1 = 0, head_b1 = 0, head_w2 = 0, head_b2 = 0;
    size_t total = 0;       // number of weights
};

struct MbBlockDef {
    double expansion;
    int filters, k, stride;
    bool se;
    int act;
};
// keras mobilenet_v3.MobileNetV3Small stack_fn (alpha 1.0, minimalistic False)
inline const MbBlockDef* mobilenet_v3_small_blocks() {
    static const MbBlockDef B[11] = {
        {1.0, 16, 3, 2, true, ACT_RELU},          {72.0 / 16, 24, 3, 2, false, ACT_RELU},
        {88.0 / 24, 24, 3, 1, false, ACT_RELU},   {4.0, 40, 5, 2, true, ACT_HSWISH},
        {6.0, 40, 5, 1, true, ACT_HSWISH},        {6.0, 40, 5, 1, true, ACT_HSWISH},
        {3.0, 48, 5, 1, true, ACT_HSWISH},        {3.0, 48, 5, 1, true, ACT_HSWISH},
        {6.0, 96, 5, 2, true, ACT_HSWISH},        {6.0, 96, 5, 1, true, ACT_HSWISH},
        {6.0, 96, 5, 1, true, ACT_HSWISH},
    };
    return B;
}

inline int make_divisible(double v, int divisor = 8) {   // mobilenet_v3._depth
    int nv = std::max(divisor, (int)(v + divisor / 2.0) / divisor * divisor);
    if (nv < 0.9 * v) nv += divisor;
    return nv;
}

inline void same_pad(int n, int k, int s, int* out, int* before) {
    *out = (n + s - 1) / s;
    const int total = std::max((*out - 1) * s + k - n, 0);
    *before = total / 2;
}

inline int build_predictor_plan(const rst_predictor_shape* s, PPlan* P) {
    if (!s || s->h <= 0 || s->w <= 0 || s->c <= 0 || s->num_top_parameters <= 0 || s->num_style_parameters <= 0 ||
        s->max_batch <= 0)
        return set_error(RST_ERR_INVALID, "rst_predictor_shape: all dimensions must be positive");
    if (s->num_style_parameters > 1024)
        return set_error(RST_ERR_UNSUPPORTED, "rst_predictor: num_style_parameters > 1024");
    *P = PPlan();
    size_t off = 0;
    auto take = [&](size_t n) { const size_t o = off; off += n; return o; };
    int H = s->h, W = s->w, C = s->c;
    if (s->feature_extractor == RST_EXTRACTOR_DUMMY) {
        PUnit u{PU_DUMMY};
        u.H = H; u.W = W; u.cin = C; u.k = 9; u.stride = 5; u.cout = 1;
        same_pad(H, 9, 5, &u.Ho, &u.pad_t);
        same_pad(W, 9, 5, &u.Wo, &u.pad_l);
        u.woff = take((size_t)81 * C);
        u.goff = take(1);
        u.stage = true;
        P->units.push_back(u);
        P->feat_unit = 0;
        P->feat_c = 1;
        P->feat_hw = u.Ho * u.Wo;
    } else if (s->feature_extractor == RST_EXTRACTOR_MOBILE_NET) {
        if (C != 3) return set_error(RST_ERR_INVALID, "rst_predictor: MobileNetV3Small takes 3-channel images");
        PUnit st{PU_STEM};   // Conv2D(16, 3, s2, same, no bias) -> BN -> hard_swish
        st.H = H; st.W = W; st.cin = 3; st.cout = 16; st.k = 3; st.stride = 2; st.act = ACT_HSWISH;
        same_pad(H, 3, 2, &st.Ho, &st.pad_t);
        same_pad(W, 3, 2, &st.Wo, &st.pad_l);
        st.woff = take(3 * 3 * 3 * 16);
        st.goff = take(4 * 16);
        st.stage = true;
        P->units.push_back(st);
        H = st.Ho; W = st.Wo; C = 16;
        int cur = 0;
        const MbBlockDef* blocks = mobilenet_v3_small_blocks();
        for (int bi = 0; bi < 11; ++bi) {
            const MbBlockDef& blk = blocks[bi];
            const int shortcut = cur, cin = C;
            const int ce = make_divisible(cin * blk.expansion);
            if (bi) {   // 1x1 expand -> BN -> act
                PUnit u{PU_PW};
                u.H = u.Ho = H; u.W = u.Wo = W; u.cin = cin; u.cout = ce; u.act = blk.act; u.in = cur; u.block = bi;
                u.woff = take((size_t)cin * ce);
                u.goff = take(4 * (size_t)ce);
                P->units.push_back(u);
                cur = (int)P->units.size() - 1;
            }
            PUnit d{PU_DW};   // [ZeroPadding2D(correct_pad)] DepthwiseConv2D -> BN -> act
            d.H = H; d.W = W; d.cin = d.cout = ce; d.k = blk.k; d.stride = blk.stride; d.act = blk.act; d.in = cur;
            d.block = bi;
            if (blk.stride == 2) {
                const int c = blk.k / 2;
                d.pad_t = c - (1 - H % 2);
                d.pad_l = c - (1 - W % 2);
                d.Ho = (H + d.pad_t + c - blk.k) / 2 + 1;
                d.Wo = (W + d.pad_l + c - blk.k) / 2 + 1;
            } else {
                same_pad(H, blk.k, 1, &d.Ho, &d.pad_t);
                same_pad(W, blk.k, 1, &d.Wo, &d.pad_l);
            }
            d.woff = take((size_t)blk.k * blk.k * ce);
            d.goff = take(4 * (size_t)ce);
            P->units.push_back(d);
            const int dw = (int)P->units.size() - 1;
            int se = -1;
            if (blk.se) {   // GAP -> Conv2D(R, 1) -> ReLU -> Conv2D(C, 1) -> hard_sigmoid -> x * se
                PSE e;
                e.C = ce; e.R = make_divisible(ce * 0.25); e.Ho = d.Ho; e.Wo = d.Wo; e.src = dw;
                e.w1 = take((size_t)ce * e.R);
                e.b1 = take(e.R);
                e.w2 = take((size_t)e.R * ce);
                e.b2 = take(ce);
                P->ses.push_back(e);
                se = (int)P->ses.size() - 1;
            }
            H = d.Ho; W = d.Wo;
            PUnit pj{PU_PW};   // 1x1 project -> BN [+ shortcut]
            pj.H = pj.Ho = H; pj.W = pj.Wo = W; pj.cin = ce; pj.cout = blk.filters; pj.act = ACT_NONE; pj.in = dw;
            pj.se = se; pj.block = bi; pj.stage = true;
            pj.woff = take((size_t)ce * blk.filters);
            pj.goff = take(4 * (size_t)blk.filters);
            if (blk.stride == 1 && cin == blk.filters) pj.res = shortcut;
            P->units.push_back(pj);
            cur = (int)P->units.size() - 1;
            C = blk.filters;
        }
        const int last = make_divisible(C * 6.0);   // Conv_1: 1x1 -> BN -> hard_swish
        PUnit u{PU_PW};
        u.H = u.Ho = H; u.W = u.Wo = W; u.cin = C; u.cout = last; u.act = ACT_HSWISH; u.in = cur; u.stage = true;
        u.woff = take((size_t)C * last);
        u.goff = take(4 * (size_t)last);
        P->units.push_back(u);
        P->feat_unit = (int)P->units.size() - 1;
        P->feat_c = last;
        P->feat_hw = H * W;
    } else {
        return set_error(RST_ERR_UNSUPPORTED, "rst_predictor: feature_extractor must be DUMMY or MOBILE_NET "
                                              "(EFFICIENT_NET is not built)");
    }
    const int NS = s->num_style_parameters, NP = s->num_top_parameters, CF = P->feat_c;
    P->head_w1 = take((size_t)CF * NS);
    P->head_b1 = take(NS);
    P->head_w2 = take((size_t)NS * NP);
    P->head_b2 = take(NP);
    P->total = off;
    return RST_OK;
}

}  // namespace rst
