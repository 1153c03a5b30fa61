// predictor_api.hip — C ABI of the style predictor (include/rst.h, rst_predictor_*).
//
// Restates create_style_prediction_model (realtime_style_transfer/models/stylePrediction.py:25-75):
// feature extractor (DUMMY: Conv2D(1, 9, s5, same) :31-32; MOBILE_NET: Rescaling(2,-1) +
// keras.applications.MobileNetV3Small(include_top=False, include_preprocessing=False) :33-38),
// GlobalAveragePooling2D :55, StylePredictor Conv2D(100, 1) :60-64, StyleNormPredictor
// Conv2D(P, 1) :67-71, squeeze :73. The MobileNetV3Small layer list (Keras 2.9
// keras/applications/mobilenet_v3.py) is derived below from the input size exactly as Keras builds
// it; weights arrive in Keras get_weights() order and BatchNormalization (inference: moving
// statistics, eps 1e-3) is folded into a per-channel affine at create time.
//
// The style predictor runs once per style image (predict_video_using_checkpoint.py:77-83 caches
// the parameters; styleTransferInferenceModel.py:23-26 runs it per call): every buffer is
// allocated once for max_batch, rst_predictor_forward only launches kernels on the caller's stream
// (hipGraph-capturable).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "predictor.h"

using namespace rst;

namespace {

constexpr float BN_EPS = 1e-3f;

struct MbBlock {
    double expansion;
    int filters, k, stride;
    bool se;
    int act;
};
// keras mobilenet_v3.MobileNetV3Small stack_fn (alpha 1.0, minimalistic False)
const MbBlock MOBILENET_V3_SMALL[11] = {
    {1.0, 16, 3, 2, true, ACT_RELU},          {72.0 / 16, 24, 3, 2, false, ACT_RELU},
    {88.0 / 24, 24, 3, 1, false, ACT_RELU},   {4.0, 40, 5, 2, true, ACT_HSWISH},
    {6.0, 40, 5, 1, true, ACT_HSWISH},        {6.0, 40, 5, 1, true, ACT_HSWISH},
    {3.0, 48, 5, 1, true, ACT_HSWISH},        {3.0, 48, 5, 1, true, ACT_HSWISH},
    {6.0, 96, 5, 2, true, ACT_HSWISH},        {6.0, 96, 5, 1, true, ACT_HSWISH},
    {6.0, 96, 5, 1, true, ACT_HSWISH},
};

int make_divisible(double v, int divisor = 8) {   // mobilenet_v3._depth
    int nv = std::max(divisor, (int)(v + divisor / 2.0) / divisor * divisor);
    if (nv < 0.9 * v) nv += divisor;
    return nv;
}

void same_pad(int n, int k, int s, int* out, int* before) {
    *out = (n + s - 1) / s;
    const int total = std::max((*out - 1) * s + k - n, 0);
    *before = total / 2;
}

enum OpType { OP_STEM = 0, OP_DUMMY = 1, OP_PW = 2, OP_DW = 3, OP_SE = 4 };

struct Op {
    int type;
    int H = 0, W = 0, cin = 0, Ho = 0, Wo = 0, cout = 0, k = 1, stride = 1, pad_t = 0, pad_l = 0, act = ACT_NONE;
    int in = -1, out = -1, res = -1, se = -1, part = -1;   // buffer indices (-1: none / network input)
    int n_part = 0, hw = 0, r = 0;                          // SE
    size_t w = 0, ba = 0, bb = 0, b1 = 0, w2 = 0, b2 = 0;  // offsets into the device parameter image
    int stage = -1;                                          // debug stage index of the output
};

}  // namespace

struct rst_predictor {
    rst_predictor_shape shape;
    std::vector<Op> ops;
    std::vector<float*> bufs;            // per-op outputs + SE partials / scales, [max_batch][...]
    std::vector<size_t> buf_elems;       // per image
    std::vector<int> stage_buf;          // debug stages -> buffer
    std::vector<int> stage_hwc;          // 3 per stage
    int feat_buf = -1, feat_hw = 0, feat_c = 0;
    int feat_part = -1, feat_nparts = 0; // per-tile channel sums of the features (global average pool)
    float* d_params = nullptr;           // packed parameter image (kernels' layouts)
    float* d_hidden = nullptr;           // [max_batch][num_style_parameters]
    size_t head_w1 = 0, head_b1 = 0, head_w2 = 0, head_b2 = 0;
    std::vector<void*> allocs;
    ~rst_predictor() {
        for (void* p : allocs) (void)hipFree(p);
    }
};

namespace {

// Host-side plan + parameter packing. Consumes the Keras-ordered weights when `wsrc` is non-null;
// with wsrc == nullptr it only counts them (rst_predictor_num_weights).
struct Builder {
    const float* wsrc;
    size_t wpos = 0;
    std::vector<float> params;    // device parameter image
    rst_predictor* p;

    const float* take(size_t n) {
        const float* r = wsrc ? wsrc + wpos : nullptr;
        wpos += n;
        return r;
    }
    size_t put(const float* src, size_t n) {
        const size_t off = params.size();
        params.resize(off + ((n + 3) & ~size_t(3)), 0.f);   // keep every array 16-byte aligned
        if (src) std::copy(src, src + n, params.begin() + off);
        return off;
    }
    // BatchNormalization(eps 1e-3): gamma, beta, moving_mean, moving_variance -> (a, b)
    void bn(int C, size_t* oa, size_t* ob) {
        const float* g = take(C);
        const float* be = take(C);
        const float* m = take(C);
        const float* v = take(C);
        std::vector<float> a(C, 1.f), b(C, 0.f);
        if (wsrc)
            for (int c = 0; c < C; ++c) {
                const double s = (double)g[c] / std::sqrt((double)v[c] + (double)BN_EPS);
                a[c] = (float)s;
                b[c] = (float)((double)be[c] - (double)m[c] * s);
            }
        *oa = put(a.data(), C);
        *ob = put(b.data(), C);
    }
    int new_buf(size_t per_image) {
        p->buf_elems.push_back(per_image);
        return (int)p->buf_elems.size() - 1;
    }
    void stage(int buf, int H, int W, int C) {
        p->stage_buf.push_back(buf);
        p->stage_hwc.insert(p->stage_hwc.end(), {H, W, C});
    }
};

int build(Builder& B, const rst_predictor_shape* s) {
    rst_predictor* P = B.p;
    int H = s->h, W = s->w, C = s->c;
    if (s->feature_extractor == RST_EXTRACTOR_DUMMY) {
        Op op{OP_DUMMY};
        op.H = H; op.W = W; op.cin = C; op.k = 9; op.stride = 5; op.cout = 1;
        same_pad(H, 9, 5, &op.Ho, &op.pad_t);
        same_pad(W, 9, 5, &op.Wo, &op.pad_l);
        op.w = B.put(B.take((size_t)81 * C), (size_t)81 * C);
        op.ba = B.put(B.take(1), 1);
        op.out = B.new_buf((size_t)op.Ho * op.Wo);
        op.part = B.new_buf((size_t)dummy_conv_parts(op.Ho * op.Wo));
        B.stage(op.out, op.Ho, op.Wo, 1);
        P->ops.push_back(op);
        P->feat_buf = op.out;
        P->feat_hw = op.Ho * op.Wo;
        P->feat_c = 1;
        P->feat_part = op.part;
        P->feat_nparts = dummy_conv_parts(op.Ho * op.Wo);
        return RST_OK;
    }
    if (s->feature_extractor != RST_EXTRACTOR_MOBILE_NET)
        return set_error(RST_ERR_UNSUPPORTED, "rst_predictor: feature_extractor must be DUMMY or MOBILE_NET "
                                              "(EFFICIENT_NET is not built)");
    if (C != 3) return set_error(RST_ERR_INVALID, "rst_predictor: MobileNetV3Small takes 3-channel images");
    // stem: Conv2D(16, 3, s2, same, no bias) -> BN -> hard_swish
    {
        Op op{OP_STEM};
        op.H = H; op.W = W; op.cin = 3; op.cout = 16; op.k = 3; op.stride = 2; op.act = ACT_HSWISH;
        same_pad(H, 3, 2, &op.Ho, &op.pad_t);
        same_pad(W, 3, 2, &op.Wo, &op.pad_l);
        op.w = B.put(B.take(3 * 3 * 3 * 16), 3 * 3 * 3 * 16);
        B.bn(16, &op.ba, &op.bb);
        op.out = B.new_buf((size_t)op.Ho * op.Wo * 16);
        B.stage(op.out, op.Ho, op.Wo, 16);
        P->ops.push_back(op);
        H = op.Ho; W = op.Wo; C = 16;
    }
    int cur = P->ops.back().out;
    for (int bi = 0; bi < 11; ++bi) {
        const MbBlock& blk = MOBILENET_V3_SMALL[bi];
        const int shortcut = cur;
        const int cin = C;
        const int ce = make_divisible(cin * blk.expansion);
        if (bi) {   // expand
            Op op{OP_PW};
            op.H = op.Ho = H; op.W = op.Wo = W; op.cin = cin; op.cout = ce; op.act = blk.act; op.in = cur;
            op.w = B.put(B.take((size_t)cin * ce), (size_t)cin * ce);
            B.bn(ce, &op.ba, &op.bb);
            op.out = B.new_buf((size_t)H * W * ce);
            P->ops.push_back(op);
            cur = op.out;
        }
        Op dw{OP_DW};
        dw.H = H; dw.W = W; dw.cin = dw.cout = ce; dw.k = blk.k; dw.stride = blk.stride; dw.act = blk.act; dw.in = cur;
        if (blk.stride == 2) {   // ZeroPadding2D(correct_pad) + 'valid'
            const int c = blk.k / 2;
            dw.pad_t = c - (1 - H % 2);
            dw.pad_l = c - (1 - W % 2);
            dw.Ho = (H + dw.pad_t + c - blk.k) / 2 + 1;
            dw.Wo = (W + dw.pad_l + c - blk.k) / 2 + 1;
        } else {
            same_pad(H, blk.k, 1, &dw.Ho, &dw.pad_t);
            same_pad(W, blk.k, 1, &dw.Wo, &dw.pad_l);
        }
        dw.w = B.put(B.take((size_t)blk.k * blk.k * ce), (size_t)blk.k * blk.k * ce);
        B.bn(ce, &dw.ba, &dw.bb);
        dw.out = B.new_buf((size_t)dw.Ho * dw.Wo * ce);
        int se_buf = -1;
        Op se{OP_SE};
        if (blk.se) {
            int block, slots, ppw, n_wg;
            dw_geometry(ce, dw.Ho * dw.Wo, &block, &slots, &ppw, &n_wg);
            dw.part = B.new_buf((size_t)n_wg * ce);
            dw.n_part = n_wg;
            const int r = make_divisible(ce * 0.25);
            se.cin = ce; se.r = r; se.part = dw.part; se.n_part = n_wg; se.hw = dw.Ho * dw.Wo;
            se.w = B.put(B.take((size_t)ce * r), (size_t)ce * r);
            se.b1 = B.put(B.take(r), r);
            se.w2 = B.put(B.take((size_t)r * ce), (size_t)r * ce);
            se.b2 = B.put(B.take(ce), ce);
            se.out = se_buf = B.new_buf(ce);
        }
        P->ops.push_back(dw);
        if (blk.se) P->ops.push_back(se);
        H = dw.Ho; W = dw.Wo;
        cur = dw.out;
        Op pj{OP_PW};   // project (+ SE scale on its input, + shortcut)
        pj.H = pj.Ho = H; pj.W = pj.Wo = W; pj.cin = ce; pj.cout = blk.filters; pj.act = ACT_NONE; pj.in = cur;
        pj.se = se_buf;
        pj.w = B.put(B.take((size_t)ce * blk.filters), (size_t)ce * blk.filters);
        B.bn(blk.filters, &pj.ba, &pj.bb);
        if (blk.stride == 1 && cin == blk.filters) pj.res = shortcut;
        pj.out = B.new_buf((size_t)H * W * blk.filters);
        B.stage(pj.out, H, W, blk.filters);
        P->ops.push_back(pj);
        cur = pj.out;
        C = blk.filters;
    }
    // Conv_1: 1x1 to _depth(C * 6) = 576, BN, hard_swish
    const int last = make_divisible(C * 6.0);
    Op op{OP_PW};
    op.H = op.Ho = H; op.W = op.Wo = W; op.cin = C; op.cout = last; op.act = ACT_HSWISH; op.in = cur;
    op.w = B.put(B.take((size_t)C * last), (size_t)C * last);
    B.bn(last, &op.ba, &op.bb);
    op.out = B.new_buf((size_t)H * W * last);
    op.part = B.new_buf((size_t)pw_parts(H * W) * last);
    B.stage(op.out, H, W, last);
    P->ops.push_back(op);
    P->feat_buf = op.out;
    P->feat_hw = H * W;
    P->feat_c = last;
    P->feat_part = op.part;
    P->feat_nparts = pw_parts(H * W);
    return RST_OK;
}

int build_all(Builder& B, const rst_predictor_shape* s) {
    if (!s || s->h <= 0 || s->w <= 0 || s->c <= 0 || s->num_top_parameters <= 0 || s->num_style_parameters <= 0 ||
        s->max_batch <= 0)
        return set_error(RST_ERR_INVALID, "rst_predictor_shape: all dimensions must be positive");
    if (s->num_style_parameters > 1024)
        return set_error(RST_ERR_UNSUPPORTED, "rst_predictor: num_style_parameters > 1024");
    int st = build(B, s);
    if (st != RST_OK) return st;
    const int C = B.p->feat_c, NS = s->num_style_parameters, P = s->num_top_parameters;
    B.p->head_w1 = B.put(B.take((size_t)C * NS), (size_t)C * NS);
    B.p->head_b1 = B.put(B.take(NS), NS);
    B.p->head_w2 = B.put(B.take((size_t)NS * P), (size_t)NS * P);
    B.p->head_b2 = B.put(B.take(P), P);
    return RST_OK;
}

}  // namespace

extern "C" {

size_t rst_predictor_num_weights(const rst_predictor_shape* shape) {
    rst_predictor tmp;
    Builder B{nullptr};
    B.p = &tmp;
    if (build_all(B, shape) != RST_OK) return 0;
    return B.wpos;
}

int rst_predictor_create(const rst_predictor_shape* shape, const float* weights_host, size_t num_weights,
                         rst_predictor** out) {
    if (!shape || !weights_host || !out) return set_error(RST_ERR_INVALID, "rst_predictor_create: null argument");
    *out = nullptr;
    const size_t want = rst_predictor_num_weights(shape);
    if (want == 0) return RST_ERR_INVALID;
    if (num_weights != want)
        return set_error(RST_ERR_INVALID, "rst_predictor_create: expected " + std::to_string(want) + " weights, got " +
                                              std::to_string(num_weights));
    rst_predictor* p = new rst_predictor();
    p->shape = *shape;
    Builder B{weights_host};
    B.p = p;
    int st = build_all(B, shape);
    if (st != RST_OK) { delete p; return st; }
    auto alloc = [&](float** d, size_t n) -> int {
        if (hipMalloc((void**)d, std::max<size_t>(n, 1) * sizeof(float)) != hipSuccess) {
            *d = nullptr;
            return set_error(RST_ERR_ALLOC, "rst_predictor_create: hipMalloc failed");
        }
        p->allocs.push_back(*d);
        return RST_OK;
    };
    if ((st = alloc(&p->d_params, B.params.size())) != RST_OK) { delete p; return st; }
    if (hipMemcpy(p->d_params, B.params.data(), B.params.size() * sizeof(float), hipMemcpyHostToDevice) !=
        hipSuccess) {
        delete p;
        return set_error(RST_ERR_HIP, "rst_predictor_create: hipMemcpy failed");
    }
    for (size_t e : p->buf_elems) {
        float* d;
        if ((st = alloc(&d, e * shape->max_batch)) != RST_OK) { delete p; return st; }
        p->bufs.push_back(d);
    }
    if ((st = alloc(&p->d_hidden, (size_t)shape->num_style_parameters * shape->max_batch)) != RST_OK) {
        delete p;
        return st;
    }
    *out = p;
    return RST_OK;
}

void rst_predictor_destroy(rst_predictor* p) { delete p; }

int rst_predictor_forward(rst_predictor* p, const float* style, int batch, float* style_params, void* stream) {
    if (!p || !style || !style_params) return set_error(RST_ERR_INVALID, "rst_predictor_forward: null argument");
    if (batch < 1 || batch > p->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_predictor_forward: batch outside [1, max_batch]");
    hipStream_t st = (hipStream_t)stream;
    const float* prm = p->d_params;
    auto buf = [&](int i) -> float* { return i < 0 ? nullptr : p->bufs[i]; };
    for (const Op& op : p->ops) {
        const float* in = op.in < 0 ? style : buf(op.in);
        switch (op.type) {
            case OP_STEM:
                RST_HIP_TRY(stem_launch(style, prm + op.w, prm + op.ba, prm + op.bb, buf(op.out), batch, op.H, op.W,
                                        op.Ho, op.Wo, op.pad_t, op.pad_l, st));
                break;
            case OP_DUMMY:
                RST_HIP_TRY(dummy_conv_launch(style, prm + op.w, prm + op.ba, buf(op.out), buf(op.part), batch, op.H,
                                              op.W, op.cin, op.Ho, op.Wo, op.pad_t, op.pad_l, st));
                break;
            case OP_PW:
                RST_HIP_TRY(pw_launch(in, buf(op.se), prm + op.w, prm + op.ba, prm + op.bb, buf(op.res), buf(op.out),
                                      buf(op.part), batch, op.H * op.W, op.cin, op.cout, op.act, st));
                break;
            case OP_DW:
                RST_HIP_TRY(dw_launch(in, prm + op.w, prm + op.ba, prm + op.bb, buf(op.out), buf(op.part), batch, op.H,
                                      op.W, op.cin, op.Ho, op.Wo, op.k, op.stride, op.pad_t, op.pad_l, op.act, st));
                break;
            case OP_SE:
                RST_HIP_TRY(se_launch(buf(op.part), op.n_part, op.hw, batch, op.cin, op.r, prm + op.w, prm + op.b1,
                                      prm + op.w2, prm + op.b2, buf(op.out), st));
                break;
        }
    }
    RST_HIP_TRY(head_launch(buf(p->feat_part), p->feat_nparts, p->feat_hw, batch, p->feat_c,
                            p->shape.num_style_parameters, p->shape.num_top_parameters, prm + p->head_w1,
                            prm + p->head_b1, prm + p->head_w2, prm + p->head_b2, p->d_hidden, style_params,
                            p->shape.num_top_parameters, st));
    return RST_OK;
}

int rst_predictor_num_stages(const rst_predictor* p) { return p ? (int)p->stage_buf.size() : 0; }

int rst_predictor_stage_shape(const rst_predictor* p, int idx, int* hwc3) {
    if (!p || !hwc3 || idx < 0 || idx >= (int)p->stage_buf.size())
        return set_error(RST_ERR_INVALID, "rst_predictor_stage_shape: bad argument");
    for (int i = 0; i < 3; ++i) hwc3[i] = p->stage_hwc[3 * idx + i];
    return RST_OK;
}

int rst_predictor_copy_stage(rst_predictor* p, int idx, float* dst, size_t count, int batch, void* stream) {
    if (!p || !dst || idx < 0 || idx >= (int)p->stage_buf.size() || batch < 1 || batch > p->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_predictor_copy_stage: bad argument");
    const size_t n = (size_t)p->stage_hwc[3 * idx] * p->stage_hwc[3 * idx + 1] * p->stage_hwc[3 * idx + 2] * batch;
    if (count != n) return set_error(RST_ERR_INVALID, "rst_predictor_copy_stage: count mismatch");
    RST_HIP_TRY(hipMemcpyAsync(dst, p->bufs[p->stage_buf[idx]], n * sizeof(float), hipMemcpyDeviceToDevice,
                               (hipStream_t)stream));
    return RST_OK;
}

}  // extern "C"
