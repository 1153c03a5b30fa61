// predictor_api.hip — C ABI of the style predictor, inference (include/rst.h, rst_predictor_*).
//
// Restates create_style_prediction_model (realtime_style_transfer/models/stylePrediction.py:25-75):
// feature extractor (DUMMY: Conv2D(1, 9, s5, same) :31-32; MOBILE_NET: Rescaling(2,-1) +
// keras.applications.MobileNetV3Small(include_top=False, include_preprocessing=False) :33-38),
// GlobalAveragePooling2D :55, StylePredictor Conv2D(100, 1) :60-64, StyleNormPredictor
// Conv2D(P, 1) :67-71, squeeze :73. The layer plan (predictor_plan.h) is derived from the input
// size exactly as Keras builds it. The Keras weight layouts are the kernels' layouts, so the
// get_weights() list is uploaded as-is; BatchNormalization (inference: moving statistics, eps 1e-3)
// is folded into a per-channel affine (a, b) at create time.
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
#include "predictor_plan.h"

using namespace rst;

constexpr float PRED_BN_EPS = 1e-3f;

struct rst_predictor {
    rst_predictor_shape shape;
    PPlan plan;
    float* d_w = nullptr;                 // the Keras-ordered weights
    float* d_ab = nullptr;                // folded BN per unit: a at ab_off[u], b at ab_off[u] + C
    std::vector<size_t> ab_off;
    std::vector<float*> out;              // per unit: activated output [max_batch][Ho][Wo][cout]
    std::vector<float*> se_part, se_val;  // per SE block: squeeze partials [B][n_wg][C], scale [B][C]
    std::vector<int> se_nwg;
    std::vector<int> se_of_dw;            // unit -> SE block fed by this depthwise unit (or -1)
    float* feat_part = nullptr;           // per-tile channel sums of the features (global average pool)
    int feat_nparts = 0;
    float* d_hidden = nullptr;            // [max_batch][num_style_parameters]
    std::vector<int> stage_unit;
    std::vector<void*> allocs;
    ~rst_predictor() {
        for (void* p : allocs) (void)hipFree(p);
    }
    int alloc(float** d, size_t n) {
        if (hipMalloc((void**)d, std::max<size_t>(n, 1) * sizeof(float)) != hipSuccess) {
            *d = nullptr;
            return set_error(RST_ERR_ALLOC, "rst_predictor: hipMalloc failed");
        }
        allocs.push_back(*d);
        return RST_OK;
    }
};

namespace rst {
// shared with the trainer: stage list = units flagged in the plan
std::vector<int> predictor_stage_units(const PPlan& P) {
    std::vector<int> s;
    for (size_t i = 0; i < P.units.size(); ++i)
        if (P.units[i].stage) s.push_back((int)i);
    return s;
}
}  // namespace rst

extern "C" {

size_t rst_predictor_num_weights(const rst_predictor_shape* shape) {
    PPlan P;
    if (build_predictor_plan(shape, &P) != RST_OK) return 0;
    return P.total;
}

int rst_predictor_create(const rst_predictor_shape* shape, const float* weights_host, size_t num_weights,
                         rst_predictor** out) {
    if (!shape || !weights_host || !out) return set_error(RST_ERR_INVALID, "rst_predictor_create: null argument");
    *out = nullptr;
    rst_predictor* p = new rst_predictor();
    p->shape = *shape;
    int st = build_predictor_plan(shape, &p->plan);
    if (st != RST_OK) { delete p; return st; }
    const PPlan& P = p->plan;
    if (num_weights != P.total) {
        delete p;
        return set_error(RST_ERR_INVALID, "rst_predictor_create: expected " + std::to_string(P.total) +
                                              " weights, got " + std::to_string(num_weights));
    }
    for (const PUnit& u : P.units)
        if ((u.kind == PU_PW || u.kind == PU_DW) && (u.woff % 4) != 0) {   // float4 weight loads
            delete p;
            return set_error(RST_ERR_UNSUPPORTED, "rst_predictor_create: misaligned weight offset");
        }
    // fold BatchNormalization into (a, b) per unit
    std::vector<float> ab;
    for (const PUnit& u : P.units) {
        p->ab_off.push_back(ab.size());
        const int C = u.cout;
        if (u.kind == PU_DUMMY) {
            ab.push_back(1.f);
            ab.push_back(weights_host[u.goff]);   // conv bias
            continue;
        }
        std::vector<float> a(C), b(C);
        const float* g = weights_host + u.goff;
        for (int c = 0; c < C; ++c) {
            const double s = (double)g[c] / std::sqrt((double)g[3 * C + c] + (double)PRED_BN_EPS);
            a[c] = (float)s;
            b[c] = (float)((double)g[C + c] - (double)g[2 * C + c] * s);
        }
        ab.insert(ab.end(), a.begin(), a.end());
        ab.insert(ab.end(), b.begin(), b.end());
        while (ab.size() % 4) ab.push_back(0.f);   // keep every unit's (a, b) 16-byte aligned
        // b must also be 16-byte aligned: C is a multiple of 8 for every BN unit
    }
    const int B = shape->max_batch;
    if ((st = p->alloc(&p->d_w, P.total)) != RST_OK || (st = p->alloc(&p->d_ab, ab.size())) != RST_OK) {
        delete p;
        return st;
    }
    if (hipMemcpy(p->d_w, weights_host, P.total * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p->d_ab, ab.data(), ab.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        delete p;
        return set_error(RST_ERR_HIP, "rst_predictor_create: hipMemcpy failed");
    }
    p->se_of_dw.assign(P.units.size(), -1);
    for (size_t i = 0; i < P.units.size(); ++i) {
        const PUnit& u = P.units[i];
        float* d;
        if ((st = p->alloc(&d, (size_t)B * u.Ho * u.Wo * u.cout)) != RST_OK) { delete p; return st; }
        p->out.push_back(d);
    }
    for (size_t e = 0; e < P.ses.size(); ++e) {
        const PSE& s = P.ses[e];
        int block, slots, ppw, n_wg;
        dw_geometry(s.C, s.Ho * s.Wo, &block, &slots, &ppw, &n_wg);
        float *part, *val;
        if ((st = p->alloc(&part, (size_t)B * n_wg * s.C)) != RST_OK || (st = p->alloc(&val, (size_t)B * s.C)) != RST_OK) {
            delete p;
            return st;
        }
        p->se_part.push_back(part);
        p->se_val.push_back(val);
        p->se_nwg.push_back(n_wg);
        p->se_of_dw[s.src] = (int)e;
    }
    const PUnit& fu = P.units[P.feat_unit];
    p->feat_nparts = fu.kind == PU_DUMMY ? dummy_conv_parts(fu.Ho * fu.Wo) : pw_parts(fu.Ho * fu.Wo);
    if ((st = p->alloc(&p->feat_part, (size_t)B * p->feat_nparts * P.feat_c)) != RST_OK ||
        (st = p->alloc(&p->d_hidden, (size_t)B * shape->num_style_parameters)) != RST_OK) {
        delete p;
        return st;
    }
    p->stage_unit = predictor_stage_units(P);
    *out = p;
    return RST_OK;
}

void rst_predictor_destroy(rst_predictor* p) { delete p; }

int rst_predictor_forward(rst_predictor* p, const float* style, int batch, float* style_params, void* stream) {
    if (!p || !style || !style_params) return set_error(RST_ERR_INVALID, "rst_predictor_forward: null argument");
    if (batch < 1 || batch > p->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_predictor_forward: batch outside [1, max_batch]");
    hipStream_t st = (hipStream_t)stream;
    const PPlan& P = p->plan;
    const float* w = p->d_w;
    for (size_t i = 0; i < P.units.size(); ++i) {
        const PUnit& u = P.units[i];
        const float* in = u.in < 0 ? style : p->out[u.in];
        const float* a = p->d_ab + p->ab_off[i];
        const float* b = a + u.cout;
        const bool feat = (int)i == P.feat_unit;
        switch (u.kind) {
            case PU_STEM:
                RST_HIP_TRY(stem_launch(style, w + u.woff, a, b, p->out[i], batch, u.H, u.W, u.Ho, u.Wo, u.pad_t,
                                        u.pad_l, ACT_HSWISH, st));
                break;
            case PU_DUMMY:
                RST_HIP_TRY(dummy_conv_launch(style, w + u.woff, w + u.goff, p->out[i], p->feat_part, batch, u.H,
                                              u.W, u.cin, u.Ho, u.Wo, u.pad_t, u.pad_l, st));
                break;
            case PU_PW:
                RST_HIP_TRY(pw_launch(in, u.se >= 0 ? p->se_val[u.se] : nullptr, w + u.woff, a, b,
                                      u.res >= 0 ? p->out[u.res] : nullptr, p->out[i], feat ? p->feat_part : nullptr,
                                      batch, u.H * u.W, u.cin, u.cout, u.act, st));
                break;
            case PU_DW: {
                const int e = p->se_of_dw[i];
                RST_HIP_TRY(dw_launch(in, w + u.woff, a, b, p->out[i], e >= 0 ? p->se_part[e] : nullptr, batch, u.H,
                                      u.W, u.cin, u.Ho, u.Wo, u.k, u.stride, u.pad_t, u.pad_l, u.act, st));
                if (e >= 0) {
                    const PSE& s = P.ses[e];
                    RST_HIP_TRY(se_launch(p->se_part[e], p->se_nwg[e], s.Ho * s.Wo, batch, s.C, s.R, w + s.w1,
                                          w + s.b1, w + s.w2, w + s.b2, p->se_val[e], nullptr, nullptr, nullptr, st));
                }
                break;
            }
        }
    }
    RST_HIP_TRY(head_launch(p->feat_part, p->feat_nparts, P.feat_hw, batch, P.feat_c, p->shape.num_style_parameters,
                            p->shape.num_top_parameters, w + P.head_w1, w + P.head_b1, w + P.head_w2,
                            w + P.head_b2, p->d_hidden, style_params, p->shape.num_top_parameters, nullptr, st));
    return RST_OK;
}

int rst_predictor_num_stages(const rst_predictor* p) { return p ? (int)p->stage_unit.size() : 0; }

int rst_predictor_stage_shape(const rst_predictor* p, int idx, int* hwc3) {
    if (!p || !hwc3 || idx < 0 || idx >= (int)p->stage_unit.size())
        return set_error(RST_ERR_INVALID, "rst_predictor_stage_shape: bad argument");
    const PUnit& u = p->plan.units[p->stage_unit[idx]];
    hwc3[0] = u.Ho;
    hwc3[1] = u.Wo;
    hwc3[2] = u.cout;
    return RST_OK;
}

int rst_predictor_copy_stage(rst_predictor* p, int idx, float* dst, size_t count, int batch, void* stream) {
    if (!p || !dst || idx < 0 || idx >= (int)p->stage_unit.size() || batch < 1 || batch > p->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_predictor_copy_stage: bad argument");
    const int ui = p->stage_unit[idx];
    const PUnit& u = p->plan.units[ui];
    const size_t n = (size_t)u.Ho * u.Wo * u.cout * batch;
    if (count != n) return set_error(RST_ERR_INVALID, "rst_predictor_copy_stage: count mismatch");
    RST_HIP_TRY(hipMemcpyAsync(dst, p->out[ui], n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return RST_OK;
}

}  // extern "C"
