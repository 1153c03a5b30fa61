// predictor_train_api.hip — C ABI of the style predictor's training step (rst_predictor_trainer_*).
//
// train_network.py:86-138 fits the style predictor (stylePrediction.py:25-75, MobileNetV3Small or
// DUMMY extractor, trainable) jointly with the transfer network: the predictor's output is the
// transfer network's style_params input (styleTransferInferenceModel.py:23-37), so one Keras
// train_step is
//   style_params = predictor(style, training=True)        rst_predictor_trainer_forward
//   transfer forward / loss / backward                     rst_trainer_compute_gradients (-> d style_params)
//   predictor backward                                     rst_predictor_trainer_backward
//   RMSprop on both weight sets                            rst_*_apply_gradients
// In training mode every BatchNormalization normalises with the batch statistics over (B, H, W)
// and updates its moving statistics (Keras mobilenet_v3: momentum 0.999, eps 1e-3).
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/rst.h"
#include "common.h"
#include "predictor.h"
#include "predictor_plan.h"
#include "predictor_train.h"
#include "train.h"

using namespace rst;

namespace {
constexpr float PT_BN_EPS = 1e-3f;
constexpr float PT_BN_MOMENTUM = 0.999f;
}  // namespace

struct rst_predictor_trainer {
    rst_predictor_shape shape;
    PPlan plan;
    int batch = 0;                          // batch of the most recent forward
    const float* style = nullptr;           // its input (caller-owned; must stay valid until backward)
    float* d_wc = nullptr;                  // weights, Keras order (BN moving statistics updated in place)
    float* d_ms = nullptr;                  // RMSprop slots
    float* d_ones = nullptr;                // 1024 ones / zeros: the raw (unnormalised) conv epilogue
    float* d_zeros = nullptr;
    std::vector<float*> z, y, dyb, dres;    // per unit
    std::vector<float2*> ab, mr;
    std::vector<bool> res_consumer;         // unit is the shortcut of a later project unit
    std::vector<int> se_of_dw;
    // per SE block
    std::vector<float*> se_part, se_val, se_g, se_s1, se_s2, se_dpart, se_ds1, se_ds2, se_dgb;
    std::vector<int> se_nwg;
    float* feat_part = nullptr;
    int feat_nparts = 0;
    float *gap = nullptr, *hidden = nullptr, *dhid = nullptr, *dfeat = nullptr;
    float* dz = nullptr;                    // norm-backward output (largest unit); ring slot 0
    // the weight gradients (and the SE / head outer products) run on `wside` beside the input-gradient chain; the
    // norm-backward outputs go round a ring of DZR buffers, each released by the weight gradient that reads it
    // (RST_PBWD_DZR at creation, default 3; at most one per unit)
    int n_dzr = 3;
    std::vector<float*> dzr;
    hipStream_t wside = nullptr;
    // every fork / join of one backward records a fresh event (evs[ev_next++]): no event is recorded twice within a
    // call, so a hipGraph capture of the step sees each dependency once (re-recording the ring's events within one
    // capture crashed the capture's end on this stack, tools/train_graph_check.py, profiles/r06)
    std::vector<hipEvent_t> evs;
    size_t ev_next = 0;
    bool serial_wgrad = false;              // RST_SERIAL_PREDICTOR_WGRAD=1 at creation: everything on the caller's stream
    float4* bn_part = nullptr;
    float2* consts = nullptr;
    float* slab = nullptr;
    float* wt = nullptr;                    // transposed 1x1 weights (dgrad): every pointwise unit's at wt_off[unit]
    std::vector<size_t> wt_off;
    TransposeJobs wt_jobs;                  // all of them in one launch at the start of each backward
    int* stat_index = nullptr;              // weight index of every BN moving_mean / moving_variance entry
    size_t n_stat = 0;
    std::vector<void*> allocs;
    ~rst_predictor_trainer() {
        if (wside) {
            (void)hipStreamSynchronize(wside);
            (void)hipStreamDestroy(wside);
        }
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
        for (void* p : allocs) (void)hipFree(p);
    }
    template <typename T>
    int alloc(T** d, size_t bytes) {
        if (hipMalloc((void**)d, std::max<size_t>(bytes, 16)) != hipSuccess) {
            *d = nullptr;
            return set_error(RST_ERR_ALLOC, "rst_predictor_trainer: hipMalloc failed");
        }
        allocs.push_back((void*)*d);
        return RST_OK;
    }
};

extern "C" {

int rst_predictor_trainer_create(const rst_predictor_shape* shape, const float* weights_host, size_t num_weights,
                                 rst_predictor_trainer** out) {
    if (!shape || !weights_host || !out) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_create: null argument");
    *out = nullptr;
    auto* t = new rst_predictor_trainer();
    t->shape = *shape;
    int st = build_predictor_plan(shape, &t->plan);
    if (st != RST_OK) { delete t; return st; }
    const PPlan& P = t->plan;
    if (num_weights != P.total) {
        delete t;
        return set_error(RST_ERR_INVALID, "rst_predictor_trainer_create: expected " + std::to_string(P.total) +
                                              " weights, got " + std::to_string(num_weights));
    }
    for (const PUnit& u : P.units)
        if ((u.kind == PU_PW || u.kind == PU_DW) && (u.woff % 4 != 0 || u.goff % 4 != 0)) {
            delete t;
            return set_error(RST_ERR_UNSUPPORTED, "rst_predictor_trainer_create: misaligned weight offset");
        }
    const size_t B = shape->max_batch;
    const size_t nw = P.total;
#define TRY(x)                        \
    do {                              \
        if ((st = (x)) != RST_OK) {   \
            delete t;                 \
            return st;                \
        }                             \
    } while (0)
    TRY(t->alloc(&t->d_wc, nw * 4));
    TRY(t->alloc(&t->d_ms, nw * 4));
    TRY(t->alloc(&t->d_ones, 1024 * 4));
    TRY(t->alloc(&t->d_zeros, 1024 * 4));
    {
        std::vector<float> ones(1024, 1.f);
        if (hipMemcpy(t->d_wc, weights_host, nw * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(t->d_ms, 0, nw * 4) != hipSuccess ||
            hipMemcpy(t->d_ones, ones.data(), 1024 * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemset(t->d_zeros, 0, 1024 * 4) != hipSuccess) {
            delete t;
            return set_error(RST_ERR_HIP, "rst_predictor_trainer_create: upload failed");
        }
    }
    {   // BN moving statistics in get_weights() order (the units are laid out in weight order)
        std::vector<int> idx;
        for (const PUnit& u : P.units)
            if (u.kind != PU_DUMMY)
                for (int i = 0; i < 2 * u.cout; ++i) idx.push_back((int)(u.goff + 2 * (size_t)u.cout + i));
        t->n_stat = idx.size();
        if (!idx.empty()) {
            TRY(t->alloc(&t->stat_index, idx.size() * 4));
            if (hipMemcpy(t->stat_index, idx.data(), idx.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
                delete t;
                return set_error(RST_ERR_HIP, "rst_predictor_trainer_create: upload failed");
            }
        }
    }
    const size_t nu = P.units.size();
    t->res_consumer.assign(nu, false);
    for (const PUnit& u : P.units)
        if (u.res >= 0) t->res_consumer[u.res] = true;
    t->se_of_dw.assign(nu, -1);
    size_t max_act = 0, max_part = 0, max_slab = 0, max_wt = 0;
    for (size_t i = 0; i < nu; ++i) {
        const PUnit& u = P.units[i];
        const size_t n = B * u.Ho * u.Wo * u.cout;
        max_act = std::max(max_act, n);
        float *zi = nullptr, *yi = nullptr, *dyi = nullptr, *dri = nullptr;
        float2 *abi = nullptr, *mri = nullptr;
        TRY(t->alloc(&yi, n * 4));
        if (u.kind != PU_DUMMY) {
            TRY(t->alloc(&zi, n * 4));
            TRY(t->alloc(&abi, (size_t)u.cout * 8));
            TRY(t->alloc(&mri, (size_t)u.cout * 8));
            int block, slots, ppw, nt;
            dw_geometry(u.cout, u.Ho * u.Wo, &block, &slots, &ppw, &nt);
            max_part = std::max(max_part, B * nt * (size_t)u.cout / 4 * 2);
        }
        if ((int)i != P.feat_unit) TRY(t->alloc(&dyi, n * 4));
        if (t->res_consumer[i]) TRY(t->alloc(&dri, n * 4));
        t->z.push_back(zi);
        t->y.push_back(yi);
        t->dyb.push_back(dyi);
        t->dres.push_back(dri);
        t->ab.push_back(abi);
        t->mr.push_back(mri);
        if (u.kind == PU_PW) {
            int pps;
            const int S = pw_wgrad_splits((int)B, u.H * u.W, u.cin, u.cout, &pps);
            max_slab = std::max(max_slab, (size_t)S * u.cin * u.cout);
            max_wt += (size_t)u.cin * u.cout;   // (the sum: one transposed image per pointwise unit)
        } else if (u.kind == PU_DW) {
            int pps, block, slots;
            const int S = dw_wgrad_splits((int)B, u.Ho * u.Wo, u.cout, &pps, &block, &slots);
            max_slab = std::max(max_slab, (size_t)S * u.k * u.k * u.cout);
        } else if (u.kind == PU_STEM) {
            int pps;
            const int S = stem_wgrad_splits((int)B, u.Ho * u.Wo, &pps);
            max_slab = std::max(max_slab, (size_t)S * 432);
        }
    }
    for (size_t e = 0; e < P.ses.size(); ++e) {
        const PSE& s = P.ses[e];
        int block, slots, ppw, nwg;
        dw_geometry(s.C, s.Ho * s.Wo, &block, &slots, &ppw, &nwg);
        float *part, *val, *g, *s1, *s2, *dpart, *ds1, *ds2, *dgb;
        TRY(t->alloc(&part, B * nwg * s.C * 4));
        TRY(t->alloc(&val, B * s.C * 4));
        TRY(t->alloc(&g, B * s.C * 4));
        TRY(t->alloc(&s1, B * s.R * 4));
        TRY(t->alloc(&s2, B * s.C * 4));
        TRY(t->alloc(&dpart, B * nwg * s.C * 4));
        TRY(t->alloc(&ds1, B * s.R * 4));
        TRY(t->alloc(&ds2, B * s.C * 4));
        TRY(t->alloc(&dgb, B * s.C * 4));
        t->se_part.push_back(part); t->se_val.push_back(val); t->se_g.push_back(g); t->se_s1.push_back(s1);
        t->se_s2.push_back(s2); t->se_dpart.push_back(dpart); t->se_ds1.push_back(ds1); t->se_ds2.push_back(ds2);
        t->se_dgb.push_back(dgb); t->se_nwg.push_back(nwg);
        t->se_of_dw[s.src] = (int)e;
    }
    const PUnit& fu = P.units[P.feat_unit];
    if (fu.kind == PU_DUMMY) {
        t->feat_nparts = dummy_conv_parts(fu.Ho * fu.Wo);
    } else {
        int block, slots, ppw, nt;
        dw_geometry(fu.cout, fu.Ho * fu.Wo, &block, &slots, &ppw, &nt);
        t->feat_nparts = nt;
    }
    const int NS = shape->num_style_parameters;
    TRY(t->alloc(&t->feat_part, B * t->feat_nparts * P.feat_c * 4));
    TRY(t->alloc(&t->gap, B * P.feat_c * 4));
    TRY(t->alloc(&t->dfeat, B * P.feat_c * 4));
    TRY(t->alloc(&t->hidden, B * NS * 4));
    TRY(t->alloc(&t->dhid, B * NS * 4));
    TRY(t->alloc(&t->dz, max_act * 4));
    TRY(t->alloc(&t->bn_part, std::max<size_t>(max_part, 1) * 16));
    TRY(t->alloc(&t->consts, 1024 * 8));
    TRY(t->alloc(&t->slab, std::max<size_t>(max_slab, 1) * 4));
    TRY(t->alloc(&t->wt, std::max<size_t>(max_wt, 1) * 4));
    {
        t->wt_off.assign(P.units.size(), 0);
        size_t off = 0;
        long long end = 0;
        for (size_t i = 0; i < P.units.size(); ++i) {
            const PUnit& u = P.units[i];
            if (u.kind != PU_PW) continue;
            TransposeJobs& J = t->wt_jobs;
            if (J.n >= TransposeJobs::MAX) {
                delete t;
                return set_error(RST_ERR_UNSUPPORTED, "rst_predictor_trainer_create: too many pointwise units");
            }
            t->wt_off[i] = off;
            end += (long long)u.cin * u.cout;
            J.src[J.n] = (long long)u.woff;
            J.dst[J.n] = (long long)off;
            J.end[J.n] = end;
            J.rows[J.n] = u.cin;
            J.cols[J.n] = u.cout;
            ++J.n;
            off += (size_t)u.cin * u.cout;
        }
    }
    {
        const char* dv = getenv("RST_PBWD_DZR");
        const int want = dv != nullptr ? atoi(dv) : 3, nu = (int)t->plan.units.size();
        t->n_dzr = want < 1 ? 1 : (want > nu ? (nu > 0 ? nu : 1) : want);
    }
    t->dzr.assign((size_t)t->n_dzr, nullptr);
    t->dzr[0] = t->dz;
    for (int k = 1; k < t->n_dzr; ++k) TRY(t->alloc(&t->dzr[k], max_act * 4));
    {
        const char* sw = getenv("RST_SERIAL_PREDICTOR_WGRAD");
        t->serial_wgrad = sw != nullptr && sw[0] == '1';
        bool ok = hipStreamCreateWithFlags(&t->wside, hipStreamNonBlocking) == hipSuccess;
        // forks: the heads' and one per SE unit; two per unit (norm-backward output handed over, released); the join
        t->evs.assign(2 * t->plan.units.size() + t->plan.ses.size() + 4, nullptr);
        for (size_t k = 0; ok && k < t->evs.size(); ++k)
            ok = hipEventCreateWithFlags(&t->evs[k], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            delete t;
            return set_error(RST_ERR_HIP, "rst_predictor_trainer_create: stream / event creation failed");
        }
    }
#undef TRY
    *out = t;
    return RST_OK;
}

void rst_predictor_trainer_destroy(rst_predictor_trainer* t) { delete t; }

size_t rst_predictor_trainer_num_weights(const rst_predictor_trainer* t) { return t ? t->plan.total : 0; }

int rst_predictor_trainer_forward(rst_predictor_trainer* t, const float* style, int batch, float* style_params,
                                  void* stream) {
    if (!t || !style || !style_params) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_forward: null argument");
    if (batch < 1 || batch > t->shape.max_batch)
        return set_error(RST_ERR_INVALID, "rst_predictor_trainer_forward: batch outside [1, max_batch]");
    hipStream_t st = (hipStream_t)stream;
    const PPlan& P = t->plan;
    const int B = batch;
    float* w = t->d_wc;
    t->batch = B;
    t->style = style;
    for (size_t i = 0; i < P.units.size(); ++i) {
        const PUnit& u = P.units[i];
        const float* in = u.in < 0 ? style : t->y[u.in];
        const bool feat = (int)i == P.feat_unit;
        const int HWo = u.Ho * u.Wo;
        switch (u.kind) {
            case PU_DUMMY:
                RST_HIP_TRY(dummy_conv_launch(style, w + u.woff, w + u.goff, t->y[i], t->feat_part, B, u.H, u.W,
                                              u.cin, u.Ho, u.Wo, u.pad_t, u.pad_l, st));
                continue;
            case PU_STEM:
                RST_HIP_TRY(stem_launch(style, w + u.woff, t->d_ones, t->d_zeros, t->z[i], B, u.H, u.W, u.Ho, u.Wo,
                                        u.pad_t, u.pad_l, ACT_NONE, st));
                break;
            case PU_PW:
                RST_HIP_TRY(pw_launch(in, u.se >= 0 ? t->se_val[u.se] : nullptr, w + u.woff, t->d_ones, t->d_zeros,
                                      nullptr, t->z[i], nullptr, B, u.H * u.W, u.cin, u.cout, ACT_NONE, st));
                break;
            case PU_DW:
                RST_HIP_TRY(dw_launch(in, w + u.woff, t->d_ones, t->d_zeros, t->z[i], nullptr, B, u.H, u.W, u.cin,
                                      u.Ho, u.Wo, u.k, u.stride, u.pad_t, u.pad_l, ACT_NONE, st));
                break;
        }
        const int e = t->se_of_dw[i];
        float* ypart = feat ? t->feat_part : (e >= 0 ? t->se_part[e] : nullptr);
        RST_HIP_TRY(bn_forward_launch(t->z[i], B, HWo, u.cout, w + u.goff, PT_BN_EPS, PT_BN_MOMENTUM, t->bn_part,
                                      t->ab[i], t->mr[i], u.res >= 0 ? t->y[u.res] : nullptr, t->y[i], u.act, ypart,
                                      st));
        if (e >= 0) {
            const PSE& s = P.ses[e];
            RST_HIP_TRY(se_launch(t->se_part[e], t->se_nwg[e], s.Ho * s.Wo, B, s.C, s.R, w + s.w1, w + s.b1,
                                  w + s.w2, w + s.b2, t->se_val[e], t->se_g[e], t->se_s1[e], t->se_s2[e], st));
        }
    }
    RST_HIP_TRY(head_launch(t->feat_part, t->feat_nparts, P.feat_hw, B, P.feat_c, t->shape.num_style_parameters,
                            t->shape.num_top_parameters, w + P.head_w1, w + P.head_b1, w + P.head_w2, w + P.head_b2,
                            t->hidden, style_params, t->shape.num_top_parameters, t->gap, st));
    return RST_OK;
}

int rst_predictor_trainer_backward(rst_predictor_trainer* t, const float* d_style_params, float* grad, void* stream) {
    if (!t || !d_style_params || !grad) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_backward: null argument");
    if (t->batch < 1) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_backward: no forward to differentiate");
    hipStream_t st = (hipStream_t)stream;
    const PPlan& P = t->plan;
    const int B = t->batch, NS = t->shape.num_style_parameters, NP = t->shape.num_top_parameters;
    const float* w = t->d_wc;
    // Off the input-gradient chain (weight gradients, the SE / head outer products) on t->wside when par: every such
    // launch follows a fork (ev_chain recorded on the chain, waited on wside) placed after the chain's last write of
    // its operands; the chain's norm-backward outputs round a ring of DZR buffers released by ev_wg; joined at the end.
    // Same kernels on the same operands: bitwise the serial order.
    const bool par = !t->serial_wgrad;
    hipStream_t ws = par ? t->wside : st;
    t->ev_next = 0;
    auto next_ev = [&](hipEvent_t* ev) -> hipError_t {
        if (t->ev_next >= t->evs.size()) return hipErrorInvalidValue;
        *ev = t->evs[t->ev_next++];
        return hipSuccess;
    };
    auto fork = [&]() -> hipError_t {
        if (!par) return hipSuccess;
        hipEvent_t ev;
        hipError_t e = next_ev(&ev);
        if (e == hipSuccess) e = hipEventRecord(ev, st);
        return e != hipSuccess ? e : hipStreamWaitEvent(ws, ev, 0);
    };
    std::vector<hipEvent_t> ev_wg((size_t)t->n_dzr, nullptr);   // the weight gradient that last read ring slot k
    RST_HIP_TRY(hipMemsetAsync(grad, 0, P.total * sizeof(float), st));
    // the input-gradient convs' transposed 1x1 weights, all in one launch (22 separate transposes on the chain were
    // 1.1 ms of a config-4 step: each small launch waited for CUs beside the transfer network's backward)
    if (t->wt_jobs.n > 0) RST_HIP_TRY(transpose_batch_launch(w, t->wt_jobs, t->wt, st));
    // heads (stylePrediction.py:60-71): P = W2^T h + b2, h = W1^T gap + b1
    RST_HIP_TRY(rowdot_launch(d_style_params, B, NP, w + P.head_w2, NS, 1.f, t->dhid, st));
    RST_HIP_TRY(fork());
    RST_HIP_TRY(outer_launch(t->hidden, NS, d_style_params, NP, B, 0, grad + P.head_w2, grad + P.head_b2, ws));
    const PUnit& fu = P.units[P.feat_unit];
    // gradient of the pooled features; spread over the feature map as dgap / HW (DUMMY: dgap itself)
    RST_HIP_TRY(rowdot_launch(t->dhid, B, NS, w + P.head_w1, P.feat_c, fu.kind == PU_DUMMY ? 1.f : 1.f / P.feat_hw,
                              t->dfeat, st));
    RST_HIP_TRY(outer_launch(t->gap, P.feat_c, t->dhid, NS, B, 0, grad + P.head_w1, grad + P.head_b1, ws));
    int j = 0;
    for (int i = (int)P.units.size() - 1; i >= 0; --i, ++j) {
        const PUnit& u = P.units[i];
        const int slot = j % t->n_dzr;
        float* const dz = par ? t->dzr[slot] : t->dz;
        const float* in = u.in < 0 ? t->style : t->y[u.in];
        if (u.kind == PU_DUMMY) {
            RST_HIP_TRY(dummy_wgrad_launch(t->style, t->dfeat, B, u.H, u.W, u.cin, u.Ho, u.Wo, u.pad_t, u.pad_l,
                                           grad + u.woff, grad + u.goff, st));
            continue;
        }
        const bool feat = i == P.feat_unit;
        const int e = t->se_of_dw[i];
        BnBwdArgs a{};
        a.z = t->z[i];
        a.dy = feat ? nullptr : t->dyb[i];
        a.mul = e >= 0 ? t->se_val[e] : nullptr;
        a.bcast = feat ? t->dfeat : (e >= 0 ? t->se_dgb[e] : nullptr);
        a.ab = t->ab[i];
        a.mr = t->mr[i];
        a.consts = t->consts;
        a.part = t->bn_part;
        a.dz = dz;
        a.dgamma = grad + u.goff;
        a.B = B;
        a.HW = u.Ho * u.Wo;
        a.C = u.cout;
        a.act = u.act;
        if (par && ev_wg[slot] != nullptr) RST_HIP_TRY(hipStreamWaitEvent(st, ev_wg[slot], 0));
        RST_HIP_TRY(bn_backward_launch(a, st));
        if (par) {
            hipEvent_t ev_dz;
            RST_HIP_TRY(next_ev(&ev_dz));
            RST_HIP_TRY(hipEventRecord(ev_dz, st));
            RST_HIP_TRY(hipStreamWaitEvent(ws, ev_dz, 0));
        }
        if (u.res >= 0)   // y = BN(z) + shortcut: the shortcut's consumer adds this in its dgrad
            RST_HIP_TRY(hipMemcpyAsync(t->dres[u.res], t->dyb[i], (size_t)B * u.Ho * u.Wo * u.cout * sizeof(float),
                                       hipMemcpyDeviceToDevice, st));
        switch (u.kind) {
            case PU_STEM:
                RST_HIP_TRY(stem_wgrad_launch(t->style, dz, B, u.H, u.W, u.Ho, u.Wo, u.pad_t, u.pad_l, t->slab,
                                              grad + u.woff, ws));
                break;
            case PU_PW: {
                const float* se = u.se >= 0 ? t->se_val[u.se] : nullptr;
                RST_HIP_TRY(pw_wgrad_launch(in, se, dz, B, u.H * u.W, u.cin, u.cout, t->slab, grad + u.woff, ws));
                // dgrad: the 1x1 conv with the transposed kernel; the shortcut gradient rides on its residual input
                RST_HIP_TRY(pw_launch(dz, nullptr, t->wt + t->wt_off[i], t->d_ones, t->d_zeros,
                                      t->res_consumer[u.in] ? t->dres[u.in] : nullptr, t->dyb[u.in], nullptr, B,
                                      u.H * u.W, u.cout, u.cin, ACT_NONE, st));
                if (u.se >= 0) {   // dyb[in] is d/d(u * se): SE backward (the dw unit applies mul/bcast)
                    const PSE& s = P.ses[u.se];
                    int np;
                    RST_HIP_TRY(se_dscale_launch(t->dyb[u.in], t->y[u.in], B, u.H * u.W, u.cin, t->se_dpart[u.se], &np,
                                                 st));
                    RST_HIP_TRY(se_bwd_launch(t->se_dpart[u.se], np, B, s.C, s.R, s.Ho * s.Wo, w + s.w1, w + s.w2,
                                              t->se_s1[u.se], t->se_s2[u.se], t->se_ds1[u.se], t->se_ds2[u.se],
                                              t->se_dgb[u.se], st));
                    RST_HIP_TRY(fork());
                    RST_HIP_TRY(outer_launch(t->se_g[u.se], s.C, t->se_ds1[u.se], s.R, B, 0, grad + s.w1, grad + s.b1,
                                             ws));
                    RST_HIP_TRY(outer_launch(t->se_s1[u.se], s.R, t->se_ds2[u.se], s.C, B, 1, grad + s.w2, grad + s.b2,
                                             ws));
                }
                break;
            }
            case PU_DW:
                RST_HIP_TRY(dw_wgrad_launch(in, dz, B, u.H, u.W, u.cout, u.Ho, u.Wo, u.k, u.stride, u.pad_t, u.pad_l,
                                            t->slab, grad + u.woff, ws));
                RST_HIP_TRY(dw_dgrad_launch(dz, w + u.woff, t->dyb[u.in], B, u.H, u.W, u.cout, u.Ho, u.Wo, u.k,
                                            u.stride, u.pad_t, u.pad_l, st));
                break;
        }
        if (par) {
            RST_HIP_TRY(next_ev(&ev_wg[slot]));
            RST_HIP_TRY(hipEventRecord(ev_wg[slot], ws));
        }
    }
    if (par) {   // join: every gradient is in `grad` when the caller's stream goes on
        hipEvent_t ev_done;
        RST_HIP_TRY(next_ev(&ev_done));
        RST_HIP_TRY(hipEventRecord(ev_done, ws));
        RST_HIP_TRY(hipStreamWaitEvent(st, ev_done, 0));
    }
    return RST_OK;
}

int rst_predictor_trainer_apply_gradients(rst_predictor_trainer* t, const float* grad, float learning_rate, float rho,
                                          float epsilon, void* stream) {
    if (!t || !grad) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_apply_gradients: null argument");
    RST_HIP_TRY(rmsprop_launch(t->d_wc, t->d_ms, grad, t->plan.total, learning_rate, rho, epsilon, (hipStream_t)stream));
    return RST_OK;
}

int rst_predictor_trainer_copy_weights(rst_predictor_trainer* t, float* dst, size_t count, void* stream) {
    if (!t || !dst || count != t->plan.total) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_copy_weights");
    RST_HIP_TRY(hipMemcpyAsync(dst, t->d_wc, count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return RST_OK;
}

int rst_predictor_trainer_set_weights(rst_predictor_trainer* t, const float* src, size_t count, void* stream) {
    if (!t || !src || count != t->plan.total) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_set_weights");
    RST_HIP_TRY(hipMemcpyAsync(t->d_wc, src, count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return RST_OK;
}

size_t rst_predictor_trainer_num_moving_statistics(const rst_predictor_trainer* t) { return t ? t->n_stat : 0; }

int rst_predictor_trainer_get_moving_statistics(rst_predictor_trainer* t, float* dst, size_t count, void* stream) {
    if (!t || !dst || count != t->n_stat)
        return set_error(RST_ERR_INVALID, "rst_predictor_trainer_get_moving_statistics: bad argument");
    if (count) RST_HIP_TRY(gather_launch(t->d_wc, t->stat_index, dst, count, (hipStream_t)stream));
    return RST_OK;
}

int rst_predictor_trainer_set_moving_statistics(rst_predictor_trainer* t, const float* src, size_t count, float divisor,
                                                void* stream) {
    if (!t || !src || count != t->n_stat || !(divisor > 0.f))
        return set_error(RST_ERR_INVALID, "rst_predictor_trainer_set_moving_statistics: bad argument");
    RST_HIP_TRY(scatter_div_launch(src, t->stat_index, t->d_wc, count, divisor, (hipStream_t)stream));
    return RST_OK;
}

int rst_predictor_trainer_copy_slots(rst_predictor_trainer* t, float* dst, size_t count, void* stream) {
    if (!t || !dst || count != t->plan.total) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_copy_slots");
    RST_HIP_TRY(hipMemcpyAsync(dst, t->d_ms, count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return RST_OK;
}

int rst_predictor_trainer_set_slots(rst_predictor_trainer* t, const float* src, size_t count, void* stream) {
    if (!t || !src || count != t->plan.total) return set_error(RST_ERR_INVALID, "rst_predictor_trainer_set_slots");
    RST_HIP_TRY(hipMemcpyAsync(t->d_ms, src, count * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return RST_OK;
}

}  // extern "C"
