// wino_x6_bench.hip — residual conv of rst-960-120-128-17 (B x 120 x 240 x Cin -> 128, CIN affine prologue
// of the given mode) on wino_x6 (split-bf16 Winograd) against wino (f32-MFMA Winograd): timing of both, the
// max difference of the outputs relative to the output scale (both restate the same convolution), and the
// statistics partials / materialised block input of wino_x6 against wino's.
// Build: bash tools/build_wino_x6_bench.sh   Run: tools/wino_x6_bench [B] [Cin] [pro_mode] [cold copies]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
#ifdef X6_PROF
namespace rst { void x6_timeline_print(int nwg, int nwave); }
#endif

using namespace rst;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static std::vector<float> host_rand(size_t n, float lo, float hi, unsigned seed) {
    std::vector<float> h(n); srand(seed);
    for (auto& v : h) v = lo + (hi - lo) * (rand() / (float)RAND_MAX);
    return h;
}
template <typename T> static T* dev(const std::vector<T>& h) {
    T* d; CK(hipMalloc(&d, h.size() * sizeof(T))); CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}
template <typename T> static std::vector<T> host(const T* d, size_t n) {
    std::vector<T> h(n);
    CK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
    return h;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1, C = argc > 2 ? atoi(argv[2]) : 128, H = 120, W = 240;
    const int pro = argc > 3 ? atoi(argv[3]) : PRO_AFF_RELU;
    // cold > 0: cycle the timed launches over `cold` copies of the input / residual / output / materialised
    // buffers and the weights (about 61 MB a copy at B=1, Cin=128), so a launch reads inputs and weights the L2 does
    // not hold, as in the frame (ten residual convs, each with its own weights)
    const int cold = argc > 4 ? atoi(argv[4]) : 0;
    // zm = 1: zero-mean inputs and prologue bias 0 (a ReLU prologue then zeroes about half the patch, as the
    // CIN + ReLU inputs of the frame's conv1 layers)
    const int zm = argc > 5 ? atoi(argv[5]) : 0;
    // chain = 1: each timed launch reads the output the previous launch wrote (ping-pong, Cin = 128), as the
    // frame's residual convs do; chain = 2: the chain's zero-mean weights without the chaining
    const int chain = argc > 6 ? atoi(argv[6]) : 0;
    // fin = 1: a CIN finalize launch (norm.hip) after every conv launch, as in the frame; the time reported
    // is per (conv + finalize) pair, and a finalize-only loop is timed beside it
    const int fin = argc > 7 ? atoi(argv[7]) : 0;
    // nomat = 1: no materialised block output (the frame's conv1 layers: a.mat == nullptr)
    const int nomat = argc > 8 ? atoi(argv[8]) : 0;
    // accm (x6 only): 1 = CIN statistics into f64 accumulators and the prologue affine formed from them (the
    // round-3 frame), 2 = producer side only (accumulators out, pro_ab in), 3 = consumer side only
    const int accm = argc > 9 ? atoi(argv[9]) : 0;
    auto hin = host_rand((size_t)B * H * W * C, zm ? -2.f : -1.f, zm ? 2.f : 3.f, 1);
    auto hres = host_rand((size_t)B * H * W * C, -1, 1, 5);
    // residual init U(0, 0.05); zero-mean in chain mode (a gain near 1 per layer keeps the chained values finite)
    auto hk = host_rand((size_t)9 * C * 128, chain ? -0.05f : 0.f, 0.05f, 2);
    auto hb = host_rand(128, -0.1f, 0.1f, 3);
    auto hab = host_rand((size_t)B * C * 2, 0.5f, 1.f, 4);
    if (zm)
        for (size_t i = 1; i < hab.size(); i += 2) hab[i] = 0.f;
    float* in = dev(hin);
    float* res = dev(hres);
    float* pp[2] = {dev(hin), dev(hin)};   // chain ping-pong buffers (B x H x W x 128)
    float* U32 = dev(wino_pack_weights(hk.data(), C));
    float* U6 = dev(wino_x6_pack_weights(hk.data(), C));
    float* bias = dev(hb);
    float* ab = dev(hab);
    const size_t n_out = (size_t)B * H * W * 128, n_mat = (size_t)B * H * W * C;
    WinoArgs a{};
    a.in = in; a.res = res; a.pro_ab = reinterpret_cast<const float2*>(ab); a.bias = bias;
    a.batch = B; a.H = H; a.W = W; a.cin = C; a.tiles_y = wino_tiles_y(H); a.tiles_x = wino_tiles_x(W);
    a.pro_mode = pro;
    const size_t n_part = (size_t)B * 128 * a.tiles_y * a.tiles_x;
    CK(wino_prepare()); CK(wino_x6_prepare());
    float* outs[2];
    float* mats[2];
    float4* parts[2];
    for (int v = 0; v < 2; ++v) {
        CK(hipMalloc(&outs[v], n_out * 4));
        CK(hipMalloc(&mats[v], n_mat * 4));
        CK(hipMalloc(&parts[v], n_part * 16));
        CK(hipMemset(mats[v], 0, n_mat * 4));
    }
    std::vector<float*> cin_(cold), cres(cold), cout_(cold), cmat(cold), cu32(cold), cu6(cold);
    const size_t nu32 = wino_pack_weights(hk.data(), C).size(), nu6 = wino_x6_pack_weights(hk.data(), C).size();
    for (int i = 0; i < cold; ++i) {
        CK(hipMalloc(&cin_[i], n_mat * 4)); CK(hipMalloc(&cres[i], n_mat * 4));
        CK(hipMalloc(&cout_[i], n_out * 4)); CK(hipMalloc(&cmat[i], n_mat * 4));
        CK(hipMemcpy(cin_[i], in, n_mat * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(cres[i], res, n_mat * 4, hipMemcpyDeviceToDevice));
        CK(hipMalloc(&cu32[i], nu32 * 4)); CK(hipMalloc(&cu6[i], nu6 * 4));
        CK(hipMemcpy(cu32[i], U32, nu32 * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(cu6[i], U6, nu6 * 4, hipMemcpyDeviceToDevice));
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float2* fab;
    CK(hipMalloc(&fab, (size_t)B * 128 * sizeof(float2)));
    auto fin_args = [&](const float4* part) {
        FinalizeArgs f{};
        f.part = part;
        f.ab = fab;
        f.batch = B;
        f.C = 128;
        f.ntot = 128;
        f.n_part = a.tiles_y * a.tiles_x;
        f.phases = 1;
        f.eps = 1e-5f;
        return f;
    };
    if (fin) {
        const FinalizeArgs f = fin_args(parts[1]);
        for (int i = 0; i < 20; ++i) CK(finalize_launch(f, 0));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 200; ++i) CK(finalize_launch(f, 0));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("finalize alone: %.2f us/launch\n", ms * 1e3 / 200);
    }
    // accumulator modes: the consumer side reads seeded accumulators (acc_in: slot 0 holds the fixed-point limbs of the
    // input's own per-(image, channel) sums, the others zero), the producer side adds into acc_out (timing only); the f32
    // kernel's prologue affine is the host restatement of cin_affine_table on the same sums, so the outputs compare
    cin_word* acc_in = nullptr;
    cin_word* acc_out = nullptr;
    float* sty = nullptr;
    if (accm) {
        const size_t n_acc = (size_t)8 * B * 2 * CIN_LIMBS * C;
        CK(hipMalloc(&acc_out, n_acc * sizeof(cin_word)));
        CK(hipMemset(acc_out, 0, n_acc * sizeof(cin_word)));
        std::vector<cin_word> ha(n_acc, 0);
        const auto hsty = host_rand((size_t)B * 2 * C, 0.5f, 1.f, 9);
        sty = dev(hsty);
        auto split = [](double v, cin_word* l) {   // kernels.h cin_fixed_split
            const double m = std::fabs(v), h = std::floor(m * 0x1p-32), r = m - h * 0x1p32, q = std::floor(r * 0x1p8);
            const double r2 = r - q * 0x1p-8;
            const cin_word k[3] = {(cin_word)std::floor(r2 * 0x1p48), (cin_word)q, (cin_word)h};
            for (int i = 0; i < 3; ++i) l[i] = v < 0 ? -k[i] : k[i];
        };
        for (int b = 0; b < B; ++b)
            for (int c = 0; c < C; ++c) {
                double S = 0, Q = 0;
                for (size_t p = 0; p < (size_t)H * W; ++p) {
                    const double x = hin[((size_t)b * H * W + p) * C + c];
                    S += x;
                    Q += x * x;
                }
                cin_word l[3];
                double v[2];
                for (int w = 0; w < 2; ++w) {
                    split(w ? Q : S, l);
                    for (int i = 0; i < 3; ++i) ha[((size_t)(b * 2 + w) * CIN_LIMBS + i) * C + c] = l[i];   // slot 0
                    // the value the device merges back (kernels.h cin_fixed_value of one canonical copy)
                    const double mag = (double)std::llabs(l[2]) * 0x1p32 +
                                       ((double)std::llabs(l[1]) * 0x1p-8 + (double)std::llabs(l[0]) * 0x1p-48);
                    v[w] = (w ? Q : S) < 0 ? -mag : mag;
                }
                S = v[0];
                Q = v[1];
                // the affine as cin_affine_table forms it (from the limbs' exact sums: S, Q truncated at 2^-48)
                const double N = (double)H * W, mean = S / N, var = std::fmax(Q - S * mean, 0.0) / N;
                const float rstd = (float)(1.0 / std::sqrt(var + (double)1e-5f)), g = hsty[b * 2 * C + c], be = hsty[b * 2 * C + C + c];
                hab[((size_t)b * C + c) * 2] = g * rstd;
                hab[((size_t)b * C + c) * 2 + 1] = be - (float)mean * (g * rstd);
            }
        acc_in = dev(ha);
        CK(hipMemcpy(ab, hab.data(), hab.size() * 4, hipMemcpyHostToDevice));
    }
    const int iters = 200;
    const char* names[2] = {"wino   ", "wino_x6"};
    for (int v = 0; v < 2; ++v) {
        WinoArgs x = a;
        x.U = v ? U6 : U32; x.out = outs[v]; x.mat = nomat ? nullptr : mats[v]; x.part = parts[v];
        if (v && (accm == 1 || accm == 2)) {
            x.part = nullptr;
            x.stat.acc = acc_out;
            x.stat.nslot = 8;
        }
        if (v && (accm == 1 || accm == 3) && pro != PRO_NONE) {
            x.pro_stat.acc = acc_in;
            x.pro_stat.nslot = 8;
            x.pro_stat.C = C;
            x.pro_stat.batch = B;
            x.pro_stat.n = (double)H * W;
            x.pro_stat.style = sty;
            x.pro_stat.style_stride = 2 * C;
            x.pro_stat.style_offset = 0;
            x.pro_stat.style1_offset = -1;
            x.pro_stat.eps = 1e-5f;
        }
        auto launch = [&]() { return v ? wino_x6_launch(x, 0) : wino_launch(x, 0); };
        for (int i = 0; i < 20; ++i) CK(launch());
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) {
            if (cold) {
                const int j = i % cold;
                x.in = cin_[j]; x.res = cres[j]; x.out = cout_[j]; x.mat = nomat ? nullptr : cmat[j];
                x.U = v ? cu6[j] : cu32[j];
            }
            if (chain == 1 && C == 128) {
                x.in = pp[i & 1];
                x.out = pp[(i + 1) & 1];
            }
            CK(launch());
            if (fin) CK(finalize_launch(fin_args(x.part), 0));
        }
        x.in = in; x.res = res; x.out = outs[v]; x.mat = nomat ? nullptr : mats[v]; x.U = v ? U6 : U32;
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / iters;
        const double direct = 2.0 * B * H * W * C * 128 * 9, exec = 2.0 * B * H * W / 4 * 16 * C * 128;
#ifdef X6_PROF
        if (v) rst::x6_timeline_print(B * a.tiles_y * a.tiles_x, 8);
#endif
        if (v) printf("%s B=%d Cin=%d pro=%d%s%s: %.2f us/launch, bf16 pipe %.3f (6 terms), direct-equivalent %.1f TF/s\n",
                      names[v], B, C, pro, accm == 1 ? " acc" : (accm == 2 ? " acc-out" : (accm == 3 ? " acc-in" : "")), cold ? " cold" : (chain == 1 ? " chain" : (chain == 2 ? " zero-mean weights" : "")), us, 6 * exec / (us * 1e-6) / 2.5e15, direct / (us * 1e-6) / 1e12);
        else printf("%s B=%d Cin=%d pro=%d%s: %.2f us/launch, f32 pipe %.3f, direct-equivalent %.1f TF/s\n", names[v], B,
                    C, pro, cold ? " cold" : (chain == 1 ? " chain" : (chain == 2 ? " zero-mean weights" : "")), us, exec / (us * 1e-6) / 157.3e12, direct / (us * 1e-6) / 1e12);
    }
    const auto h32 = host(outs[0], n_out), h6 = host(outs[1], n_out);
    double md = 0, mx = 0;
    size_t bad = 0;
    for (size_t i = 0; i < n_out; ++i) {
        if (!std::isfinite(h6[i])) ++bad;
        md = std::fmax(md, std::fabs((double)h6[i] - h32[i]));
        mx = std::fmax(mx, std::fabs((double)h32[i]));
    }
    printf("max |x6 - f32| = %.3e, max |f32| = %.3e, relative %.3e, non-finite %zu\n", md, mx, md / mx, bad);
    // materialised block input (the same prologue arithmetic in both kernels: bitwise), statistics partials
    const auto m0 = host(mats[0], n_mat), m1 = host(mats[1], n_mat);
    size_t mdiff = 0;
    // (accumulator consumer modes: the device forms the affine itself; its last bit may differ from the host's)
    const bool cons_acc = (accm == 1 || accm == 3) && pro != PRO_NONE;
    for (size_t i = 0; i < n_mat; ++i)
        mdiff += cons_acc ? std::fabs(m0[i] - m1[i]) > 2e-6f * std::fmax(1.f, std::fabs(m0[i])) : m0[i] != m1[i];
    const auto p0 = host(parts[0], n_part), p1 = host(parts[1], n_part);
    double ds = 0, dm = 0, sc = 0, mc = 0;
    size_t dn = 0;
    for (size_t i = 0; i < n_part; ++i) {
        ds = std::fmax(ds, std::fabs((double)p0[i].x - p1[i].x));
        dm = std::fmax(dm, std::fabs((double)p0[i].y - p1[i].y));
        sc = std::fmax(sc, std::fabs((double)p0[i].x));
        mc = std::fmax(mc, std::fabs((double)p0[i].y));
        dn += p0[i].z != p1[i].z;
    }
    printf("x6 vs f32: materialised input differs in %zu of %zu; partial sums rel %.3e, M2 rel %.3e, counts differ %zu\n",
           mdiff, n_mat, ds / sc, dm / mc, dn);
    // accumulator modes: the outputs compare (the f32 kernel's affine restates the seeded accumulators' one); the
    // statistics go to acc_out instead of partials (producer modes 1, 2), so the partials are not compared there
    const bool prod_acc = accm == 1 || accm == 2;
    const bool ok = md / mx < 1e-5 && bad == 0 && mdiff == 0 && (prod_acc || (ds / sc < 1e-5 && dm / mc < 1e-5 && dn == 0));
    printf("correctness gate: %s\n", ok ? "pass" : "FAIL");
    return ok ? 0 : 2;
}
