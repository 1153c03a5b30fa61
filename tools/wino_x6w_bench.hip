// wino_x6w_bench.hip — residual conv of rst-960-120-128-17 (B x 120 x 240 x Cin -> 128, CIN affine prologue of
// the given mode) on wino (f32 MFMA Winograd, the reference of the comparison), wino_x6 (8x16 px x 128 channels)
// and wino_x6w (16x16 px x 64 channels): time per launch of each, max output difference to wino relative to the
// output scale, materialised block input bitwise, and the per-(image, channel) totals of the statistics partials
// {sum S, sum of M2 + S^2/n} (the quantity the CIN merge uses) relative to wino's.
// Build: bash tools/build_wino_x6w_bench.sh   Run: tools/wino_x6w_bench [B] [Cin] [pro_mode] [acc]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"

namespace rst {   // tools/wino_x6w.hip (experiment, not in the library)
bool wino_x6w_supported(int kh, int stride, int cin, int cout);
std::vector<float> wino_x6w_pack_weights(const float* kern, int cin);
int wino_x6w_tiles_y(int H);
int wino_x6w_tiles_x(int W);
hipError_t wino_x6w_prepare();
hipError_t wino_x6w_launch(const WinoArgs& a, hipStream_t st);
}
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
    const int B = argc > 1 ? atoi(argv[1]) : 1, C = argc > 2 ? atoi(argv[2]) : 128;
    const int pro = argc > 3 ? atoi(argv[3]) : PRO_AFF_RELU;
    const int accm = argc > 4 ? atoi(argv[4]) : 0;   // 1: statistics into f64 accumulators + prologue from them
    const int H = argc > 5 ? atoi(argv[5]) : 120, W = argc > 6 ? atoi(argv[6]) : 240;
    auto hin = host_rand((size_t)B * H * W * C, -1.f, 3.f, 1);
    auto hres = host_rand((size_t)B * H * W * C, -1, 1, 5);
    auto hk = host_rand((size_t)9 * C * 128, 0.f, 0.05f, 2);
    auto hb = host_rand(128, -0.1f, 0.1f, 3);
    auto hab = host_rand((size_t)B * C * 2, 0.5f, 1.f, 4);
    float* in = dev(hin);
    float* res = dev(hres);
    float* Us[3] = {dev(wino_pack_weights(hk.data(), C)), dev(wino_x6_pack_weights(hk.data(), C)),
                    dev(wino_x6w_pack_weights(hk.data(), C))};
    float* bias = dev(hb);
    float* ab = dev(hab);
    const size_t n_out = (size_t)B * H * W * 128, n_mat = (size_t)B * H * W * C;
    CK(wino_prepare()); CK(wino_x6_prepare()); CK(wino_x6w_prepare());
    const int tys[3] = {wino_tiles_y(H), wino_tiles_y(H), wino_x6w_tiles_y(H)};
    const int txs[3] = {wino_tiles_x(W), wino_tiles_x(W), wino_x6w_tiles_x(W)};
    float* outs[3];
    float* mats[3];
    float4* parts[3];
    size_t nparts[3];
    for (int v = 0; v < 3; ++v) {
        nparts[v] = (size_t)B * 128 * tys[v] * txs[v];
        CK(hipMalloc(&outs[v], n_out * 4));
        CK(hipMalloc(&mats[v], n_mat * 4));
        CK(hipMalloc(&parts[v], nparts[v] * 16));
        CK(hipMemset(mats[v], 0, n_mat * 4));
        CK(hipMemset(outs[v], 0, n_out * 4));
    }
    double* acc = nullptr;
    float* sty = nullptr;
    if (accm) {
        CK(hipMalloc(&acc, (size_t)8 * B * 2 * 128 * sizeof(double)));
        std::vector<double> ha((size_t)8 * B * 2 * 128);
        for (size_t i = 0; i < ha.size(); ++i) ha[i] = ((i / 128) % 2) ? 2.0e4 : 1.0e2;
        CK(hipMemcpy(acc, ha.data(), ha.size() * 8, hipMemcpyHostToDevice));
        sty = dev(host_rand((size_t)B * 2 * C, 0.5f, 1.f, 9));
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const char* names[3] = {"wino    ", "wino_x6 ", "wino_x6w"};
    const int iters = 200;
    double us_v[3] = {0, 0, 0};
    for (int v = 0; v < 3; ++v) {
        WinoArgs x{};
        x.in = in; x.res = res; x.pro_ab = reinterpret_cast<const float2*>(ab); x.bias = bias;
        x.batch = B; x.H = H; x.W = W; x.cin = C; x.tiles_y = tys[v]; x.tiles_x = txs[v];
        x.pro_mode = pro;
        x.U = Us[v]; x.out = outs[v]; x.mat = mats[v]; x.part = parts[v];
        if (v && accm) {   // timed with the accumulators (the frame's form); the checked launch below uses partials
            x.part = nullptr;
            x.stat.acc = acc;
            x.stat.nslot = 8;
            if (pro != PRO_NONE) {
                x.pro_stat.acc = acc; x.pro_stat.nslot = 8; x.pro_stat.C = C; x.pro_stat.batch = B;
                x.pro_stat.n = (double)H * W; x.pro_stat.style = sty; x.pro_stat.style_stride = 2 * C;
                x.pro_stat.style_offset = 0; x.pro_stat.style1_offset = -1; x.pro_stat.eps = 1e-5f;
            }
        }
        auto launch = [&](const WinoArgs& y) {
            return v == 0 ? wino_launch(y, 0) : (v == 1 ? wino_x6_launch(y, 0) : wino_x6w_launch(y, 0));
        };
        for (int i = 0; i < 20; ++i) CK(launch(x));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(launch(x));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        us_v[v] = 1e3 * ms / iters;
        if (v && accm) {   // the checked launch: partials, affine from pro_ab
            WinoArgs y = x;
            y.stat = CinAcc{};
            y.pro_stat = CinSrc{};
            y.part = parts[v];
            CK(launch(y));
            CK(hipDeviceSynchronize());
        }
        const double exec = 2.0 * B * H * W / 4 * 16 * C * 128;
        printf("%s B=%d Cin=%d pro=%d%s: %.2f us/launch, exec frac %.3f\n", names[v], B, C, pro, accm ? " acc" : "",
               us_v[v], (v ? 6 : 1) * exec / (us_v[v] * 1e-6) / (v ? 2.5e15 : 157.3e12));
    }
    const auto h32 = host(outs[0], n_out);
    const auto m0 = host(mats[0], n_mat);
    const auto p0 = host(parts[0], nparts[0]);
    auto totals = [&](const std::vector<float4>& p, int np) {   // per (b, channel): {sum S, sum M2 + S^2/n}
        std::vector<double> t((size_t)B * 128 * 2, 0.0);
        for (int b = 0; b < B; ++b)
            for (int c = 0; c < 128; ++c)
                for (int k = 0; k < np; ++k) {
                    const float4 q = p[((size_t)b * 128 + c) * np + k];
                    if (q.z > 0) {
                        t[((size_t)b * 128 + c) * 2] += q.x;
                        t[((size_t)b * 128 + c) * 2 + 1] += (double)q.y + (double)q.x * q.x / q.z;
                    }
                }
        return t;
    };
    const auto t0 = totals(p0, tys[0] * txs[0]);
    int rc = 0;
    for (int v = 1; v < 3; ++v) {
        const auto h = host(outs[v], n_out);
        double md = 0, mx = 0;
        size_t bad = 0;
        for (size_t i = 0; i < n_out; ++i) {
            if (!std::isfinite(h[i])) ++bad;
            md = std::fmax(md, std::fabs((double)h[i] - h32[i]));
            mx = std::fmax(mx, std::fabs((double)h32[i]));
        }
        const auto m = host(mats[v], n_mat);
        size_t mdiff = 0;
        for (size_t i = 0; i < n_mat; ++i) mdiff += m0[i] != m[i];
        const auto t = totals(host(parts[v], nparts[v]), tys[v] * txs[v]);
        double ds = 0, dq = 0;
        for (size_t i = 0; i < t.size(); i += 2) {
            ds = std::fmax(ds, std::fabs(t[i] - t0[i]) / (std::fabs(t0[i]) + 1e-30));
            dq = std::fmax(dq, std::fabs(t[i + 1] - t0[i + 1]) / (std::fabs(t0[i + 1]) + 1e-30));
        }
        printf("%s vs wino: max |d| rel %.3e, non-finite %zu, materialised differs %zu of %zu, S totals rel %.3e, Q totals rel %.3e\n",
               names[v], md / mx, bad, pro == PRO_NONE ? (size_t)0 : mdiff, n_mat, ds, dq);
        if (!(md / mx < 1e-5 && bad == 0 && (pro == PRO_NONE || mdiff == 0) && ds < 1e-5 && dq < 1e-5)) rc = 2;
    }
    printf("speedup x6w over x6: %.3f\n", us_v[1] / us_v[2]);
    return rc;
}
