// wino9_x6_bench.hip — the 9x9 start conv of rst-960-120-128-17 (B x 480 x 960 x 17 -> 32, inference BN
// epilogue) on wino9_x6 (split-bf16 composite Winograd) against wino9 (f32-MFMA composite Winograd):
// timing of both and the max difference of their outputs relative to the output scale.
// Build: bash tools/build_wino9_x6_bench.sh   Run: tools/wino9_x6_bench [B]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
#ifdef W9_PROF
namespace rst { void w9_timeline_print(int nwg); }
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

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1, C = 17, H = 480, W = 960;
    auto hin = host_rand((size_t)B * H * W * C, 0, 1, 1);
    auto hk = host_rand((size_t)81 * C * 32, -0.04f, 0.04f, 2);
    auto hb = host_rand(32, -0.1f, 0.1f, 3);
    auto hbn = host_rand(64, 0.5f, 1.f, 4);
    float* in = dev(hin);
    float* U32 = dev(wino9_pack_weights(hk.data(), C));
    float* U6 = dev(wino9_x6_pack_weights(hk.data(), C));
    float* bias = dev(hb);
    float* bn = dev(hbn);
    size_t n_out = (size_t)B * H * W * 32;
    float *o32, *o6;
    CK(hipMalloc(&o32, n_out * 4)); CK(hipMalloc(&o6, n_out * 4));
    Wino9Args a{};
    a.in = in; a.bias = bias; a.bn_ab = reinterpret_cast<const float2*>(bn);
    a.batch = B; a.H = H; a.W = W; a.cin = C; a.tiles_y = wino9_tiles_y(H); a.tiles_x = wino9_tiles_x(W);
    CK(wino9_x6_prepare());
    Wino9Args a32 = a, a6 = a;
    a6.tiles_y = wino9_x6_tiles_y(H);
    a6.tiles_x = wino9_x6_tiles_x(W);
    a32.U = U32; a32.out = o32;
    a6.U = U6; a6.out = o6;
    if (getenv("W9_QUEUE")) {   // the inference work queue (rst_api passes it), zeroed once, self-resetting
        unsigned* q;
        CK(hipMalloc(&q, 8));
        CK(hipMemset(q, 0, 8));
        a6.queue = q;
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 50;
    for (int v = 0; v < 2; ++v) {
        const Wino9Args& x = v ? a6 : a32;
        for (int i = 0; i < 5; ++i) CK(v ? wino9_x6_launch(x, 0) : wino9_launch(x, 0));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(v ? wino9_x6_launch(x, 0) : wino9_launch(x, 0));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%s B=%d: %.2f us/launch\n", v ? "wino9_x6" : "wino9   ", B, 1e3 * ms / iters);
#ifdef W9_PROF
        if (v) rst::w9_timeline_print(B * a6.tiles_y * a6.tiles_x);
#endif
    }
    std::vector<float> h32(n_out), h6(n_out);
    CK(hipMemcpy(h32.data(), o32, n_out * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h6.data(), o6, n_out * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    size_t bad = 0;
    for (size_t i = 0; i < n_out; ++i) {
        if (!std::isfinite(h6[i])) ++bad;
        md = std::fmax(md, std::fabs((double)h6[i] - h32[i]));
        mx = std::fmax(mx, std::fabs((double)h32[i]));
    }
    printf("max |x6 - f32| = %.3e, max |f32| = %.3e, relative %.3e, non-finite %zu\n", md, mx, md / mx, bad);
    return (md / mx < 1e-5 && bad == 0) ? 0 : 2;
}
