// wino9f3_bench.hip — the 9x9 start conv of rst-960-120-128-17 (B x 480 x 960 x 17 -> 32, inference BN epilogue) on
// wino9f3 (split-bf16 x6, F(3x3, 3x3) tiles) against wino9_x6 (F(2x2, 3x3) composite) and wino9 (f32 MFMA): timing
// of each and the max difference of wino9f3's output from wino9's relative to the output scale.
// Build: bash tools/build_wino9f3_bench.sh   Run: tools/wino9f3_bench [B]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
#ifdef W9F3_PROF
namespace rst { void f3_timeline_print(int nwg); }
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
    const int B = argc > 1 ? atoi(argv[1]) : 1, C = argc > 2 ? atoi(argv[2]) : 17, H = 480, W = 960;
    auto hin = host_rand((size_t)B * H * W * C, 0, 1, 1);
    auto hk = host_rand((size_t)81 * C * 32, -0.04f, 0.04f, 2);
    auto hb = host_rand(32, -0.1f, 0.1f, 3);
    auto hbn = host_rand(64, 0.5f, 1.f, 4);
    float* in = dev(hin);
    float* U32 = dev(wino9_pack_weights(hk.data(), C));
    float* U6 = dev(wino9_x6_pack_weights(hk.data(), C));
    float* UF = dev(wino9f3_pack_weights(hk.data(), C));
    float* bias = dev(hb);
    float* bn = dev(hbn);
    size_t n_out = (size_t)B * H * W * 32;
    float *o32, *o6, *of;
    CK(hipMalloc(&o32, n_out * 4)); CK(hipMalloc(&o6, n_out * 4)); CK(hipMalloc(&of, n_out * 4));
    Wino9Args a{};
    a.in = in; a.bias = bias; a.bn_ab = reinterpret_cast<const float2*>(bn);
    a.batch = B; a.H = H; a.W = W; a.cin = C;
    CK(wino9_x6_prepare());
    CK(wino9f3_prepare());
    Wino9Args a32 = a, a6 = a, af = a;
    a32.tiles_y = wino9_tiles_y(H); a32.tiles_x = wino9_tiles_x(W); a32.U = U32; a32.out = o32;
    a6.tiles_y = wino9_x6_tiles_y(H); a6.tiles_x = wino9_x6_tiles_x(W); a6.U = U6; a6.out = o6;
    af.tiles_y = wino9f3_tiles_y(H); af.tiles_x = wino9f3_tiles_x(W); af.U = UF; af.out = of;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 50;
    for (int v = 0; v < 3; ++v) {
        auto launch = [&]() { return v == 0 ? wino9_launch(a32, 0) : v == 1 ? wino9_x6_launch(a6, 0) : wino9f3_launch(af, 0); };
        for (int i = 0; i < 5; ++i) CK(launch());
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(launch());
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%s B=%d C=%d: %.2f us/launch\n", v == 0 ? "wino9   " : v == 1 ? "wino9_x6" : "wino9f3 ", B, C, 1e3 * ms / iters);
#ifdef W9F3_PROF
        if (v == 2) rst::f3_timeline_print(B * af.tiles_y * af.tiles_x);
#endif
    }
    std::vector<float> h32(n_out), hf(n_out);
    CK(hipMemcpy(h32.data(), o32, n_out * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hf.data(), of, n_out * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    size_t bad = 0;
    for (size_t i = 0; i < n_out; ++i) {
        if (!std::isfinite(hf[i])) ++bad;
        md = std::fmax(md, std::fabs((double)hf[i] - h32[i]));
        mx = std::fmax(mx, std::fabs((double)h32[i]));
    }
    printf("max |f3 - f32| = %.3e, max |f32| = %.3e, relative %.3e, non-finite %zu\n", md, mx, md / mx, bad);
    return 0;
}
