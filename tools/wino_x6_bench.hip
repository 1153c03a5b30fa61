// wino_x6_bench.hip — residual conv of rst-960-120-128-17 (B x 120 x 240 x Cin -> 128, CIN affine + ReLU
// prologue) on wino_x6 (split-bf16 Winograd) against wino (f32-MFMA Winograd): timing of both and the
// max difference of their outputs relative to the output scale (both restate the same convolution).
// Build: bash tools/build_wino_x6_bench.sh   Run: tools/wino_x6_bench [B] [Cin]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
#ifdef X6_PROF
namespace rst { void x6_timeline_print(int nwg); }
#endif
#ifdef X6_PROF2
namespace rst { void x6_points_print(int nwg, int nchunks); }
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
    const int B = argc > 1 ? atoi(argv[1]) : 1, C = argc > 2 ? atoi(argv[2]) : 128, H = 120, W = 240;
    auto hin = host_rand((size_t)B * H * W * C, -1, 3, 1);
    auto hk = host_rand((size_t)9 * C * 128, 0.f, 0.05f, 2);          // residual init U(0, 0.05)
    auto hb = host_rand(128, -0.1f, 0.1f, 3);
    auto hab = host_rand((size_t)B * C * 2, 0.5f, 1.f, 4);
    float* in = dev(hin);
    float* U32 = dev(wino_pack_weights(hk.data(), C));
    float* U6 = dev(wino_x6_pack_weights(hk.data(), C));
    float* bias = dev(hb);
    float* ab = dev(hab);
    size_t n_out = (size_t)B * H * W * 128;
    float *o32, *o6, *mat;
    CK(hipMalloc(&o32, n_out * 4)); CK(hipMalloc(&o6, n_out * 4)); CK(hipMalloc(&mat, (size_t)B * H * W * C * 4));
    WinoArgs a{};
    a.in = in; a.res = in; a.mat = mat; a.pro_ab = reinterpret_cast<const float2*>(ab); a.bias = bias;
    a.batch = B; a.H = H; a.W = W; a.cin = C; a.tiles_y = wino_tiles_y(H); a.tiles_x = wino_tiles_x(W);
    a.pro_mode = PRO_AFF_RELU;
    float4* part; CK(hipMalloc(&part, (size_t)B * 128 * a.tiles_y * a.tiles_x * 16));
    a.part = part;
    CK(wino_prepare()); CK(wino_x6_prepare());
    WinoArgs a32 = a, a6 = a;
    a32.U = U32; a32.out = o32;
    a6.U = U6; a6.out = o6;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 200;
    for (int v = 0; v < 2; ++v) {
        const WinoArgs& x = v ? a6 : a32;
        for (int i = 0; i < 20; ++i) CK(v ? wino_x6_launch(x, 0) : wino_launch(x, 0));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(v ? wino_x6_launch(x, 0) : wino_launch(x, 0));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / iters;
        const double direct = 2.0 * B * H * W * C * 128 * 9, exec = 2.0 * B * H * W / 4 * 16 * C * 128;
#ifdef X6_PROF
        if (v) rst::x6_timeline_print(B * a.tiles_y * a.tiles_x);
#endif
#ifdef X6_PROF2
        if (v) rst::x6_points_print(B * a.tiles_y * a.tiles_x, C / 16);
#endif
        if (v) printf("wino_x6 B=%d Cin=%d: %.2f us/launch, bf16 pipe %.3f (6 terms), direct-equivalent %.1f TF/s\n", B, C,
                      us, 6 * exec / (us * 1e-6) / 2.5e15, direct / (us * 1e-6) / 1e12);
        else printf("wino    B=%d Cin=%d: %.2f us/launch, f32 pipe %.3f, direct-equivalent %.1f TF/s\n", B, C, us,
                    exec / (us * 1e-6) / 157.3e12, direct / (us * 1e-6) / 1e12);
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
