// wgrad_bench.hip — weight gradient of a residual conv of rst-960-120-128-17 (3x3 s1 SAME, 128 -> 128,
// B x 120 x 240) on the f32-MFMA kernel and on the split-bf16 x6 kernel: timing of both (kernel + slab
// reduction) and the max difference of the two gradients relative to their scale.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc \
//            tools/wgrad_bench.hip realtime_style_transfer_amd/csrc/wgrad.hip -o tools/wgrad_bench
// Run: tools/wgrad_bench [B]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "kernels.h"
#include "train.h"

using namespace rst;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static float* dev_rand(size_t n, float lo, float hi, unsigned seed) {
    std::vector<float> h(n);
    srand(seed);
    for (auto& v : h) v = lo + (hi - lo) * (rand() / (float)RAND_MAX);
    float* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 4, H = 120, W = 240, C = 128;
    float* X = dev_rand((size_t)B * H * W * C, 0.f, 3.f, 1);      // post-ReLU-like input
    float* D = dev_rand((size_t)B * H * W * C, -1.f, 1.f, 2);     // output gradient
    WgradArgs a{};
    a.X = X;
    a.D = D;
    a.batch = B;
    a.XH = H; a.XW = W; a.C1 = C;
    a.DH = H; a.DW = W; a.C2 = C;
    a.Qh = H; a.Qw = W;
    a.kh = a.kw = 3; a.stride = 1; a.pad_t = a.pad_l = 1;
    a.transposed = 0;
    // each variant's own split count (x6 = 1: the tap-row kernel unless RST_WGRAD_X6R=0); one slab for the larger
    size_t slab_bytes = 0;
    for (int v = 0; v < 2; ++v) {
        WgradArgs x = a;
        x.x6 = v;
        x.nsplit = wgrad_choose_splits(x);
        slab_bytes = std::max(slab_bytes, wgrad_slab_bytes(x));
    }
    float* slab;
    CK(hipMalloc(&slab, slab_bytes));
    a.slab = slab;
    const size_t nw = (size_t)9 * C * C;
    float *dw0, *dw1;
    CK(hipMalloc(&dw0, nw * 4));
    CK(hipMalloc(&dw1, nw * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 50;
    for (int v = 0; v < 2; ++v) {
        WgradArgs x = a;
        x.x6 = v;
        x.nsplit = wgrad_choose_splits(x);
        x.dW = v ? dw1 : dw0;
        for (int i = 0; i < 3; ++i) CK(wgrad_launch(x, 0));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(wgrad_launch(x, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / iters, flops = 2.0 * B * H * W * 9.0 * C * C;
        printf("%s B=%d nsplit=%d: %.1f us (kernel + reduce), %.1f TFLOP/s algorithmic\n", v ? "wgrad_x6  " : "wgrad_mfma",
               B, x.nsplit, us, flops / us * 1e-6);
    }
    std::vector<float> h0(nw), h1(nw);
    CK(hipMemcpy(h0.data(), dw0, nw * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), dw1, nw * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    size_t bad = 0;
    for (size_t i = 0; i < nw; ++i) {
        if (!std::isfinite(h1[i])) ++bad;
        md = std::fmax(md, std::fabs((double)h1[i] - h0[i]));
        mx = std::fmax(mx, std::fabs((double)h0[i]));
    }
    printf("max |x6 - f32| = %.3e, max |f32| = %.3e, relative %.3e, non-finite %zu\n", md, mx, md / mx, bad);
    return (md / mx < 1e-5 && bad == 0) ? 0 : 2;
}
