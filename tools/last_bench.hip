// last_bench.hip — standalone timing of the final 9x9 transposed conv kernels at 480x960x16 -> 3
// (B = 1, 8): last_x6 (conv_last.hip) beside the VALU small_conv_kernel (conv_small.hip).
// Build: bash tools/build_last_bench.sh   Run: ./tools/last_bench [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../realtime_style_transfer_amd/csrc/conv_last.hip"
#include "../realtime_style_transfer_amd/csrc/conv_small.hip"

using namespace rst;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float* dev_rand(size_t n, float lo, float hi, unsigned seed) {
    std::vector<float> h(n);
    srand(seed);
    for (auto& v : h) v = lo + (hi - lo) * (rand() / (float)RAND_MAX);
    float* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}

template <typename F>
static double time_us(F&& f, int iters, hipStream_t st) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) f();
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 100;
    const int H = 480, W = 960, C = 16;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    CK(last_x6_prepare());
    for (int B : {1, 8}) {
        float* in = dev_rand((size_t)B * H * W * C, -1.f, 1.f, 1);
        float* ab = dev_rand((size_t)2 * B * C, 0.5f, 1.f, 2);
        std::vector<float> kern(9 * 9 * 3 * C);
        srand(3);
        for (auto& v : kern) v = -0.05f + 0.1f * (rand() / (float)RAND_MAX);
        std::vector<float> wpk = last_x6_pack_weights(kern.data(), C);
        float* w;
        CK(hipMalloc(&w, wpk.size() * 4));
        CK(hipMemcpy(w, wpk.data(), wpk.size() * 4, hipMemcpyHostToDevice));
        float* bias = dev_rand(3, -0.1f, 0.1f, 4);
        float* out;
        CK(hipMalloc(&out, (size_t)B * H * W * 3 * 4));
        float4* part;
        CK(hipMalloc(&part, (size_t)B * 3 * 2048 * 16));
        LastArgs a{};
        a.in = in; a.pro_ab = reinterpret_cast<const float2*>(ab); a.w = w; a.bias = bias; a.out = out; a.part = part;
        a.batch = B; a.H = H; a.W = W; a.cin = C; a.tiles_y = last_x6_tiles_y(H); a.tiles_x = last_x6_tiles_x(W);
        const double us = time_us([&] { CK(last_x6_launch(a, st)); }, iters, st);
#ifdef LAST_PROF
        last_timeline_print(a.batch * ((H + lastx6::RB - 1) / lastx6::RB) * a.tiles_x);
#endif
        const double flops = 2.0 * B * H * W * 81 * C * 3;
        printf("B=%d last_x6      %8.2f us  %6.1f TFLOP/s direct-equivalent (grid %d)\n", B, us, flops / us * 1e-6,
               B * a.tiles_y * a.tiles_x);
        CK(hipFree(in)); CK(hipFree(ab)); CK(hipFree(w)); CK(hipFree(bias)); CK(hipFree(out)); CK(hipFree(part));
    }
    return 0;
}
