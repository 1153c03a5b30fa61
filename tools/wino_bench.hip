// wino_bench.hip — standalone timing + phase profile of wino_conv_kernel (no torch).
// Residual conv of rst-960-120-128-17: 1 x 120 x 240 x 128 -> 128, prologue affine + ReLU.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DWINO_PROF=225 -I include
//        -I realtime_style_transfer_amd/csrc tools/wino_bench.hip -o tools/wino_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../realtime_style_transfer_amd/csrc/wino.hip"

using namespace rst;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static float* dev_rand(size_t n, float lo, float hi, unsigned seed) {
    std::vector<float> h(n); srand(seed);
    for (auto& v : h) v = lo + (hi - lo) * (rand() / (float)RAND_MAX);
    float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1, H = 120, W = 240, C = 128;
    float* in = dev_rand((size_t)B * H * W * C, -1, 1, 1);
    float* U = dev_rand((size_t)C / 8 * 16 * 128 * 8, -0.05f, 0.05f, 2);
    float* bias = dev_rand(128, -0.1f, 0.1f, 3);
    float* ab = dev_rand((size_t)B * C * 2, 0.5f, 1.f, 4);
    float* out; CK(hipMalloc(&out, (size_t)B * H * W * C * 4));
    float* mat; CK(hipMalloc(&mat, (size_t)B * H * W * C * 4));
    WinoArgs a{};
    a.in = in; a.res = in; a.mat = mat; a.pro_ab = reinterpret_cast<const float2*>(ab); a.U = U; a.bias = bias;
    a.out = out; a.batch = B; a.H = H; a.W = W; a.cin = C; a.tiles_y = wino_tiles_y(H); a.tiles_x = wino_tiles_x(W);
    a.pro_mode = PRO_AFF_RELU;
    float4* part; CK(hipMalloc(&part, (size_t)B * 128 * a.tiles_y * a.tiles_x * 16));
    a.part = part;
    CK(wino_prepare());
    for (int i = 0; i < 20; ++i) CK(wino_launch(a, 0));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 200;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) CK(wino_launch(a, 0));
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = 2.0 * B * H * W * C * C * 9;
    printf("wino B=%d: %.2f us/launch, %.1f TFLOP/s direct-equivalent, MFMA pipe %.3f\n", B, 1e3 * ms / iters,
           flops / (ms / iters * 1e-3) / 1e12, flops / (ms / iters * 1e-3) / 1e12 * 16 / 36 / 157.3);
#ifdef WINO_PROF
    const int nwg = WINO_PROF;
    std::vector<unsigned long long> pr((size_t)nwg * 4 * 16 * 8);
    CK(hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(wino_prof), pr.size() * 8));
    double ph[8] = {0}; double tot = 0; int n = 0;
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 4; ++w) {
            const unsigned long long* p = &pr[((size_t)g * 4 + w) * 128];
            for (int c = 1; c < 15; ++c) {   // steady-state chunks
                const unsigned long long* q = p + c * 8;
                for (int k = 0; k < 3; ++k) ph[k] += (double)(q[k + 1] - q[k]);
                ph[3] += (double)(p[(c + 1) * 8] - q[3]);
                tot += (double)(p[(c + 1) * 8] - q[0]);
                ++n;
            }
        }
    const char* nm[4] = {"stage+load", "mfma loop", "barrier", "loop"};
    printf("per-chunk phase (s_memtime ticks, mean over %d wave-chunks): total %.1f\n", n, tot / n);
    for (int k = 0; k < 4; ++k) printf("  %-11s %8.1f  (%.1f%%)\n", nm[k], ph[k] / n, 100 * ph[k] / tot);
    const unsigned long long* p0 = &pr[0];
    printf("WG0 wave0 first chunk start->end of chunk 15: %llu ticks\n", p0[15 * 8 + 3] - p0[0]);
    // timeline of the LAST launch (100 MHz clock, 10 ns ticks), over all profiled workgroups
    std::vector<unsigned long long> tl((size_t)nwg * 4 * 4);
    CK(hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(wino_tl), tl.size() * 8));
    unsigned long long t0 = ~0ull, tend = 0, s_last = 0;
    double fill = 0, loop = 0, epi = 0;
    for (int g = 0; g < nwg; ++g)
        for (int w = 0; w < 4; ++w) {
            const unsigned long long* q = &tl[((size_t)g * 4 + w) * 4];
            t0 = q[0] < t0 ? q[0] : t0;
            tend = q[3] > tend ? q[3] : tend;
            s_last = q[0] > s_last ? q[0] : s_last;
            fill += (double)(q[1] - q[0]); loop += (double)(q[2] - q[1]); epi += (double)(q[3] - q[2]);
        }
    const double nw = nwg * 4.0;
    printf("timeline (us): first start -> last end %.2f, last wave start at +%.2f; per wave: fill %.2f, "
           "chunk loop %.2f, epilogue %.2f\n", (tend - t0) * 0.01, (s_last - t0) * 0.01, fill / nw * 0.01,
           loop / nw * 0.01, epi / nw * 0.01);
    // histogram of wave end times
    int hist[10] = {0};
    for (int g = 0; g < nwg; ++g) {
        const unsigned long long e = tl[((size_t)g * 4 + 0) * 4 + 3];
        int k = (int)(10.0 * (e - t0) / (double)(tend - t0 + 1)); hist[k > 9 ? 9 : k]++;
    }
    printf("WG end-time deciles:"); for (int k = 0; k < 10; ++k) printf(" %d", hist[k]); printf("\n");
#endif
    return 0;
}
