// icache_x6.hip — does a residual conv pay for its code the first time it runs in a frame? The frame's first
// launches of wino_x6<1>, <2> and <3> ran 3.6-4.5 us longer in the graph replay than their later launches
// (profiles/r06/r06c: layer 4 <1> 34.4 us vs 29.6-30.2, layer 7 <3> 38.8 vs 35.1), and each template is 22 KB of
// code, so the CU pair's 64 KB instruction cache holds two of them at a time.
// Two graphs of B=1 Cin-128 residual convs (random data, prologue affine given), timed per launch inside the replay by
// the in-kernel end stamps (kernels.h tl_stamp_end; share = end(k) - end(k - 1)):
//   warm:  <1> <1> <1> <1> <1> <1> <1> <1>           (the same code every launch)
//   cycle: <0> <2> <3> <1> <0> <2> <3> <1>           (four templates, 88 KB of code: every launch starts cold)
// Build: bash tools/build_icache_x6.sh   Run: tools/icache_x6 [replays]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"

using namespace rst;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static std::vector<float> host_rand(size_t n, float lo, float hi, unsigned seed) {
    std::vector<float> h(n);
    srand(seed);
    for (auto& v : h) v = lo + (hi - lo) * (rand() / (float)RAND_MAX);
    return h;
}
template <typename T> static T* dev(const std::vector<T>& h) {
    T* d;
    CK(hipMalloc(&d, h.size() * sizeof(T)));
    CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 50;
    const int B = 1, C = 128, H = 120, W = 240, L = 8;
    const size_t n = (size_t)B * H * W * C;
    std::vector<float*> buf(L + 1), mat(L);
    const auto hx = host_rand(n, -1.f, 3.f, 1);
    for (auto& p : buf) p = dev(hx);
    for (auto& p : mat) CK(hipMalloc(&p, n * 4));
    float* res = dev(host_rand(n, -1.f, 1.f, 5));
    float* U = dev(wino_x6_pack_weights(host_rand((size_t)9 * C * 128, -0.05f, 0.05f, 2).data(), C));
    float* U32 = dev(wino_x6_pack_weights(host_rand((size_t)9 * 32 * 128, -0.05f, 0.05f, 2).data(), 32));
    float* bias = dev(host_rand(128, -0.1f, 0.1f, 3));
    float* ab = dev(host_rand((size_t)B * C * 2, 0.5f, 1.f, 4));
    float4* part;
    const int ty = wino_tiles_y(H), tx = wino_tiles_x(W);
    CK(hipMalloc(&part, (size_t)B * 128 * ty * tx * 16));
    unsigned long long* tl;
    CK(hipMalloc(&tl, (size_t)L * TL_SLOTS * 8));
    CK(hipMemset(tl, 0, (size_t)L * TL_SLOTS * 8));
    CK(wino_x6_prepare());
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto launch = [&](int k, int pro) {
        WinoArgs a{};
        a.in = buf[k];
        a.res = res;
        a.mat = pro == PRO_AFF || pro == PRO_AFF_RES ? mat[k] : nullptr;
        a.pro_ab = pro == PRO_NONE ? nullptr : reinterpret_cast<const float2*>(ab);
        a.U = pro == PRO_NONE ? U32 : U;
        a.bias = bias;
        a.out = buf[k + 1];
        a.part = part;
        a.batch = B; a.H = H; a.W = W; a.cin = pro == PRO_NONE ? 32 : C;
        a.tiles_y = ty; a.tiles_x = tx;
        a.pro_mode = pro;
        a.wt_stores = 3;
        a.tl = tl + (size_t)k * TL_SLOTS;
        CK(wino_x6_launch(a, st));
    };
    const int warm[L] = {1, 1, 1, 1, 1, 1, 1, 1};
    const int cycle[L] = {0, 2, 3, 1, 0, 2, 3, 1};
    for (int v = 0; v < 2; ++v) {
        const int* seq = v == 0 ? warm : cycle;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < L; ++k) launch(k, seq[k]);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        std::vector<double> sum(L, 0.0);
        std::vector<unsigned long long> h((size_t)L * TL_SLOTS);
        for (int r = 0; r < R; ++r) {
            CK(hipGraphLaunch(ge, st));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(h.data(), tl, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long prev = 0;
            for (int k = 0; k < L; ++k) {
                unsigned long long m = 0;
                for (int s = 0; s < TL_SLOTS; ++s) m = std::max(m, h[(size_t)k * TL_SLOTS + s]);
                if (k > 0) sum[k] += (double)(m - prev) * 0.01;
                prev = m;
            }
        }
        printf("%s:", v == 0 ? "warm " : "cycle");
        for (int k = 1; k < L; ++k) printf("  <%d> %.2f", seq[k], sum[k] / R);
        printf("  (us, in-graph share, %d replays)\n", R);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
