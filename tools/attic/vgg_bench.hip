// RECORD ONLY (not built): the standalone timing of tools/attic/conv_vgg.hip against conv_bf3 (round 5).
// vgg_bench.hip — VGG16 3x3 conv layers at 480x960 (B = 4) on conv_bf3's production tiles (134 / 135) and on
// conv_vgg.hip (160 / 161), plain bf16, random data, timing only (parity: tests/test_gpu_loss.py, test_gpu_train.py).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc tools/vgg_bench.hip
//        -o tools/vgg_bench      Run: tools/vgg_bench [B] [mask]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>
#include "../realtime_style_transfer_amd/csrc/conv_bf3.hip"
#include "../realtime_style_transfer_amd/csrc/conv_vgg.hip"

using namespace rst;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <typename F>
static float time_ms(F&& launch, int iters) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}
static float* dev_rand(size_t n, float lo, float hi, unsigned seed) {
    std::vector<float> h(n); srand(seed);
    for (auto& v : h) v = lo + (hi - lo) * (rand() / (float)RAND_MAX);
    float* d; CK(hipMalloc(&d, n * 4)); CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}
struct L { const char* name; int H, W, Cin, Cout; };
int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 4, msk = argc > 2 ? atoi(argv[2]) : 0;
    const L ls[] = {{"b1c2", 480, 960, 64, 64}, {"b2c1", 240, 480, 64, 128}, {"b2c2", 240, 480, 128, 128},
                    {"b3c2", 120, 240, 256, 256}, {"b4c2", 60, 120, 512, 512}, {"b5c2", 30, 60, 512, 512}};
    size_t maxact = 0, maxw = 0;
    for (const auto& l : ls) {
        maxact = std::max(maxact, (size_t)B * l.H * l.W * std::max(l.Cin, l.Cout));
        maxw = std::max(maxw, (size_t)9 * l.Cin * l.Cout);
    }
    float* in = dev_rand(maxact, -1.f, 1.f, 11);
    float* res = dev_rand(maxact, -1.f, 1.f, 14);
    float* out; CK(hipMalloc(&out, maxact * 4));
    float* w = dev_rand(maxw, -0.05f, 0.05f, 12);   // (as packed bf16 bits: timing only)
    float* bias = dev_rand(512, -0.1f, 0.1f, 13);
    for (const auto& l : ls) {
        const double fl = 2.0 * l.H * l.W * 9.0 * l.Cin * l.Cout * B;
        const double bytes = (double)B * l.H * l.W * (l.Cin * (msk ? 2 : 1) + l.Cout) * 4;
        std::vector<std::function<void()>> launches;
        std::vector<std::string> names;
        auto args = [&](const ConvTile& t) {
            ConvArgs a{};
            a.in = in; a.res = res; a.wpk = w; a.bias = bias; a.out = out;
            a.batch = B; a.H = l.H; a.W = l.W; a.cin = l.Cin; a.Ho = l.H; a.Wo = l.W;
            a.ntot = l.Cout; a.cout = l.Cout; a.pad_t = 1; a.pad_l = 1;
            a.tiles_y = (l.H + t.th - 1) / t.th; a.tiles_x = (l.W + t.tw - 1) / t.tw;
            a.n_blocks = l.Cout / t.nt; a.nchunks = (l.Cin + t.ck - 1) / t.ck;
            a.pro_mode = msk ? PRO_MASK : PRO_NONE; a.epi_mode = msk ? EPI_NONE : EPI_RELU_STATS;
            return a;
        };
        ConvTile t0, t1;
        setenv("RST_VGG_CONV", "0", 1);
        if (conv_bf3_select(3, 1, l.Cin, l.Cout, 1, (long long)B * l.H * l.W, &t0)) {
            CK(conv_bf3_prepare(t0));
            const ConvArgs a = args(t0);
            launches.push_back([=] { CK(conv_bf3_launch(t0, a, 0)); });
            names.push_back("conv_bf3 " + std::to_string(t0.id));
        }
        setenv("RST_VGG_CONV", "2", 1);
        if (conv_vgg_select(l.Cin, l.Cout, B, l.H, l.W, &t1)) {
            CK(conv_vgg_prepare(t1));
            const ConvArgs a = args(t1);
            launches.push_back([=] { CK(conv_vgg_launch(t1, a, 0)); });
            names.push_back("conv_vgg " + std::to_string(t1.id));
        }
        const int nv = (int)launches.size(), rounds = 5, iters = 10;
        for (auto& f : launches) f();
        CK(hipDeviceSynchronize());
        std::vector<std::vector<float>> t(nv);
        for (int r = 0; r < rounds; ++r)
            for (int i = 0; i < nv; ++i) t[i].push_back(time_ms(launches[i], iters));
        for (int i = 0; i < nv; ++i) {
            std::sort(t[i].begin(), t[i].end());
            const float med = t[i][rounds / 2];
            printf("%-5s %-14s B=%d %s  median %8.2f us  %7.1f TF/s  %6.2f TB/s (f32 in%s + out)\n", l.name,
                   names[i].c_str(), B, msk ? "dgrad" : "fwd  ", med * 1e3, fl / (med * 1e-3) / 1e12,
                   bytes / (med * 1e-3) / 1e12, msk ? " + mask" : "");
        }
    }
    return 0;
}
