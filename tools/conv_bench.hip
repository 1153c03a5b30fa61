// conv_bench.hip — standalone timing harness for conv_mfma_kernel variants (no torch).
// Times kernel variants interleaved in one process (cdna_hip_programming.md §5.4 rule 24) on
// the residual-block conv of rst-960-120-128-17 (B x 120 x 240 x 128 -> 128, 3x3 s1) and the
// start conv (480 x 960 x 17 -> 32, 9x9). Build: see tools/build_conv_bench.sh.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>
#include <string>
#include "../realtime_style_transfer_amd/csrc/conv_mfma.hip"
#include "../realtime_style_transfer_amd/csrc/conv_small.hip"
#include "../realtime_style_transfer_amd/csrc/conv_bf3.hip"

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

struct Layer { int H, W, Cin, Ntot, kh, s, pad; double flops; };

template <RST_TP, int OPT>
static ConvArgs make_args(const Layer& L, int B, float* in, float* w, float* bias, float2* ab, float* out, float4* part) {
    using C = ConvCfg<RST_TA>;
    ConvArgs a{};
    a.in = in; a.res = in; a.mat = nullptr; a.pro_ab = ab; a.wpk = w; a.bias = bias; a.bn_ab = ab; a.out = out; a.part = part;
    a.batch = B; a.H = L.H; a.W = L.W; a.cin = L.Cin;
    a.Ho = (L.H + L.s - 1) / L.s; a.Wo = (L.W + L.s - 1) / L.s; a.ntot = L.Ntot; a.cout = L.Ntot;
    a.pad_t = L.pad; a.pad_l = L.pad;
    a.tiles_y = (a.Ho + TH - 1) / TH; a.tiles_x = (a.Wo + TW - 1) / TW;
    a.n_blocks = (L.Ntot + NT - 1) / NT; a.nchunks = (L.Cin + CK - 1) / CK;
    a.pro_mode = L.Cin % 4 == 0 ? PRO_AFF_RELU : PRO_NONE; a.epi_mode = L.Cin % 4 == 0 ? EPI_RELU_STATS : EPI_RELU_BN;
    a.shuffle = 0;
    return a;
}

template <RST_TP, int OPT>
struct Variant {
    const char* name;
    ConvArgs a;
    unsigned grid;
    void setup(const char* n, const Layer& L, int B, float* in, float* w, float* bias, float2* ab, float* out, float4* part) {
        using C = ConvCfg<RST_TA>;
        name = n;
        a = make_args<RST_TA, OPT>(L, B, in, w, bias, ab, out, part);
        grid = (unsigned)(B * a.tiles_y * a.tiles_x * a.n_blocks);
        CK(hipFuncSetAttribute((const void*)conv_mfma_kernel<RST_TA, OPT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)C::LDS_BYTES));
        printf("%-40s LDS %6zu B  grid %u\n", n, (size_t)C::LDS_BYTES, grid);
    }
    void launch() {
        using C = ConvCfg<RST_TA>;
        hipLaunchKernelGGL((conv_mfma_kernel<RST_TA, OPT>), dim3(grid), dim3(256), C::LDS_BYTES, 0, a);
    }
};

// VGG16 3x3 layers of the training loss (480 x 960 input, B images), plain bf16 (NP = 1) tiles
struct VggLayer { const char* name; int H, W, Cin, Cout; };
static int run_vgg(int B) {
    const VggLayer L[] = {{"b1c2", 480, 960, 64, 64},   {"b2c1", 240, 480, 64, 128}, {"b2c2", 240, 480, 128, 128},
                          {"b3c2", 120, 240, 256, 256}, {"b4c2", 60, 120, 512, 512}, {"b5c2", 30, 60, 512, 512}};
    const int iters = 10, rounds = 5;
    size_t maxact = 0, maxw = 0;
    for (const auto& l : L) {
        maxact = std::max(maxact, (size_t)B * l.H * l.W * std::max(l.Cin, l.Cout));
        maxw = std::max(maxw, (size_t)9 * l.Cin * l.Cout);
    }
    float* in = dev_rand(maxact, 0.f, 1.f, 11);
    float* out; CK(hipMalloc(&out, maxact * 4));
    float* w = dev_rand(maxw, -0.05f, 0.05f, 12);
    float* bias = dev_rand(512, -0.1f, 0.1f, 13);
    for (const auto& l : L) {
        const double fl = 2.0 * l.H * l.W * 9.0 * l.Cin * l.Cout * B;
        std::vector<std::function<void()>> launches;
        std::vector<const char*> names;
#define VV(CK_, NT, TH, TW, WM, WN, TPS, PF, NAME)                                                            \
        if (l.Cout % NT == 0) {                                                                            \
            using BC = Bf3Cfg<3, 3, 1, CK_, NT, TH, TW, WM, WN, TPS, 1, PF>;                                   \
            ConvArgs a{};                                                                                  \
            a.in = in; a.res = in; a.wpk = w; a.bias = bias; a.out = out;                                  \
            a.batch = B; a.H = l.H; a.W = l.W; a.cin = l.Cin; a.Ho = l.H; a.Wo = l.W;                      \
            a.ntot = l.Cout; a.cout = l.Cout; a.pad_t = 1; a.pad_l = 1;                                    \
            a.tiles_y = (l.H + TH - 1) / TH; a.tiles_x = (l.W + TW - 1) / TW;                              \
            a.n_blocks = l.Cout / NT; a.nchunks = (l.Cin + CK_ - 1) / CK_;                                 \
            a.pro_mode = PRO_NONE; a.epi_mode = EPI_RELU_STATS;                                            \
            const unsigned g = (unsigned)(B * a.tiles_y * a.tiles_x * a.n_blocks);                         \
            CK(hipFuncSetAttribute((const void*)conv_bf3_kernel<3, 3, 1, CK_, NT, TH, TW, WM, WN, TPS, 1, PF>, \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)BC::LDS_BYTES));       \
            launches.push_back([=] {                                                                       \
                hipLaunchKernelGGL((conv_bf3_kernel<3, 3, 1, CK_, NT, TH, TW, WM, WN, TPS, 1, PF>), dim3(g),   \
                                   dim3(256), BC::LDS_BYTES, 0, a);                                        \
            });                                                                                            \
            names.push_back(NAME);                                                                         \
        }
        VV(32, 64, 8, 16, 4, 1, 3, 0, "134 NT64 8x16 WM4 TPS3 (prod)")
        VV(32, 128, 8, 16, 2, 2, 3, 0, "135 NT128 8x16 WM2 TPS3 (prod)")
        VV(32, 128, 8, 16, 2, 2, 3, 2, "136 = 135 + 2-stage weight prefetch")
        VV(32, 128, 8, 16, 2, 2, 3, 3, "135 + 2-stage wts + halo PF")
        VV(32, 64, 8, 16, 4, 1, 3, 2, "134 + 2-stage weight prefetch")
#undef VV
        const int nv = (int)launches.size();
        std::vector<std::vector<float>> t(nv);
        for (int r = 0; r < rounds; ++r)
            for (int i = 0; i < nv; ++i) t[i].push_back(time_ms(launches[i], iters));
        for (int i = 0; i < nv; ++i) {
            std::sort(t[i].begin(), t[i].end());
            const float med = t[i][rounds / 2];
            printf("%-5s %-34s B=%d  median %8.2f us  %7.1f TF/s\n", l.name, names[i], B, med * 1e3,
                   fl / (med * 1e-3) / 1e12);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}


// The small transfer-net layers of rst-960-120-128-17 at B=1: stride-2 contract convs and the
// 4-phase (2x2) expand convs (output channel shuffle to 2H x 2W)
struct SmallLayer { const char* name; int kh, s, H, W, Cin, Ntot, shuffle; };
static int run_small(int B) {
    const SmallLayer L[] = {{"c0", 3, 2, 480, 960, 32, 16, 0}, {"c1", 3, 2, 240, 480, 16, 32, 0},
                            {"e0", 2, 1, 120, 240, 128, 128, 1}, {"e1", 2, 1, 240, 480, 32, 64, 1}};
    const int iters = 20, rounds = 7;
    const size_t maxact = (size_t)B * 480 * 960 * 64;
    float* in = dev_rand(maxact, 0.f, 1.f, 21);
    float* out; CK(hipMalloc(&out, maxact * 4));
    float* w = dev_rand((size_t)9 * 128 * 256 * 2, -0.05f, 0.05f, 22);
    float* bias = dev_rand(512, -0.1f, 0.1f, 23);
    float2* ab = (float2*)dev_rand(2 * 512 * B, 0.5f, 1.5f, 24);
    float4* part; CK(hipMalloc(&part, (size_t)B * 256 * 8192 * 16));
    for (const auto& l : L) {
        const int Ho = l.shuffle ? l.H : (l.H + l.s - 1) / l.s, Wo = l.shuffle ? l.W : (l.W + l.s - 1) / l.s;
        const double fl = l.shuffle ? 2.0 * Ho * Wo * 4 * l.Cin * l.Ntot * B
                                    : 2.0 * Ho * Wo * 9.0 * l.Cin * l.Ntot * B;
        const double by = 4.0 * B * ((double)l.H * l.W * l.Cin + (double)Ho * Wo * l.Ntot);
        std::vector<std::function<void()>> launches;
        std::vector<const char*> names;
#define VM(KH, S, CK_, NT, TH, TW, WM, WN, TPS, NAME)                                                          \
        if (l.kh == KH && l.s == S && (l.Ntot % NT == 0 || l.Ntot < NT) && l.Cin % CK_ == 0) {                                   \
            using C = ConvCfg<KH, KH, S, CK_, NT, TH, TW, WM, WN, TPS, 1>;                                      \
            ConvArgs a{};                                                                                       \
            a.in = in; a.res = in; a.pro_ab = ab; a.wpk = w; a.bias = bias; a.bn_ab = ab; a.out = out;          \
            a.part = part;                                                                                      \
            a.batch = B; a.H = l.H; a.W = l.W; a.cin = l.Cin; a.Ho = Ho; a.Wo = Wo;                             \
            a.ntot = l.Ntot; a.cout = l.shuffle ? l.Ntot / 4 : l.Ntot; a.shuffle = l.shuffle;                  \
            a.pad_t = l.shuffle ? 0 : 0; a.pad_l = a.pad_t;                                                     \
            a.tiles_y = (Ho + TH - 1) / TH; a.tiles_x = (Wo + TW - 1) / TW;                                     \
            a.n_blocks = (l.Ntot + NT - 1) / NT; a.nchunks = (l.Cin + CK_ - 1) / CK_;                              \
            a.pro_mode = PRO_AFF_RELU; a.epi_mode = EPI_RELU_STATS;                                            \
            const unsigned g = (unsigned)(B * a.tiles_y * a.tiles_x * a.n_blocks);                              \
            CK(hipFuncSetAttribute((const void*)conv_mfma_kernel<KH, KH, S, CK_, NT, TH, TW, WM, WN, TPS, 1, 1>, \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::LDS_BYTES));             \
            launches.push_back([=] {                                                                             \
                hipLaunchKernelGGL((conv_mfma_kernel<KH, KH, S, CK_, NT, TH, TW, WM, WN, TPS, 1, 1>), dim3(g),   \
                                   dim3(256), C::LDS_BYTES, 0, a);                                              \
            });                                                                                                  \
            names.push_back(NAME);                                                                               \
        }
        VM(3, 2, 16, 32, 8, 16, 4, 1, 3, "3 s2 CK16 NT32 8x16 TPS3 (prod)")
        VM(3, 2, 16, 32, 16, 16, 4, 1, 3, "s2 CK16 NT32 16x16 TPS3")
        VM(3, 2, 16, 32, 8, 16, 4, 1, 9, "s2 CK16 NT32 8x16 TPS9")
        VM(3, 2, 16, 32, 8, 16, 4, 1, 1, "s2 CK16 NT32 8x16 TPS1")
        VM(3, 2, 32, 32, 8, 16, 4, 1, 3, "s2 CK32 NT32 8x16 TPS3")
        VM(3, 2, 32, 32, 8, 16, 4, 1, 1, "s2 CK32 NT32 8x16 TPS1")
        VM(3, 2, 8, 32, 8, 16, 4, 1, 3, "4 s2 CK8 NT32 8x16 TPS3")
        VM(2, 1, 32, 128, 4, 16, 2, 2, 1, "8 2x2 CK32 NT128 4x16 (prod)")
        VM(2, 1, 32, 64, 8, 16, 2, 2, 1, "9 2x2 CK32 NT64 8x16 (prod)")
        VM(2, 1, 32, 128, 8, 16, 2, 2, 1, "2x2 CK32 NT128 8x16")
        VM(2, 1, 32, 32, 8, 16, 4, 1, 4, "10 2x2 CK32 NT32 8x16 TPS4")
        VM(2, 1, 32, 64, 4, 16, 2, 2, 1, "2x2 CK32 NT64 4x16")
        VM(2, 1, 32, 64, 16, 16, 4, 1, 1, "2x2 CK32 NT64 16x16 WM4")
        VM(2, 1, 16, 64, 8, 16, 2, 2, 1, "2x2 CK16 NT64 8x16")
#undef VM
        const int nv = (int)launches.size();
        std::vector<std::vector<float>> t(nv);
        for (int r = 0; r < rounds; ++r)
            for (int i = 0; i < nv; ++i) t[i].push_back(time_ms(launches[i], iters));
        for (int i = 0; i < nv; ++i) {
            std::sort(t[i].begin(), t[i].end());
            const float med = t[i][rounds / 2];
            printf("%-3s %-34s B=%d  median %7.2f us  %6.1f TF/s  %6.0f GB/s\n", l.name, names[i], B, med * 1e3,
                   fl / (med * 1e-3) / 1e12, by / (med * 1e-3) / 1e9);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}

int main(int argc, char** argv) {
    int B = argc > 1 ? atoi(argv[1]) : 1;
    if (argc > 2 && std::string(argv[2]) == "vgg") return run_vgg(B);
    if (argc > 2 && std::string(argv[2]) == "small") return run_small(B);
    const int iters = 20, rounds = 7;
    Layer res{120, 240, 128, 128, 3, 1, 1, 2.0 * 120 * 240 * 9 * 128 * 128};
    float* in = dev_rand((size_t)B * 120 * 240 * 128, 0.f, 1.f, 1);
    float* w = dev_rand((size_t)9 * 128 * 128 * 2, -0.05f, 0.05f, 2);
    float* bias = dev_rand(256, -0.1f, 0.1f, 3);
    float2* ab = (float2*)dev_rand(2 * 128 * B, 0.5f, 1.5f, 4);
    float* out; CK(hipMalloc(&out, (size_t)B * 120 * 240 * 128 * 4));
    float4* part; CK(hipMalloc(&part, (size_t)B * 128 * 4096 * 16));

    Layer start{480, 960, 17, 32, 9, 1, 4, 2.0 * 480 * 960 * 81 * 17 * 32};
    float* in_s = dev_rand((size_t)B * 480 * 960 * 17, 0.f, 1.f, 5);
    float* out_s; CK(hipMalloc(&out_s, (size_t)B * 480 * 960 * 32 * 4));
    float* w_s = dev_rand((size_t)81 * 18 * 32, -0.05f, 0.05f, 6);
#define VARIANTS(X)                                                   \
    X(3, 3, 1, 32, 128, 4, 16, 2, 2, 1, 1, 1, "res CK32 NT128 4x16 TPS1 HB1 (prod)", res, in, w, out) \
    X(3, 3, 1, 32, 128, 4, 16, 2, 2, 1, 2, 1, "res CK32 NT128 4x16 TPS1 HB2", res, in, w, out) \
    X(3, 3, 1, 32, 64, 8, 16, 2, 2, 1, 1, 1, "res CK32 NT64 8x16 TPS1 HB1", res, in, w, out) \
    X(3, 3, 1, 32, 64, 8, 16, 2, 2, 3, 1, 1, "res CK32 NT64 8x16 TPS3 HB1", res, in, w, out) \
    X(3, 3, 1, 16, 128, 4, 16, 2, 2, 3, 1, 1, "res CK16 NT128 4x16 TPS3 HB1", res, in, w, out) \
    X(3, 3, 1, 16, 128, 4, 16, 2, 2, 9, 1, 1, "res CK16 NT128 4x16 TPS9 HB1", res, in, w, out) \
    X(3, 3, 1, 32, 128, 4, 16, 2, 2, 3, 1, 1, "res CK32 NT128 4x16 TPS3 HB1", res, in, w, out) \
    X(3, 3, 1, 32, 128, 8, 16, 4, 1, 1, 1, 1, "res CK32 NT128 8x16 WM4 TPS1", res, in, w, out) \
    X(3, 3, 1, 32, 64, 4, 16, 2, 2, 1, 1, 1, "res CK32 NT64 4x16 TPS1 HB1", res, in, w, out) \
    X(3, 3, 1, 32, 64, 4, 16, 2, 2, 3, 1, 1, "res CK32 NT64 4x16 TPS3 HB1", res, in, w, out) \
    X(9, 9, 1, 18, 32, 8, 16, 4, 1, 3, 1, 1, "start CK18 NT32 8x16 TPS3 (prod)", start, in_s, w_s, out_s) \
    X(9, 9, 1, 18, 32, 8, 16, 4, 1, 9, 1, 1, "start CK18 NT32 8x16 TPS9", start, in_s, w_s, out_s) \
    X(9, 9, 1, 18, 32, 16, 16, 4, 1, 3, 1, 1, "start CK18 NT32 16x16 TPS3", start, in_s, w_s, out_s)
    int nv = 0;
    std::vector<std::function<void()>> launches;
    std::vector<const char*> names;
    std::vector<double> flops;
#define X(KH, KW, S, CK_, NT, TH, TW, WM, WN, TPS, HB, OPT, NAME, LAY, IN, WW, OUT)      \
    {                                                                                     \
        auto* v = new Variant<KH, KW, S, CK_, NT, TH, TW, WM, WN, TPS, HB, OPT>();         \
        v->setup(NAME, LAY, B, IN, WW, bias, ab, OUT, part);                              \
        flops.push_back(LAY.flops);                                                       \
        launches.push_back([v] { v->launch(); });                                         \
        names.push_back(NAME);                                                            \
        ++nv;                                                                             \
    }
    VARIANTS(X)
#undef X
    // final 9x9 -> 3 channel layer (VALU kernel), 480 x 960 x 16
    float* in_l = dev_rand((size_t)B * 480 * 960 * 16, 0.f, 1.f, 7);
    float* w_l = dev_rand((size_t)9 * 16 * 28, -0.05f, 0.05f, 8);
    float* out_l; CK(hipMalloc(&out_l, (size_t)B * 480 * 960 * 3 * 4));
    SmallConvArgs sa{};
    sa.in = in_l; sa.pro_ab = ab; sa.w = w_l; sa.bias = bias; sa.out = out_l; sa.part = part;
    sa.batch = B; sa.H = 480; sa.W = 960; sa.cin = 16; sa.tiles_y = small_conv_tiles_y(480); sa.tiles_x = small_conv_tiles_x(960);
    const unsigned sgrid = (unsigned)(B * sa.tiles_y * sa.tiles_x);
    const double sflops = 2.0 * 480 * 960 * 81 * 16 * 3;
#define SV(OPTV, NAME)                                                                                  \
    launches.push_back([=] { hipLaunchKernelGGL(small_conv_kernel<OPTV>, dim3(sgrid), dim3(256), 0, 0, sa, w_l, in_l); }); \
    names.push_back(NAME); flops.push_back(sflops); ++nv;
    SV(0, "small opt0 (s_load, q loop)")
    SV(1, "small opt1 (s_load, q unrolled)")
    SV(2, "small opt2 (LDS weights)")
    SV(3, "small opt3 (LDS weights, q unrolled)")
    // split-bf16 (bf16x3) residual conv variants: timing only (random weight bits)
#define BV(KH, KW, S, CK_, NT, TH, TW, WM, WN, TPS, NP, PF, NAME)                                               \
    {                                                                                                    \
        using BC = Bf3Cfg<KH, KW, S, CK_, NT, TH, TW, WM, WN, TPS, NP, PF>;                                  \
        ConvArgs ba = make_args<KH, KW, S, CK_, NT, TH, TW, WM, WN, 1, 1, 1>(res, B, in, w, bias, ab, out, part); \
        const unsigned bgrid = (unsigned)(B * ba.tiles_y * ba.tiles_x * ba.n_blocks);                    \
        CK(hipFuncSetAttribute((const void*)conv_bf3_kernel<KH, KW, S, CK_, NT, TH, TW, WM, WN, TPS, NP, PF>, \
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)BC::LDS_BYTES));         \
        printf("%-40s LDS %6zu B  grid %u\n", NAME, (size_t)BC::LDS_BYTES, bgrid);                        \
        launches.push_back([=] {                                                                         \
            hipLaunchKernelGGL((conv_bf3_kernel<KH, KW, S, CK_, NT, TH, TW, WM, WN, TPS, NP, PF>), dim3(bgrid), \
                               dim3(256), BC::LDS_BYTES, 0, ba);                                         \
        });                                                                                              \
        names.push_back(NAME); flops.push_back(res.flops); ++nv;                                         \
    }
    BV(3, 3, 1, 32, 64, 4, 16, 2, 2, 1, 2, 0, "bf16x3 res NT64 4x16 (prod)")
    BV(3, 3, 1, 32, 64, 4, 16, 2, 2, 1, 2, 1, "bf16x3 res NT64 4x16 PF")
    BV(3, 3, 1, 32, 64, 8, 16, 2, 2, 3, 2, 1, "bf16x3 res NT64 8x16 TPS3 PF")
    BV(3, 3, 1, 32, 64, 8, 16, 2, 2, 1, 3, 0, "bf16x6 res NT64 8x16 (prod)")
    BV(3, 3, 1, 32, 64, 8, 16, 2, 2, 1, 3, 1, "bf16x6 res NT64 8x16 PF")
    BV(3, 3, 1, 32, 64, 8, 16, 2, 2, 3, 3, 1, "bf16x6 res NT64 8x16 TPS3 PF")
    BV(3, 3, 1, 32, 64, 8, 16, 2, 2, 3, 1, 1, "bf16 res NT64 8x16 TPS3 PF (133)")
    BV(3, 3, 1, 32, 128, 8, 16, 2, 2, 3, 1, 1, "bf16 res NT128 8x16 TPS3 PF (132)")
    std::vector<std::vector<float>> t(nv);
    for (int r = 0; r < rounds; ++r)
        for (int i = 0; i < nv; ++i) t[i].push_back(time_ms(launches[i], iters));
    for (int i = 0; i < nv; ++i) {
        std::sort(t[i].begin(), t[i].end());
        const float med = t[i][rounds / 2];
        printf("%-40s B=%d  median %8.2f us  min %8.2f us  %7.2f TF/s\n", names[i], B, med * 1e3, t[i][0] * 1e3,
               flops[i] * B / (med * 1e-3) / 1e12);
    }
    return 0;
}
