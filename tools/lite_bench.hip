// lite_bench.hip — standalone timing of the narrow-conv kernels (conv_lite.hip) on the headline shapes
// (rst-960-120-128-17, B = 1 and 8): contract_0 480x960x32 -> 16, contract_1 240x480x16 -> 32,
// expand_0 120x240x128 -> 32 (x4 phases), expand_1 240x480x32 -> 16 (x4 phases).
// Build: bash tools/build_lite_bench.sh   Run: ./tools/lite_bench [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <vector>

#ifndef LITE_X6
#define LITE_X6 0
#endif
#include "../realtime_style_transfer_amd/csrc/conv_lite.hip"

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

struct Shape { const char* name; int kind, H, W, cin, cout, pro; };

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const Shape shapes[] = {{"contract_0", 0, 480, 960, 32, 16, PRO_NONE},
                            {"contract_1", 0, 240, 480, 16, 32, PRO_NONE},
                            {"expand_0", 1, 120, 240, 128, 32, PRO_AFF_RES},
                            {"expand_1", 1, 240, 480, 32, 16, PRO_AFF_RELU}};
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int B : {1, 8})
        for (const Shape& s : shapes) {
            LiteTile t{};
            if (!conv_lite_select(s.kind, 3, 2, s.cin, s.cout, LITE_X6 != 0, &t)) { printf("no tile for %s\n", s.name); return 1; }
            CK(conv_lite_prepare(t));
            const int Ho = s.kind == 0 ? (s.H + 1) / 2 : s.H, Wo = s.kind == 0 ? (s.W + 1) / 2 : s.W;
            const size_t nin = (size_t)B * s.H * s.W * s.cin;
            const size_t nout = (size_t)B * (s.kind == 0 ? Ho * Wo : 4 * Ho * Wo) * s.cout;
            float* in = dev_rand(nin, -1.f, 1.f, 1);
            float* res = dev_rand(nin, -1.f, 1.f, 2);
            // the packed weight image of a random kernel (the x6 image is 1.5x the f32 one)
            std::vector<float> hk((size_t)9 * s.cin * s.cout);
            srand(3);
            for (auto& v : hk) v = -0.1f + 0.2f * (rand() / (float)RAND_MAX);
            const std::vector<float> pk = conv_lite_pack_weights(t, hk.data());
            float* w;
            CK(hipMalloc(&w, pk.size() * 4));
            CK(hipMemcpy(w, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
            float* bias = dev_rand(s.cout, -0.1f, 0.1f, 4);
            // prologue affine [B][cin] and the epilogue BatchNorm affine [cout] read from one buffer
            const size_t nab = (size_t)2 * B * (s.cin > s.cout ? s.cin : s.cout);
            float* ab = dev_rand(nab, 0.5f, 1.f, 5);
            float* out;
            CK(hipMalloc(&out, nout * 4));
            const int tiles_y = (Ho + t.th - 1) / t.th, tiles_x = (Wo + t.tw - 1) / t.tw;
            float4* part;
            CK(hipMalloc(&part, (size_t)B * s.cout * tiles_y * tiles_x * 16));
            ConvArgs a{};
            a.in = in;
            a.res = res;
            a.pro_ab = reinterpret_cast<const float2*>(ab);
            a.wpk = w;
            a.bias = bias;
            a.bn_ab = reinterpret_cast<const float2*>(ab);
            a.out = out;
            // transposed convs feed a CIN: their statistics go to fixed-point accumulators as in the frame
            // (LITE_PART=1: the per-tile partials of the training path instead)
            cin_word* acc = nullptr;
            CK(hipMalloc(&acc, (size_t)32 * B * 2 * CIN_LIMBS * s.cout * sizeof(cin_word)));
            CK(hipMemset(acc, 0, (size_t)32 * B * 2 * CIN_LIMBS * s.cout * sizeof(cin_word)));
            const bool use_part = getenv("LITE_PART") != nullptr;
            a.part = s.kind == 1 && use_part ? part : nullptr;
            if (s.kind == 1 && !use_part) {
                a.stat.acc = acc;
                a.stat.nslot = 32;
            }
            a.batch = B;
            a.H = s.H;
            a.W = s.W;
            a.cin = s.cin;
            a.Ho = Ho;
            a.Wo = Wo;
            a.ntot = s.cout;
            a.cout = s.cout;
            a.pad_t = a.pad_l = 0;
            a.tiles_y = tiles_y;
            a.tiles_x = tiles_x;
            a.pro_mode = s.pro;
            // LITE_PROACC=n: the prologue affine formed from n producer accumulator copies (zeroed) as in the frame,
            // instead of the given pro_ab (the output check is then skipped: the affine differs)
            const int proacc = getenv("LITE_PROACC") ? atoi(getenv("LITE_PROACC")) : 0;
            cin_word* pacc = nullptr;
            float* pstyle = nullptr;
            if (proacc > 0 && s.pro != PRO_NONE) {
                CK(hipMalloc(&pacc, (size_t)proacc * B * 2 * CIN_LIMBS * s.cin * sizeof(cin_word)));
                CK(hipMemset(pacc, 0, (size_t)proacc * B * 2 * CIN_LIMBS * s.cin * sizeof(cin_word)));
                pstyle = dev_rand((size_t)B * 2 * s.cin, 0.5f, 1.f, 6);
                a.pro_stat.acc = pacc;
                a.pro_stat.nslot = proacc;
                a.pro_stat.C = s.cin;
                a.pro_stat.batch = B;
                a.pro_stat.n = (double)s.H * s.W;
                a.pro_stat.style = pstyle;
                a.pro_stat.style_stride = 2 * s.cin;
                a.pro_stat.eps = 1e-5f;
            }
            for (int i = 0; i < 5; ++i) CK(conv_lite_launch(t, a, st));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; ++i) CK(conv_lite_launch(t, a, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            if (pacc == nullptr) {   // sampled CPU check of the output (f64 sums): max |err| / (sum of |terms| + |bias|) over 4096 points
                std::vector<float> hin(nin), hres(nin), hb(s.cout), hab(nab), hout(nout);
                CK(hipMemcpy(hin.data(), in, nin * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hres.data(), res, nin * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hb.data(), bias, s.cout * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hab.data(), ab, hab.size() * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hout.data(), out, nout * 4, hipMemcpyDeviceToHost));
                const int OH = s.kind == 0 ? Ho : 2 * Ho, OW = s.kind == 0 ? Wo : 2 * Wo;
                double worst = 0;
                srand(7);
                for (int i = 0; i < 4096; ++i) {
                    const int b = rand() % B, oy = rand() % OH, ox = rand() % OW, n = rand() % s.cout;
                    double acc = 0, mag = 0;
                    for (int ky = 0; ky < 3; ++ky)
                        for (int kx = 0; kx < 3; ++kx) {
                            int iy, ix;
                            if (s.kind == 0) { iy = 2 * oy + ky; ix = 2 * ox + kx; }
                            else {   // out(2p + py) takes in(p - 1 + ty) through ky = py + 2 (1 - ty)
                                const int py = oy & 1, px = ox & 1;
                                if ((ky - py) & 1 || (kx - px) & 1) continue;
                                iy = (oy >> 1) - 1 + (1 - (ky - py) / 2);
                                ix = (ox >> 1) - 1 + (1 - (kx - px) / 2);
                            }
                            if (iy < 0 || iy >= s.H || ix < 0 || ix >= s.W) continue;
                            for (int ci = 0; ci < s.cin; ++ci) {
                                const size_t gi = (((size_t)b * s.H + iy) * s.W + ix) * s.cin + ci;
                                double x = hin[gi];
                                if (s.pro == PRO_AFF_RES) x = (double)fmaf(hab[2 * (b * s.cin + ci)], hin[gi], hab[2 * (b * s.cin + ci) + 1]) + hres[gi];
                                if (s.pro == PRO_AFF_RELU) x = fmaxf(fmaf(hab[2 * (b * s.cin + ci)], hin[gi], hab[2 * (b * s.cin + ci) + 1]), 0.f);
                                const double wv = s.kind == 0 ? hk[((size_t)(ky * 3 + kx) * s.cin + ci) * s.cout + n]
                                                              : hk[((size_t)(ky * 3 + kx) * s.cout + n) * s.cin + ci];
                                acc += x * wv;
                                mag += fabs(x * wv);
                            }
                        }
                    double ref = acc + hb[n];
                    if (s.kind == 0) { ref = fmax(ref, 0.0); ref = fmax(hab[2 * n] * ref + hab[2 * n + 1], 0.0); }
                    const double got = hout[(((size_t)b * OH + oy) * OW + ox) * s.cout + n];
                    worst = fmax(worst, fabs(got - ref) / (mag + fabs(hb[n]) + 1e-30));
                }
                printf("B=%d %-11s check: max |err| / sum|terms| = %.2e%s\n", B, s.name, worst, worst > 2e-6 ? "   <-- MISMATCH" : "");
            }
            const double flops = 2.0 * B * (s.kind == 0 ? (double)Ho * Wo : (double)s.H * s.W) * 9 * s.cin * s.cout;
            const double bytes = 4.0 * (nin * (s.pro == PRO_AFF_RES ? 2 : 1) + nout);
#ifdef LITE_PROF
            lite_timeline_print(16);
#endif
            printf("B=%d %-11s %8.2f us   %6.1f TFLOP/s (%.2f of f32 MFMA)   %7.1f GB/s (%.2f of HBM)   grid %d\n", B,
                   s.name, us, flops / us * 1e-6, flops / us * 1e-6 / 157.3, bytes / us * 1e-3,
                   bytes / us * 1e-3 / 8000.0, B * tiles_y * tiles_x);
            CK(hipFree(in)); CK(hipFree(res)); CK(hipFree(w)); CK(hipFree(bias)); CK(hipFree(ab));
            CK(hipFree(out)); CK(hipFree(part)); CK(hipFree(acc));
            if (pacc) { CK(hipFree(pacc)); CK(hipFree(pstyle)); }
        }
    return 0;
}
