// affine_probe.hip — cost of forming the CIN prologue affine from the fixed-point accumulators (kernels.h
// cin_affine_table), as every residual conv's workgroups do at their start: 225 workgroups x 512 threads, C = 128,
// nslot = 8 (the residual convs' geometry at B = 1). Modes: 0 the whole table; 1 the accumulator loads and the
// limb merge only (no f64 math); 2 the f64 math only (limbs from registers); 3 nothing (launch + LDS write floor).
// Build: hipcc -O3 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc tools/affine_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels.h"
using namespace rst;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int MODE>
__global__ __launch_bounds__(512) void probe(CinSrc s, float2* sink) {
    __shared__ float2 tab[256];
    if constexpr (MODE == 0) {
        cin_affine_table<512>(s, 0, 1, tab, nullptr, nullptr, nullptr);
    } else if constexpr (MODE == 1) {
        const int c = threadIdx.x & 127, k0 = threadIdx.x >> 7;   // 4 lanes per channel, 2 copies each
        cin_word w[6] = {};
        for (int r = 0; r < 2; ++r) {
            const cin_word* p = s.acc + ((size_t)(k0 + 4 * r) * 2 * CIN_LIMBS) * s.C + c;
#pragma unroll
            for (int q = 0; q < 6; ++q) w[q] += p[q * s.C];
        }
        if (threadIdx.x < 128) tab[c] = make_float2((float)(w[0] + w[3]), (float)(w[1] + w[4] + w[2] + w[5]));
    } else if constexpr (MODE == 2) {
        if (threadIdx.x < 128) {
            const cin_word base = (cin_word)blockIdx.x * 977 + threadIdx.x;
            const double S = cin_fixed_value(base, base * 3, 7), Q = cin_fixed_value(base * 5, base, 11);
            const double N = s.n, mean = S / N, var = fmax(Q - S * mean, 0.0) / N;
            const float rstd = (float)(1.0 / sqrt(var + (double)s.eps));
            tab[threadIdx.x] = make_float2(rstd, (float)mean);
        }
    } else {
        if (threadIdx.x < 128) tab[threadIdx.x] = make_float2(1.f, 0.f);
    }
    __syncthreads();
    if (threadIdx.x == 0 && tab[blockIdx.x & 127].x == 12345.f) sink[blockIdx.x] = tab[0];
}

int main() {
    const int C = 128, nslot = 8, nwg = 225;
    std::vector<cin_word> h((size_t)nslot * 2 * CIN_LIMBS * C);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (cin_word)((i * 2654435761u) % 100000);
    cin_word* acc; float* sty; float2* sink;
    CK(hipMalloc(&acc, h.size() * 8)); CK(hipMemcpy(acc, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<float> hs(2 * C, 0.7f);
    CK(hipMalloc(&sty, 2 * C * 4)); CK(hipMemcpy(sty, hs.data(), 2 * C * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&sink, nwg * 8));
    // a buffer the size of the L2s to evict the accumulators between launches (as in the frame, where they were
    // written by another kernel's atomics)
    const size_t nev = (size_t)64 << 20;
    float* ev; CK(hipMalloc(&ev, nev * 4));
    CinSrc s{};
    s.acc = acc; s.nslot = nslot; s.C = C; s.batch = 1; s.n = 28800.0; s.style = sty; s.style_stride = 2 * C;
    s.style_offset = 0; s.style1_offset = -1; s.eps = 1e-5f;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const char* names[4] = {"whole table", "loads + merge", "f64 math", "floor"};
    for (int cold = 0; cold < 2; ++cold)
        for (int m = 0; m < 4; ++m) {
            float tot = 0.f;
            const int it = 50;
            for (int i = 0; i < it + 5; ++i) {
                if (cold) CK(hipMemsetAsync(ev, i & 0xFF, nev * 4, 0));
                CK(hipEventRecord(e0, 0));
                switch (m) {
                    case 0: hipLaunchKernelGGL(probe<0>, dim3(nwg), dim3(512), 0, 0, s, sink); break;
                    case 1: hipLaunchKernelGGL(probe<1>, dim3(nwg), dim3(512), 0, 0, s, sink); break;
                    case 2: hipLaunchKernelGGL(probe<2>, dim3(nwg), dim3(512), 0, 0, s, sink); break;
                    default: hipLaunchKernelGGL(probe<3>, dim3(nwg), dim3(512), 0, 0, s, sink); break;
                }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                if (i >= 5) tot += ms;
            }
            printf("%s %-14s %7.2f us per launch\n", cold ? "cold" : "warm", names[m], tot * 1e3f / it);
        }
    return 0;
}
