// fin_probe.hip — where does a CIN finalize launch's time go? Times, with HIP events over 2000
// back-to-back launches on one stream (and as one captured hipGraph): an empty kernel, the
// finalize shapes of the headline frame (residual: C=128 x 225 partials; expand_0: C=32 x 4 phases x 900;
// expand_1: C=16 x 4 x 3600; expand_last: C=3 x 450), and each finalize preceded by a 15 MB "producer" write so the
// partials are freshly written by another kernel as in the frame.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I realtime_style_transfer_amd/csrc tools/fin_probe.hip -o tools/fin_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "../realtime_style_transfer_amd/csrc/norm.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void empty_kernel() {}
// expand_1-shaped read of the partials without the statistics arithmetic: DIV = 1 keeps the
// (image, phase, tile) index decode with integer divisions, DIV = 0 walks a flat range
template <int DIV>
__global__ __launch_bounds__(256) void read_only_kernel(const float4* __restrict__ part, float* out, int C, int phases,
                                                        int n_part, int nsplit) {
    const int c = blockIdx.x, total = phases * n_part, chunk = (total + nsplit - 1) / nsplit;
    const int lo = blockIdx.z * chunk, hi = min(total, lo + chunk);
    float acc = 0.f;
    for (int base = lo + threadIdx.x; base < hi; base += 4 * 256) {
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = min(base + k * 256, hi - 1);
            if (DIV) {
                const int ph = i / n_part, t = i - ph * n_part;
                v[k] = part[(size_t)(ph * C + c) * n_part + t];
            } else {
                v[k] = part[(size_t)c * total + i];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + k * 256 < hi) acc += v[k].x + v[k].y;
    }
    if (acc == 12345.f) out[c] = acc;
}
__global__ void producer_kernel(float4* p, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) p[i] = make_float4(1.f, 0.5f, 128.f, 0.f);
}

int main() {
    using namespace rst;
    const int REPS = 2000;
    float4* part;
    const long NP = 16L * 4 * 3600 + 4096;
    CK(hipMalloc(&part, 16 * NP));
    float4* big;
    const long NBIG = 15L * 1024 * 1024 / 16;
    CK(hipMalloc(&big, 16 * NBIG));
    float2* ab;
    CK(hipMalloc(&ab, 8 * 4096));

    std::vector<float4> h(NP, make_float4(1.f, 0.5f, 128.f, 0.f));
    CK(hipMemcpy(part, h.data(), 16 * NP, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    struct Case { const char* name; int C, phases, n_part; };
    const Case cases[] = {{"residual C=128 x 225", 128, 1, 225}, {"expand_0 C=32 x 4 x 900", 32, 4, 900},
                          {"expand_1 C=16 x 4 x 3600", 16, 4, 3600}, {"expand_last C=3 x 450", 3, 1, 450}};
    auto time_it = [&](const char* name, auto&& body) -> int {
        for (int i = 0; i < 50; ++i) body();
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < REPS; ++i) body();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // graph of 20 launches, replayed REPS/20 times
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 20; ++i) body();
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < REPS / 20; ++i) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float gms;
        CK(hipEventElapsedTime(&gms, e0, e1));
        printf("%-44s stream %7.2f us/iter   graph %7.2f us/iter\n", name, 1e3f * ms / REPS, 1e3f * gms / REPS);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return 0;
    };
    if (time_it("empty kernel", [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st); })) return 1;
    if (time_it("producer 15 MB write", [&] { hipLaunchKernelGGL(producer_kernel, dim3(1024), dim3(256), 0, st, big, NBIG); })) return 1;
    {
        float* o;
        CK(hipMalloc(&o, 4096));
        if (time_it("read-only expand_1 shape, div, 15 splits", [&] {
                hipLaunchKernelGGL(read_only_kernel<1>, dim3(16, 1, 15), dim3(256), 0, st, part, o, 16, 4, 3600, 15); }))
            return 1;
        if (time_it("read-only expand_1 shape, flat, 15 splits", [&] {
                hipLaunchKernelGGL(read_only_kernel<0>, dim3(16, 1, 15), dim3(256), 0, st, part, o, 16, 4, 3600, 15); }))
            return 1;
        if (time_it("read-only expand_1 shape, flat, 1 split", [&] {
                hipLaunchKernelGGL(read_only_kernel<0>, dim3(16, 1, 1), dim3(256), 0, st, part, o, 16, 4, 3600, 1); }))
            return 1;
    }
    for (const Case& c : cases) {
        FinalizeArgs f{};
        f.part = part;
        f.ab = ab;
        f.batch = 1;
        f.C = c.C;
        f.ntot = c.C * c.phases;
        f.n_part = c.n_part;
        f.phases = c.phases;
        f.eps = 1e-5f;
        char nm[96];
        snprintf(nm, sizeof nm, "finalize %s", c.name);
        if (time_it(nm, [&] { (void)finalize_launch(f, st); })) return 1;

        snprintf(nm, sizeof nm, "producer + finalize %s", c.name);
        if (time_it(nm, [&] {
                hipLaunchKernelGGL(producer_kernel, dim3(1024), dim3(256), 0, st, big, NBIG);
                (void)finalize_launch(f, st);
            }))
            return 1;
    }
    CK(hipStreamSynchronize(st));
    printf("done\n");
    return 0;
}
