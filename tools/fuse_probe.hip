// fuse_probe.hip — what does folding the CIN finalize into the producing conv cost?
// A "producer" shaped like the residual conv (225 workgroups x 256 threads, each writing a 64 KB output
// tile and 128 per-tile {sum, M2, n} partials) is timed, as one captured hipGraph replayed 2000 times:
//   mode 0: producer only                       (+ the separate finalize launch, as today)
//   mode 1: producer + last-arriver merge       (agent-scope acq_rel counter; the last workgroup of the
//                                                image merges all 225 x 128 partials)
//   mode 2: producer + two-level merge          (groups of 15 workgroups; the last of each group merges
//                                                its 15 partials and publishes a group partial; the last
//                                                group merges the 15 group partials)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I realtime_style_transfer_amd/csrc tools/fuse_probe.hip -o tools/fuse_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "../realtime_style_transfer_amd/csrc/norm.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int NWG = 225, C = 128, GRP = 15;

__device__ __forceinline__ void merge_add(double& S, double& Q, float& N, float4 v) {
    if (v.z > 0.f) {
        const double sv = v.x, nv = v.z;
        double r = __builtin_amdgcn_rcp(nv);
        r = fma(fma(-nv, r, 1.0), r, r);
        S += sv;
        N += v.z;
        Q += (double)v.y + sv * sv * r;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void producer(float4* out, float4* part, double4* gpart, unsigned* cnt, float2* ab) {
    const int tid = threadIdx.x, wg = blockIdx.x;
    float4* o = out + (size_t)wg * 4096;
#pragma unroll
    for (int k = 0; k < 16; ++k) o[tid + 256 * k] = make_float4(tid, k, wg, 1.f);
    if (tid < C) part[(size_t)tid * NWG + wg] = make_float4(1.f + tid, 0.5f, 128.f, 0.f);
    if constexpr (MODE == 0) return;
    __shared__ unsigned last;
    __shared__ double red[2][C];
    __syncthreads();
    if constexpr (MODE == 1) {
        if (tid == 0) {
            const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last = t == NWG - 1;
        }
        __syncthreads();
        if (!last) return;
        const int c = tid & 127, h = tid >> 7;
        double S = 0, Q = 0;
        float N = 0;
        for (int t = h; t < NWG; t += 2) merge_add(S, Q, N, part[(size_t)c * NWG + t]);
        if (h == 1) { red[0][c] = S; red[1][c] = Q; }
        __syncthreads();
        if (h == 0) {
            S += red[0][c];
            Q += red[1][c];
            const double mean = S / (2 * N), var = (Q - S * mean) / (2 * N);
            ab[c] = make_float2((float)(1.0 / sqrt(var + 1e-5)), (float)mean);
            if (c == 0) cnt[0] = 0;
        }
    } else {
        const int g = wg / GRP;
        if (tid == 0) {
            const unsigned t = __hip_atomic_fetch_add(cnt + 1 + g, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last = t == GRP - 1;
        }
        __syncthreads();
        if (!last) return;
        const int c = tid & 127, h = tid >> 7;
        double S = 0, Q = 0;
        float N = 0;
        for (int t = g * GRP + h; t < (g + 1) * GRP; t += 2) merge_add(S, Q, N, part[(size_t)c * NWG + t]);
        if (h == 1) { red[0][c] = S; red[1][c] = Q; }
        __syncthreads();
        if (h == 0) {
            S += red[0][c];
            Q += red[1][c];
            gpart[(size_t)c * GRP + g] = make_double4(S, Q, 0.0, 0.0);
            if (c == 0) cnt[1 + g] = 0;
        }
        __syncthreads();
        if (tid == 0) {
            const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last = t == NWG / GRP - 1;
        }
        __syncthreads();
        if (!last) return;
        if (tid < C) {
            double S2 = 0, Q2 = 0;
            for (int t = 0; t < NWG / GRP; ++t) {
                const double4 v = gpart[(size_t)tid * GRP + t];
                S2 += v.x;
                Q2 += v.y;
            }
            const double n = 128.0 * NWG, mean = S2 / n, var = (Q2 - S2 * mean) / n;
            ab[tid] = make_float2((float)(1.0 / sqrt(var + 1e-5)), (float)mean);
            if (tid == 0) cnt[0] = 0;
        }
    }
}

int main() {
    float4 *out, *part;
    double4* gpart;
    unsigned* cnt;
    float2 *ab, *ab2;
    CK(hipMalloc(&out, (size_t)NWG * 4096 * 16));
    CK(hipMalloc(&part, (size_t)NWG * C * 16));
    CK(hipMalloc(&gpart, (size_t)GRP * C * 32));
    CK(hipMalloc(&cnt, 64 * 4));
    CK(hipMemset(cnt, 0, 64 * 4));
    CK(hipMalloc(&ab, C * 8));
    CK(hipMalloc(&ab2, C * 8));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    rst::FinalizeArgs f{};
    f.part = part;
    f.ab = ab2;
    f.batch = 1;
    f.C = C;
    f.ntot = C;
    f.n_part = NWG;
    f.phases = 1;
    f.eps = 1e-5f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int R = 2000;
    auto run = [&](const char* name, auto body) -> int {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < 20; ++i) body();
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < R / 20; ++i) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-44s graph %7.2f us/iter\n", name, ms * 1e3 / R);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        return 0;
    };
    if (run("producer only", [&] { producer<0><<<NWG, 256, 0, st>>>(out, part, gpart, cnt, ab); })) return 1;
    if (run("producer + finalize launch", [&] {
            producer<0><<<NWG, 256, 0, st>>>(out, part, gpart, cnt, ab);
            rst::finalize_launch(f, st);
        })) return 1;
    if (run("producer + last-arriver merge", [&] { producer<1><<<NWG, 256, 0, st>>>(out, part, gpart, cnt, ab); })) return 1;
    if (run("producer + two-level merge", [&] { producer<2><<<NWG, 256, 0, st>>>(out, part, gpart, cnt, ab); })) return 1;
    std::vector<float2> h(C);
    CK(hipMemcpy(h.data(), ab, C * 8, hipMemcpyDeviceToHost));
    std::vector<unsigned> hc(64);
    CK(hipMemcpy(hc.data(), cnt, 64 * 4, hipMemcpyDeviceToHost));
    unsigned nz = 0;
    for (unsigned v : hc) nz += v != 0;
    printf("ab[5] = (%g, %g), nonzero counters after the runs: %u\n", h[5].x, h[5].y, nz);
    return 0;
}
