// Round-6 probes (one tool, three questions; tools/build_probe_r06.sh, run under rocprofv3 for the cross-checks):
//   graphev  Can a hipGraph replay report per-kernel durations live? Compares, for ten back-to-back 512-thread x 256-WG
//            kernels: eager hipExtLaunchKernel start/stop events (kernel-execution timestamps), the same launches captured
//            into a graph (do the ext events survive capture?), event-record nodes around each captured launch, and the
//            plain graph's replay time per kernel. rocprofv3 --kernel-trace of the same run is the reference.
//   fetch    FETCH_SIZE / WRITE_SIZE calibration on known byte counts (MI355X_MICROARCH.md §HBM: "other access widths are
//            uncalibrated"): coalesced reads with 4-, 8- and 16-byte lanes, the one-dword-per-128-B-line L2 touch the conv
//            kernels use for next-layer prefetch, and 4- / 16-byte stores. One launch each, 512 MiB per pattern (twice the
//            Infinity Cache), every pattern on its own buffer.
//   barrier  What a grid-wide seam costs inside one launch against a kernel boundary, in the residual stack's geometry
//            (225 workgroups of 512 threads, one per CU): ten "layers" of fixed MFMA work + a 64 KB write-through output per
//            workgroup + a read of the neighbour workgroup's previous output, as ten graph-captured launches vs one
//            persistent launch with an XCD-hierarchical barrier (per-XCD arrival counter -> top counter, agent-scope
//            release before arrive and acquire after, bounded spin with a give-up flag).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ graphev ------------------------------------------
__global__ __launch_bounds__(512) void spin_kernel(float* out, int iters) {
    floatx16 acc = {};
    short8 a = {1, 2, 3, 4, 5, 6, 7, 8};
    for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
    if (acc[0] == 1.2345f) out[blockIdx.x * 512 + threadIdx.x] = acc[1];
}

static void graphev(int iters) {
    const int G = 256, N = 10, R = 50;
    float* out;
    CK(hipMalloc(&out, G * 512 * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * N);
    for (auto& e : ev) CK(hipEventCreate(&e));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(spin_kernel, dim3(G), dim3(512), 0, st, out, iters);
    CK(hipStreamSynchronize(st));
    float ms;
    // A: eager, plain launches, total / N
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(spin_kernel, dim3(G), dim3(512), 0, st, out, iters);
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("graphev A eager plain: %.2f us per kernel (total / %d)\n", ms * 1e3 / N, N);
    // B: eager hipExtLaunchKernel with start/stop events
    for (int i = 0; i < N; ++i)
        hipExtLaunchKernelGGL(spin_kernel, dim3(G), dim3(512), 0, st, ev[2 * i], ev[2 * i + 1], 0, out, iters);
    CK(hipStreamSynchronize(st));
    double s = 0;
    for (int i = 0; i < N; ++i) {
        CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
        s += ms;
    }
    printf("graphev B eager ext events: %.2f us per kernel\n", s * 1e3 / N);
    // C: graph of N plain launches, R replays
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(spin_kernel, dim3(G), dim3(512), 0, st, out, iters);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("graphev C graph plain: %.2f us per kernel (replay total / %d)\n", ms * 1e3 / (N * R), N * R);
    // D: graph of N hipExtLaunchKernel launches with per-launch events
    hipGraph_t gd;
    hipGraphExec_t ged;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) {
        hipError_t e = hipExtLaunchKernel(reinterpret_cast<const void*>(spin_kernel), dim3(G), dim3(512),
                                          (void*[]){&out, &iters}, 0, st, ev[2 * i], ev[2 * i + 1], 0);
        if (e != hipSuccess) printf("graphev D capture ext launch %d: %s\n", i, hipGetErrorString(e));
    }
    CK(hipStreamEndCapture(st, &gd));
    size_t nn = 0;
    CK(hipGraphGetNodes(gd, nullptr, &nn));
    printf("graphev D captured nodes: %zu (for %d launches)\n", nn, N);
    CK(hipGraphInstantiate(&ged, gd, nullptr, nullptr, 0));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ged, st));
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ged, st));
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("graphev D graph ext: %.2f us per kernel (replay total)\n", ms * 1e3 / (N * R));
    s = 0;
    int ok = 0;
    for (int i = 0; i < N; ++i) {
        hipError_t e = hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
        if (e == hipSuccess) { s += ms; ++ok; printf("  D event pair %d: %.2f us\n", i, ms * 1e3); }
        else printf("  D event pair %d: %s\n", i, hipGetErrorString(e));
    }
    if (ok) printf("graphev D graph ext events: %.2f us per kernel (%d pairs)\n", s * 1e3 / ok, ok);
    // E: graph with event-record nodes around each plain launch
    hipGraph_t gE;
    hipGraphExec_t geE;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) {
        CK(hipEventRecord(ev[2 * i], st));
        hipLaunchKernelGGL(spin_kernel, dim3(G), dim3(512), 0, st, out, iters);
        CK(hipEventRecord(ev[2 * i + 1], st));
    }
    CK(hipStreamEndCapture(st, &gE));
    CK(hipGraphGetNodes(gE, nullptr, &nn));
    printf("graphev E captured nodes: %zu\n", nn);
    CK(hipGraphInstantiate(&geE, gE, nullptr, nullptr, 0));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(geE, st));
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < R; ++i) CK(hipGraphLaunch(geE, st));
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("graphev E graph with record nodes: %.2f us per kernel (replay total)\n", ms * 1e3 / (N * R));
    s = 0;
    ok = 0;
    for (int i = 0; i < N; ++i) {
        hipError_t e = hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
        if (e == hipSuccess) { s += ms; ++ok; }
        else printf("  E event pair %d: %s\n", i, hipGetErrorString(e));
    }
    if (ok) printf("graphev E record-node pairs: %.2f us per kernel (%d pairs)\n", s * 1e3 / ok, ok);
    CK(hipStreamSynchronize(st));
    CK(hipFree(out));
}

// ------------------------------------------------------------------ fetch --------------------------------------------
template <int W>   // coalesced read, W bytes per lane
__global__ __launch_bounds__(256) void rd_kernel(const unsigned char* p, size_t bytes, unsigned* sink) {
    unsigned f = 0;
    const size_t n = bytes / W, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if constexpr (W == 16) { const uint4 v = reinterpret_cast<const uint4*>(p)[i]; f ^= v.x ^ v.y ^ v.z ^ v.w; }
        if constexpr (W == 8) { const uint2 v = reinterpret_cast<const uint2*>(p)[i]; f ^= v.x ^ v.y; }
        if constexpr (W == 4) f ^= reinterpret_cast<const unsigned*>(p)[i];
    }
    if (f == 0x9E3779B9u) sink[threadIdx.x] = f;
}
template <int LINE>   // one dword per LINE bytes (the L2 touch)
__global__ __launch_bounds__(256) void touch_kernel(const unsigned char* p, size_t bytes, unsigned* sink) {
    unsigned f = 0;
    const size_t n = bytes / LINE, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        f ^= *reinterpret_cast<const unsigned*>(p + i * LINE);
    if (f == 0x9E3779B9u) sink[threadIdx.x] = f;
}
template <int W>
__global__ __launch_bounds__(256) void wr_kernel(unsigned char* p, size_t bytes) {
    const size_t n = bytes / W, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if constexpr (W == 16) reinterpret_cast<uint4*>(p)[i] = make_uint4(i, i, i, i);
        if constexpr (W == 4) reinterpret_cast<unsigned*>(p)[i] = (unsigned)i;
    }
}

static void fetch() {
    const size_t B = (size_t)512 << 20;
    const int npat = 7;
    unsigned char* buf[npat];
    for (auto& b : buf) {
        CK(hipMalloc(&b, B));
        CK(hipMemset(b, 1, B));
    }
    unsigned* sink;
    CK(hipMalloc(&sink, 4096));
    CK(hipDeviceSynchronize());
    const int G = 2048;
    hipLaunchKernelGGL(rd_kernel<16>, dim3(G), dim3(256), 0, 0, buf[0], B, sink);
    hipLaunchKernelGGL(rd_kernel<8>, dim3(G), dim3(256), 0, 0, buf[1], B, sink);
    hipLaunchKernelGGL(rd_kernel<4>, dim3(G), dim3(256), 0, 0, buf[2], B, sink);
    hipLaunchKernelGGL(touch_kernel<128>, dim3(G), dim3(256), 0, 0, buf[3], B, sink);
    hipLaunchKernelGGL(touch_kernel<64>, dim3(G), dim3(256), 0, 0, buf[4], B, sink);
    hipLaunchKernelGGL(wr_kernel<16>, dim3(G), dim3(256), 0, 0, buf[5], B);
    hipLaunchKernelGGL(wr_kernel<4>, dim3(G), dim3(256), 0, 0, buf[6], B);
    CK(hipDeviceSynchronize());
    printf("fetch: 7 patterns over %zu bytes each (rd16 rd8 rd4 touch128 touch64 wr16 wr4); read the counters per kernel\n", B);
    for (auto& b : buf) CK(hipFree(b));
}

// ------------------------------------------------------------------ barrier ------------------------------------------
constexpr int BT = 512;
constexpr int SLAB = 64 * 1024 / 16;   // uint4 per workgroup output (64 KB)

struct BarrierState {
    unsigned xcnt[8 * 32];   // per-XCD arrival counters, 128 B apart
    unsigned top[32];
    unsigned fail[32];
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one "layer": fixed MFMA work, then read the previous layer's output of workgroup (wg + 1) % G and write this layer's
// 64 KB (write-through) = f(layer, wg, neighbour value); returns the number of wrong neighbour values seen
__device__ __forceinline__ unsigned layer_body(int layer, int wg, int G, int iters, uint4* slabs_prev, uint4* slabs_cur) {
    floatx16 acc = {};
    short8 a = {1, 2, 3, 4, 5, 6, 7, 8};
    for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
    unsigned bad = 0;
    const int nb = (wg + 1) % G;
    for (int i = threadIdx.x; i < SLAB; i += BT) {
        unsigned v = 0;
        if (layer > 0) {
            const uint4 q = slabs_prev[(size_t)nb * SLAB + i];
            const unsigned want = (unsigned)((layer - 1) * 1000003u + nb * 7919u + i);
            bad += q.x != want;
            v = q.x;
        }
        (void)v;
        const unsigned w = (unsigned)(layer * 1000003u + wg * 7919u + i);
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){w, w, w, acc[0] == 1.5f ? 1u : 0u},
                                               __builtin_amdgcn_make_buffer_rsrc(slabs_cur + (size_t)wg * SLAB, 0, SLAB * 16, 0x00020000),
                                               i * 16, 0, 16);
    }
    return bad;
}

__global__ __launch_bounds__(BT) void layer_kernel(int layer, int iters, uint4* s0, uint4* s1, unsigned* bad) {
    uint4* prev = (layer & 1) ? s0 : s1;
    uint4* cur = (layer & 1) ? s1 : s0;
    const unsigned b = layer_body(layer, blockIdx.x, gridDim.x, iters, prev, cur);
    if (b) atomicAdd(bad, b);
}

__global__ __launch_bounds__(BT) void persistent_kernel(int layers, int iters, uint4* s0, uint4* s1, unsigned* bad,
                                                        BarrierState* bs, unsigned gen0) {
    const int G = gridDim.x, wg = blockIdx.x, r = wg & 7;
    const unsigned nr = (unsigned)((G - r + 7) >> 3);   // workgroups of residue r
    unsigned tb = 0;
    for (int l = 0; l < layers; ++l) {
        uint4* prev = (l & 1) ? s0 : s1;
        uint4* cur = (l & 1) ? s1 : s0;
        tb += layer_body(l, wg, G, iters, prev, cur);
        if (l + 1 == layers) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are done
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned gen = gen0 + (unsigned)l + 1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const unsigned old = __hip_atomic_fetch_add(&bs->xcnt[r * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == nr * gen) __hip_atomic_fetch_add(&bs->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (ld_sc1(&bs->top[0]) < 8u * gen) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {   // 20 ms: give up, flag it
                    __hip_atomic_fetch_add(&bs->fail[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    if (tb) atomicAdd(bad, tb);
}

static void barrier(int iters, int G) {
    const int L = 10, R = 30;
    uint4 *s0, *s1;
    unsigned* bad;
    BarrierState* bs;
    CK(hipMalloc(&s0, (size_t)G * SLAB * 16));
    CK(hipMalloc(&s1, (size_t)G * SLAB * 16));
    CK(hipMalloc(&bad, 4));
    CK(hipMalloc(&bs, sizeof(BarrierState)));
    CK(hipMemset(bad, 0, 4));
    CK(hipMemset(bs, 0, sizeof(BarrierState)));
    int dev, ncu, occ;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent_kernel, BT, 0));
    printf("barrier: G=%d, CUs %d, occupancy %d per CU, iters %d\n", G, ncu, occ, iters);
    if (occ * ncu < G) { printf("barrier: grid not co-resident, skipped\n"); return; }
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    float ms;
    // launches: L layer kernels in one graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < L; ++l) hipLaunchKernelGGL(layer_kernel, dim3(G), dim3(BT), 0, st, l, iters, s0, s1, bad);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    unsigned hb = 0;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("barrier launches: %.2f us per layer (%d layers x %d replays), wrong neighbour values %u\n",
           ms * 1e3 / (L * R), L, R, hb);
    // one layer alone (the body's own span, for reference)
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(layer_kernel, dim3(G), dim3(BT), 0, st, 1, iters, s0, s1, bad);
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("barrier single layer eager: %.2f us\n", ms * 1e3 / R);
    // persistent: one launch per replay; the generation base advances by L - 1 per launch (counters monotonic)
    CK(hipMemset(bad, 0, 4));
    unsigned gen0 = 0;
    for (int i = 0; i < 3; ++i) {
        hipLaunchKernelGGL(persistent_kernel, dim3(G), dim3(BT), 0, st, L, iters, s0, s1, bad, bs, gen0);
        gen0 += L - 1;
    }
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(t0, st));
    for (int i = 0; i < R; ++i) {
        hipLaunchKernelGGL(persistent_kernel, dim3(G), dim3(BT), 0, st, L, iters, s0, s1, bad, bs, gen0);
        gen0 += L - 1;
    }
    CK(hipEventRecord(t1, st));
    CK(hipEventSynchronize(t1));
    CK(hipEventElapsedTime(&ms, t0, t1));
    BarrierState h;
    CK(hipMemcpy(&h, bs, sizeof(h), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("barrier persistent: %.2f us per layer, wrong neighbour values %u, give-ups %u\n", ms * 1e3 / (L * R), hb, h.fail[0]);
    CK(hipStreamSynchronize(st));
}

int main(int argc, char** argv) {
    const char* what = argc > 1 ? argv[1] : "all";
    const int iters = argc > 2 ? atoi(argv[2]) : 1000;
    if (!strcmp(what, "graphev") || !strcmp(what, "all")) graphev(iters);
    if (!strcmp(what, "fetch") || !strcmp(what, "all")) fetch();
    if (!strcmp(what, "barrier") || !strcmp(what, "all")) {
        barrier(iters, 225);
        barrier(iters / 4, 225);
    }
    return 0;
}
