// icache_probe.hip — does a kernel's first pass over straight-line code pay instruction-cache misses? One launch of a
// different kernel, then a kernel of N straight-line VALU instructions (asm .rept) stamped with s_memrealtime before and
// after, against the same N as a 16-iteration loop over N/16 (the loop body is fetched once). 256 workgroups x 512
// threads, as the residual convs. Build: hipcc -O3 --offload-arch=gfx950 tools/icache_probe.hip -o tools/icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void other_kernel(float* p) {
    float v = p[threadIdx.x];
    asm volatile(".rept 64\n v_mul_f32 %0, %0, %0\n .endr" : "+v"(v));
    if (v == 123.f) p[threadIdx.x] = v;
}
template <int MODE>
__global__ __launch_bounds__(512) void probe(float* p, unsigned long long* t) {
    float a = p[threadIdx.x], b = a * 0.5f, c = a * 0.25f, d = a * 2.f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (MODE == 0) {
        asm volatile(".rept 1024\n v_add_f32 %0, %0, %1\n v_add_f32 %2, %2, %3\n .endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else {
        for (int i = 0; i < 16; ++i) {
            asm volatile(".rept 64\n v_add_f32 %0, %0, %1\n v_add_f32 %2, %2, %3\n .endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) t[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
    if (a + b + c + d == 1234.f) p[threadIdx.x] = a;
}
int main() {
    float* p;
    unsigned long long* t;
    CK(hipMalloc(&p, 4096));
    CK(hipMemset(p, 0, 4096));
    CK(hipMalloc(&t, 256 * 8 * 8));
    std::vector<unsigned long long> h(256 * 8);
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 2; ++mode) {
            hipLaunchKernelGGL(other_kernel, dim3(256), dim3(512), 0, 0, p);
            if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(256), dim3(512), 0, 0, p, t);
            else hipLaunchKernelGGL(probe<1>, dim3(256), dim3(512), 0, 0, p, t);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
            double s = 0;
            for (auto v : h) s += (double)v;
            printf("%s: 2048 v_add_f32 per wave, mean %.3f us per wave\n", mode ? "loop 16 x 128 " : "straight line ",
                   s / h.size() * 0.01);
        }
    return 0;
}
