// Check (GPU): the three-piece bf16 split of an f32 pair formed with v_dot2c_f32_bf16 (x - piece as
// dot2(piece, (-1, 0)) + x) is bitwise the split formed with shifts and subtractions (wino_x6.hip, wino9_x6.hip),
// over random pairs of many magnitudes and signs, zeros and values near bf16 rounding ties.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <random>
#include <cstring>
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void split_ref(const float2* in, uint4* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[i].x, y = in[i].y;
    unsigned p[3];
    for (int k = 0; k < 2; ++k) {
        p[k] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
        x = x - __uint_as_float(p[k] << 16);
        y = y - __uint_as_float(p[k] & 0xFFFF0000u);
    }
    p[2] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
    out[i] = make_uint4(p[0], p[1], p[2], __float_as_uint(x) ^ __float_as_uint(y));
}
__global__ void split_dot2(const float2* in, uint4* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[i].x, y = in[i].y;
    const bf16x2 mlo = {(__bf16)-1.0f, (__bf16)0.0f}, mhi = {(__bf16)0.0f, (__bf16)-1.0f};
    unsigned p[3];
    for (int k = 0; k < 2; ++k) {
        const bf16x2 pb = __builtin_convertvector((f32x2){x, y}, bf16x2);
        p[k] = __builtin_bit_cast(unsigned, pb);
        x = __builtin_amdgcn_fdot2_f32_bf16(pb, mlo, x, false);
        y = __builtin_amdgcn_fdot2_f32_bf16(pb, mhi, y, false);
    }
    p[2] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x, y}, bf16x2));
    out[i] = make_uint4(p[0], p[1], p[2], __float_as_uint(x) ^ __float_as_uint(y));
}

int main() {
    const int n = 1 << 24;
    std::vector<float2> h(n);
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::uniform_int_distribution<int> ex(-60, 60);
    for (int i = 0; i < n; ++i) {
        float v[2];
        for (int k = 0; k < 2; ++k) {
            const int mode = (int)(rng() % 8);
            if (mode == 0) v[k] = 0.f;
            else if (mode == 1) {   // bf16 tie / near-tie patterns: low 16 bits 0x8000 +- small
                uint32_t b = (uint32_t)rng() & 0xFFFF0000u;
                b = (b & 0x807FFFFFu) | ((uint32_t)(100 + rng() % 56) << 23);
                b |= 0x8000u + (uint32_t)((int)(rng() % 5) - 2);
                std::memcpy(&v[k], &b, 4);
            } else v[k] = (float)std::ldexp(u(rng), ex(rng));
        }
        h[i] = make_float2(v[0], v[1]);
    }
    float2* d; uint4 *o1, *o2;
    CK(hipMalloc(&d, n * sizeof(float2))); CK(hipMalloc(&o1, n * 16)); CK(hipMalloc(&o2, n * 16));
    CK(hipMemcpy(d, h.data(), n * sizeof(float2), hipMemcpyHostToDevice));
    split_ref<<<n / 256, 256>>>(d, o1, n);
    split_dot2<<<n / 256, 256>>>(d, o2, n);
    CK(hipDeviceSynchronize());
    std::vector<uint4> a(n), b(n);
    CK(hipMemcpy(a.data(), o1, n * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o2, n * 16, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int i = 0; i < n; ++i)
        if (a[i].x != b[i].x || a[i].y != b[i].y || a[i].z != b[i].z || a[i].w != b[i].w) {
            if (bad < 5) printf("diff at %d: (%a, %a)\n", i, h[i].x, h[i].y);
            ++bad;
        }
    printf("dot2 split vs sub split: %zu of %d pairs differ\n", bad, n);
    return bad ? 2 : 0;
}
