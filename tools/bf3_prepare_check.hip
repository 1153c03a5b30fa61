// Diagnostic: hipFuncSetAttribute on the split-bf16 conv configurations vs the f32 conv kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../realtime_style_transfer_amd/csrc/conv_mfma.hip"
#include "../realtime_style_transfer_amd/csrc/conv_bf3.hip"
using namespace rst;
int main() {
    auto kb = conv_bf3_kernel<3, 3, 1, 32, 128, 4, 16, 2, 2, 1>;
    auto kf = conv_mfma_kernel<3, 3, 1, 32, 128, 4, 16, 2, 2, 1, 1>;
    for (int v : {1024, 54144, 65536, 100000, 163840}) {
        hipError_t e1 = hipFuncSetAttribute((const void*)kb, hipFuncAttributeMaxDynamicSharedMemorySize, v);
        (void)hipGetLastError();
        hipError_t e2 = hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, v);
        (void)hipGetLastError();
        printf("value %6d: bf3 %d (%s)  f32 %d (%s)\n", v, (int)e1, hipGetErrorString(e1), (int)e2, hipGetErrorString(e2));
    }
    return 0;
}
