// common.h — host helpers shared by the C-ABI translation units of librst.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "kernels.h"

namespace rst {

// bf16 planes of a split-bf16 precision mode (include/rst.h RST_PRECISION_*), 0 for the f32 modes
inline int bf16_planes(int precision) {
    return precision == 1 ? 2 : (precision == 2 ? 3 : (precision == 4 ? 1 : 0));   // BF16X3, BF16X6, BF16
}

// Record the thread-local error message returned by rst_last_error(); returns code.
int set_error(int code, const std::string& msg);

// Pack a GEMM-form conv kernel Wg[tap][ci][n] (taps = kh*kw, row-major) into the LDS stage image
// [n_block][cin_chunk][tap_group][tap][kgroup][lane_half][n][VEC] that conv_mfma_kernel stages.
std::vector<float> pack_conv_tiles(const std::vector<float>& Wg, int taps, int cin, int ntot, const ConvTile& t);
// Same for the split-bf16 kernel: [n_block][cin_chunk][tap_group][tap][kstep][hi/lo][lane_half][n][8]
// bf16, returned as the float-sized buffer that holds those bits (2 bf16 per float).
std::vector<float> pack_conv_tiles_bf3(const std::vector<float>& Wg, int taps, int cin, int ntot, const ConvTile& t);
// source index in Wg of every bf16 element of the one-plane pack_conv_tiles_bf3 image (-1: padding)
std::vector<int> pack_conv_tiles_bf3_index(int taps, int cin, int ntot, const ConvTile& t);

// Diagnostic guard bands (RST_ALLOC_PAD=<bytes>, default 0 = plain hipMalloc): the trainer's and the loss network's
// buffers get a canary-filled band of that many bytes on both sides; guard_check reports every band a kernel wrote
// (an out-of-bounds store) to stderr and returns their count. guard_free takes the pointer guard_malloc returned.
size_t guard_pad();
hipError_t guard_malloc(void** p, size_t bytes);
void guard_free(void* p);
int guard_check(const char* when);

}  // namespace rst

#define RST_HIP_TRY(expr)                                                                         \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) return rst::set_error(3, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)
