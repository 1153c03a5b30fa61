// ingest.hip — G-buffer ingest on the device: the per-channel EXR planes of an
// Unreal HDR screenshot are assembled into one NHWC content tensor, bilinearly resized and
// center-cropped in ONE pass.
//
// Reference: dataloaders/hdrScreenshots.py:14-30 (stack / expand_dims / concatenate of the channel
// images in `expected_channels` order) followed by dataloaders/common.py:44-57
// (preprocess_numpy_image):
//     new_size = (ceil(W * h/w), W) if h/w > H/W else (H, ceil(H / (h/w)))
//     image = tf.image.resize(image, new_size)                  # bilinear, half-pixel centers, no antialias
//     image = tf.image.resize_with_crop_or_pad(image, H, W)     # crop offset (new - target) // 2
// tf.image.resize (TF 2.9) runs ResizeBilinear(half_pixel_centers=True): per output coordinate
//     in = (float(o) + 0.5f) * (float(in_size) / out_size) - 0.5f,  lo = max(floor(in), 0),
//     hi = min(ceil(in), in_size - 1),  lerp = in - floor(in)
// and blends top = tl + (tr - tl) * xl, bottom = bl + (br - bl) * xl, out = top + (bottom - top) * yl,
// all in f32. The kernel does exactly those f32 operations (FMA contraction off), so it is
// bit-identical to that arithmetic (oracle/ingest_ref.py).
//
// Memory: a workgroup owns 256 consecutive output pixels (a contiguous 256 x C run of the NHWC
// output). Per plane, thread t resamples pixel t (consecutive threads read consecutive source
// columns of one plane: coalesced) into an LDS tile [pixel][C+1]; the tile then leaves as one
// contiguous, fully coalesced store. The tap coordinates and weights are computed once per pixel
// for all planes. HBM-bound: the source is read about once, the output written once.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace rst {

// hipcc contracts a*b+c into an FMA by default (HIP's __fmul_rn / __fadd_rn are plain operators in a
// header, outside any pragma): contraction is off for the expressions of this file, so every
// product and sum below rounds separately, as in TF's kernel
#pragma clang fp contract(off)

__device__ __forceinline__ void tf_half_pixel(int o, float scale, int in_size, int& lo, int& hi, float& lerp) {
    const float in = ((float)o + 0.5f) * scale - 0.5f;
    const float f = floorf(in);
    lo = max((int)f, 0);
    hi = min((int)ceilf(in), in_size - 1);
    lerp = in - f;
}

constexpr int GB_PIX = 256;                            // output pixels per workgroup

__global__ __launch_bounds__(256) void gbuffer_resize_crop_kernel(GbufferArgs a) {
    __shared__ float tile[GB_PIX * (GBUFFER_MAX_PLANES + 1)];
    const int C = a.num_planes, CS = C + 1;            // odd row stride: conflict-free column writes
    const int npix = a.dst_h * a.dst_w;                // 32-bit index math: the host checks npix * C < 2^31
    const int p0 = blockIdx.x * GB_PIX, p = p0 + threadIdx.x;
    const int cnt = min(GB_PIX, npix - p0);
    if (p < npix) {
        const int y = p / a.dst_w, x = p - y * a.dst_w;
        const int ry = y + a.off_y, rx = x + a.off_x;   // coordinates in the resized image
        if (ry < 0 || ry >= a.new_h || rx < 0 || rx >= a.new_w) {   // resize_with_crop_or_pad: zero pad
            for (int c = 0; c < C; ++c) tile[threadIdx.x * CS + c] = 0.f;
        } else {
            int y0, y1, x0, x1;
            float yl, xl;
            tf_half_pixel(ry, a.scale_y, a.src_h, y0, y1, yl);
            tf_half_pixel(rx, a.scale_x, a.src_w, x0, x1, xl);
            const long o00 = y0 * a.row_stride + x0 * a.pixel_stride, o01 = y0 * a.row_stride + x1 * a.pixel_stride;
            const long o10 = y1 * a.row_stride + x0 * a.pixel_stride, o11 = y1 * a.row_stride + x1 * a.pixel_stride;
            for (int c = 0; c < C; ++c) {
                const float* pl = a.planes[c];
                const float tl = pl[o00], tr = pl[o01], bl = pl[o10], br = pl[o11];
                const float top = tl + (tr - tl) * xl;
                const float bottom = bl + (br - bl) * xl;
                tile[threadIdx.x * CS + c] = top + (bottom - top) * yl;
            }
        }
    }
    __syncthreads();
    float* dst = a.dst + (size_t)p0 * C;
    for (int i = threadIdx.x; i < cnt * C; i += GB_PIX) {
        const int q = i / C;
        dst[i] = tile[q * CS + (i - q * C)];
    }
}

hipError_t gbuffer_resize_crop_launch(const GbufferArgs& a, hipStream_t st) {
    const int npix = a.dst_h * a.dst_w;
    const unsigned blocks = (unsigned)((npix + GB_PIX - 1) / GB_PIX);
    hipLaunchKernelGGL(gbuffer_resize_crop_kernel, dim3(blocks), dim3(GB_PIX), 0, st, a);
    return hipGetLastError();
}

}  // namespace rst
