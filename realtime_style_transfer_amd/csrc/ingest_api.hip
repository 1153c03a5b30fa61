// ingest_api.hip — C ABI of the G-buffer ingest (include/rst.h, rst_gbuffer_*).
// Host side of dataloaders/common.py:44-57 (preprocess_numpy_image): the resize target and the
// crop/pad offsets are derived here in f64 exactly as the reference derives them in Python floats.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/rst.h"
#include "common.h"
#include "kernels.h"

using namespace rst;

static int fail(int code, const std::string& msg) { return set_error(code, msg); }

int rst_gbuffer_resized_size(int src_h, int src_w, int dst_h, int dst_w, int* new_hw2) {
    if (new_hw2 == nullptr || src_h <= 0 || src_w <= 0 || dst_h <= 0 || dst_w <= 0)
        return fail(RST_ERR_INVALID, "rst_gbuffer_resized_size: sizes must be positive");
    // aspect_ratio_image = image.shape[0] / image.shape[1]; aspect_ratio_target = shape[0] / shape[1]
    const double ai = (double)src_h / (double)src_w, at = (double)dst_h / (double)dst_w;
    if (ai > at) {   // should_scale_to_target_y: (ceil(shape[1] * aspect_ratio_image), shape[1])
        new_hw2[0] = (int)std::ceil((double)dst_w * ai);
        new_hw2[1] = dst_w;
    } else {         // (shape[0], ceil(shape[0] / aspect_ratio_image))
        new_hw2[0] = dst_h;
        new_hw2[1] = (int)std::ceil((double)dst_h / ai);
    }
    return RST_OK;
}

// Python floor division (TF resize_with_crop_or_pad uses `//` on ints)
static int floordiv2(int v) { return v >= 0 ? v / 2 : -((-v + 1) / 2); }

int rst_gbuffer_preprocess(const float* const* planes, int num_planes, int src_h, int src_w, long long row_stride,
                           long long pixel_stride, float* dst, int dst_h, int dst_w, void* stream) {
    if (planes == nullptr || dst == nullptr) return fail(RST_ERR_INVALID, "rst_gbuffer_preprocess: null argument");
    if (num_planes <= 0 || num_planes > GBUFFER_MAX_PLANES)
        return fail(RST_ERR_INVALID, "rst_gbuffer_preprocess: num_planes must be in [1, " +
                                         std::to_string(GBUFFER_MAX_PLANES) + "], got " + std::to_string(num_planes));
    if (row_stride <= 0 || pixel_stride <= 0)
        return fail(RST_ERR_INVALID, "rst_gbuffer_preprocess: strides must be positive");
    if ((long long)dst_h * dst_w * num_planes >= (1LL << 31))
        return fail(RST_ERR_UNSUPPORTED, "rst_gbuffer_preprocess: output has 2^31 or more elements");
    int nhw[2];
    int st = rst_gbuffer_resized_size(src_h, src_w, dst_h, dst_w, nhw);
    if (st != RST_OK) return st;
    GbufferArgs a{};
    for (int k = 0; k < num_planes; ++k) {
        if (planes[k] == nullptr) return fail(RST_ERR_INVALID, "rst_gbuffer_preprocess: null plane pointer");
        a.planes[k] = planes[k];
    }
    a.num_planes = num_planes;
    a.src_h = src_h;
    a.src_w = src_w;
    a.row_stride = (long)row_stride;
    a.pixel_stride = (long)pixel_stride;
    a.dst = dst;
    a.dst_h = dst_h;
    a.dst_w = dst_w;
    a.new_h = nhw[0];
    a.new_w = nhw[1];
    // resize_with_crop_or_pad: crop offset max((in - target) // 2, 0), pad offset max((target - in) // 2, 0)
    const int crop_y = std::max(floordiv2(nhw[0] - dst_h), 0), pad_y = std::max(floordiv2(dst_h - nhw[0]), 0);
    const int crop_x = std::max(floordiv2(nhw[1] - dst_w), 0), pad_x = std::max(floordiv2(dst_w - nhw[1]), 0);
    a.off_y = crop_y - pad_y;
    a.off_x = crop_x - pad_x;
    // CalculateResizeScale(in, out, align_corners=false) = static_cast<float>(in) / out  (f32 division)
    a.scale_y = (float)src_h / (float)nhw[0];
    a.scale_x = (float)src_w / (float)nhw[1];
    const hipError_t e = gbuffer_resize_crop_launch(a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(RST_ERR_HIP, std::string("rst_gbuffer_preprocess: ") + hipGetErrorString(e));
    return RST_OK;
}
