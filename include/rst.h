/*
 * rst.h — C ABI of the MI355X-native realtime style-transfer hot path (librst.so).
 *
 * Plain C: pointers, sizes and ints only (no torch / TF / HIP types), so ctypes, cgo,
 * JNI or N-API can bind it. Streams are passed as `void*` and interpreted as
 * `hipStream_t`. All tensor pointers are DEVICE pointers owned by the caller, fp32,
 * NHWC (channels last), densely packed. Every call is asynchronous on the given
 * stream, allocates nothing and never synchronises, so it can be captured into a
 * hipGraph. Errors: every entry point returns an rst_status; rst_last_error() gives a
 * thread-local message for the last failing call on this thread.
 *
 * Reference interfaces each entry point replaces (realtime_style_transfer @ /root/reference):
 *   rst_create / rst_destroy     create_style_transfer_model(input_shape, output_shape,
 *                                bottleneck_res_y, bottleneck_num_filters, num_styles)
 *                                -> (tf.keras.Model, P)          models/styleTransfer.py:213-214,332
 *                                plus Model.set_weights/load_weights (predict_using_checkpoint.py:84)
 *   rst_num_style_params         the returned P                  models/styleTransfer.py:278-279,332
 *   rst_forward                  Model.__call__ / predict({'content','style_params'[,'style_weights']})
 *                                                                 models/styleTransfer.py:281-331,
 *                                                                 predict_video_using_checkpoint.py:96
 *   rst_gram                     gram_matrix / get_gram_matrix_model  models/styleLoss.py:11-37
 *   rst_instance_norm            ConditionalInstanceNormalization.call models/styleTransfer.py:57-71
 *   rst_copy_activation          (debug) per-block outputs of the Keras sub-models
 *   rst_predictor_*              create_style_prediction_model(input_shape, feature_extractor,
 *                                num_top_parameters, num_style_parameters=100) -> tf.keras.Model
 *                                                                 models/stylePrediction.py:25-75
 *   rst_gbuffer_preprocess       hdrScreenshots.load_unreal_hdr_screenshot channel assembly +
 *                                common.preprocess_numpy_image     dataloaders/hdrScreenshots.py:14-30,
 *                                                                  dataloaders/common.py:44-57
 *   rst_loss_create / _forward   StyleLossModelVGG + make_style_loss_function(..., with_depth_loss=False)
 *                                -> compute_loss(y_pred, y_true) dict      models/styleLoss.py:69-109,295-369
 */
#ifndef RST_H_
#define RST_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum rst_status {
    RST_OK = 0,
    RST_ERR_INVALID = 1,      /* bad argument / shape mismatch (reference: Python assert / ValueError) */
    RST_ERR_UNSUPPORTED = 2,  /* configuration this build does not implement */
    RST_ERR_HIP = 3,          /* HIP runtime error */
    RST_ERR_ALLOC = 4         /* device allocation failed (only in rst_create) */
} rst_status;

/* Network geometry — the arguments of create_style_transfer_model (styleTransfer.py:213). */
typedef struct rst_shape {
    int in_h, in_w, in_c;        /* content input (H, W, C)                      */
    int out_h, out_w;            /* stylised output (H, W); always 3 channels    */
    int bottleneck_res_y;        /* ShapeConfig.bottleneck_res_y                 */
    int bottleneck_num_filters;  /* ShapeConfig.bottleneck_num_filters           */
    int num_styles;              /* ShapeConfig.num_styles (this build: 1)       */
    int max_batch;               /* largest batch rst_forward will be called with */
} rst_shape;

typedef struct rst_handle rst_handle;

/* Build the network on the current HIP device: derive the block plan exactly as the
 * reference does, upload the weights (HOST pointer, Keras get_weights() order, see
 * realtime_style_transfer_amd/plan.py) into device layouts, allocate the activation /
 * statistics workspace for max_batch. num_weights must equal the plan's total. */
int rst_create(const rst_shape* shape, const float* weights_host, size_t num_weights, rst_handle** out);
void rst_destroy(rst_handle* h);

/* Arithmetic of the convolutions. FP32: exact f32 products (v_mfma_f32_32x32x2_f32), the default.
 * BF16X6: each fp32 operand split exactly into three bf16 pieces (8+8+8 = 24 significant bits, the
 * whole fp32 mantissa) and the six product terms down to 2^-16 accumulated in fp32
 * (6 x v_mfma_f32_32x32x16_bf16): fp32-level products (dropped terms <= 2^-24) at 6/16 of the
 * f32-MFMA cost. BF16X3: two pieces, three terms (16 significant bits per operand; TF32,
 * TensorFlow's default for "fp32" convs on NVIDIA Ampere, keeps 11) at 3/16 of the cost.
 * The split modes are used for the 3x3 s1 convs with Cin % 32 == 0 (the residual blocks); the
 * other layers stay FP32.
 * FP32_WINOGRAD: fp32 arithmetic (exact-f32 MFMA products, f32 accumulation) with the residual
 * convs computed as Winograd F(2x2,3x3) (16 instead of 36 multiplies per 2x2 output tile); single
 * style only (two-style blending keeps the direct kernel).
 * WINOGRAD_BF16X6: as FP32_WINOGRAD, with the residual convs' transform-domain products (V = B^T d B times
 * U = G g G^T) computed as BF16X6 terms: each fp32 operand split exactly into three bf16 pieces, six
 * terms, fp32 accumulation (dropped terms <= 2^-25 of each product) — fp32-level products on the bf16
 * MFMA pipe; the 9x9 start conv likewise (its nine 3x3 sub-kernels' Winograd products as BF16X6 terms).
 * BF16: plain bf16 operands (round-to-nearest-even), fp32 accumulation — a Keras mixed_bfloat16
 * policy's arithmetic (BASELINE config 4 trains in bf16) — on the same layers as the split modes. */
enum { RST_PRECISION_FP32 = 0, RST_PRECISION_BF16X3 = 1, RST_PRECISION_BF16X6 = 2, RST_PRECISION_FP32_WINOGRAD = 3,
       RST_PRECISION_BF16 = 4, RST_PRECISION_WINOGRAD_BF16X6 = 5 };
int rst_create_ex(const rst_shape* shape, const float* weights_host, size_t num_weights, int precision,
                  rst_handle** out);
int rst_precision(const rst_handle* h);

/* Number of style parameters P per style (2662 for rst-960-120-128-17). */
int rst_num_style_params(const rst_handle* h);
/* Total weight count expected by rst_create for this shape (no device work). */
size_t rst_num_weights_for_shape(const rst_shape* shape);

/* out (B, out_h, out_w, 3) = transfer(content (B, in_h, in_w, in_c), style_params (B, S, P)).
 * style_weights must be NULL when num_styles == 1. */
int rst_forward(rst_handle* h, const float* content, const float* style_params, const float* style_weights,
                float* out, int batch, void* stream);

/* Debug: number of conv layers, and a copy of layer idx's most recent output
 * (post-normalisation/activation as the reference block emits it) into dst. */
int rst_num_layers(const rst_handle* h);
int rst_layer_output_shape(const rst_handle* h, int idx, int batch, int* hwc3);
int rst_copy_activation(rst_handle* h, int idx, float* dst, size_t count, int batch, void* stream);

/* Per-layer timing with HIP events recorded on the forward's stream (for bench roofline):
 * rst_profile_begin allocates 3 events per layer for up to max_steps forwards (call outside
 * graph capture); rst_profile_end waits for the last event and returns, per conv layer, the
 * summed conv-kernel time and conv+CIN-finalize time (ms) over the recorded steps. */
int rst_profile_begin(rst_handle* h, int max_steps);
int rst_profile_end(rst_handle* h, float* conv_ms, float* layer_ms, int* steps);

/* In-graph kernel timeline (measurement; no reference counterpart). rst_timeline_begin (outside graph capture)
 * allocates a per-layer stamp buffer that the forwards issued afterwards (eager or captured into a hipGraph) pass to
 * the residual convs (wino_x6) and the narrow convs (conv_lite): every wave stores the 100-MHz realtime counter as it
 * ends. rst_timeline_read synchronises the device and returns, per layer (n = number of layers), the latest end
 * stamp of the most recent forward in microseconds after the first stamped layer's, or -1 for layers whose kernel
 * does not stamp; end[k] - end[k - 1] is layer k's share of a back-to-back graph replay (what rocprofv3's kernel
 * trace reports as its duration there). rst_timeline_end frees the buffer (after any graph holding it is gone). */
int rst_timeline_begin(rst_handle* h);
int rst_timeline_read(rst_handle* h, double* end_us, int n);
int rst_timeline_end(rst_handle* h);
/* Which compiled kernel configuration runs layer idx (100 = VALU 9x9 Cout=3 kernel). */
int rst_layer_kernel_id(const rst_handle* h, int idx);

/* Gram matrices: out[b][c][d] = sum_p feat[b][p][c] * feat[b][p][d] / hw.
 * feat (B, hw, C) fp32; out (B, C, C). workspace: rst_gram_workspace_size() bytes. */
size_t rst_gram_workspace_size(int batch, int hw, int channels);
int rst_gram(const float* feat, int batch, int hw, int channels, float* out, void* workspace, void* stream);

/* Per-pixel style parameters of a two-style model (num_styles == 2): out (B, hw, n) =
 * (1 - w1) * style_params[b][0] + w1 * style_params[b][1], w1 = style_weights (B, hw) — the
 * model's style_weights input (B, out_h, out_w, S-1) at one mip level. Replaces
 * _apply_style_weights(concat[1 - w1, w1], style_params)          models/styleTransfer.py:36-44,297-302
 * with the same device formula the conv prologues blend the CIN affine with (debug / KAT entry). */
int rst_style_param_map(const float* style_weights, const float* style_params, int batch, int hw, int num_styles,
                        int n, float* out, void* stream);

/* Conditional instance norm: y = bias + scale * (x - mean) * rsqrt(var + eps) per (b, c)
 * over H*W, optional ReLU. scale/bias (B, C). workspace: rst_instance_norm_workspace_size(). */
size_t rst_instance_norm_workspace_size(int batch, int hw, int channels);
int rst_instance_norm(const float* x, int batch, int hw, int channels, const float* scale, const float* bias,
                      float eps, int relu, float* y, void* workspace, void* stream);

/* ---- VGG16 / Gram style loss (StyleLossModelVGG + make_style_loss_function, no depth term) ---- */
typedef struct rst_loss_shape {
    int h, w;                 /* prediction / content / style image size (multiples of 16)        */
    int max_batch;
    float content_factor;     /* StyleLossModelVGG: 1e4   (styleLoss.py:101)                      */
    float style_factor;       /*                    1e-3  (styleLoss.py:102)                      */
    float tv_factor;          /*                    1e-1  (styleLoss.py:103)                      */
    int precision;            /* RST_PRECISION_* of the VGG16 3x3 convs (Cin % 32 == 0)            */
} rst_loss_shape;
typedef struct rst_loss_handle rst_loss_handle;

/* Number of VGG16 trunk weights (13 x [kernel (3,3,cin,cout), bias]) in Keras order. */
size_t rst_loss_num_weights(void);
int rst_loss_create(const rst_loss_shape* shape, const float* vgg_weights_host, size_t num_weights,
                    rst_loss_handle** out);
void rst_loss_destroy(rst_loss_handle* h);
/* prediction, gt_content: (B, h, w, 3); gt_style: (B, 1, h, w, 3) == (B, h, w, 3), all in [0, 1].
 * losses (device, B x 4): [loss, feature_loss, style_loss, total_variation_loss] per image. */
int rst_loss_forward(rst_loss_handle* h, const float* prediction, const float* gt_content, const float* gt_style,
                     int batch, float* losses, void* stream);
/* Debug: VGG16 conv layer (0..12) output of the most recent run (the prediction). */
int rst_loss_copy_feature(rst_loss_handle* h, int layer, float* dst, size_t count, int batch, void* stream);

/* ---- Training step (train_network.py:102-138: Keras fit, RMSprop; BASELINE config 4) ----
 * Replaces StyleTransferTrainingModel.train_step (styleTransferTrainingModel.py:26-29 +
 * keras Model.train_step) for the transfer network: forward with BatchNorm in training mode
 * (batch statistics, moving statistics updated with momentum 0.99), the VGG16/Gram loss
 * (rst_loss_*), the gradient of the batch-summed loss with respect to every transfer weight
 * (Keras get_weights() order; BN moving statistics get 0) and to the style parameters (the
 * style predictor's output, styleTransferInferenceModel.py:23-37), and the RMSprop update
 * (OptimizerV2, momentum 0: ms = rho ms + (1 - rho) g^2; w -= lr g / (sqrt(ms) + eps)).
 * Gradients land in a caller-owned buffer so data-parallel callers can all-reduce them
 * (RCCL) before rst_trainer_apply_gradients. Images must have even H, W at every stride-2
 * level (the reference's configs all do). */
typedef struct rst_trainer rst_trainer;
int rst_trainer_create(const rst_shape* shape, const float* weights_host, size_t num_weights,
                       const rst_loss_shape* loss, const float* vgg_weights_host, size_t num_vgg_weights,
                       rst_trainer** out);
/* As rst_trainer_create with the transfer network's conv arithmetic: RST_PRECISION_FP32 (exact-f32
 * MFMA, what rst_trainer_create uses), RST_PRECISION_FP32_WINOGRAD (the residual-block 3x3 convs,
 * forward and input gradient, and the 9x9 start conv forward as Winograd F(2x2,3x3) on f32 MFMA; weight
 * images re-transformed on the device after every update) or RST_PRECISION_WINOGRAD_BF16X6 (as
 * FP32_WINOGRAD with the residual convs' forward, input gradient and weight gradient on exact 3-piece
 * split-bf16 MFMA products, fp32-level). Same training loop as train_network.py:128-138 (Keras fit). */
int rst_trainer_create_ex(const rst_shape* shape, const float* weights_host, size_t num_weights,
                          const rst_loss_shape* loss, const float* vgg_weights_host, size_t num_vgg_weights,
                          int precision, rst_trainer** out);
void rst_trainer_destroy(rst_trainer* t);
int rst_trainer_num_style_params(const rst_trainer* t);
size_t rst_trainer_num_weights(const rst_trainer* t);
/* The trainer's own loss model (e.g. rst_loss_copy_feature of the last prediction). Owned by t. */
rst_loss_handle* rst_trainer_loss(rst_trainer* t);
/* content (B, in_h, in_w, in_c), style_params (B, 1, P), gt_content / gt_style (B, out_h, out_w, 3).
 * Writes prediction (B, out_h, out_w, 3), losses (B x 4, as rst_loss_forward), grad (num_weights)
 * and, when non-NULL, grad_style_params (B, P). All device pointers. */
int rst_trainer_compute_gradients(rst_trainer* t, const float* content, const float* style_params,
                                  const float* gt_content, const float* gt_style, int batch, float* prediction,
                                  float* losses, float* grad, float* grad_style_params, void* stream);
/* Optional, before the step's style-predictor forward (train_network.py:61's model.fit step runs the loss model's
 * ground truth through VGG16 as part of the same step): start the loss targets of the next
 * rst_trainer_compute_gradients — the style image's Gram matrices and the content image's block5_conv3 features —
 * on the trainer's own stream, ordered after the work already in `stream`, so they run beside the predictor
 * forward. The next compute_gradients must pass the same gt_content, gt_style and batch (else it fails with
 * RST_ERR_INVALID) and joins them; without this call compute_gradients starts them itself, beside the transfer
 * network's forward. Bitwise the same results either way. Targets still pending from a step that never reached
 * compute_gradients are joined into `stream` and replaced; compute_gradients joins them on every path, its own
 * failures included. */
int rst_trainer_compute_targets(rst_trainer* t, const float* gt_content, const float* gt_style, int batch,
                                void* stream);
/* Drop pending targets (the caller's step failed between compute_targets and compute_gradients): joins the side
 * stream into `stream`. No-op when none are pending. */
int rst_trainer_cancel_targets(rst_trainer* t, void* stream);
// Makes `stream` wait until grad_style_params of the most recent rst_trainer_compute_gradients is final — recorded
// after the backward's last conditional-instance-norm layer, before the contract layers' backward and the start
// conv's weight gradient — so the style predictor's backward (rst_predictor_trainer_backward) can run on `stream`
// beside the rest of the transfer network's backward. The caller joins `stream` back before using either gradient.
// Replaces the serial predictor backward after compute_gradients (reference: train_network.py:102 fits predictor and
// transfer network in one tape, styleTransferTrainingModel.py:26-33).
int rst_trainer_wait_style_gradient(rst_trainer* t, void* stream);
/* RMSprop on the device-resident weights with gradient grad (num_weights), then re-pack them
 * into the kernels' weight images. Keras defaults: lr 1e-3, rho 0.9, epsilon 1e-7. */
int rst_trainer_apply_gradients(rst_trainer* t, const float* grad, float learning_rate, float rho, float epsilon,
                                void* stream);
/* Device copies of the current weights (Keras order) / RMSprop slots; set_weights re-packs. */
int rst_trainer_copy_weights(rst_trainer* t, float* dst, size_t count, void* stream);
int rst_trainer_copy_slots(rst_trainer* t, float* dst, size_t count, void* stream);
int rst_trainer_set_weights(rst_trainer* t, const float* src, size_t count, void* stream);
/* Restore the RMSprop `rms` slots (a checkpoint's .OPTIMIZER_SLOT values, Checkpoint.restore,
 * save_using_checkpoint.py:65-66 / train_network.py:112-113). */
int rst_trainer_set_slots(rst_trainer* t, const float* src, size_t count, void* stream);
/* Data parallel: the BatchNormalization moving statistics (every BN layer's moving_mean then
 * moving_variance, get_weights() order), which each rank updates from its own batch. get copies them
 * into dst (e.g. the tail of the gradient bucket, so ONE all-reduce carries both); set writes
 * src[i] / divisor back (divisor = world size after a SUM all-reduce: tf.distribute.MirroredStrategy's
 * MEAN aggregation of the moving-average assignments, styleTransfer.py:201, train_network.py:61) without
 * re-packing any kernel image (no training kernel reads them). Replaces the reference's implicit
 * MirroredStrategy sync; the reference itself trains on one GPU (train_network.py:14-23). */
size_t rst_trainer_num_moving_statistics(const rst_trainer* t);
int rst_trainer_get_moving_statistics(rst_trainer* t, float* dst, size_t count, void* stream);
int rst_trainer_set_moving_statistics(rst_trainer* t, const float* src, size_t count, float divisor, void* stream);
/* Debug: gradient of the batch loss w.r.t. conv layer `layer`'s activated output (before any skip
 * add; the last layer's is d loss / d prediction) from the most recent compute_gradients. */
int rst_trainer_copy_output_gradient(rst_trainer* t, int layer, float* dst, size_t count, int batch, void* stream);
/* Debug: d loss / d (VGG16 conv `layer` output). The first call for a layer arms the tap (it
 * allocates; dst may be NULL); later calls copy the value of the most recent compute_gradients. */
int rst_trainer_debug_vgg_gradient(rst_trainer* t, int layer, float* dst, size_t count, int batch, void* stream);

/* ---- Style predictor (create_style_prediction_model, models/stylePrediction.py:25-75) ----
 * Replaces the Keras predictor that make_style_transfer_inference_model runs once per style image
 * (styleTransferInferenceModel.py:23-26; predict_video_using_checkpoint.py:77-83):
 *   DUMMY:      Conv2D(1, 9, strides=5, padding='same') on the raw image            (:31-32)
 *   MOBILE_NET: Rescaling(2, -1) + keras.applications.MobileNetV3Small(include_top=False,
 *               include_preprocessing=False), BatchNormalization in inference mode   (:33-38)
 * then GlobalAveragePooling2D (:55), Conv2D(num_style_parameters, 1) (:60-64) and
 * Conv2D(num_top_parameters, 1) (:67-71), squeezed to (B, num_top_parameters) (:73-74).
 * Weights: Keras get_weights() order (per layer kernel[, bias]; BN gamma, beta, moving_mean,
 * moving_variance), HOST pointer; rst_predictor_num_weights gives the count for a shape. */
enum { RST_EXTRACTOR_DUMMY = 0, RST_EXTRACTOR_MOBILE_NET = 1 };
typedef struct rst_predictor_shape {
    int h, w, c;                  /* style image (H, W, C): ShapeConfig.input_shape['style'][1:]     */
    int feature_extractor;        /* RST_EXTRACTOR_* (EFFICIENT_NET: RST_ERR_UNSUPPORTED)             */
    int num_top_parameters;       /* P, the transfer network's style-parameter count (num_top_parameters) */
    int num_style_parameters;     /* width of the StylePredictor bottleneck (default 100)            */
    int max_batch;                /* largest batch (= images) rst_predictor_forward is called with    */
} rst_predictor_shape;
typedef struct rst_predictor rst_predictor;
size_t rst_predictor_num_weights(const rst_predictor_shape* shape);
int rst_predictor_create(const rst_predictor_shape* shape, const float* weights_host, size_t num_weights,
                         rst_predictor** out);
void rst_predictor_destroy(rst_predictor* p);
/* style (B, h, w, c) -> style_params (B, num_top_parameters). Device pointers, async on stream.
 * For num_styles S pass the (B, S, h, w, c) style stack as B*S images: the output is (B, S, P). */
int rst_predictor_forward(rst_predictor* p, const float* style, int batch, float* style_params, void* stream);
/* Debug: stage outputs (MOBILE_NET: stem, the 11 inverted-residual blocks, Conv_1 features;
 * DUMMY: the conv output) of the most recent forward. */
int rst_predictor_num_stages(const rst_predictor* p);
int rst_predictor_stage_shape(const rst_predictor* p, int idx, int* hwc3);
int rst_predictor_copy_stage(rst_predictor* p, int idx, float* dst, size_t count, int batch, void* stream);

/* ---- Style-predictor training (train_network.py:86-138 fits the predictor jointly) ----
 * Forward in Keras training mode: BatchNormalization normalises with the batch statistics over
 * (B, H, W) and updates its moving statistics (MobileNetV3: momentum 0.999, eps 1e-3) in the
 * device-resident weights. Backward: gradient of sum(style_params * d_style_params) with respect to
 * every predictor weight (Keras get_weights() order; moving statistics get 0) — chain it to
 * rst_trainer_compute_gradients' grad_style_params. The style tensor passed to forward must stay
 * valid until the matching backward. */
typedef struct rst_predictor_trainer rst_predictor_trainer;
int rst_predictor_trainer_create(const rst_predictor_shape* shape, const float* weights_host, size_t num_weights,
                                 rst_predictor_trainer** out);
void rst_predictor_trainer_destroy(rst_predictor_trainer* t);
size_t rst_predictor_trainer_num_weights(const rst_predictor_trainer* t);
int rst_predictor_trainer_forward(rst_predictor_trainer* t, const float* style, int batch, float* style_params,
                                  void* stream);
int rst_predictor_trainer_backward(rst_predictor_trainer* t, const float* d_style_params, float* grad, void* stream);
int rst_predictor_trainer_apply_gradients(rst_predictor_trainer* t, const float* grad, float learning_rate, float rho,
                                          float epsilon, void* stream);
int rst_predictor_trainer_copy_weights(rst_predictor_trainer* t, float* dst, size_t count, void* stream);
int rst_predictor_trainer_set_weights(rst_predictor_trainer* t, const float* src, size_t count, void* stream);
int rst_predictor_trainer_copy_slots(rst_predictor_trainer* t, float* dst, size_t count, void* stream);
int rst_predictor_trainer_set_slots(rst_predictor_trainer* t, const float* src, size_t count, void* stream);
/* As rst_trainer_*_moving_statistics for the predictor's BatchNormalization layers (MobileNetV3Small). */
size_t rst_predictor_trainer_num_moving_statistics(const rst_predictor_trainer* t);
int rst_predictor_trainer_get_moving_statistics(rst_predictor_trainer* t, float* dst, size_t count, void* stream);
int rst_predictor_trainer_set_moving_statistics(rst_predictor_trainer* t, const float* src, size_t count, float divisor,
                                                void* stream);

/* ---- G-buffer ingest ----
 * Replaces the host-side numpy/TF preprocessing of an Unreal HDR screenshot:
 *   dataloaders/hdrScreenshots.py:14-30   per-channel EXR images stacked / concatenated (channel order
 *                                         = `expected_channels` order) into (h, w, C)
 *   dataloaders/common.py:44-57           preprocess_numpy_image(image, shape): tf.image.resize (bilinear,
 *                                         half-pixel centers) to the aspect-preserving size, then
 *                                         tf.image.resize_with_crop_or_pad to (shape[0], shape[1])
 * in one device pass. planes: HOST array of num_planes DEVICE pointers; element (y, x) of plane k
 * is planes[k][y * row_stride + x * pixel_stride] (planar EXR channels: pixel_stride 1, row_stride w;
 * an interleaved (h, w, C) image: planes[k] = base + k, pixel_stride C, row_stride w * C).
 * dst: device (dst_h, dst_w, num_planes) NHWC fp32 — directly the `content` input of rst_forward.
 * f32 arithmetic identical to TF's ResizeBilinear kernel (no FMA contraction). */
#define RST_GBUFFER_MAX_PLANES 32
int rst_gbuffer_resized_size(int src_h, int src_w, int dst_h, int dst_w, int* new_hw2);
int rst_gbuffer_preprocess(const float* const* planes, int num_planes, int src_h, int src_w, long long row_stride,
                           long long pixel_stride, float* dst, int dst_h, int dst_w, void* stream);

/* ---- Checkpoint I/O helper ----
 * CRC-32C (Castagnoli) of n bytes continuing from crc (0 to start): the checksum TF tensor bundles
 * store for every tensor and SSTable block (tracing/checkpoint.py:21-37 writes them through
 * tf.train.Checkpoint / Model.save_weights; predict_using_checkpoint.py:84 reads them). Host-only. */
unsigned int rst_crc32c_extend(unsigned int crc, const void* data, size_t n);

const char* rst_last_error(void);
const char* rst_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RST_H_ */
