#!/usr/bin/env python3
"""Benchmark: stylised frames/s of the rst-960-120-128-17 transfer network on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched
by torch.distributed.run (one rank per GPU, RCCL). One "step" = one forward of the transfer
network over one batch of synthetic 480x960x17 G-buffer frames (BASELINE config 2:
single-frame fp32 inference, B=1, unless --batch). Frames shard across ranks with no
data-path collective (weak scaling); the timed region is bracketed by barrier + device sync,
and the max time over ranks is used. Rank 0 prints ONE JSON line.

Extra fields: ``roofline`` (dominant kernel, HIP-event timed inside the timed region),
``cpu_baseline`` (torch-CPU f32 restatement of the same graph on the host cores — TF-CPU is not
installed; a bounded sample), ``max_abs_delta_vs_oracle`` (same frame, GPU vs that restatement),
and the batch-8 hipGraph stream throughput (BASELINE config 3).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402

SPEC = "rst-960-120-128-17"
METRIC = "stylized FPS/GPU at 960p×17ch (rst-960-120-128-17); max-abs Δ vs TF ref"
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: Peak FP32 (matrix) = vector peak
BF16_MFMA_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md: Peak BF16 MFMA ~2.5 PF dense
HBM_PEAK_GBS = 8000.0


def layer_flops(layer) -> float:
    """Algorithmic FLOPs (2 x MAC) of one conv layer for one image (SURVEY §8d convention)."""
    if layer.kind == 'conv':
        return 2.0 * layer.out_hw[0] * layer.out_hw[1] * layer.k * layer.k * layer.cin * layer.cout
    # transposed conv: counted as H_in * W_in * k^2 * Cin * Cout MACs
    return 2.0 * layer.in_hw[0] * layer.in_hw[1] * layer.k * layer.k * layer.cin * layer.cout


KERNEL_NAMES = {
    1: "conv_mfma<9x9 s1 CK18 NT32>", 2: "conv_mfma<9x9 s1 CK4 NT32>", 3: "conv_mfma<3x3 s2 CK16 NT32>",
    4: "conv_mfma<3x3 s2 CK8 NT32>", 5: "conv_mfma<3x3 s1 CK32 NT128>", 6: "conv_mfma<3x3 s1 CK32 NT32>",
    7: "conv_mfma<3x3 s1 CK8 NT32>", 8: "conv_mfma<2x2 phase CK32 NT128>", 9: "conv_mfma<2x2 phase CK32 NT64>",
    10: "conv_mfma<2x2 phase CK32 NT32>", 11: "conv_mfma<2x2 phase CK16 NT32>", 12: "conv_mfma<2x2 phase CK8 NT32>",
    13: "conv_mfma<3x3 s1 CK16 NT32>", 14: "conv_mfma<3x3 s2 CK4 NT32>", 15: "conv_mfma<3x3 s1 CK4 NT32>",
    16: "conv_mfma<2x2 phase CK4 NT32>", 17: "conv_mfma<3x3 s1 CK32 NT64>", 100: "small_conv_kernel<9x9 Cout3 VALU>",
    101: "conv_bf3<3x3 s1 CK32 NT128 bf16x3>", 102: "conv_bf3<3x3 s1 CK32 NT64 bf16x3>",
    111: "conv_bf3<3x3 s1 CK32 NT128 bf16x6>", 112: "conv_bf3<3x3 s1 CK32 NT64 bf16x6>",
    113: "conv_bf3<3x3 s1 CK32 NT64 8x16 bf16x6>",
    200: "wino_conv<F(2x2,3x3) 8x16 N128 f32 MFMA>", 201: "wino9_conv<9x9 as 9 x F(2x2,3x3) 8x16 N32 f32 MFMA>",
}


DTYPE_DESC = {
    "fp32": "fp32 (exact-f32 MFMA products, f32 accumulate), every conv direct (implicit GEMM)",
    "fp32_winograd": "fp32 (exact-f32 MFMA products, f32 accumulate); the residual convs as fused Winograd "
                     "F(2x2,3x3) (16 instead of 36 multiplies per 2x2 output tile, f32 transforms), other layers "
                     "direct",
    "bf16x6": "fp32 via exact 3-piece split bf16 (24 significant bits, 6 product terms, dropped terms <= 2^-24), "
              "fp32 accumulate, on the residual convs; other layers fp32 MFMA",
    "bf16x3": "fp32 via 2-piece split bf16 (3 product terms, 16 significant bits per operand), fp32 accumulate, "
              "on the residual convs; other layers fp32 MFMA",
    "bf16": "bf16 operands (8 significant bits), fp32 accumulate, on the residual convs; other layers fp32 MFMA",
}


def dominant_kernel(model, plan, conv_ms, nsteps, B) -> dict:
    """The kernel (config id) with the largest summed time over the timed launches, with its
    algorithmic TFLOP/s (direct-conv FLOPs per launch / average launch duration)."""
    groups = {}
    for i, l in enumerate(plan.layers):
        kid = model.layer_kernel_id(i)
        g = groups.setdefault(kid, {"ms": 0.0, "flops": 0.0, "launches": 0})
        g["ms"] += conv_ms[i]
        g["flops"] += layer_flops(l) * B * nsteps
        g["launches"] += nsteps
    kid = max(groups, key=lambda k: groups[k]["ms"])
    g = groups[kid]
    avg_ms = g["ms"] / max(g["launches"], 1)
    fpl = g["flops"] / max(g["launches"], 1)
    return {"id": kid, "kernel": KERNEL_NAMES.get(kid, str(kid)), "avg_ms": avg_ms, "flops_per_launch": fpl,
            "launches": g["launches"], "tflops": fpl / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0}


def cpu_threads() -> int:
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env))) if env else aff


def train_flops_per_sample(plan, H, W) -> dict:
    """Algorithmic FLOPs (2 x MAC) of one training sample: transfer forward + backward (wgrad on
    every conv, dgrad on every conv but the first), VGG16 forward x3 (style, content, prediction),
    VGG16 dgrad on the prediction branch down to the image, Gram forward x2 and backward x1."""
    fwd = sum(layer_flops(l) for l in plan.layers)
    dgrad = sum(layer_flops(l) for l in plan.layers[1:])
    vgg_fwd, gram, cin, h, w = 0.0, 0.0, 3, H, W
    chans = [64, 64, 128, 128, 256, 256, 256, 512, 512, 512, 512, 512, 512]
    pools = {1, 3, 6, 9}
    for i, c in enumerate(chans):
        vgg_fwd += 2.0 * h * w * 9 * cin * c
        if i in pools:
            gram += 2.0 * h * w * c * c
            h, w = h // 2, w // 2
        cin = c
    return {"transfer_fwd": fwd, "transfer_bwd": fwd + dgrad, "vgg_fwd_x3": 3 * vgg_fwd, "vgg_dgrad": vgg_fwd,
            "gram_fwd_x2_bwd_x1": 3 * gram}


def bench_split(args, world, dev, cfg, ins, outs, plan, weights, P, inputs, timed, precision):
    """The same B=1 hipGraph frame loop with a split-bf16 precision mode on the residual convs."""
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    B = args.batch
    model, _ = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=weights, max_batch=B, device=dev, precision=precision)
    out = torch.empty((B,) + outs, dtype=torch.float32, device=dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        model(inputs, out=out)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        model(inputs, out=out)
    for _ in range(args.warmup):
        g.replay()
    torch.cuda.synchronize()
    el = timed(g.replay, args.steps)
    model.profile_begin(args.steps)
    timed(lambda: model(inputs, out=out), args.steps)
    conv_ms, _, nsteps = model.profile_end()
    ids = [model.layer_kernel_id(i) for i in range(len(plan.layers))]
    bf3 = [i for i, k in enumerate(ids) if k >= 101]
    terms = {"bf16x3": 3, "bf16x6": 6, "bf16": 1}.get(precision, 6)
    ms = sum(conv_ms[i] for i in bf3) / max(nsteps, 1) / max(len(bf3), 1)
    fl = sum(layer_flops(plan.layers[i]) for i in bf3) * B / max(len(bf3), 1)
    eff_tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    if precision == "fp32":
        dom = dominant_kernel(model, plan, conv_ms, nsteps, B)
        return model, {
            "value": round(world * B * args.steps / el, 3), "unit": "frames/s",
            "ms_per_step": round(el * 1e3 / args.steps, 4), "dtype": DTYPE_DESC["fp32"],
            "roofline": {"bound": "mfma", "kernel": dom["kernel"], "achieved": round(dom["tflops"], 2),
                         "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(dom["tflops"] / FP32_MFMA_PEAK_TFLOPS, 4),
                         "avg_launch_ms": round(dom["avg_ms"], 5)},
            "layers_ms": [round(c / max(nsteps, 1), 4) for c in conv_ms],
        }
    if precision == "fp32_winograd":
        return model, {
            "value": round(world * B * args.steps / el, 3), "unit": "frames/s",
            "ms_per_step": round(el * 1e3 / args.steps, 4),
            "dtype": "fp32 (exact-f32 MFMA products, f32 accumulate); the residual convs as fused Winograd "
                     "F(2x2,3x3) (16 instead of 36 multiplies per 2x2 output tile), other layers direct",
            "roofline": {"bound": "mfma", "kernel": KERNEL_NAMES.get(200), "achieved": round(eff_tf, 2),
                         "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s (algorithmic = direct-conv FLOPs)",
                         "frac": round(eff_tf / FP32_MFMA_PEAK_TFLOPS, 4), "avg_launch_ms": round(ms, 5),
                         "mfma_pipe_frac": round(eff_tf * 16.0 / 36.0 / FP32_MFMA_PEAK_TFLOPS, 4)},
            "layers_ms": [round(c / max(nsteps, 1), 4) for c in conv_ms],
        }
    return model, {
        "value": round(world * B * args.steps / el, 3), "unit": "frames/s", "ms_per_step": round(el * 1e3 / args.steps, 4),
        "dtype": DTYPE_DESC.get(precision, precision),
        "roofline": {"bound": "mfma", "kernel": KERNEL_NAMES.get(ids[bf3[0]], "?") if bf3 else None,
                     "achieved": round(terms * eff_tf, 2), "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s (bf16 MFMA)",
                     "frac": round(terms * eff_tf / BF16_MFMA_PEAK_TFLOPS, 4), "avg_launch_ms": round(ms, 5),
                     "fp32_equivalent_tflops": round(eff_tf, 2)},
        "layers_ms": [round(c / max(nsteps, 1), 4) for c in conv_ms],
    }


def bench_training(args, world, rank, dev, cfg, ins, outs, plan, weights, P, timed, precision="fp32"):
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    TB = args.train_batch
    lm = StyleLossModelVGG(outs, max_batch=TB, device=dev, precision=precision)
    from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer
    sins = tuple(cfg.input_shape['style'][1:])
    # train_network.py fits the MobileNetV3Small style predictor jointly (stylePrediction.py:25-75)
    pr = StylePredictionTrainer(sins, cfg.style_feature_extractor_type, P, max_batch=TB, device=dev)
    tr = StyleTransferTrainingModel(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, loss_model=lm,
                                    weights=weights, max_batch=TB, device=dev, style_predictor=pr)
    rng = np.random.default_rng(3000 + rank)
    x = {'content': torch.from_numpy(rng.random((TB,) + ins, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((TB, 1) + sins, dtype=np.float32)).to(dev)}
    y = {'content': torch.from_numpy(rng.random((TB,) + outs, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((TB, 1) + outs, dtype=np.float32)).to(dev)}
    for _ in range(2):
        m = tr.train_step(x, y)
    torch.cuda.synchronize()
    el = timed(lambda: tr.train_step(x, y), args.train_steps)
    loss = float(tr.compute_metrics()['loss'])
    fl = train_flops_per_sample(plan, outs[0], outs[1])
    per_sample = sum(fl.values())
    ms = el * 1e3 / args.train_steps
    tfs = per_sample * TB / (ms * 1e-3) / 1e12
    return {"workload": f"{SPEC} train_network.py step (BASELINE config 4): MobileNetV3Small style predictor + "
                        f"transfer net, training-mode forward, VGG16/Gram loss (no depth term), backward of both, " +
                        ("RCCL gradient all-reduce (SUM, one bucket), " if world > 1 else "") +
                        "RMSprop on both", "batch_per_gpu": TB, "steps": args.train_steps, "ms_per_step": round(ms, 3),
            "frames_per_s": round(world * TB * args.train_steps / el, 3),
            "dtype": {"fp32": "fp32 (f32 MFMA)",
                      "bf16x6": "VGG16 3x3 convs: exact 3-piece split bf16 MFMA (fp32-level products, fp32 accumulate); "
                                "transfer net and the rest fp32 (transfer_precision)",
                      "bf16x3": "VGG16 3x3 convs: 2-piece split bf16 MFMA (16-bit operands, fp32 accumulate); "
                                "transfer net and the rest fp32 (transfer_precision)",
                      "bf16": "VGG16 3x3 convs: bf16 operands, fp32 accumulate (mixed_bfloat16 arithmetic); "
                              "transfer net and the rest fp32 (transfer_precision)"}[precision],
            "transfer_precision": {"fp32": "exact f32 MFMA",
                                   "fp32_winograd": "residual 3x3 convs (forward + input gradient) as Winograd "
                                                    "F(2x2,3x3) on f32 MFMA, the other transfer convs exact f32"}[
                tr.precision],
            "tflop_per_sample": round(per_sample / 1e12, 4),
            "achieved_tflops_per_gpu": round(tfs, 2), "frac_fp32_mfma_peak": round(tfs / FP32_MFMA_PEAK_TFLOPS, 4),
            "frac_note": "algorithmic (direct-conv, f32-equivalent) FLOPs over the f32 MFMA peak; the bf16 VGG16 "
                         "convs and the Winograd transfer convs execute fewer f32 MFMA operations, so > 1 is possible",
            "flop_breakdown_per_sample_gflop": {k: round(v / 1e9, 2) for k, v in fl.items()},
            "last_loss_mean": loss}


def predictor_bytes_per_image(ins) -> float:
    """Algorithmic HBM bytes of one MobileNetV3Small style-predictor pass (stylePrediction.py:25-75): every
    layer reads its input and writes its output once (fp32), plus all weights once."""
    from realtime_style_transfer_amd.stylePrediction import _MOBILENET_V3_SMALL, _depth
    H, W = ins[0], ins[1]
    by = H * W * 3
    H, W = -(-H // 2), -(-W // 2)
    by += H * W * 16
    cin = 16
    for i, (e, f, k, s, se, _) in enumerate(_MOBILENET_V3_SMALL):
        ce = _depth(cin * e)
        if i:
            by += 2 * H * W * ce + H * W * cin        # expand: read cin, write ce; dw reads ce
        else:
            by += H * W * ce
        H, W = -(-H // s), -(-W // s)
        by += H * W * ce * (2 if se else 1)           # dw write (+ SE-scaled re-read by project)
        by += H * W * f + (H * W * f if (s == 1 and cin == f) else 0)
        cin = f
    by += H * W * cin + H * W * 576 * 2              # Conv_1 in/out, GAP read
    return 4.0 * by


def bench_ingest(args, dev, cfg, timed, rank):
    """G-buffer ingest: a 1080x1920 Unreal screenshot's 17 channel planes (already in
    HBM, as after the per-channel EXR uploads) -> rst_gbuffer_preprocess -> the 480x960x17 content tensor
    (hdrScreenshots.py:14-30 + common.py:44-57 in one pass). HBM-bound: algorithmic bytes = the source
    rows x columns the bilinear taps touch + the output."""
    from realtime_style_transfer_amd.dataloaders.common import preprocess_planes, resized_size
    src, C = (1080, 1920), cfg.num_channels
    shape = cfg.input_shape['content'][:2]
    planes = [torch.rand(src, device=dev) for _ in range(C)]
    out = torch.empty(shape + (C,), device=dev)
    fn = lambda: preprocess_planes(planes, shape, out=out)   # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    steps = max(args.steps, 50)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    el = timed(fn, steps)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    nh, nw = resized_size(src, shape)

    def touched(n_out, n_in, off, n):
        sc = np.float32(np.float32(n_in) / np.float32(n_out))
        pos = (np.arange(off, off + n, dtype=np.float32) + np.float32(0.5)) * sc - np.float32(0.5)
        lo = np.maximum(np.floor(pos).astype(np.int64), 0)
        hi = np.minimum(np.ceil(pos).astype(np.int64), n_in - 1)
        return len(set(lo.tolist()) | set(hi.tolist()))
    rows = touched(nh, src[0], (nh - shape[0]) // 2, shape[0])
    cols = touched(nw, src[1], (nw - shape[1]) // 2, shape[1])
    alg = (rows * cols + shape[0] * shape[1]) * C * 4.0
    res = {"workload": f"1080x1920x{C} G-buffer planes -> {shape[0]}x{shape[1]}x{C} content (TF bilinear "
                       f"half-pixel resize to {nh}x{nw} + center crop), one frame per call",
           "ms_per_frame": round(ms, 5), "frames_per_s": round(1e3 / ms, 1),
           "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes": alg}}
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.ingest_ref import preprocess_numpy_image
        x = np.random.default_rng(5).random(src + (C,), dtype=np.float32)
        n, t = 0, 0.0
        while n < 5 and t < 5.0:
            t0 = time.perf_counter()
            preprocess_numpy_image(x, shape)
            t += time.perf_counter() - t0
            n += 1
        res["cpu_baseline"] = {"value": round(n / t, 3), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{n} frames through oracle/ingest_ref.py (numpy f32, TF not installed)"}
    return res


def bench_predictor(args, dev, cfg, transfer_model, transfer_inputs, P, timed):
    """make_style_transfer_inference_model path: the MobileNetV3Small style predictor on a 480x960x3 style image
    (once per style in the video loop, predict_video_using_checkpoint.py:77-83) and predictor + transfer per
    frame (the Keras inference model runs both per call, styleTransferInferenceModel.py:23-37)."""
    from realtime_style_transfer_amd.stylePrediction import create_style_prediction_model
    sins = tuple(cfg.input_shape['style'][1:])
    pred = create_style_prediction_model(sins, cfg.style_feature_extractor_type, P, max_batch=1, device=dev)
    rng = np.random.default_rng(4000)
    style = torch.from_numpy(rng.random((1,) + sins, dtype=np.float32)).to(dev)
    sp = torch.empty((1, P), dtype=torch.float32, device=dev)        # the predictor writes the transfer's input
    tin = {'content': transfer_inputs['content'][:1], 'style_params': sp.view(1, 1, P)}
    out = torch.empty((1,) + transfer_model.output_shape, dtype=torch.float32, device=dev)

    def graph_of(fn):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        return g

    gp = graph_of(lambda: pred(style, out=sp))
    el_p = timed(gp.replay, args.steps)
    gi = graph_of(lambda: (pred(style, out=sp), transfer_model(tin, out=out)))
    el_i = timed(gi.replay, args.steps)
    ms_p = el_p * 1e3 / args.steps
    by = predictor_bytes_per_image(sins)
    return {"workload": f"MobileNetV3Small style predictor + GAP + 1x1 heads (P={P}) on one {sins[0]}x{sins[1]}x3 "
                        f"style image, hipGraph replay", "ms_per_style_image": round(ms_p, 4),
            "roofline": {"bound": "hbm", "achieved": round(by / (ms_p * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(by / (ms_p * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes": by,
                         "note": "~45 small launches; latency-bound at B=1 (whole graph, not one kernel)"},
            "inference_model_fps": round(args.steps / el_i, 3),
            "inference_model_workload": "predictor + transfer per frame (B=1), as the Keras inference model runs"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1, help="frames per step per GPU (config 2: 1)")
    ap.add_argument("--stream-batch", type=int, default=8, help="config 3 (hipGraph stream) batch; 0 to skip")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0, help="bounded CPU-baseline sample (seconds)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="headline from eager launches instead of hipGraph replay")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    ap.add_argument("--train-batch", type=int, default=4, help="config 4 training step batch per GPU; 0 to skip")
    ap.add_argument("--train-steps", type=int, default=5)
    ap.add_argument("--precision", default="fp32_winograd",
                    help="headline precision mode: fp32_winograd (default: fp32 arithmetic, residual convs as "
                         "fused Winograd F(2x2,3x3)), fp32 (all direct), bf16x6, bf16x3")
    ap.add_argument("--no-bf16x3", action="store_true", help="skip the other precision-mode measurements")
    ap.add_argument("--no-predictor", action="store_true", help="skip the style-predictor measurement")
    ap.add_argument("--no-ingest", action="store_true", help="skip the G-buffer ingest measurement")
    ap.add_argument("--pcie-steps", type=int, default=50, help="host-resident frame loop (PCIe-inclusive); 0 to skip")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{torch.cuda.current_device()}")

    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model

    cfg = ShapeConfig.from_spec(SPEC)
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    weights = init_weights(plan, seed=2)
    B = args.batch
    max_b = max(B, args.stream_batch)
    model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=weights, max_batch=max_b, device=dev, precision=args.precision)
    # synthetic frames (distinct per rank), resident in HBM before the timed region
    rng = np.random.default_rng(1000 + rank)
    content = torch.from_numpy(rng.random((B,) + ins, dtype=np.float32)).to(dev)
    sp_np = synthetic_style_params(B, 1, P, plan, seed=1)
    style = torch.from_numpy(sp_np).to(dev)
    out = torch.empty((B,) + outs, dtype=torch.float32, device=dev)
    inputs = {'content': content, 'style_params': style}

    for _ in range(args.warmup):
        model(inputs, out=out)
    torch.cuda.synchronize()

    def timed(fn, steps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # ---------------- timed region 1 (headline): one hipGraph replay per step -------------------
    # The forward (~30 kernel launches) is captured once into a hipGraph on torch's stream —
    # how a real-time frame loop drives it; the per-frame host cost is one graph launch.
    graph = None
    if not args.eager:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            model(inputs, out=out)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            model(inputs, out=out)
        for _ in range(args.warmup):
            graph.replay()
        torch.cuda.synchronize()
        elapsed = timed(graph.replay, args.steps)
    # ---------------- PCIe-inclusive rate (reported beside the headline, never as `value`) ------
    # The C-ABI hands over device pointers; a host-resident frame loop adds H2D of the 31 MB
    # G-buffer and D2H of the 5.5 MB output per frame. "serial": upload -> graph -> download on one
    # stream. "pipelined": two input/output buffer pairs and two graphs; frame i+1 is uploaded and
    # frame i-1 downloaded on a copy stream while frame i computes (pinned host buffers).
    pcie = None
    if graph is not None and args.pcie_steps > 0:
        n = args.pcie_steps
        h_in = [torch.from_numpy(rng.random((B,) + ins, dtype=np.float32)).pin_memory() for _ in range(2)]
        h_out = [torch.empty((B,) + outs, dtype=torch.float32).pin_memory() for _ in range(2)]

        def serial():
            content.copy_(h_in[0], non_blocking=True)
            graph.replay()
            h_out[0].copy_(out, non_blocking=True)

        serial()
        torch.cuda.synchronize()
        el_serial = timed(serial, n)
        d_in = [content, torch.empty_like(content)]
        d_out = [out, torch.empty_like(out)]
        graphs = [graph, torch.cuda.CUDAGraph()]
        inputs2 = {'content': d_in[1], 'style_params': style}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            model(inputs2, out=d_out[1])
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(graphs[1]):
            model(inputs2, out=d_out[1])
        # uploads and downloads on one copy stream (two separate copy streams measured slower: 661 vs
        # 747 FPS); every buffer reuse waits on the event of its previous user
        comp = torch.cuda.current_stream()
        up = down = torch.cuda.Stream()
        up_done = [torch.cuda.Event(), torch.cuda.Event()]
        comp_done = [torch.cuda.Event(), torch.cuda.Event()]
        down_done = [torch.cuda.Event(), torch.cuda.Event()]

        def pipelined():
            # frame i in slot s = i & 1: upload(i), compute(i) on `comp`, download(i) (copy stream)
            torch.cuda.synchronize()
            with torch.cuda.stream(up):
                d_in[0].copy_(h_in[0], non_blocking=True)
                up_done[0].record(up)
            for i in range(n):
                s = i & 1
                comp.wait_event(up_done[s])
                if i >= 2:
                    comp.wait_event(down_done[s])        # d_out[s] read back (frame i-2)
                graphs[s].replay()
                comp_done[s].record(comp)
                if i + 1 < n:
                    with torch.cuda.stream(up):
                        if i >= 1:
                            up.wait_event(comp_done[s ^ 1])   # d_in[s^1] consumed (frame i-1)
                        d_in[s ^ 1].copy_(h_in[s ^ 1], non_blocking=True)
                        up_done[s ^ 1].record(up)
                with torch.cuda.stream(down):
                    down.wait_event(comp_done[s])
                    h_out[s].copy_(d_out[s], non_blocking=True)
                    down_done[s].record(down)
            comp.wait_stream(up)

        el_pipe = timed(pipelined, 1)
        frame_bytes = B * (int(np.prod(ins)) + int(np.prod(outs))) * 4
        pcie = {"serial_fps": round(world * B * n / el_serial, 3),
                "pipelined_fps": round(world * B * n / el_pipe, 3),
                "frames": n, "bytes_per_frame_h2d_d2h": frame_bytes // B,
                "note": "pinned host frames; serial = H2D + graph + D2H per frame on one stream; pipelined = "
                        "double-buffered, copies on a second stream overlapping the compute"}
        torch.cuda.synchronize()
    # ---------------- timed region 2: eager launches with per-layer HIP events -----------------
    # (every kernel recorded between events on the forward's stream -> per-kernel durations for
    # the roofline; also the eager FPS)
    model.profile_begin(args.steps)
    elapsed_eager = timed(lambda: model(inputs, out=out), args.steps)
    conv_ms, layer_ms, nsteps = model.profile_end()
    if graph is None:
        elapsed = elapsed_eager
    frames = world * B * args.steps
    fps = frames / elapsed
    fps_eager = frames / elapsed_eager
    ms_per_step = elapsed * 1e3 / args.steps

    # ---------------- dominant kernel roofline (from the timed region's events) ----------------
    flops = [layer_flops(l) * B for l in plan.layers]
    dom = dominant_kernel(model, plan, conv_ms, nsteps, B)
    dom_id, avg_ms, flops_per_launch, achieved_tf = dom["id"], dom["avg_ms"], dom["flops_per_launch"], dom["tflops"]
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get("per_launch_bytes", {}).get(KERNEL_NAMES.get(dom_id, ""), None)
        except Exception:
            traffic = None
    total_flops = sum(flops) / B
    conv_ms_per_frame = sum(conv_ms) / max(nsteps, 1) / B
    layer_table = [{"layer": l.name, "kernel": KERNEL_NAMES.get(model.layer_kernel_id(i), "?"),
                    "ms": round(conv_ms[i] / max(nsteps, 1), 4),
                    "tflops": round(flops[i] / (conv_ms[i] / max(nsteps, 1) * 1e-3) / 1e12, 2) if conv_ms[i] > 0 else None}
                   for i, l in enumerate(plan.layers)]

    # ---------------- config 3: batch-8 stream, hipGraph steady state -------------------------
    stream_fps = None
    if args.stream_batch > 0:
        SB = args.stream_batch
        rng2 = np.random.default_rng(2000 + rank)
        c8 = torch.from_numpy(rng2.random((SB,) + ins, dtype=np.float32)).to(dev)
        s8 = torch.from_numpy(synthetic_style_params(SB, 1, P, plan, seed=1)).to(dev)
        o8 = torch.empty((SB,) + outs, dtype=torch.float32, device=dev)
        in8 = {'content': c8, 'style_params': s8}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                model(in8, out=o8)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            model(in8, out=o8)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        reps = 20
        if world > 1:
            dist.barrier()
        ts = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        te = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([te], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            te = float(t.item())
        stream_fps = world * SB * reps / te

    # ---------------- precision mode: split-bf16 residual convs (reported beside the fp32 headline) --
    split_models, split = {}, {}
    if not args.no_bf16x3:
        for prec in [p for p in ("fp32", "fp32_winograd", "bf16x6", "bf16x3", "bf16") if p != args.precision]:
            split_models[prec], split[prec] = bench_split(args, world, dev, cfg, ins, outs, plan, weights, P, inputs,
                                                          timed, prec)

    # ---------------- style predictor / inference model -----------------------
    predictor = None
    if not args.no_predictor:
        predictor = bench_predictor(args, dev, cfg, model, inputs, P, timed)

    ingest = None if args.no_ingest else bench_ingest(args, dev, cfg, timed, rank)

    # ---------------- config 4: training step (fwd + VGG loss + bwd + [RCCL all-reduce] + RMSprop) --
    train = None
    if args.train_batch > 0:
        # BASELINE config 4 trains in bf16: the headline training figure runs the VGG16 3x3 convs with bf16
        # operands and fp32 accumulation; the split-bf16 (bf16x3, bf16x6) and fp32 runs are reported beside it
        train = bench_training(args, world, rank, dev, cfg, ins, outs, plan, weights, P, timed, "bf16")
        train["other_precisions"] = {p: {k: v for k, v in bench_training(args, world, rank, dev, cfg, ins, outs, plan,
                                                                          weights, P, timed, p).items()
                                         if k in ("ms_per_step", "frames_per_s", "achieved_tflops_per_gpu", "dtype")}
                                     for p in ("bf16x3", "bf16x6", "fp32")}

    # ---------------- parity + CPU baseline (rank 0 only, bounded sample) -----------------------
    max_abs = None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.torch_ref import TorchTransfer
        threads = cpu_threads()
        torch.set_num_threads(threads)
        ref = TorchTransfer(weights, ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
        x0 = content[:1].cpu().numpy()
        ts = time.perf_counter()
        y_ref = ref(x0, sp_np[:1])
        first = time.perf_counter() - ts
        y_gpu = model({'content': content[:1].contiguous(), 'style_params': style[:1].contiguous()})
        torch.cuda.synchronize()
        max_abs = float(np.abs(y_gpu.cpu().numpy() - y_ref).max())
        for prec, m3 in split_models.items():
            y3 = m3({'content': content[:1].contiguous(), 'style_params': style[:1].contiguous()})
            torch.cuda.synchronize()
            split[prec]["max_abs_delta_vs_oracle"] = float(np.abs(y3.cpu().numpy() - y_ref).max())
        n, tsum = 0, 0.0
        while tsum < args.cpu_budget_s and n < 20:
            ts = time.perf_counter()
            ref(x0, sp_np[:1])
            tsum += time.perf_counter() - ts
            n += 1
            if first > args.cpu_budget_s:
                break
        cpu = {"value": round(n / tsum, 4), "unit": "frames/s", "cores": threads, "kind": "port",
               "sample": f"{n} frames of 480x960x17 (B=1) after 1 warm-up frame; torch-CPU f32 restatement of the "
                         f"same graph (oracle/torch_ref.py; TF-CPU not installed), {n} x {tsum / n:.3f} s"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(fps, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "precision_mode": args.precision,
            "arithmetic": DTYPE_DESC.get(args.precision, args.precision),
            "data": "synthetic (U[0,1) 480x960x17 G-buffer frames, seeded weights; no checkpoints offline)",
            "config": {"workload": f"{SPEC} single-frame transfer inference (BASELINE config 2)", "spec": SPEC,
                       "frames_per_step_per_gpu": B, "input": list(ins), "output": list(outs),
                       "parallelism": f"frame-sharded x{world}, no data-path collective"},
            "fps_per_gpu": round(fps / world, 3),
            "timing": "hipGraph replay per step" if graph is not None else "eager launches",
            "eager_fps": round(fps_eager, 3),
            "pcie_inclusive": pcie,
            "max_abs_delta_vs_oracle": max_abs,
            "roofline": {
                "bound": "mfma",
                "kernel": KERNEL_NAMES.get(dom_id, str(dom_id)),
                "achieved": round(achieved_tf, 3),
                "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s" if dom_id != 200 else "TFLOP/s (algorithmic = direct-conv FLOPs)",
                "frac": round(achieved_tf / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "avg_launch_ms": round(avg_ms, 5),
                "flops_per_launch": flops_per_launch,
                "launches": dom["launches"],
                # Winograd executes 16/36 of the direct multiplies on the MFMA pipe
                "mfma_pipe_frac": round(achieved_tf * (16.0 / 36.0 if dom_id == 200 else 1.0) / FP32_MFMA_PEAK_TFLOPS, 4),
            },
            "network_roofline": {
                "gflop_per_frame": round(total_flops / 1e9, 3),
                "conv_kernel_ms_per_frame": round(conv_ms_per_frame, 4),
                "achieved_tflops_conv_kernels": round(total_flops / (conv_ms_per_frame * 1e-3) / 1e12, 3),
                "achieved_tflops_end_to_end": round(total_flops * fps / world / 1e12, 3),
                "frac_end_to_end": round(total_flops * fps / world / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
            },
            "stream_graph_fps": None if stream_fps is None else round(stream_fps, 3),
            "stream_graph_batch": args.stream_batch,
            "layers": layer_table,
            "split_bf16_modes": split,
            "training": train,
            "style_predictor": predictor,
            "gbuffer_ingest": ingest,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
