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
    202: "wino_x6_conv<F(2x2,3x3) 8x16 N128 split-bf16 x6 MFMA>",
    204: "last_x6<9x9 transposed Cin16 Cout3 as N=(kx,co) split-bf16 x6 MFMA>",
    301: "conv_lite<3x3 s2 Cin32 Cout16 f32 16x16x4 MFMA>", 302: "conv_lite<3x3 s2 Cin16 Cout32 f32 32x32x2 MFMA>",
    303: "conv_lite<3x3 s2 transposed Cin128 Cout32 f32 32x32x2 MFMA>",
    304: "conv_lite<3x3 s2 transposed Cin32 Cout16 f32 16x16x4 MFMA>",
    305: "conv_lite<3x3 s2 transposed Cin128 Cout32 split-bf16 x6 32x32x16 MFMA>",
    306: "conv_lite<3x3 s2 Cin32 Cout16 split-bf16 x6 16x16x32 MFMA>",
    307: "conv_lite<3x3 s2 Cin16 Cout32 split-bf16 x6 32x32x16 MFMA>",
    308: "conv_lite<3x3 s2 transposed Cin32 Cout16 split-bf16 x6 16x16x32 MFMA>",
    203: "wino9_x6_conv<9x9 as 9 x F(2x2,3x3) 16x16 N32 split-bf16 x6 MFMA persistent>",
    205: "wino9f3<9x9 as 9 x F(3x3,3x3) on one tile grid, 24x24 N32 split-bf16 x6 MFMA persistent>",
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
    "winograd_bf16x6": "fp32-level: the residual convs as fused Winograd F(2x2,3x3) and the 9x9 start conv as nine 3x3 "
                       "sub-kernels on one F(3x3,3x3) tile grid, whose transform-domain products are exact 3-piece "
                       "split-bf16 MFMA terms (each "
                       "fp32 operand = 3 bf16 pieces holding all 24 significant bits, 6 product terms, dropped "
                       "terms <= 2^-25 of each product, fp32 accumulate); the final 9x9 transposed conv as a GEMM "
                       "over (kx, co) columns and the narrow stride-2 (transposed) convs with the same exact "
                       "split-bf16 products",
}


def executed_mfma(model, plan, i: int, B: int):
    """(FLOPs the kernel of layer i actually issues on its pipe for B images, peak TFLOP/s of that pipe).

    Direct implicit-GEMM convs issue the algorithmic 2*MAC. Winograd F(2x2,3x3) issues 16 products per
    2x2 output tile and (cin, cout) pair instead of 36 (tiles counted over the padded 8x16-pixel workgroup
    blocks); the composite 9x9 start conv issues 16 x 9 sub-kernels x 18 channels (17 + one zero) per tile
    and output channel. The split-bf16 kernels issue `terms` bf16 products per fp32 product on the bf16
    pipe. The VALU 9x9 Cout=3 kernel issues the algorithmic FMAs on the f32 vector pipe (same peak)."""
    kid = model.layer_kernel_id(i)
    l = plan.layers[i]
    Ho, Wo = l.out_hw
    tiles = B * (-(-Ho // 8) * 4) * (-(-Wo // 16) * 8)
    if kid == 200:
        return 2.0 * tiles * 16 * l.cin * l.cout, FP32_MFMA_PEAK_TFLOPS
    if kid == 201:
        return 2.0 * tiles * 16 * 9 * 18 * l.cout, FP32_MFMA_PEAK_TFLOPS
    if kid == 202:
        return 6 * 2.0 * tiles * 16 * l.cin * l.cout, BF16_MFMA_PEAK_TFLOPS
    if kid == 203:   # 9 sub-kernels x 16 channels + the gathered channel-16 K-step (16 wide), 6 terms
        return 6 * 2.0 * tiles * 16 * (9 * 16 + 16) * l.cout, BF16_MFMA_PEAK_TFLOPS
    if kid == 205:   # 24x24 blocks of 64 F(3x3) tiles, 25 points: points 0..23 on 32x32x16 K-steps (5 per 8-channel chunk,
        # one for channel 16), point 24 on 16x16x32 K-steps (3 per chunk, one for channel 16); 6 terms, padded K issued
        blocks = B * (-(-Ho // 24)) * (-(-Wo // 24))
        ks = 5 + (5 if l.cin > 8 else 0) + (1 if l.cin > 16 else 0)
        k24 = 3 + (3 if l.cin > 8 else 0) + (1 if l.cin > 16 else 0)
        return 6 * 2.0 * blocks * 64 * l.cout * (24 * 16 * ks + 32 * k24), BF16_MFMA_PEAK_TFLOPS
    if kid == 204:   # per output row and 88-column strip: 3 x' tiles of 32, N = 32 columns (27 used), K = 9 x 16
        return 6 * 2.0 * B * Ho * (-(-Wo // 88)) * 3 * 32 * 32 * 144, BF16_MFMA_PEAK_TFLOPS
    if kid in (305, 308):   # 9 (phase, tap) slots x Cin x Cout per input pixel, 6 bf16 terms, tiles of 4 x Cout
        tiles = B * (-(-l.in_hw[0] // 4)) * (-(-l.in_hw[1] // l.cout)) * 4 * l.cout
        return 6 * 2.0 * tiles * 9 * l.cin * l.cout, BF16_MFMA_PEAK_TFLOPS
    if kid in (306, 307):   # strided: 9 taps x Cin x Cout per output pixel, 6 bf16 terms, tiles of 4 x Cout
        tiles = B * (-(-Ho // 4)) * (-(-Wo // l.cout)) * 4 * l.cout
        return 6 * 2.0 * tiles * 9 * l.cin * l.cout, BF16_MFMA_PEAK_TFLOPS
    if 101 <= kid < 200:
        terms = {"bf16x3": 3, "bf16x6": 6, "bf16": 1}.get(model.precision, 6)
        return terms * layer_flops(l) * B, BF16_MFMA_PEAK_TFLOPS
    return layer_flops(l) * B, FP32_MFMA_PEAK_TFLOPS


def dominant_kernel(model, plan, conv_ms, nsteps, B) -> dict:
    """The kernel (config id) with the largest summed time over the timed launches: its executed-work
    rate (executed_mfma FLOPs per launch / average launch duration, against the peak of the pipe it
    issues on) and, separately, the algorithmic (direct-conv) rate."""
    groups = {}
    for i, l in enumerate(plan.layers):
        kid = model.layer_kernel_id(i)
        ex, peak = executed_mfma(model, plan, i, B)
        g = groups.setdefault(kid, {"ms": 0.0, "flops": 0.0, "exec": 0.0, "launches": 0, "peak": peak})
        g["ms"] += conv_ms[i]
        g["flops"] += layer_flops(l) * B * nsteps
        g["exec"] += ex * nsteps
        g["launches"] += nsteps
    kid = max(groups, key=lambda k: groups[k]["ms"])
    g = groups[kid]
    avg_ms = g["ms"] / max(g["launches"], 1)
    fpl = g["flops"] / max(g["launches"], 1)
    epl = g["exec"] / max(g["launches"], 1)
    sec = avg_ms * 1e-3
    return {"id": kid, "kernel": KERNEL_NAMES.get(kid, str(kid)), "avg_ms": avg_ms, "flops_per_launch": fpl,
            "exec_flops_per_launch": epl, "launches": g["launches"], "peak": g["peak"],
            "tflops": fpl / sec / 1e12 if avg_ms > 0 else 0.0, "exec_tflops": epl / sec / 1e12 if avg_ms > 0 else 0.0}


def graph_layer_ms(model, inputs, out, n_replays: int):
    """Per-layer share of a back-to-back hipGraph replay of the frame (the configuration the headline times): the
    frame captured with in-kernel end stamps (rst_timeline_*; the residual convs and the narrow convs stamp every
    wave's end with the 100-MHz realtime counter), replayed n_replays times, each replay read back; layer k's share
    is end(k) - end(k - 1), which is what rocprofv3's kernel trace reports as the duration of a kernel inside a graph
    replay (its start is the predecessor's completion). -> [L] ms (NaN where layer k or k - 1 does not stamp)."""
    model.timeline_begin()
    try:
        g = capture_graph(lambda: model(inputs, out=out))
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        rows = []
        for _ in range(n_replays):
            g.replay()
            rows.append(model.timeline_read())
        del g
        torch.cuda.synchronize()
    finally:
        model.timeline_end()
    E = np.array(rows)
    d = np.full(E.shape[1], np.nan)
    d[1:] = np.mean(E[:, 1:] - E[:, :-1], axis=0) * 1e-3
    return d


def dominant_kernel_graph(model, plan, graph_ms, B, kid: int):
    """dominant_kernel's record for kernel `kid` from the in-graph per-layer shares (graph_layer_ms)."""
    ms, ex, fl, n, peak = 0.0, 0.0, 0.0, 0, BF16_MFMA_PEAK_TFLOPS
    for i, l in enumerate(plan.layers):
        if model.layer_kernel_id(i) != kid:
            continue
        if not np.isfinite(graph_ms[i]):
            return None
        e, peak = executed_mfma(model, plan, i, B)
        ms += graph_ms[i]
        ex += e
        fl += layer_flops(l) * B
        n += 1
    if n == 0:
        return None
    avg, sec = ms / n, ms / n * 1e-3
    return {"id": kid, "kernel": KERNEL_NAMES.get(kid, str(kid)), "avg_ms": avg, "flops_per_launch": fl / n,
            "exec_flops_per_launch": ex / n, "launches": n, "peak": peak, "tflops": fl / n / sec / 1e12,
            "exec_tflops": ex / n / sec / 1e12}


def roofline_of(dom: dict, traffic=None) -> dict:
    """BASELINE roofline object of the dominant kernel: `achieved` = executed FLOPs per launch / average
    launch duration (HIP events on the forward's stream in the timed region), `frac` = achieved / peak of the
    pipe those FLOPs issue on; the direct-conv-equivalent rate is reported beside it, never as `frac`."""
    peak = dom["peak"]
    return {"bound": "mfma", "kernel": dom["kernel"], "achieved": round(dom["exec_tflops"], 3), "peak": peak,
            "unit": "TFLOP/s", "frac": round(dom["exec_tflops"] / peak, 4), "traffic": traffic,
            "avg_launch_ms": round(dom["avg_ms"], 5), "exec_flops_per_launch": dom["exec_flops_per_launch"],
            "launches": dom["launches"],
            "pipe": "bf16 MFMA" if peak == BF16_MFMA_PEAK_TFLOPS else "f32 MFMA",
            "direct_equivalent": {"flops_per_launch": dom["flops_per_launch"],
                                  "tflops": round(dom["tflops"], 3),
                                  "note": "algorithmic direct-conv FLOPs / launch time; > peak is possible for "
                                          "Winograd (it issues fewer products), so this is not a roofline fraction"}}


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


def capture_graph(fn):
    """Capture fn (one forward on torch's current stream) into a hipGraph after a warm-up launch on a side
    stream (torch.cuda.graphs' recipe)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def bench_split(args, ctx, cfg, ins, outs, plan, weights, P, inputs, precision):
    """The same B=1 hipGraph frame loop with another precision mode (reported beside the headline)."""
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    B = args.batch
    model, _ = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=weights, max_batch=B, device=ctx.device, precision=precision,
                                           allow_reduced_precision=precision == "bf16")
    out = torch.empty((B,) + outs, dtype=torch.float32, device=ctx.device)
    g = capture_graph(lambda: model(inputs, out=out))
    for _ in range(args.warmup):
        g.replay()
    torch.cuda.synchronize()
    el = ctx.timed(g.replay, args.steps)
    model.profile_begin(args.steps)
    ctx.timed(lambda: model(inputs, out=out), args.steps)
    conv_ms, _, nsteps = model.profile_end()
    dom = dominant_kernel(model, plan, conv_ms, nsteps, B)
    return model, {
        "value": round(ctx.world * B * args.steps / el, 3), "unit": "frames/s",
        "ms_per_step": round(el * 1e3 / args.steps, 4), "dtype": DTYPE_DESC.get(precision, precision),
        "roofline": roofline_of(dom),
        "layers_ms": [round(c / max(nsteps, 1), 4) for c in conv_ms],
    }


def bench_two_styles(args, ctx, cfg, ins, outs, plan, weights, precision):
    """num_styles = 2 (README dual-style use; styleTransfer.py:36-44,288-303): the same B=1 hipGraph frame loop
    with a per-pixel style-weight map (the AvgPool2 mip chain and the per-pixel blend of the two CIN affines in
    the consumer prologues). Reported beside the headline."""
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    B = args.batch
    plan2 = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 2)
    model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 2,
                                           weights=weights, max_batch=B, device=ctx.device, precision=precision)
    rng = np.random.default_rng(5000 + ctx.rank)
    inputs = {'content': torch.from_numpy(rng.random((B,) + ins, dtype=np.float32)).to(ctx.device),
              'style_params': torch.from_numpy(synthetic_style_params(B, 2, P, plan2, seed=7)).to(ctx.device),
              'style_weights': torch.from_numpy(rng.random((B,) + outs[:2] + (1,), dtype=np.float32)).to(ctx.device)}
    out = torch.empty((B,) + outs, dtype=torch.float32, device=ctx.device)
    g = capture_graph(lambda: model(inputs, out=out))
    for _ in range(args.warmup):
        g.replay()
    torch.cuda.synchronize()
    el = ctx.timed(g.replay, args.steps)
    kinds = sorted({KERNEL_NAMES.get(model.layer_kernel_id(i), "?") for i in range(len(plan2.layers))})
    return {"workload": f"{SPEC} with num_styles=2: per-pixel blend of two styles' CIN parameters (style_weights "
                        f"(B,480,960,1), AvgPool2 mips), B={B}, hipGraph replay", "value": round(ctx.world * B * args.steps / el, 3),
            "unit": "frames/s", "ms_per_step": round(el * 1e3 / args.steps, 4), "precision_mode": precision,
            "kernels": kinds}


def train_executed_work(plan, H, W, vgg_precision: str, transfer_precision: str) -> dict:
    """Per-sample FLOPs the training step issues, split by the pipe they issue on (bf16 / f32 MFMA), for the
    mixed roofline: ideal time = bf16 FLOPs / bf16 peak + f32 FLOPs / f32 peak. Transfer net: forward (the
    residual and start convs on Winograd in fp32_winograd mode), weight gradient of every conv (direct GEMM),
    input gradient of every conv but the first (residual ones on Winograd). VGG16: forward of three images
    and the prediction's input gradient; the 3x3 convs after the first on bf16 with `terms` products per fp32
    product (bf16: 1, bf16x3: 3, bf16x6: 6), the 3-channel first conv and fp32 mode on f32. Gram: forward of
    two images and one backward on f32 MFMA."""
    wino = transfer_precision in ("fp32_winograd", "winograd_bf16x6")
    x6 = transfer_precision == "winograd_bf16x6"   # residual convs: 6 bf16 terms per product, on the bf16 pipe

    def conv_exec(i, l):
        Ho, Wo = l.out_hw
        tiles = (-(-Ho // 8) * 4) * (-(-Wo // 16) * 8)
        if wino and i == 0 and l.k == 9:
            return 2.0 * tiles * 16 * 9 * 18 * l.cout
        if wino and l.block.startswith('residual'):
            return 2.0 * tiles * 16 * l.cin * l.cout
        return layer_flops(l)
    t_f32, t_bf16 = 0.0, 0.0
    for i, l in enumerate(plan.layers):
        if x6 and i == 0 and l.k == 9:   # start conv forward on wino9_x6 (16x16 blocks, K = 9 x 16 + 16 per point)
            Ho, Wo = l.out_hw
            tiles = (-(-Ho // 16) * 8) * (-(-Wo // 16) * 8)
            t_bf16 += 6 * 2.0 * tiles * 16 * (9 * 16 + 16) * l.cout
            t_f32 += layer_flops(l)   # weight gradient (direct GEMM, f32)
            continue
        work = conv_exec(i, l) + layer_flops(l) + (conv_exec(i, l) if i > 0 else 0.0)   # fwd + wgrad + dgrad
        if x6 and l.block.startswith('residual'):
            t_bf16 += 6 * work
        else:
            t_f32 += work
    terms = {"bf16": 1, "bf16x3": 3, "bf16x6": 6}.get(vgg_precision, 0)
    chans = [64, 64, 128, 128, 256, 256, 256, 512, 512, 512, 512, 512, 512]
    pools = {1, 3, 6, 9}
    vgg_f32, vgg_bf16, gram, cin, h, w = 0.0, 0.0, 0.0, 3, H, W
    for i, c in enumerate(chans):
        f = 2.0 * h * w * 9 * cin * c * 4                    # three forwards + one input gradient
        if i == 0 or terms == 0:
            vgg_f32 += f
        else:
            vgg_bf16 += terms * f
        if i in pools:
            if terms == 1:   # plain bf16: the Gram forwards and the Gram backward (1x1) on the bf16 pipe
                vgg_bf16 += 3 * 2.0 * h * w * c * c
            else:
                gram += 3 * 2.0 * h * w * c * c
            h, w = h // 2, w // 2
        cin = c
    return {"transfer_f32": t_f32, "transfer_bf16": t_bf16, "vgg_f32": vgg_f32, "vgg_bf16": vgg_bf16, "gram_f32": gram}


def bench_training(args, ctx, cfg, ins, outs, plan, weights, P, precision="fp32", transfer="winograd_bf16x6"):
    from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
    from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
    dev = ctx.device
    TB = args.train_batch
    lm = StyleLossModelVGG(outs, max_batch=TB, device=dev, precision=precision)
    from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer
    sins = tuple(cfg.input_shape['style'][1:])
    # train_network.py fits the MobileNetV3Small style predictor jointly (stylePrediction.py:25-75)
    pr = StylePredictionTrainer(sins, cfg.style_feature_extractor_type, P, max_batch=TB, device=dev)
    tr = StyleTransferTrainingModel(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, loss_model=lm,
                                    weights=weights, max_batch=TB, device=dev, style_predictor=pr, precision=transfer)
    rng = np.random.default_rng(3000 + ctx.rank)
    x = {'content': torch.from_numpy(rng.random((TB,) + ins, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((TB, 1) + sins, dtype=np.float32)).to(dev)}
    y = {'content': torch.from_numpy(rng.random((TB,) + outs, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((TB, 1) + outs, dtype=np.float32)).to(dev)}
    for _ in range(args.train_warmup):   # untimed: allocations, first-use kernel attributes, clocks settle
        tr.train_step(x, y)
    torch.cuda.synchronize()
    el = ctx.timed(lambda: tr.train_step(x, y), args.train_steps)
    loss = float(tr.compute_metrics()['loss'])
    fl = train_flops_per_sample(plan, outs[0], outs[1])
    per_sample = sum(fl.values())
    ms = el * 1e3 / args.train_steps
    tfs = per_sample * TB / (ms * 1e-3) / 1e12
    ex = train_executed_work(plan, outs[0], outs[1], precision, tr.precision)
    ideal_ms = TB * ((ex["vgg_bf16"] + ex["transfer_bf16"]) / (BF16_MFMA_PEAK_TFLOPS * 1e12) +
                     (ex["transfer_f32"] + ex["vgg_f32"] + ex["gram_f32"]) / (FP32_MFMA_PEAK_TFLOPS * 1e12)) * 1e3
    return {"workload": f"{SPEC} train_network.py step (BASELINE config 4): MobileNetV3Small style predictor + "
                        f"transfer net, training-mode forward, VGG16/Gram loss (no depth term), backward of both, " +
                        ("one all-reduce per step (SUM, one bucket: gradients + BN moving statistics, the latter then / world), "
                         if ctx.world > 1 else "") + "RMSprop on both", "batch_per_gpu": TB, "steps": args.train_steps, "warmup": args.train_warmup,
            "ms_per_step": round(ms, 3),
            "frames_per_s": round(ctx.world * TB * args.train_steps / el, 3),
            "dtype": {"fp32": "fp32 (f32 MFMA)",
                      "bf16x6": "VGG16 3x3 convs: exact 3-piece split bf16 MFMA (fp32-level products, fp32 accumulate); "
                                "transfer net and the rest fp32-level (see transfer_precision)",
                      "bf16x3": "VGG16 3x3 convs: 2-piece split bf16 MFMA (16-bit operands, fp32 accumulate); "
                                "transfer net and the rest fp32-level (see transfer_precision)",
                      "bf16": "VGG16 3x3 convs and the Gram forwards/backward: bf16 operands, fp32 accumulate "
                              "(mixed_bfloat16 arithmetic); transfer net and the rest fp32-level (see "
                              "transfer_precision)"}[precision],
            "transfer_precision": {"fp32": "exact f32 MFMA",
                                   "fp32_winograd": "residual 3x3 convs (forward + input gradient) and the 9x9 start "
                                                    "conv (forward) as Winograd F(2x2,3x3) on f32 MFMA, the other "
                                                    "transfer convs exact f32",
                                   "winograd_bf16x6": "residual 3x3 convs (forward, input gradient, weight gradient) and "
                                                      "the 9x9 start conv's forward (nine 3x3 Winograd sub-kernels) on "
                                                      "exact 3-piece split-bf16 MFMA products (fp32-level), the other "
                                                      "transfer convs exact f32"}[tr.precision],
            "tflop_per_sample": round(per_sample / 1e12, 4),
            "algorithmic_tflops_per_gpu": round(tfs, 2),
            "roofline": {"bound": "mfma (mixed)", "ideal_ms": round(ideal_ms, 3), "achieved_ms": round(ms, 3),
                         "frac": round(ideal_ms / ms, 4),
                         "executed_gflop_per_sample": {k: round(v / 1e9, 2) for k, v in ex.items()},
                         "peaks_tflops": {"bf16": BF16_MFMA_PEAK_TFLOPS, "f32": FP32_MFMA_PEAK_TFLOPS},
                         "note": "ideal = bf16 FLOPs / bf16 peak + f32 FLOPs / f32 peak (executed work: Winograd "
                                 "and split-bf16 counted as issued); the style predictor (~1 GFLOP/sample, VALU) "
                                 "is left out of the ideal"},
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


def bench_ingest(args, ctx, cfg):
    """G-buffer ingest: a 1080x1920 Unreal screenshot's 17 channel planes (already in
    HBM, as after the per-channel EXR uploads) -> rst_gbuffer_preprocess -> the 480x960x17 content tensor
    (hdrScreenshots.py:14-30 + common.py:44-57 in one pass). HBM-bound: algorithmic bytes = the source
    rows x columns the bilinear taps touch + the output."""
    from realtime_style_transfer_amd.dataloaders.common import preprocess_planes, resized_size
    src, C = (1080, 1920), cfg.num_channels
    shape = cfg.input_shape['content'][:2]
    dev = ctx.device
    planes = [torch.rand(src, device=dev) for _ in range(C)]
    out = torch.empty(shape + (C,), device=dev)
    fn = lambda: preprocess_planes(planes, shape, out=out)   # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    steps = max(args.steps, 50)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    ctx.timed(fn, steps)
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
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
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


def bench_predictor(args, ctx, cfg, transfer_model, transfer_inputs, P):
    """make_style_transfer_inference_model path: the MobileNetV3Small style predictor on a 480x960x3 style image
    (once per style in the video loop, predict_video_using_checkpoint.py:77-83) and predictor + transfer per
    frame (the Keras inference model runs both per call, styleTransferInferenceModel.py:23-37)."""
    from realtime_style_transfer_amd.stylePrediction import create_style_prediction_model
    dev = ctx.device
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
    el_p = ctx.timed(gp.replay, args.steps)
    gi = graph_of(lambda: (pred(style, out=sp), transfer_model(tin, out=out)))
    el_i = ctx.timed(gi.replay, args.steps)
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


DEFAULT_PRECISION = "winograd_bf16x6"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); >1 without WORLD_SIZE launches them")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed graph replays (seconds of wall time) before the headline's warmup steps: the "
                         "GPU clock ramps out of the idle setup; reported as settle_s")
    ap.add_argument("--batch", type=int, default=1, help="frames per step per GPU (config 2: 1)")
    ap.add_argument("--stream-batch", type=int, default=8, help="config 3 (hipGraph stream) batch; 0 to skip")
    ap.add_argument("--stream-frames", type=int, default=500, help="config 3 timed frames (after 50 warm-up)")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0, help="bounded CPU-baseline sample (seconds)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="headline from eager launches instead of hipGraph replay")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06", "traffic_r06.json"),
                    help="per-launch HBM bytes of the dominant kernel (tools/pmc_traffic.py on this build's FETCH/WRITE passes)")
    ap.add_argument("--train-batch", type=int, default=4, help="config 4 training step batch per GPU; 0 to skip")
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--train-warmup", type=int, default=5)
    ap.add_argument("--train-modes", default="bf16,bf16x3,bf16x6,fp32",
                    help="VGG16 precisions of the training line, comma-separated; the first is the headline")
    ap.add_argument("--precision", default=DEFAULT_PRECISION,
                    help="headline transfer precision mode (default winograd_bf16x6: fp32-level Winograd F(2x2,3x3) "
                         "with exact split-bf16 MFMA products); also fp32, fp32_winograd, bf16x6, bf16x3 and bf16 "
                         "(bf16 is not fp32-level)")
    ap.add_argument("--no-bf16x3", action="store_true", help="skip the other precision-mode measurements")
    ap.add_argument("--no-predictor", action="store_true", help="skip the style-predictor measurement")
    ap.add_argument("--no-two-styles", action="store_true", help="skip the num_styles=2 frame loop")
    ap.add_argument("--no-ingest", action="store_true", help="skip the G-buffer ingest measurement")
    ap.add_argument("--pcie-steps", type=int, default=50, help="host-resident frame loop (PCIe-inclusive); 0 to skip")
    ap.add_argument("--dist-backend", default=None, choices=[None, "nccl", "gloo"],
                    help="process-group backend for N>1 (default RCCL; gloo lets ranks share one GPU)")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="CPU only: launch the ranks, shard, time and report with no device work (tests the "
                         "multi-rank path; prints value null)")
    return ap.parse_args(argv)


def plumbing_check(args, ctx):
    """The multi-rank path of main() with the per-step device work removed: rank setup, the frame stream
    sharded over ranks (frames.shard_batches), the barrier-bracketed timed region with the MAX over ranks,
    the SUM of frames processed, and rank 0's JSON line. Used by the CPU gloo test."""
    from realtime_style_transfer_amd.frames import shard_batches, sum_over_ranks
    B = args.batch
    n_frames = ctx.world * B * args.steps
    mine = shard_batches(n_frames, B, ctx.rank, ctx.world)
    it, done = iter(mine), [0]

    def step():                     # "process" the next owned batch: count its frames
        done[0] += len(next(it))

    el = ctx.timed(step, args.steps)
    total = sum_over_ranks(float(done[0]))
    if ctx.rank == 0:
        print(json.dumps({"metric": "plumbing-check (no device work)", "value": None, "unit": "frames/s",
                          "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
                          "frames_processed": int(total), "frames_expected": n_frames, "elapsed_max_s": el,
                          "backend": ctx.backend, "scaling": "weak"}), flush=True)


def main(argv=None):
    args = parse_args(argv)
    from realtime_style_transfer_amd.frames import init_ranks, launch_ranks
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # driver contract: `python bench.py --gpus N` runs N ranks. Start them as children before anything
        # touches the GPU (this process never initialises HIP and is not replaced).
        return launch_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:] if argv is None else list(argv))
    ctx = init_ranks(args.dist_backend, "cpu" if args.plumbing_check else "cuda")
    if ctx.world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ctx.world}")
    try:
        if args.plumbing_check:
            plumbing_check(args, ctx)
        else:
            run(args, ctx)
    finally:
        ctx.close()
    return 0


def run(args, ctx):
    from realtime_style_transfer_amd.frames import shard_batches
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    rank, world, dev = ctx.rank, ctx.world, ctx.device
    cfg = ShapeConfig.from_spec(SPEC)
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    weights = init_weights(plan, seed=2)
    B = args.batch
    max_b = max(B, args.stream_batch)
    model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                           weights=weights, max_batch=max_b, device=dev, precision=args.precision)
    # The synthetic stream has world * B * steps frames; rank r owns the batches r, r + world, ...
    # (frames.shard_batches). Frame i's content is drawn from a generator seeded with i, so every rank's
    # frames differ; the first owned batch is resident in HBM before the timed region starts.
    first = shard_batches(world * B * args.steps, B, rank, world)[0]
    content = torch.from_numpy(np.concatenate([np.random.default_rng(1000 + i).random((1,) + ins, dtype=np.float32)
                                               for i in first])).to(dev)
    sp_np = synthetic_style_params(B, 1, P, plan, seed=1)
    style = torch.from_numpy(sp_np).to(dev)
    out = torch.empty((B,) + outs, dtype=torch.float32, device=dev)
    inputs = {'content': content, 'style_params': style}
    rng = np.random.default_rng(1000 + rank)

    for _ in range(args.warmup):
        model(inputs, out=out)
    torch.cuda.synchronize()

    # ---------------- timed region 1 (headline): one hipGraph replay per step -------------------
    # The forward (~30 kernel launches) is captured once into a hipGraph on torch's stream —
    # how a real-time frame loop drives it; the per-frame host cost is one graph launch.
    graph = None
    settle_s = 0.0
    if not args.eager:
        graph = capture_graph(lambda: model(inputs, out=out))
        # clock settle: untimed replays for a fixed wall time before the W warmup steps, so a short driver
        # run (--steps 20 --warmup 5, ~17 ms) does not time the GPU's clock ramp out of the idle setup
        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < args.settle_s:
            for _ in range(50):
                graph.replay()
            torch.cuda.synchronize()
        settle_s = time.perf_counter() - t_settle
        for _ in range(args.warmup):
            graph.replay()
        torch.cuda.synchronize()
        elapsed = ctx.timed(graph.replay, args.steps)
    # ---------------- config 4: training step (fwd + VGG loss + bwd + [RCCL all-reduce] + RMSprop) --
    # measured right after the headline's timed region, before any side leg: the PCIe leg's copy stream alone cost the
    # step 0.75 ms when it ran first (20.5 vs 19.7 ms, profiles/r06/r06as; GPU_MAX_HW_QUEUES = 4 hardware queues carry
    # every stream of the process), and the later side legs another 0.7 ms (profiles/r06/r06ar)
    train = None
    if args.train_batch > 0:
        # BASELINE config 4 trains in bf16: the headline training figure runs the VGG16 3x3 convs with bf16
        # operands and fp32 accumulation; the split-bf16 (bf16x3, bf16x6) and fp32 runs are reported beside it
        modes = [m for m in args.train_modes.split(",") if m]
        train = bench_training(args, ctx, cfg, ins, outs, plan, weights, P, modes[0])
        keep = ("ms_per_step", "frames_per_s", "algorithmic_tflops_per_gpu", "dtype", "roofline")
        train["other_precisions"] = {p: {k: v for k, v in bench_training(args, ctx, cfg, ins, outs, plan, weights, P,
                                                                          p).items() if k in keep}
                                     for p in modes[1:]}

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
        el_serial = ctx.timed(serial, n)
        d_in = [content, torch.empty_like(content)]
        d_out = [out, torch.empty_like(out)]
        inputs2 = {'content': d_in[1], 'style_params': style}
        graphs = [graph, capture_graph(lambda: model(inputs2, out=d_out[1]))]
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

        el_pipe = ctx.timed(pipelined, 1)
        frame_bytes = B * (int(np.prod(ins)) + int(np.prod(outs))) * 4
        pcie = {"serial_fps": round(world * B * n / el_serial, 3),
                "pipelined_fps": round(world * B * n / el_pipe, 3),
                "frames": n, "bytes_per_frame_h2d_d2h": frame_bytes // B,
                "note": "pinned host frames; serial = H2D + graph + D2H per frame on one stream; pipelined = "
                        "double-buffered, copies on a second stream overlapping the compute"}
        torch.cuda.synchronize()
        content.copy_(d_in[0])
    # ---------------- timed region 2: eager launches with per-layer HIP events -----------------
    # (every kernel recorded between events on the forward's stream -> per-kernel durations for
    # the roofline; also the eager FPS)
    model.profile_begin(args.steps)
    elapsed_eager = ctx.timed(lambda: model(inputs, out=out), args.steps)
    conv_ms, layer_ms, nsteps = model.profile_end()
    if graph is None:
        elapsed = elapsed_eager
    frames = world * B * args.steps
    fps = frames / elapsed
    fps_eager = frames / elapsed_eager
    ms_per_step = elapsed * 1e3 / args.steps

    # ---------------- dominant kernel roofline ------------------------------------------------------------
    # The kernel with the most eager time (HIP events above); its average launch duration from the in-graph timeline
    # of the same frame graph the headline replays (graph_layer_ms): back to back, the residual convs run ~4 % longer
    # than eager launches, and rocprofv3's kernel trace of a graph replay is what profiles/ holds
    flops = [layer_flops(l) * B for l in plan.layers]
    dom_eager = dominant_kernel(model, plan, conv_ms, nsteps, B)
    graph_ms = None
    dom = dom_eager
    if graph is not None:
        graph_ms = graph_layer_ms(model, inputs, out, max(20, min(args.steps, 100)))
        dg = dominant_kernel_graph(model, plan, graph_ms, B, dom_eager["id"])
        if dg is not None:
            dom = dg
    traffic, traffic_note = None, None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get("per_launch_bytes", {}).get(dom["kernel"], None)
            traffic_note = tj.get("correction")
        except Exception:
            traffic = None
    total_flops = sum(flops) / B
    conv_ms_per_frame = sum(conv_ms) / max(nsteps, 1) / B
    layer_table = []
    for i, l in enumerate(plan.layers):
        ms_i = conv_ms[i] / max(nsteps, 1)
        ex, peak = executed_mfma(model, plan, i, B)
        layer_table.append({"layer": l.name, "kernel": KERNEL_NAMES.get(model.layer_kernel_id(i), "?"),
                            "ms": round(ms_i, 4),
                            "graph_ms": (round(float(graph_ms[i]), 4) if graph_ms is not None and
                                         np.isfinite(graph_ms[i]) else None),
                            "tflops_direct_equiv": round(flops[i] / (ms_i * 1e-3) / 1e12, 2) if ms_i > 0 else None,
                            "exec_frac": round(ex / (ms_i * 1e-3) / 1e12 / peak, 4) if ms_i > 0 else None})

    # ---------------- config 3: batch-8 stream, hipGraph steady state (50 warm-up + 500 frames) ----------
    stream = None
    if args.stream_batch > 0:
        SB = args.stream_batch
        c8 = torch.from_numpy(np.random.default_rng(2000 + rank).random((SB,) + ins, dtype=np.float32)).to(dev)
        s8 = torch.from_numpy(synthetic_style_params(SB, 1, P, plan, seed=1)).to(dev)
        o8 = torch.empty((SB,) + outs, dtype=torch.float32, device=dev)
        in8 = {'content': c8, 'style_params': s8}
        g = capture_graph(lambda: model(in8, out=o8))
        for _ in range(-(-50 // SB)):
            g.replay()
        torch.cuda.synchronize()
        reps = -(-args.stream_frames // SB)
        te = ctx.timed(g.replay, reps)
        stream = {"fps": round(world * SB * reps / te, 3), "batch": SB, "frames_per_gpu": SB * reps,
                  "warmup_frames": SB * -(-50 // SB), "ms_per_batch": round(te * 1e3 / reps, 4),
                  "workload": "predict_video_using_checkpoint.py stream (BASELINE config 3): batch-8 480x960x17 "
                              "frames, one hipGraph replay per batch"}

    # ---------------- other precision modes (reported beside the headline) ---------------------
    split_models, split = {}, {}
    if not args.no_bf16x3:
        for prec in [p for p in ("fp32", "fp32_winograd", "winograd_bf16x6", "bf16x6", "bf16x3", "bf16")
                     if p != args.precision]:
            split_models[prec], split[prec] = bench_split(args, ctx, cfg, ins, outs, plan, weights, P, inputs, prec)

    two_styles = None if args.no_two_styles else bench_two_styles(args, ctx, cfg, ins, outs, plan, weights,
                                                                   args.precision)

    # ---------------- style predictor / inference model -----------------------
    predictor = None if args.no_predictor else bench_predictor(args, ctx, cfg, model, inputs, P)
    ingest = None if args.no_ingest else bench_ingest(args, ctx, cfg)

    # ---------------- parity + CPU baseline (rank 0 at N=1 only, bounded sample) ----------------
    max_abs = None
    cpu = None
    if rank == 0:
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
        if world == 1 and not args.no_cpu_baseline:
            n, tsum = 0, 0.0
            while tsum < args.cpu_budget_s and n < 200:
                ts = time.perf_counter()
                ref(x0, sp_np[:1])
                tsum += time.perf_counter() - ts
                n += 1
                if first > args.cpu_budget_s:
                    break
            cpu = {"value": round(n / tsum, 4), "unit": "frames/s", "cores": threads, "kind": "port",
                   "sample": f"{n} frames of 480x960x17 (B=1) after 1 warm-up frame; torch-CPU f32 restatement of "
                             f"the same graph (oracle/torch_ref.py; TF-CPU not installed), {n} x {tsum / n:.3f} s"}

    # config-4 CPU baseline: the same training step (transfer training-mode forward, VGG16/Gram loss, backward,
    # RMSprop) as torch-CPU autograd in fp32 at B=1 on the host cores, reported only
    if rank == 0 and world == 1 and not args.no_cpu_baseline and train is not None:
        from oracle import torch_train as TT
        from realtime_style_transfer_amd.styleLoss import init_vgg16_weights
        threads = cpu_threads()
        torch.set_num_threads(threads)
        vgg_w = init_vgg16_weights(seed=3)
        crng = np.random.default_rng(4000)
        c1 = crng.random((1,) + ins, dtype=np.float32)
        gc1, gs1 = crng.random((1,) + outs, dtype=np.float32), crng.random((1, 1) + outs, dtype=np.float32)
        n, tsum = 0, 0.0
        while n < 3 and (n == 0 or tsum < args.cpu_budget_s / 2):
            ts = time.perf_counter()
            TT.training_step(weights, vgg_w, c1, sp_np[:1], gc1, gs1, ins, outs, cfg.bottleneck_res_y,
                             cfg.bottleneck_num_filters, dtype=torch.float32)
            tsum += time.perf_counter() - ts
            n += 1
        train["cpu_baseline"] = {
            "value": round(n / tsum, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "ms_per_step_b1": round(tsum / n * 1e3, 1),
            "sample": f"{n} training steps at B=1 (480x960x17 -> 480x960x3, style params as input; no style predictor), "
                      f"torch-CPU fp32 autograd restatement of the transfer net + VGG16/Gram loss + RMSprop "
                      f"(oracle/torch_train.py; TF-CPU not installed), {n} x {tsum / n:.2f} s"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(fps, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_s": round(settle_s, 3),
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
                       "parallelism": f"frame-sharded x{world}, no data-path collective"
                                      + (f" ({ctx.backend} bookkeeping)" if world > 1 else "")},
            "fps_per_gpu": round(fps / world, 3),
            "timing": "hipGraph replay per step" if graph is not None else "eager launches",
            "eager_fps": round(fps_eager, 3),
            "pcie_inclusive": pcie,
            "max_abs_delta_vs_oracle": max_abs,
            "roofline": dict(roofline_of(dom, traffic),
                             timing=("in-graph: per-launch share of the headline's hipGraph frame replay from in-kernel "
                                     "end stamps (bench.graph_layer_ms), %d replays" % max(20, min(args.steps, 100))
                                     if dom is not dom_eager else "eager launches, hipExtLaunchKernel events"),
                             eager_avg_launch_ms=round(dom_eager["avg_ms"], 5),
                             traffic_note=traffic_note),
            "network_roofline": {
                "gflop_per_frame": round(total_flops / 1e9, 3),
                "conv_kernel_ms_per_frame": round(conv_ms_per_frame, 4),
                "direct_equiv_tflops_conv_kernels": round(total_flops / (conv_ms_per_frame * 1e-3) / 1e12, 3),
                "direct_equiv_tflops_end_to_end": round(total_flops * fps / world / 1e12, 3),
            },
            "stream_graph": stream,
            "layers": layer_table,
            "split_bf16_modes": split,
            "two_styles": two_styles,
            "training": train,
            "style_predictor": predictor,
            "gbuffer_ingest": ingest,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    sys.exit(main())
