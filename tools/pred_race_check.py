"""Repeatability of the training forward's prediction with the loss targets beside it (diagnostic).
The config-4 480x960 trainer (winograd_bf16x6 transfer convs, VGG16 in plain bf16 or fp32) runs compute_gradients
N times on the same inputs; every prediction must be bitwise the first one (the targets run on the trainer's side
stream beside the forward). Prints the max |difference| per call and the differing pixel count.
Usage: python tools/pred_race_check.py [bf16|fp32] [N] [B] [save.npy]   (save.npy: call 0's prediction, for comparing
runs under different environments, e.g. RST_LDS_POISON)"""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("tgt", os.path.join(ROOT, "tests", "test_gpu_train.py"))
tgt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tgt)


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    sc = ShapeConfig.from_spec("rst-960-120-128-17")
    cfg = dict(input_shape=sc.input_shape['content'], output_shape=sc.output_shape,
               bottleneck_res_y=sc.bottleneck_res_y, bottleneck_num_filters=sc.bottleneck_num_filters)
    plan, w, vgg, content, sp, gtc, gts = tgt._case(cfg, B, seed=9)
    tr = tgt._trainer(cfg, w, vgg, B, prec, "winograd_bf16x6")
    c, s, gc, gs = tgt._cuda(content, sp, gtc, gts)
    first = None
    first_loss = None
    for i in range(n):
        pred, losses, grad, gsp = tr.compute_gradients(c, s, gc, gs)
        torch.cuda.synchronize()
        p = pred.cpu().numpy()
        lo = losses.cpu().numpy()
        if first_loss is None:
            first_loss = lo
        elif not np.array_equal(lo, first_loss):
            print(f"call {i}: losses differ from call 0 ({lo.ravel()} vs {first_loss.ravel()})", flush=True)
        if first is None:
            first = p
            if len(sys.argv) > 4:
                np.save(sys.argv[4], p)
            print(f"call 0: prediction range [{p.min():.4f}, {p.max():.4f}]", flush=True)
            continue
        d = np.abs(p - first)
        bad = np.argwhere(d.reshape(B, -1, 3).max(-1) > 0)
        print(f"call {i}: max |diff| {d.max():.3e}, pixels differing {len(bad)}"
              + (f", first at {np.unravel_index(bad[0][1], (cfg['output_shape'][0], cfg['output_shape'][1]))}"
                 if len(bad) else ""), flush=True)


if __name__ == "__main__":
    main()
