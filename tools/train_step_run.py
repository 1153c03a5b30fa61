"""Run a few full-size training steps (rst-960-120-128-17, B=4) — the command profiled by rocprofv3."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402
from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG  # noqa: E402
from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--spec", default="rst-960-120-128-17")
    ap.add_argument("--precision", default="bf16", help="VGG16 conv arithmetic (bench.py's training headline: bf16)")
    ap.add_argument("--transfer", default="fp32_winograd", help="transfer-network conv arithmetic (fp32 | fp32_winograd)")
    ap.add_argument("--losses", action="store_true", help="print the loss of every step (syncs per step)")
    a = ap.parse_args()
    cfg = ShapeConfig.from_spec(a.spec)
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    dev = torch.device("cuda:0")
    B = a.batch
    lm = StyleLossModelVGG(outs, max_batch=B, device=dev, precision=a.precision)
    tr = StyleTransferTrainingModel(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, loss_model=lm,
                                    weights=init_weights(plan, seed=2), max_batch=B, device=dev,
                                    precision=a.transfer)
    rng = np.random.default_rng(0)
    x = {'content': torch.from_numpy(rng.random((B,) + ins, dtype=np.float32)).to(dev),
         'style_params': torch.from_numpy(synthetic_style_params(B, 1, plan.num_style_params, plan)).to(dev)}
    y = {'content': torch.from_numpy(rng.random((B,) + outs, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((B, 1) + outs, dtype=np.float32)).to(dev)}
    m = tr.train_step(x, y)
    torch.cuda.synchronize()
    if a.losses:
        print(f"step 0: loss {float(m['loss']):.9g}")
    t0 = time.perf_counter()
    for i in range(a.steps):
        m = tr.train_step(x, y)
        if a.losses:
            print(f"step {i + 1}: loss {float(m['loss']):.9g}")
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{a.steps} steps B={B}: {el / a.steps * 1e3:.2f} ms/step, loss {float(m['loss']):.6g}")


if __name__ == "__main__":
    main()
