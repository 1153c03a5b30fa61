"""Capture one full training step (bench.py's config-4 step: style predictor + transfer net + VGG16 loss,
backward of both, RMSprop) into a hipGraph and check that a replay does exactly what an eager step does:
two trainers with the same initial state, one eager step vs one graph replay -> bitwise-equal weights and
losses. Prints eager vs replay ms/step.  Usage: python tools/train_graph_check.py [batch] [steps] [--small]
(--small: a 32x64 frame, seconds). The step's stream overlaps (loss targets, the predictor's backward and its weight
gradients) follow their RST_SERIAL_* switches at creation."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_style_transfer_amd.plan import init_weights, network_plan  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402
from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG  # noqa: E402
from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer  # noqa: E402
from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel  # noqa: E402


def make(cfg, plan, B, dev):
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    sins = tuple(cfg.input_shape['style'][1:])
    lm = StyleLossModelVGG(outs, max_batch=B, device=dev, precision="bf16")
    pr = StylePredictionTrainer(sins, cfg.style_feature_extractor_type, plan.num_style_params, max_batch=B, device=dev)
    return StyleTransferTrainingModel(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, loss_model=lm,
                                      weights=init_weights(plan, seed=2), max_batch=B, device=dev, style_predictor=pr)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if len(args) > 0 else 4
    steps = int(args[1]) if len(args) > 1 else 5
    if "--small" in sys.argv:   # 32x64 frames, 8-row bottleneck of 32 filters: a seconds-long check
        cfg = ShapeConfig.explicit((32, 64), (32, 64), num_channels=17, bottleneck_res_y=8, bottleneck_num_filters=32)
    else:
        cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    sins = tuple(cfg.input_shape['style'][1:])
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(3000)
    x = {'content': torch.from_numpy(rng.random((B,) + ins, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((B, 1) + sins, dtype=np.float32)).to(dev)}
    y = {'content': torch.from_numpy(rng.random((B,) + outs, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((B, 1) + outs, dtype=np.float32)).to(dev)}
    a, b = make(cfg, plan, B, dev), make(cfg, plan, B, dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            a.train_step(x, y)
            b.train_step(x, y)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.train_step(x, y)
    a.train_step(x, y)
    g.replay()
    torch.cuda.synchronize()
    wa = np.concatenate([w.ravel() for w in a.get_weights()] + [w.ravel() for w in a.style_predictor.get_weights()])
    wb = np.concatenate([w.ravel() for w in b.get_weights()] + [w.ravel() for w in b.style_predictor.get_weights()])
    la, lb = a.compute_metrics()['loss'], b.compute_metrics()['loss']
    same_w = bool(np.array_equal(wa, wb))
    same_l = bool(torch.equal(torch.as_tensor(la), torch.as_tensor(lb)))
    print(f"weights bitwise equal: {same_w}  loss equal: {same_l}  ({float(la):.6g} vs {float(lb):.6g})")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        a.train_step(x, y)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager {1e3 * (t1 - t0) / steps:.3f} ms/step, graph replay {1e3 * (t2 - t1) / steps:.3f} ms/step (B={B})")
    return 0 if same_w and same_l else 1


if __name__ == "__main__":
    sys.exit(main())
