"""Host-side enqueue cost of the config-4 training step's pieces (no device sync inside the timed calls): how long the
host takes to queue the style predictor's forward (~150 launches), the loss targets (~40) and a whole train_step,
against a trivial torch launch. Usage: python tools/host_launch_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from realtime_style_transfer_amd.plan import init_weights, network_plan  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402
from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG  # noqa: E402
from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer  # noqa: E402
from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel  # noqa: E402

cfg = ShapeConfig.from_spec("rst-960-120-128-17")
ins, outs = cfg.input_shape['content'], cfg.output_shape
plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
TB = 4
dev = torch.device('cuda')
lm = StyleLossModelVGG(outs, max_batch=TB, device=dev, precision='bf16')
sins = tuple(cfg.input_shape['style'][1:])
pr = StylePredictionTrainer(sins, cfg.style_feature_extractor_type, plan.num_style_params, max_batch=TB, device=dev)
tr = StyleTransferTrainingModel(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, loss_model=lm,
                                weights=init_weights(plan, seed=2), max_batch=TB, device=dev, style_predictor=pr,
                                precision='winograd_bf16x6')
rng = np.random.default_rng(1)
x = {'content': torch.from_numpy(rng.random((TB,) + ins, dtype=np.float32)).to(dev),
     'style': torch.from_numpy(rng.random((TB, 1) + sins, dtype=np.float32)).to(dev)}
y = {'content': torch.from_numpy(rng.random((TB,) + outs, dtype=np.float32)).to(dev),
     'style': torch.from_numpy(rng.random((TB, 1) + outs, dtype=np.float32)).to(dev)}
for _ in range(3):
    tr.train_step(x, y)
torch.cuda.synchronize()


def host_ms(fn, n=5):
    best = 1e9
    for _ in range(n):
        torch.cuda.synchronize()
        big = torch.empty(1 << 26, device=dev)
        for _ in range(20):        # keep the device busy so the queue never drains while the host enqueues
            big.mul_(1.0001)
        t0 = time.perf_counter()
        fn()
        best = min(best, (time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    return best


t = torch.zeros(16, device=dev)
print(f"torch add_ x100: {host_ms(lambda: [t.add_(1) for _ in range(100)]) * 10:.2f} us per launch")
style = x['style'][:, 0]
print(f"predictor forward: {host_ms(lambda: pr.forward(style)):.3f} ms host")


def targets():
    tr.compute_targets(y['content'], y['style'])
    tr.cancel_targets()


print(f"loss targets: {host_ms(targets):.3f} ms host")
print(f"train_step: {host_ms(lambda: tr.train_step(x, y), 3):.3f} ms host")
