"""Run a few rst-960-120-128-17 forwards (B=1) for counter collection (rocprofv3 --pmc).
Usage: python tools/wino_probe.py [precision] [steps]"""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402
from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32_winograd"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cfg = ShapeConfig.from_spec("rst-960-120-128-17")
ins, outs = cfg.input_shape['content'], cfg.output_shape
plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
m, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                   weights=init_weights(plan, seed=2), max_batch=1, precision=prec)
x = torch.from_numpy(np.random.default_rng(0).random((1,) + ins, dtype=np.float32)).cuda()
sp = torch.from_numpy(synthetic_style_params(1, 1, P, plan, seed=1)).cuda()
for _ in range(steps):
    m({'content': x, 'style_params': sp})
torch.cuda.synchronize()
print("done", prec, steps)
