"""The per-wave timeline of the frame's last residual conv (wino_x6, X6_PROF stamps) in hipGraph replay, as the bench
runs the frame. Usage: RST_LIB=tools/prof_librst.so python tools/frame_timeline.py [replays]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402
from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
cfg = ShapeConfig.from_spec("rst-960-120-128-17")
ins, outs = cfg.input_shape['content'], cfg.output_shape
plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
m, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                   weights=init_weights(plan, seed=2), max_batch=1, precision="winograd_bf16x6")
x = torch.from_numpy(np.random.default_rng(0).random((1,) + ins, dtype=np.float32)).cuda()
sp = torch.from_numpy(synthetic_style_params(1, 1, P, plan, seed=1)).cuda()
out = torch.empty((1,) + tuple(outs), device='cuda')
inputs = {'content': x, 'style_params': sp}
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    m(inputs, out=out)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    m(inputs, out=out)
for _ in range(n):
    g.replay()
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["RST_LIB"])
print(f"frame's last wino_x6 launch (of the profiled prologue form) after {n} graph replays:", flush=True)
lib.rst_debug_x6_timeline(225, 8)
