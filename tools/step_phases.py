"""Phases of bench.py's config-4 training step on the device clock, unprofiled: timing events on the caller's stream
between the step's host calls (StyleTransferTrainingModel.train_step's body, unrolled here), averaged over steps.
  head  = loss targets started + the style predictor's forward (the style parameters ready on the caller's stream)
  main  = compute_gradients (transfer net forward, VGG16 loss, transfer backward to its start conv)
  tail  = the predictor's backward joined + both RMSprop updates
Also the host time spent issuing each phase (perf_counter around the calls; the device may lag or lead).
Usage: python tools/step_phases.py [steps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from train_graph_check import make  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_style_transfer_amd.plan import network_plan  # noqa: E402
from realtime_style_transfer_amd.shape_config import ShapeConfig  # noqa: E402


def step(tr, x, y, ev, host):
    pr = tr.style_predictor
    t0 = time.perf_counter()
    ev[0].record()
    tr.compute_targets(y['content'], y['style'])
    sp = pr.forward(x['style'][:, 0])
    ev[1].record()
    t1 = time.perf_counter()
    pred, losses, grad, gsp = tr.compute_gradients(x['content'], sp, y['content'], y['style'])
    ev[2].record()
    t2 = time.perf_counter()
    tr._predictor_backward(pr, gsp)
    tr.exchange()
    tr.apply_gradients(grad)
    o = tr.optimizer
    pr.apply_gradients(tr._pgrad, o.learning_rate, o.rho, o.epsilon)
    ev[3].record()
    t3 = time.perf_counter()
    host += np.array([t1 - t0, t2 - t1, t3 - t2]) * 1e3


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    sins = tuple(cfg.input_shape['style'][1:])
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    dev = torch.device("cuda:0")
    B = 4
    rng = np.random.default_rng(3000)
    x = {'content': torch.from_numpy(rng.random((B,) + ins, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((B, 1) + sins, dtype=np.float32)).to(dev)}
    y = {'content': torch.from_numpy(rng.random((B,) + outs, dtype=np.float32)).to(dev),
         'style': torch.from_numpy(rng.random((B, 1) + outs, dtype=np.float32)).to(dev)}
    tr = make(cfg, plan, B, dev)
    for _ in range(3):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
    host = np.zeros(3)
    t0 = time.perf_counter()
    for i in range(steps):
        step(tr, x, y, evs[i], host)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    ph = np.array([[e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]), e[2].elapsed_time(e[3])] for e in evs])
    gaps = [evs[i][3].elapsed_time(evs[i + 1][0]) for i in range(steps - 1)]
    print(f"steps {steps} B={B}: wall {wall:.3f} ms/step")
    print("device ms  head %.3f  main %.3f  tail %.3f  (between steps %.3f)" % (*ph.mean(0), float(np.mean(gaps))))
    print("host ms    head %.3f  main %.3f  tail %.3f" % tuple(host / steps))
    return 0


if __name__ == "__main__":
    sys.exit(main())
