"""Co-residency check of the inference path (diagnostic): two full-size transfer networks (480x960x17, the
headline precision) run on two streams at once, N times; every output must be bitwise the one each network gives alone.
Usage: python tools/concurrent_infer_check.py [N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import bench
    from realtime_style_transfer_amd.plan import init_weights, network_plan, synthetic_style_params
    from realtime_style_transfer_amd.shape_config import ShapeConfig
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    cfg = ShapeConfig.from_spec("rst-960-120-128-17")
    ins, outs = cfg.input_shape['content'], cfg.output_shape
    plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
    nets = []
    for k in range(2):
        ws = init_weights(plan, seed=3 + k)
        model, P = create_style_transfer_model(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters, 1,
                                               weights=ws, max_batch=1, precision=bench.DEFAULT_PRECISION)
        rng = np.random.default_rng(100 + k)
        x = torch.from_numpy(rng.random((1,) + ins, dtype=np.float32)).cuda()
        sp = torch.from_numpy(synthetic_style_params(1, 1, P, plan, seed=7 + k)).cuda()
        out = torch.empty((1,) + outs, device='cuda')
        nets.append((model, {'content': x, 'style_params': sp}, out))
    refs = []
    for model, inp, out in nets:   # alone
        model(inp, out=out)
        torch.cuda.synchronize()
        refs.append(out.clone())
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bad = 0
    for i in range(n):
        for (model, inp, out), s in zip(nets, streams):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                model(inp, out=out)
        torch.cuda.synchronize()
        diffs = [int((out != ref).sum()) for (_, _, out), ref in zip(nets, refs)]
        if any(diffs):
            bad += 1
        print(f"round {i}: values differing from the lone run {diffs}", flush=True)
    print(f"{bad} of {n} concurrent rounds differ", flush=True)


if __name__ == "__main__":
    main()
