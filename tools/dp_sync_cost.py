"""Per-step cost of the data-parallel exchange, two ranks sharing cuda:0 over gloo (the one-GPU rehearsal of
config 5's training side): the bench's config-4 step (rst-960-120-128-17, joint MobileNetV3Small predictor,
bf16 VGG16, winograd_bf16x6 transfer) at B=2 per rank, timed three ways:

  none     the step with the exchange skipped (local gradients; the floor)
  round2   the round-2 exchange: gradient all-reduce, then a second all-reduce of the BN moving statistics
           gathered from a full weight copy and written back through rst_trainer_set_weights (re-pack of
           every conv image + x6 transforms) and the predictor's set_weights
  one      this round's exchange: ONE all-reduce of [gradients | moving statistics], statistics scattered
           back with rst_*trainer_set_moving_statistics (no re-pack)

Usage (GPU box): python tools/dp_sync_cost.py [--steps 10] -> one JSON line per rank-0 run."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, steps, batch, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import realtime_style_transfer_amd.styleTransferTrainingModel as stm
        from realtime_style_transfer_amd import _lib
        from realtime_style_transfer_amd.plan import init_weights, network_plan
        from realtime_style_transfer_amd.shape_config import ShapeConfig
        from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG
        from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer
        cfg = ShapeConfig.from_spec("rst-960-120-128-17")
        ins, outs = cfg.input_shape['content'], cfg.output_shape
        plan = network_plan(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters)
        sins = tuple(cfg.input_shape['style'][1:])
        pr = StylePredictionTrainer(sins, 'MOBILE_NET', plan.num_style_params, max_batch=batch)
        lm = StyleLossModelVGG(outs, max_batch=batch, precision="bf16")
        tr = stm.StyleTransferTrainingModel(ins, outs, cfg.bottleneck_res_y, cfg.bottleneck_num_filters,
                                            loss_model=lm, weights=init_weights(plan, seed=2), max_batch=batch,
                                            precision="winograd_bf16x6", style_predictor=pr)
        rng = np.random.default_rng(100 + rank)
        x = {'content': torch.from_numpy(rng.random((batch,) + ins, dtype=np.float32)).cuda(),
             'style': torch.from_numpy(rng.random((batch, 1) + sins, dtype=np.float32)).cuda()}
        y = {'content': torch.from_numpy(rng.random((batch,) + outs, dtype=np.float32)).cuda(),
             'style': torch.from_numpy(rng.random((batch, 1) + outs, dtype=np.float32)).cuda()}
        lib = _lib.load()

        def round2_exchange():
            stm._all_reduce_sum(tr._grad_bucket)
            w = torch.empty(tr.num_weights, dtype=torch.float32, device='cuda')
            _lib.check(lib.rst_trainer_copy_weights(tr._handle, _lib.dev_ptr(w), w.numel(), _lib.stream_ptr()))
            pw = pr.weights_tensor()
            stats = torch.cat([w[tr._bn_index], pw[pr.moving_statistics_index]])
            stm._all_reduce_sum(stats)
            stats /= world
            n0 = tr._bn_index.numel()
            w[tr._bn_index] = stats[:n0]
            _lib.check(lib.rst_trainer_set_weights(tr._handle, _lib.dev_ptr(w), w.numel(), _lib.stream_ptr()))
            pw[pr.moving_statistics_index] = stats[n0:]
            pr.set_weights_tensor(pw)
            return True

        modes = {"none": lambda: False, "round2": round2_exchange, "one": tr.exchange}
        res = {}
        for name, fn in modes.items():
            tr.exchange = fn
            for _ in range(2):
                tr.train_step(x, y)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                tr.train_step(x, y)
            torch.cuda.synchronize()
            el = torch.tensor([time.perf_counter() - t0])
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            res[name] = round(float(el) * 1e3 / steps, 3)
        if rank == 0:
            with open(out, "w") as f:
                json.dump({"ranks": world, "batch_per_rank": batch, "backend": "gloo (two ranks share cuda:0)",
                           "ms_per_step": res, "exchange_ms": {k: round(v - res["none"], 3) for k, v in res.items()},
                           "bucket_values": int(tr._bucket.numel()),
                           "moving_statistics": int(tr._n_stat + tr._n_pstat)}, f)
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/dp_sync_cost.json")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    from realtime_style_transfer_amd.frames import free_port
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    mp.spawn(worker, args=(2, free_port(), a.steps, a.batch, a.out), nprocs=2, join=True)
    print(open(a.out).read())


if __name__ == "__main__":
    main()
