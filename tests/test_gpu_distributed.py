"""Multi-rank paths on the GPU box's single MI355X: ranks share cuda:0 over a gloo process group (RCCL
needs one GPU per rank; the driver's 8-GPU run exercises RCCL itself).

* data-parallel training (BASELINE config 5's training side): after steps with a different
  frame batch on each rank, every rank holds bitwise identical weights — gradients all-reduced (SUM)
  and the BatchNorm moving statistics averaged — and the averaged moving mean equals the mean of the
  per-rank updates (TF MirroredStrategy's MEAN aggregation);
* `bench.py --gpus 2` end to end (real kernels) prints one line with n_gpus 2.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _dp_worker(rank, world, port, tmp):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from realtime_style_transfer_amd.plan import init_weights, network_plan
        from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG, init_vgg16_weights
        from realtime_style_transfer_amd.stylePrediction import StylePredictionTrainer
        from realtime_style_transfer_amd.styleTransferTrainingModel import StyleTransferTrainingModel
        ins, outs, br, bf = (32, 64, 17), (32, 64, 3), 8, 8
        plan = network_plan(ins, outs, br, bf)
        lm = StyleLossModelVGG(outs, weights=init_vgg16_weights(seed=3), max_batch=2)
        pr = StylePredictionTrainer((32, 64, 3), 'MOBILE_NET', plan.num_style_params, max_batch=2)
        tr = StyleTransferTrainingModel(ins, outs, br, bf, loss_model=lm, weights=init_weights(plan, seed=2),
                                        max_batch=2, style_predictor=pr)
        rng = np.random.default_rng(100 + rank)          # a different batch on every rank
        x = {'content': torch.from_numpy(rng.random((2,) + ins, dtype=np.float32)).cuda(),
             'style': torch.from_numpy(rng.random((2, 1, 32, 64, 3), dtype=np.float32)).cuda()}
        y = {'content': torch.from_numpy(rng.random((2,) + outs, dtype=np.float32)).cuda(),
             'style': torch.from_numpy(rng.random((2, 1) + outs, dtype=np.float32)).cuda()}
        for _ in range(2):
            tr.train_step(x, y)
        torch.cuda.synchronize()
        w = np.concatenate([a.reshape(-1) for a in tr.get_weights()])
        pw = np.concatenate([a.reshape(-1) for a in pr.get_weights()])
        np.save(os.path.join(tmp, f"w{rank}.npy"), w)
        np.save(os.path.join(tmp, f"pw{rank}.npy"), pw)
        np.save(os.path.join(tmp, f"bn{rank}.npy"), tr._bn_index.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_data_parallel_training_keeps_ranks_identical(tmp_path):
    _need_gpu()
    import torch.multiprocessing as mp
    from realtime_style_transfer_amd.frames import free_port
    mp.spawn(_dp_worker, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    w0, w1 = np.load(tmp_path / "w0.npy"), np.load(tmp_path / "w1.npy")
    p0, p1 = np.load(tmp_path / "pw0.npy"), np.load(tmp_path / "pw1.npy")
    assert np.array_equal(w0, w1), "transfer weights (incl. BN moving statistics) differ across ranks"
    assert np.array_equal(p0, p1), "predictor weights (incl. BN moving statistics) differ across ranks"
    bn = np.load(tmp_path / "bn0.npy")
    assert bn.size > 0 and np.all(np.isfinite(w0[bn]))


def test_bench_two_ranks_on_one_gpu():
    """bench.py's multi-rank path with the real kernels: two ranks on cuda:0 over gloo."""
    _need_gpu()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "5", "--warmup", "2", "--stream-batch", "0", "--no-bf16x3", "--no-predictor",
                        "--no-ingest", "--train-batch", "0", "--pcie-steps", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["max_abs_delta_vs_oracle"] < 2e-4
    assert line["cpu_baseline"] is None             # rank 0 at N=1 only
