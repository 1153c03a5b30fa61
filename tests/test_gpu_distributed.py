"""Multi-rank paths on the GPU box's single MI355X: ranks share cuda:0 over a gloo process group (RCCL
needs one GPU per rank; the driver's 8-GPU run exercises RCCL itself).

* data-parallel training (BASELINE config 5's training side): after steps with a different
  frame batch on each rank, every rank holds bitwise identical weights — gradients all-reduced (SUM)
  and the BatchNorm moving statistics averaged — and the averaged moving mean equals the mean of the
  per-rank updates (TF MirroredStrategy's MEAN aggregation);
* `bench.py --gpus 2` end to end (real kernels) prints one line with n_gpus 2.
* RCCL itself with one rank (`test_rccl_step_exchange_one_rank`): the step exchange's all-reduce on the
  "nccl" backend leaves bucket and weights bitwise unchanged; a 6 MB SUM of a known pattern is exact.
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
        import realtime_style_transfer_amd.styleTransferTrainingModel as stm
        calls, local = [], []
        real = stm._all_reduce_sum

        def spy(t, group=None):            # the step's collectives, and this rank's statistics before the SUM
            calls.append(t.numel())
            local.append(t[tr._grad_bucket.numel():].clone())
            real(t, group)

        stm._all_reduce_sum = spy
        for _ in range(2):
            tr.train_step(x, y)
        stm._all_reduce_sum = real
        torch.cuda.synchronize()
        n0 = tr._grad_bucket.numel()
        np.save(os.path.join(tmp, f"calls{rank}.npy"), np.array(calls + [tr._bucket.numel(), n0]))
        np.save(os.path.join(tmp, f"local{rank}.npy"), local[-1].cpu().numpy())
        tr._get_moving_statistics()         # the synced statistics, read back from the weights
        torch.cuda.synchronize()
        np.save(os.path.join(tmp, f"synced{rank}.npy"), tr._bucket[n0:].cpu().numpy())
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
    # one collective per step, over the whole bucket [gradients | moving statistics]
    c0 = np.load(tmp_path / "calls0.npy")
    assert c0[:-2].tolist() == [c0[-2]] * 2 and c0[-2] > c0[-1]
    # the synced moving statistics are the MEAN of the ranks' own updates (not a sum, not rank 0's)
    l0, l1 = np.load(tmp_path / "local0.npy"), np.load(tmp_path / "local1.npy")
    s0, s1 = np.load(tmp_path / "synced0.npy"), np.load(tmp_path / "synced1.npy")
    assert np.array_equal(s0, s1)
    mean = (l0 + l1) / np.float32(2)
    assert np.array_equal(s0, mean)
    assert not np.array_equal(s0, l0) and not np.array_equal(s0, l1)
    # and the transfer net's part sits at the BN moving-statistic slots of the weights
    assert np.array_equal(w0[bn], s0[:bn.size])


def test_bench_two_ranks_on_one_gpu():
    """bench.py's multi-rank path with the real kernels: two ranks on cuda:0 over gloo."""
    _need_gpu()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "5", "--warmup", "2", "--stream-batch", "0", "--no-bf16x3", "--no-predictor", "--no-two-styles",
                        "--no-ingest", "--train-batch", "2", "--train-steps", "2", "--train-modes", "bf16",
                        "--pcie-steps", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["max_abs_delta_vs_oracle"] < 2e-4
    assert line["cpu_baseline"] is None             # rank 0 at N=1 only
    tr = line["training"]                           # config 5's training side: both ranks, one all-reduce per step
    assert tr["batch_per_gpu"] == 2 and tr["ms_per_step"] > 0 and np.isfinite(tr["last_loss_mean"])
    assert tr["frames_per_s"] > 0 and "one all-reduce per step" in tr["workload"]


def _rccl_worker(rank, world, port, tmp):
    import time
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        import realtime_style_transfer_amd.styleTransferTrainingModel as stm
        from realtime_style_transfer_amd.plan import init_weights, network_plan
        from realtime_style_transfer_amd.styleLoss import StyleLossModelVGG, init_vgg16_weights
        ins, outs, br, bf = (32, 64, 17), (32, 64, 3), 8, 8
        plan = network_plan(ins, outs, br, bf)
        lm = StyleLossModelVGG(outs, weights=init_vgg16_weights(seed=3), max_batch=2)
        tr = stm.StyleTransferTrainingModel(ins, outs, br, bf, loss_model=lm, weights=init_weights(plan, seed=2),
                                            max_batch=2)
        rng = np.random.default_rng(7)
        x = {'content': torch.from_numpy(rng.random((2,) + ins, dtype=np.float32)).cuda(),
             'style_params': torch.from_numpy(rng.random((2, plan.num_style_params), dtype=np.float32)).cuda()}
        y = {'content': torch.from_numpy(rng.random((2,) + outs, dtype=np.float32)).cuda(),
             'style': torch.from_numpy(rng.random((2, 1) + outs, dtype=np.float32)).cuda()}
        tr.train_step(x, y)
        torch.cuda.synchronize()
        w_before = np.concatenate([a.reshape(-1) for a in tr.get_weights()])
        # the step exchange's collective, run on RCCL in HBM: [gradients | moving statistics] SUM over one rank,
        # the statistics divided by the world size and written back into the weights
        tr._get_moving_statistics()
        before = tr._bucket.clone()
        stm._all_reduce_sum(tr._bucket, tr.process_group)
        tr._set_moving_statistics(dist.get_world_size())
        torch.cuda.synchronize()
        w_after = np.concatenate([a.reshape(-1) for a in tr.get_weights()])
        # a full-size bucket (rst-960-120-128-17's ~5.9 MB gradient): SUM of a known pattern, timed
        big = torch.arange(1_500_000, dtype=torch.float32, device="cuda") * 0.5
        ref = big.clone()
        for _ in range(3):
            dist.all_reduce(big, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            dist.all_reduce(big, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        np.save(os.path.join(tmp, "rccl.npy"), np.array([
            float(torch.equal(before, tr._bucket)), float(np.array_equal(w_before, w_after)),
            float(torch.equal(big, ref)), ms]))
        with open(os.path.join(tmp, "backend.txt"), "w") as f:
            f.write(dist.get_backend())
    finally:
        dist.destroy_process_group()


def test_rccl_step_exchange_one_rank(tmp_path):
    """BASELINE config 5's collective on RCCL (backend "nccl" on ROCm) — the one GPU of this box holds one rank, so
    the SUM is an identity: the step exchange's bucket and the weights it writes back come out bitwise unchanged,
    and a 6 MB all-reduce of a known pattern is exact. The 8-GPU curve is the driver's run."""
    _need_gpu()
    import torch.multiprocessing as mp
    from realtime_style_transfer_amd.frames import free_port
    mp.spawn(_rccl_worker, args=(1, free_port(), str(tmp_path)), nprocs=1, join=True)
    assert (tmp_path / "backend.txt").read_text() == "nccl"
    same_bucket, same_w, exact, ms = np.load(tmp_path / "rccl.npy")
    assert same_bucket == 1.0 and same_w == 1.0 and exact == 1.0
    print(f"RCCL all-reduce of 6 MB, one rank: {ms:.3f} ms")
