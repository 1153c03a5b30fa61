"""Compare two transfer-network training precisions on config A of tests/test_gpu_train.py: prediction,
VGG features of the prediction and every layer's output gradient (GPU vs GPU, no oracle)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_train as G  # noqa: E402

cfg = G.CONFIGS['A']
B = 2
plan, w, vgg, content, sp, gtc, gts = G._case(cfg, B)
res = {}
for mode in ("fp32", "fp32_winograd"):
    tr = G._trainer(cfg, w, vgg, B, "fp32", mode)
    c, s, gc, gs = G._cuda(content, sp, gtc, gts)
    pred, losses, grad, gsp = tr.compute_gradients(c, s, gc, gs)
    torch.cuda.synchronize()
    feats = {n: tr.vgg_feature(n, B).cpu().numpy() for n in ("block1_conv1", "block1_conv2", "block2_conv2",
                                                               "block3_conv3", "block4_conv3", "block5_conv3")}
    og = [tr.output_gradient(li, B).cpu().numpy() for li in range(len(plan.layers))]
    res[mode] = (pred.cpu().numpy(), losses.cpu().numpy(), feats, og)
a, b = res["fp32"], res["fp32_winograd"]
print("pred max-abs", np.abs(a[0] - b[0]).max(), "losses", a[1], b[1])
for n in a[2]:
    print(n, "feat rel max", np.abs(a[2][n] - b[2][n]).max() / np.abs(a[2][n]).max())
for li, layer in enumerate(plan.layers):
    x, y = a[3][li], b[3][li]
    print(layer.name, "out-grad rel L2", np.linalg.norm(x - y) / np.linalg.norm(x))
# discontinuities of dL/dpred: total-variation sign flips between the two predictions
pa, pb = a[0], b[0]
for ax in (1, 2):
    da, db = np.diff(pa, axis=ax), np.diff(pb, axis=ax)
    flips = np.sign(da) != np.sign(db)
    print(f"TV axis {ax}: {int(flips.sum())} sign flips of {da.size}; |d| at flips max {np.abs(da[flips]).max() if flips.any() else 0:.3g}"
          f"; exact zeros {int((da == 0).sum())}")
ga, gb = a[3][-1], b[3][-1]
dg = gb - ga
print("dL/dpred diff: L2", np.linalg.norm(dg), "max", np.abs(dg).max(), "ref L2", np.linalg.norm(ga),
      "values of diff (rounded):", np.unique(np.round(dg.ravel(), 3))[:12])
print("pred range", pa.min(), pa.max(), "fraction at min", float((pa == pa.min()).mean()))
