"""Compare the last layer's dumps (RST_RACE_DUMP) of every call with call 0's (race diagnostic).
Usage: python tools/race_dump_compare.py PREFIX N H W"""
import sys

import numpy as np

pre, n, H, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
ref = {k: np.fromfile(f"{pre}_{k}_0.bin", dtype=np.float32) for k in ("out", "part", "in")}
for i in range(1, n):
    msg = [f"call {i}:"]
    for k in ("in", "out", "part"):
        a = np.fromfile(f"{pre}_{k}_{i}.bin", dtype=np.float32)
        d = a != ref[k]
        msg.append(f"{k} {int(d.sum())} differ")
        if k == "out" and d.any():
            px = np.argwhere(d.reshape(-1, H, W, 3).any(-1))
            ys, xs = px[:, 1], px[:, 2]
            tiles = sorted({(int(y) // 32, int(x) // 32) for y, x in zip(ys, xs)})
            msg.append(f"(rows {ys.min()}..{ys.max()}, cols {xs.min()}..{xs.max()}, {len(tiles)} 32x32 tiles: "
                       f"{tiles[:8]}, max |diff| {np.abs(a - ref[k])[d].max():.3e})")
            idx = np.flatnonzero(d)[:12]
            for j in idx:   # the first differing values: flat index -> (b, y, x, c), call-0 value, this call's, bits
                bb, rem = divmod(int(j), H * W * 3)
                y, rem = divmod(rem, W * 3)
                x, c = divmod(rem, 3)
                msg.append(f"\n    ({bb},{y},{x},{c}) ref {ref[k][j]:+.6e} [{ref[k][j:j+1].view(np.uint32)[0]:08x}]"
                           f" got {a[j]:+.6e} [{a[j:j+1].view(np.uint32)[0]:08x}]")
    print(" ".join(msg), flush=True)
