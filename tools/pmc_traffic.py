#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE).

Collected in two separate passes (MI355X_MICROARCH.md §rocprofv3 PMC slots: FETCH_SIZE costs 3 TCC
slots and WRITE_SIZE 2, they cannot share a pass):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir_f> -o r01 -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir_w> -o r01 -- python bench.py ...
Units are KiB. gfx950 correction, calibrated on this chip (tools/probe_r06.hip fetch,
profiles/r06/r06a/fetch_calibration.json: 512 MiB per pattern): every read pattern the kernels issue — coalesced
4-, 8- and 16-byte lanes and the one-dword-per-128-B-line L2 touch — reports FETCH_SIZE = exactly half its bytes
(TCC_EA0_RDREQ = bytes / 128, TCC_BUBBLE = 0: each L2 miss is one 128-B request tallied at 64 B), so read bytes =
2 x FETCH_SIZE x 1024 for every kernel here; WRITE_SIZE is exact for 4- and 16-byte stores.
Infinity-Cache hits are counted too (the counters sit at the L2's memory side): these are L2 fill bytes, of which
the HBM share is smaller when the 256 MB Infinity Cache holds the data (every frame's working set does).

Usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> <out_json>
"""
import collections
import csv
import json
import re
import sys

CONFIG_NAMES = {
    (9, 9, 1, 18, 32): "conv_mfma<9x9 s1 CK18 NT32>", (9, 9, 1, 4, 32): "conv_mfma<9x9 s1 CK4 NT32>",
    (3, 3, 2, 16, 32): "conv_mfma<3x3 s2 CK16 NT32>", (3, 3, 2, 8, 32): "conv_mfma<3x3 s2 CK8 NT32>",
    (3, 3, 1, 32, 128): "conv_mfma<3x3 s1 CK32 NT128>", (3, 3, 1, 32, 32): "conv_mfma<3x3 s1 CK32 NT32>",
    (2, 2, 1, 32, 128): "conv_mfma<2x2 phase CK32 NT128>", (2, 2, 1, 32, 64): "conv_mfma<2x2 phase CK32 NT64>",
}


def short_name(k: str) -> str:
    m = re.search(r"conv_mfma_kernel<([^>]*)>", k)
    if m:
        args = tuple(int(v) for v in m.group(1).split(","))
        return CONFIG_NAMES.get(args[:5], "conv_mfma<" + ",".join(map(str, args)) + ">")
    m = re.search(r"conv_lite_kernel<([^>]*)>", k)
    if m:
        f = [int(v) for v in m.group(1).split(",")]
        mode, cin, nc = f[:3]
        if len(f) > 5 and f[5]:   # x6: 16x16x32 bf16 for Cout 16, 32x32x16 for Cout 32; the mode picks the conv kind
            shape6 = "16x16x32" if nc == 16 else "32x32x16"
            return f"conv_lite<3x3 s2 {'transposed ' if mode else ''}Cin{cin} Cout{nc} split-bf16 x6 {shape6} MFMA>"
        shape = "16x16x4" if nc == 16 else "32x32x2"
        return f"conv_lite<3x3 s2 {'transposed ' if mode else ''}Cin{cin} Cout{nc} f32 {shape} MFMA>"
    if "last_x6_kernel" in k:
        return "last_x6<9x9 transposed Cin16 Cout3 as N=(kx,co) split-bf16 x6 MFMA>"
    if "wino9f3" in k:
        return "wino9f3<9x9 as 9 x F(3x3,3x3) on one tile grid, 24x24 N32 split-bf16 x6 MFMA persistent>"
    if "wino9_x6_kernel" in k:
        return "wino9_x6_conv<9x9 as 9 x F(2x2,3x3) 16x16 N32 split-bf16 x6 MFMA persistent>"
    if "wino_x6_kernel" in k or "wino_x6w_kernel" in k:
        return "wino_x6_conv<F(2x2,3x3) 8x16 N128 split-bf16 x6 MFMA>"
    if "wino9_conv_kernel" in k:
        return "wino9_conv<9x9 as 9 x F(2x2,3x3) 8x16 N32 f32 MFMA>"
    if "wino_conv" in k:
        return "wino_conv<F(2x2,3x3) 8x16 N128 f32 MFMA>"
    if "gbuffer_resize_crop" in k:
        return "gbuffer_resize_crop"
    if "small_conv_kernel" in k:
        return "small_conv_kernel<9x9 Cout3 VALU>"
    return k.split("(")[0]


def load(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"note": __doc__.split("\n\n")[1], "per_launch_bytes": {}, "raw": {},
           "correction": "reads 2 x FETCH_SIZE (calibrated for 4/8/16-B lanes and the 128-B-line touch, "
                         "profiles/r06/r06a/fetch_calibration.json); writes WRITE_SIZE (exact for 4- and 16-B stores)"}
    # instantiations that share a short name (e.g. the prologue-mode templates of one kernel) are
    # merged launch-weighted: per_launch_bytes is the mean over every launch of that kernel
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for k, fv in fetch.items():
        wv = write.get(k, [0.0] * len(fv))
        a = agg[short_name(k)]
        a[0] += len(fv)
        a[1] += sum(fv)
        a[2] += sum(wv) * len(fv) / max(len(wv), 1)
    for name, (n, fsum, wsum) in agg.items():
        f_mean, w_mean = fsum / n, wsum / n
        out["per_launch_bytes"][name] = round(2.0 * f_mean * 1024 + w_mean * 1024)
        out["raw"][name] = {"launches": n, "fetch_kib_mean": f_mean, "write_kib_mean": w_mean,
                            "read_bytes_corrected": 2.0 * f_mean * 1024, "write_bytes": w_mean * 1024}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for n, v in sorted(out["per_launch_bytes"].items(), key=lambda t: -t[1]):
        print(f"{v / 1e6:10.2f} MB/launch  {n}")


if __name__ == "__main__":
    main()
