"""Build librst.so (gfx950) in-tree with hipcc.

The .so lands next to this file so it travels to the GPU box with the repo snapshot.
Usage: ``python -m realtime_style_transfer_amd.build [--force] [-v]``.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
ROOT = PKG.parent
LIB = PKG / "librst.so"
OBJ = PKG / "_build"
SOURCES = ["conv_mfma.hip", "conv_small.hip", "norm.hip", "gram.hip", "loss.hip", "rst_api.hip", "loss_api.hip",
           "train.hip", "train_api.hip", "wgrad.hip",
           "conv_bf3.hip", "predictor.hip", "predictor_api.hip",
           "predictor_train.hip", "predictor_train_api.hip", "wino.hip", "wino_x6.hip", "wino9.hip", "wino9_x6.hip", "wino9f3.hip", "conv_lite.hip", "conv_last.hip", "ingest.hip", "ingest_api.hip", "crc32c.hip"]
ARCH = os.environ.get("RST_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", str(ROOT / "include"), "-I", str(CSRC),
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-munsafe-fp-atomics"]


# per-source extra flags: the split-bf16 Winograd kernel keeps its transform in scalar f32 ops (packed f32
# VALU beside MFMAs costs more issue cycles than two scalar ops on gfx950)
EXTRA = {"wino_x6.hip": ["-fno-slp-vectorize"], "wino9_x6.hip": ["-fno-slp-vectorize"],
         # the last conv's scalar FMAs must stay scalar (conv_small.hip: SLP would re-pack them into v_pk_fma_f32)
         "conv_small.hip": ["-fno-slp-vectorize"]}


def _digest() -> str:
    h = hashlib.sha256()
    for f in sorted(CSRC.glob("*")) + [ROOT / "include" / "rst.h"]:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    h.update(" ".join(CFLAGS).encode())
    h.update(repr(sorted(EXTRA.items())).encode())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> Path:
    stamp = PKG / "librst.stamp"
    dig = _digest()
    if not force and LIB.exists() and stamp.exists() and stamp.read_text().strip() == dig:
        return LIB
    OBJ.mkdir(exist_ok=True)

    def compile_one(src: str) -> Path:
        obj = OBJ / (Path(src).stem + ".o")
        cmd = [HIPCC, *CFLAGS, *EXTRA.get(src, []), "-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return obj

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    stamp.write_text(dig)
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, verbose=args.verbose))


if __name__ == "__main__":
    main()
