"""Build ``librdunet_hip.so`` in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["conv_gemm.hip", "conv3_halo.hip", "conv3_ws.hip", "conv_wgrad.hip", "wgrad3_halo.hip", "pointwise.hip", "synth.hip", "metrics.hip"]
OUT = os.path.join(HERE, "librdunet_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-command-line-argument"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [
        os.path.join(CSRC, "rdn_common.h"), os.path.join(HERE, "..", "include", "rdunet_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = True) -> str:
    if not force and not _stale():
        return OUT
    objs = []
    jobs = []
    for s in SOURCES:  # compile translation units in parallel
        o = os.path.join(CSRC, s.replace(".hip", ".o"))
        cmd = [HIPCC, *FLAGS[:-2], "-c", os.path.join(CSRC, s), "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        jobs.append((subprocess.Popen(cmd), s))
        objs.append(o)
    for p, s in jobs:
        if p.wait() != 0:
            raise RuntimeError(f"hipcc failed on {s}")
    tmp = OUT + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, OUT)
    for o in objs:
        os.remove(o)
    return OUT


if __name__ == "__main__":
    build_library(force=True)
