"""Build ``librdunet_hip.so`` in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["conv_gemm.hip", "conv_pix.hip", "conv3_halo.hip", "conv3_big.hip", "conv3_ws.hip", "conv3_wsd.hip", "conv3_dw.hip", "conv3_dense.hip", "conv3_dense1.hip", "conv_wgrad.hip", "wgrad3_halo.hip", "wgrad3_glds.hip", "pointwise.hip", "synth.hip", "metrics.hip"]
OUT = os.path.join(HERE, "librdunet_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-command-line-argument"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [
        os.path.join(CSRC, "rdn_common.h"), os.path.join(CSRC, "conv3_tile.h"),
        os.path.join(HERE, "..", "include", "rdunet_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = True) -> str:
    """Compile every translation unit (in parallel) and link the library.  Objects are
    kept under build/obj so that an unforced rebuild recompiles only the sources
    newer than their object (headers touched: everything)."""
    if not force and not _stale():
        return OUT
    objdir = os.path.join(HERE, "..", "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    hdr_t = max(os.path.getmtime(os.path.join(CSRC, h)) for h in ("rdn_common.h", "conv3_tile.h"))
    hdr_t = max(hdr_t, os.path.getmtime(os.path.join(HERE, "..", "include", "rdunet_hip.h")))
    objs = []
    jobs = []
    for s in SOURCES:  # compile translation units in parallel
        src = os.path.join(CSRC, s)
        o = os.path.join(objdir, s.replace(".hip", ".o"))
        objs.append(o)
        if not force and os.path.exists(o) and os.path.getmtime(o) > max(os.path.getmtime(src), hdr_t):
            continue
        cmd = [HIPCC, *FLAGS[:-2], "-c", src, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        jobs.append((subprocess.Popen(cmd), s))
    for p, s in jobs:
        if p.wait() != 0:
            raise RuntimeError(f"hipcc failed on {s}")
    tmp = OUT + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build_library(force=True)
