"""Where a kernel's loops wait: for each instantiation matching a substring, the
loop headers and the `s_waitcnt vmcnt(0)` lines of its gfx950 assembly.

  python scripts/asm_loops.py <file.hip> <mangled-substring> [flags...]
"""
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(REPO, "vub_image_denoising_amd", "csrc", sys.argv[1])
out = "/tmp/asm_loops"
os.makedirs(out, exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                "-Wno-unused-command-line-argument", *sys.argv[3:], "-c", src, "-o", f"{out}/k.o", "-save-temps"],
               cwd=out, check=True)
s = open(glob.glob(f"{out}/*gfx950.s")[0]).read()
for m in re.finditer(r"^(_Z\S+):[^\n]*$", s, re.M):
    name = m.group(1)
    if sys.argv[2] not in name or "kernel" not in name:
        continue
    end = s.index(".Lfunc_end", m.end())
    body = s[m.end():end].split("\n")
    heads = [i for i, l in enumerate(body) if "Loop Header" in l]
    zeros = [i for i, l in enumerate(body) if "s_waitcnt vmcnt(0)" in l]
    bars = [i for i, l in enumerate(body) if "s_barrier" in l]
    print(name[:80])
    print("  lines", len(body), "loop heads", heads)
    print("  vmcnt(0) at", zeros)
    print("  s_barrier at", bars)
    with open(f"{out}/{name[:60]}.s", "w") as f:
        f.write("\n".join(body))
