"""VGPR / AGPR / scratch / LDS per kernel instantiation of one HIP source (hipcc
-Rpass-analysis=kernel-resource-usage).  python scripts/regs_dw.py <file.hip> [flags...]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(REPO, "vub_image_denoising_amd", "csrc", sys.argv[1])
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       "-Wno-unused-command-line-argument", *sys.argv[2:], "-c", src, "-o", "/tmp/regs_probe.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
name, d = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name, d = m.group(1), {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and name:
        d[m.group(1).split()[0]] = m.group(2)
        if m.group(1).startswith("LDS"):
            short = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", name)[:70]
            print(f"{short:70s} vgpr {d.get('VGPRs')} agpr {d.get('AGPRs')} scratch {d.get('ScratchSize')} "
                  f"occ {d.get('Occupancy')} lds {d.get('LDS')}")
