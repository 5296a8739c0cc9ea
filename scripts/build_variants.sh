#!/bin/bash
# build variant libraries of librdunet_hip for A/B timing (scripts/kbench.py)
set -e
cd "$(dirname "$0")/../vub_image_denoising_amd/csrc"
OUT=${OUT:-/tmp/variants}
mkdir -p $OUT
build() { # name, flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -o $OUT/lib_$name.so conv_gemm.hip conv3_halo.hip conv3_ws.hip conv3_wsd.hip conv_wgrad.hip wgrad3_halo.hip wgrad3_glds.hip pointwise.hip synth.hip metrics.hip
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$flags" = "$spec" ] && flags=""
  build $name $flags &
done
wait
ls -la $OUT
