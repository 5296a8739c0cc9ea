#!/bin/bash
# variant libraries for kernel A/B: SRC=<file.hip> VARIANTS="name:-DFLAG ..." -> build/variants/lib_<name>.so
# (the other objects come from build/obj; run the normal build first)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
OBJS=$(ls build/obj/*.o | grep -v "/$(basename ${SRC%.hip}).o")
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-command-line-argument $flags -c vub_image_denoising_amd/csrc/$SRC -o build/variants/$name.o &
done
wait
for v in $VARIANTS; do
  name=${v%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o build/variants/lib_$name.so build/variants/$name.o $OBJS
done
ls -la build/variants/*.so
