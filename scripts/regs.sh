#!/bin/bash
# register / scratch usage of every kernel in a HIP source: scripts/regs.sh file.hip [hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$f" -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
 | grep -E "VGPRs:|ScratchSize|Function Name" | paste - - - \
 | sed -E 's/.*Name: (\S+).*VGPRs: ([0-9]+).*lane\]: ([0-9]+).*/\2 \3 \1/'
rm -f /tmp/regs_$$.o
