#!/bin/bash
# kernels whose VGPR / scratch usage differs between HEAD and the working tree: scripts/regs_diff.sh name.hip
f=$1; d=$(mktemp -d)
mkdir -p $d/vub_image_denoising_amd/csrc $d/include
git -C /root/repo show HEAD:include/rdunet_hip.h > $d/include/rdunet_hip.h
for h in rdn_common.h conv3_tile.h $f; do git -C /root/repo show HEAD:vub_image_denoising_amd/csrc/$h > $d/vub_image_denoising_amd/csrc/$h; done
/root/repo/scripts/regs.sh $d/vub_image_denoising_amd/csrc/$f | awk '{print $3, $1, $2}' | sort > $d/old
/root/repo/scripts/regs.sh /root/repo/vub_image_denoising_amd/csrc/$f | awk '{print $3, $1, $2}' | sort > $d/new
join $d/old $d/new | awk '{ if ($2!=$4 || $3!=$5) printf "%4d %4d -> %4d %4d  %s\n", $2, $3, $4, $5, $1 }'
rm -rf $d
