#!/bin/bash
# GPU legs of the PSNR@sigma=25 paired protocol (scripts/psnr_parity.py --part gpu);
# the CPU-oracle legs run on any host and are merged by seed.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/psnr; export TMPDIR=/tmp
timeout -k 10 ${PSNR_TIMEOUT:-700} python -u scripts/psnr_parity.py --part gpu --bf16 --seed ${SEED:-2025} --seeds ${SEEDS:-40} \
    --steps 120 --out gpurun_out/psnr/gpu_part${PART:-}.json > gpurun_out/psnr/gpu_part${PART:-}.log 2>&1
