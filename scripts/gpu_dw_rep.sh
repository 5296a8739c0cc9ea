#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dw_repeat.py > gpurun_out/rep.log 2>&1; echo "rc=$?" >> gpurun_out/rep.log
