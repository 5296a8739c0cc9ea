#!/bin/bash
# GPU suite (no PSNR experiment) on the in-tree library, then an interleaved step A/B
# of build/variants/lib_old.so vs lib_new.so (OUT dir under gpurun_out)
cd "$GRAFT_REPO_ROOT"; OUT=${OUT:-sab}; mkdir -p gpurun_out/$OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -k "not psnr" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/$OUT/t.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ROUNDS=${ROUNDS:-2} B32=1 VARIANTS="old=RDN_LIB=build/variants/lib_old.so;new=RDN_LIB=build/variants/lib_new.so" bash scripts/ab_env.sh
