#!/bin/bash
# SQ counters (two passes) of one kbench shape: KB_ONLY=<shape> bash scripts/pmc_kb.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmck; export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  KB_REPS=5 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmck/p$i -o run --output-format csv -- python3 scripts/kbench.py > gpurun_out/pmck/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" >> gpurun_out/pmck/p$i.log
  [ $rc -eq 0 ] || exit $rc
done
