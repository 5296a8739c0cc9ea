#!/bin/bash
# SQ counters (two passes) of conv3_dw variants on one shape:
#   LIBS="base noload" DW_SHAPE=80,32 bash scripts/pmc_dw.sh   (build/variants/lib_<name>.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcdw; export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for v in $LIBS; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    DW_NOTREE=1 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmcdw/$v/p$i -o run --output-format csv -- python3 scripts/dw_kbench.py build/variants/lib_$v.so > gpurun_out/pmcdw/$v.p$i.log 2>&1
    rc=$?; echo "pass $i rc=$rc" >> gpurun_out/pmcdw/$v.p$i.log
    [ $rc -eq 0 ] || exit $rc
  done
done
