#!/bin/bash
# PMC passes (separate rocprofv3 runs, --kernel-trace only beside --pmc) of one
# command; per-dispatch csv under $PMC_OUT/pN (default gpurun_out/pmc).
# PASSES selects passes (default "1 2 3 4 5").  Usage: scripts/pmc.sh <cmd...>
cd "$GRAFT_REPO_ROOT"; O=${PMC_OUT:-gpurun_out/pmc}; mkdir -p $O; export TMPDIR=/tmp
P[1]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA"
P[2]="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P[3]="FETCH_SIZE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
P[4]="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
# MFMA pipe busy (SQ_VALU_MFMA_BUSY_CYCLES), LDS array cycles and issue stalls on LDS
P[5]="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for i in ${PASSES:-1 2 3 4 5}; do
  timeout -k 5 -s KILL 300 rocprofv3 --kernel-trace --pmc ${P[$i]} -d $O/p$i -o run --output-format csv -- "$@" > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" >> $O/p$i.log
  [ $rc -eq 0 ] || exit $rc
done
