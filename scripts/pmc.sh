#!/bin/bash
# PMC passes (separate rocprofv3 runs, --kernel-trace only beside --pmc) of one
# command; per-dispatch csv under gpurun_out/pmc/pN.  Usage: scripts/pmc.sh <cmd...>
cd "$GRAFT_REPO_ROOT"; mkdir -p ${PMC_OUT:-gpurun_out/pmc}; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d ${PMC_OUT:-gpurun_out/pmc}/p$i -o run --output-format csv -- "$@" > ${PMC_OUT:-gpurun_out/pmc}/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" >> ${PMC_OUT:-gpurun_out/pmc}/p$i.log
  [ $rc -eq 0 ] || exit $rc
done
