#!/bin/bash
# PMC passes over the persistent panel kernel (tools/prof_kernels.py: EGM solve at
# N_a = 10 000, then T periods of 1 000 006 agents).  Run on the GPU box from the repo
# root; one counter group per rocprofv3 run (MI355X_MICROARCH.md, rocprofv3 PMC slots).
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc_panel}
mkdir -p $out
pass() {
  name=$1; shift
  T=300 timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o run --output-format csv -- python3 tools/prof_kernels.py > $out/$name.log 2>&1
}
pass tlb TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum && \
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum && \
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE && \
pass tcc TCC_HIT_sum TCC_MISS_sum && \
pass sq SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS && \
echo pmc done
