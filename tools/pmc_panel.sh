#!/bin/bash
# PMC passes over the persistent panel kernel (tools/prof_kernels.py: EGM solve at
# N_a = 10 000, then T periods of 1 000 006 agents).  Run on the GPU box from the repo
# root; one counter group per rocprofv3 run (MI355X_MICROARCH.md, rocprofv3 PMC slots).
set -o pipefail
export TMPDIR=/tmp
out=${1:-gpurun_out/pmc_panel}
mkdir -p $out
rocprofv3 -L > $out/counters.txt 2>&1 || true
pass() {
  name=$1; shift
  T=300 timeout -s KILL 120 rocprofv3 --pmc "$@" -d $out/$name -o run --output-format csv -- python3 tools/prof_kernels.py > $out/$name.log 2>&1
}
pass sq SQ_WAVES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACCUM_PREV_HIRES && \
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum && \
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum && \
echo pmc done
