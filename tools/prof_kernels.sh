#!/bin/bash
# usage: scratch/prof.sh <tag>   (run on the GPU box from the repo root)
set -o pipefail
tag=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag/trace -o run --output-format csv -- python3 tools/prof_kernels.py > gpurun_out/prof_$tag/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof_$tag/pmc1 -o run --output-format csv -- python3 tools/prof_kernels.py > gpurun_out/prof_$tag/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$tag/pmc2 -o run --output-format csv -- python3 tools/prof_kernels.py > gpurun_out/prof_$tag/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$tag/pmc3 -o run --output-format csv -- python3 tools/prof_kernels.py > gpurun_out/prof_$tag/pmc3.log 2>&1 || exit 4
echo done
