#!/bin/bash
# L2 hit / miss counters of the resident panel kernels at configs[3] size (one rocprofv3 pass
# per counter group; the panel_variants child runs in-process, no exec hop).
#   bash tools/pmc_panel.sh TAG ENGINE
set -u
TAG=$1
ENG=$2
export TMPDIR=/tmp ENGINE=$ENG NAG=99999998 T=50 FUSE=0
mkdir -p gpurun_out
timeout -k 10 -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_e${ENG}_hit -o run --output-format csv -- python3 tools/panel_variants.py --child - '[[1,0,1,0,50]]' > gpurun_out/${TAG}_e${ENG}_hit.log 2>&1 || exit $?
timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_e${ENG}_fetch -o run --output-format csv -- python3 tools/panel_variants.py --child - '[[1,0,1,0,50]]' > gpurun_out/${TAG}_e${ENG}_fetch.log 2>&1 || exit $?
