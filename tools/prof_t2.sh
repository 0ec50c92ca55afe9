#!/bin/bash
# Kernel stats of the headline leg alone over several sweeps (the first launch's average over
# steps + warmup sweeps, not one cold sweep): rocprofv3 --kernel-trace --stats of
# bench.py --legs table2 --steps 5 --warmup 2.  usage: tools/prof_t2.sh <tag>
tag=${1:-r08}
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_t2trace -o run --output-format csv -- python3 bench.py --legs table2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_t2trace.log 2>&1
