#!/bin/bash
# L2 (TCC) hits and misses of configs[3]'s streaming panel: one rocprofv3 --pmc pass (its own
# gpurun call: a --pmc run may crash at teardown after the counters are written) of the
# configs3 leg alone.  AIYAGARI_LIB selects the library (A/B against an older build).
# usage: tools/prof_c3_tcc.sh <tag>
tag=${1:-r08}
export TMPDIR=/tmp
out=gpurun_out/tcc_$tag
mkdir -p $out
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $out -o run --output-format csv -- python3 bench.py --legs configs3 --steps 1 --warmup 0 --no-cpu-baseline > $out/tcc.log 2>&1
ls $out/*counter_collection.csv $out/*/*counter_collection.csv 2>/dev/null
true
