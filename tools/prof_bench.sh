#!/bin/bash
# Profiles of the bench command (run on the GPU box from the repo root), one stage per
# call -- rocprofv3 --pmc runs end with a teardown crash of the profiled process after
# the counters are written, so each PMC pass gets a gpurun call of its own:
#   trace : rocprofv3 --kernel-trace --stats of one bench step, then the bench line
#   fetch : --pmc FETCH_SIZE of one bench step
#   write : --pmc WRITE_SIZE of one bench step
#   (summary: python3 tools/pmc_traffic.py <fetch> <write> <out.json> <fetch log> [kernels])
# usage: tools/prof_bench.sh <tag> <stage> [leg]
set -o pipefail
tag=${1:-r01}
stage=${2:-trace}
export TMPDIR=/tmp
out=gpurun_out/bench_$tag
mkdir -p $out
leg=${3:-table2}   # bench leg the pass profiles (table2: the headline; configs1: the KS GE solve)
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --legs $leg"
[ "$leg" = table2 ] || out=${out}_$leg
mkdir -p $out
case $stage in
  trace)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $B > $out/trace.log 2>&1 || exit 1
    timeout -k 10 900 python3 bench.py > $out/bench.json 2> $out/bench.err || exit 5 ;;
  fetch)
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 $B > $out/pmc_fetch.log 2>&1
    ls $out/pmc_fetch/*counter_collection.csv ;;
  write)
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 $B > $out/pmc_write.log 2>&1
    ls $out/pmc_write/*counter_collection.csv ;;
esac
