#!/bin/bash
# run on the GPU box from the repo root: profiles of the bench command + the bench line
set -o pipefail
tag=${1:-r01}
export TMPDIR=/tmp
out=gpurun_out/bench_$tag
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/trace.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --act-T 400 --t-discard 100 --no-cpu-baseline > $out/pmc_fetch.log 2>&1 || exit 2
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --act-T 400 --t-discard 100 --no-cpu-baseline > $out/pmc_write.log 2>&1 || exit 3
python3 tools/pmc_traffic.py $out/pmc_fetch $out/pmc_write $out/pmc_traffic.json > $out/pmc_traffic.txt || exit 4
timeout -k 10 900 python3 bench.py > $out/bench.json 2> $out/bench.err || exit 5
echo done
