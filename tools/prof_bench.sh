#!/bin/bash
# Profiles of the bench command (run on the GPU box from the repo root), one stage per
# gpurun call (a rocprofv3 --pmc run can end with a teardown crash of the profiled process
# after the counters are written, so no GPU step may follow it in the same call):
#   trace : rocprofv3 --kernel-trace --stats of bench.py --pmc-pass (all legs)
#   fetch : rocprofv3 --pmc FETCH_SIZE of the same command
#   write : rocprofv3 --pmc WRITE_SIZE of the same command
# Each stage writes stamp_<stage>.json (the sources' digest, the digest the LOADED library was
# built from -- its .digest sidecar, $AIYAGARI_LIB or the in-tree build -- its path and mtime,
# and the git head passed in), so tools/pmc_traffic.py can stamp the traffic it derives with
# the sources profiled (a stamp whose library digest differs from the sources' is stale):
#   python3 tools/pmc_traffic.py $out/pmc_fetch $out/pmc_write $out/pmc_fetch.log \
#       $out/stamp_fetch.json profiles/pmc_traffic.json
# usage: tools/prof_bench.sh <tag> <stage> <git head> [legs]
set -o pipefail
tag=${1:-r06}
stage=${2:-trace}
head=${3:-unknown}
legs=${4:-table2,configs1,configs3,configs4}
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
python3 -c "import json, os, sys; sys.path.insert(0, '.'); from aiyagari_hark_amd import build; \
lib = os.environ.get('AIYAGARI_LIB') or build.LIB; \
d = dict(source_digest=build.source_digest(), lib_digest=build.library_digest(lib), lib_path=lib, \
         lib_mtime=os.path.getmtime(lib), git_head='$head'); \
assert d['lib_digest'] == d['source_digest'], ('stale library', d); \
json.dump(d, open('$out/stamp_$stage.json', 'w'))" || exit 3
B="bench.py --steps 1 --warmup 0 --no-cpu-baseline --pmc-pass --legs $legs"
case $stage in
  trace)
    timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $B > $out/trace.log 2>&1 ;;
  fetch)
    timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 $B > $out/pmc_fetch.log 2>&1
    ls $out/pmc_fetch/*/*counter_collection.csv $out/pmc_fetch/*counter_collection.csv 2>/dev/null ;;
  write)
    timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 $B > $out/pmc_write.log 2>&1
    ls $out/pmc_write/*/*counter_collection.csv $out/pmc_write/*counter_collection.csv 2>/dev/null ;;
esac
