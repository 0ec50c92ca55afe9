#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (tools/pmc_calib.hip), one counter per call:
#   bash tools/pmc_calib.sh fetch|write
set -o pipefail
export TMPDIR=/tmp
stage=${1:-fetch}
out=gpurun_out/pmc_calib
mkdir -p $out
case $stage in
  fetch) timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- tools/bin/pmc_calib > $out/fetch.log 2>&1 ;;
  write) timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- tools/bin/pmc_calib > $out/write.log 2>&1 ;;
esac
ls $out/$stage/*counter_collection.csv
