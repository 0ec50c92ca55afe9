#!/bin/bash
# configs[4]'s pull solve under rocprofv3 at several cluster sizes (workgroups per calibration,
# 0 = the planner's choice): one K_s(r) evaluation of the three stress cells per run
# (tools/hist_phases.py), kernel stats under gpurun_out/s6s_cl<G>/.  DESIGN.md §4g uses it to
# show that the solve's time follows its dependent load rounds, not its work.
export TMPDIR=/tmp STRESS=1
for cl in 0 64 50 43; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/s6s_cl$cl -o run --output-format csv -- python3 tools/hist_phases.py 3 $cl -1 > gpurun_out/s6s_cl$cl.log 2>&1 || exit 1
done
