"""Summarise tools/pmc_panel.sh output: per-kernel counter sums (per dispatch) for the
kernels whose name contains the given substring."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_panel"
pat = sys.argv[2] if len(sys.argv) > 2 else "resident"
for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    print(os.path.basename(os.path.dirname(f)), f"dispatches={len(disp)}",
          {k: f"{v / max(1, len(disp)):.4g}" for k, v in sorted(agg.items())})
