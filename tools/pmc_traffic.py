"""Summarise rocprofv3 PMC passes into per-launch HBM traffic for bench.py.

Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [bench_log] [kernel,kernel,...]
(entries of other kernels are kept when <out.json> exists; the optional list restricts
which kernels of these passes are taken, e.g. the Table II leg's hist_bicg_kernel only)

With the log of the profiled bench run (its "hist_point_iters=" line), the device-resident
histogram also gets hbm_bytes_per_point_iter: its launches differ in iteration count, so
bench.py scales the per-(state, node)-point-iteration traffic to its own launches.

FETCH_SIZE and WRITE_SIZE (KB) come from separate rocprofv3 --pmc passes (they do not
fit one pass on gfx950).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half the
bytes of a wide coalesced streaming read on gfx950, so it is doubled; WRITE_SIZE is
exact for streaming stores.  Both are averaged per dispatch of each kernel.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(disp[k]), len(disp[k])) for k in tot}


def point_iters(log_path):
    import re
    n = 0
    for line in open(log_path, errors="replace"):
        m = re.search(r"hist_point_iters=(\d+)", line)
        if m:
            n += int(m.group(1))
    return n


def main():
    fd, wd, out = sys.argv[1:4]
    pts = point_iters(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] else 0
    def by_short(d):   # template instantiations of one kernel pooled (mean over all their dispatches)
        agg = collections.defaultdict(lambda: [0.0, 0, []])
        for k, (mean, n) in d.items():
            short = k.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
            agg[short][0] += mean * n
            agg[short][1] += n
            agg[short][2].append(k)
        return {s: (t / max(1, n), n, names) for s, (t, n, names) in agg.items()}
    fetch = by_short(per_kernel(fd, "FETCH_SIZE"))
    write = by_short(per_kernel(wd, "WRITE_SIZE"))
    res = {}
    for short in set(fetch) | set(write):
        f_kb, nf, names_f = fetch.get(short, (0.0, 0, []))
        w_kb, nw, names_w = write.get(short, (0.0, 0, []))
        k = " | ".join(sorted(set(names_f) | set(names_w)))
        res[short] = dict(kernel=k, fetch_kb_raw=f_kb, write_kb=w_kb, dispatches=[nf, nw],
                          hbm_bytes_per_launch=(2.0 * f_kb + w_kb) * 1024.0,
                          hbm_bytes_total=(2.0 * f_kb * nf + w_kb * nw) * 1024.0,
                          correction="FETCH_SIZE x2 (gfx950 wide-read under-count), WRITE_SIZE x1")
        if short in ("hist_cluster_kernel", "hist_bicg_kernel") and pts > 0:
            res[short]["point_iters"] = pts
            res[short]["hbm_bytes_per_point_iter"] = (2.0 * f_kb * nf + w_kb * nw) * 1024.0 / pts
    merged = {}
    if os.path.exists(out):   # keep the other kernels' entries (earlier passes of other legs)
        merged = json.load(open(out))
    only = sys.argv[5].split(",") if len(sys.argv) > 5 else None   # kernels to take from these passes
    merged.update({k: v for k, v in res.items() if only is None or k in only})
    json.dump(merged, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k}: {v['hbm_bytes_per_launch'] / 1e6:.2f} MB/launch (fetch raw {v['fetch_kb_raw']:.0f} KB, "
              f"write {v['write_kb']:.0f} KB)")


if __name__ == "__main__":
    main()
