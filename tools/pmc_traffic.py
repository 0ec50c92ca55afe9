"""Summarise rocprofv3 PMC passes of bench.py into HBM traffic per kernel template.

Usage:
  python tools/pmc_traffic.py <fetch_dir> <write_dir> <fetch_log> <stamp.json> <out.json>

The passes are ``tools/prof_bench.sh <tag> fetch|write`` (rocprofv3 --pmc FETCH_SIZE, then
--pmc WRITE_SIZE, each its own process; they do not fit one pass on gfx950) of
``bench.py --pmc-pass``: every leg runs its timed work only (no warm-up launches), and bench
prints one ``[bench-alg] {...}`` line per dominant kernel to stderr with the template it
expects the library to launch, its launches and its algorithmic bytes.
``stamp.json`` is written by the pass on the GPU box: the library's source digest
(aiyagari_hark_amd.build.source_digest) and the git head of the profiled tree.

For each [bench-alg] record the dispatches of kernels whose name starts with the record's
template are pooled:
  hbm_bytes_total    = 2 x FETCH_SIZE + WRITE_SIZE over those dispatches (KB x 1024; FETCH
                       doubled: gfx950 counts half the bytes of a wide read, MI355X_MICROARCH.md
                       §HBM, calibrated for this repository's access widths in
                       profiles/r03_pmc_calibration.json)
  hbm_per_alg        = hbm_bytes_total / the record's algorithmic bytes of the same launches
                       (basis "total"), or the mean over the working dispatches (>= 1/4 of
                       the largest) / the algorithmic bytes of one launch (basis "per_launch":
                       kernels whose solve loop also launches converged no-op cycles)
bench.py reports traffic = hbm_per_alg x its own algorithmic bytes per launch, and only
while the entry's source digest equals the current sources (else null, with the reason).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def dispatches(d, counter):
    """{kernel name: {dispatch id: value}} of one counter over every CSV under d."""
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].replace("void ", "").split("(")[0].strip()
            k = re.sub(r"^aiy::", "", k)
            out[k][r["Dispatch_Id"]] = out[k].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return out


def alg_records(log_path):
    recs = []
    for line in open(log_path, errors="replace"):
        i = line.find("[bench-alg] ")
        if i >= 0:
            recs.append(json.loads(line[i + len("[bench-alg] "):]))
    return recs


def main():
    fd, wd, log, stamp_path, out = sys.argv[1:6]
    stamp = json.load(open(stamp_path))
    fetch = dispatches(fd, "FETCH_SIZE")
    write = dispatches(wd, "WRITE_SIZE")
    res = {}
    for rec in alg_records(log):
        tpl = rec["template"]
        fk = {k: v for k, v in fetch.items() if k.startswith(tpl)}
        wk = {k: v for k, v in write.items() if k.startswith(tpl)}
        fv = [x for v in fk.values() for x in v.values()]
        wv = [x for v in wk.values() for x in v.values()]
        if not fv or not wv:
            print(f"{tpl}: no dispatches in the passes (library launched another template?)")
            continue
        f_tot, w_tot = sum(fv), sum(wv)
        e = dict(leg=rec["leg"], template=tpl, kernels=sorted(set(fk) | set(wk)),
                 dispatches=[len(fv), len(wv)], source_digest=stamp["source_digest"], git_head=stamp["git_head"],
                 fetch_kb_raw_total=f_tot, write_kb_total=w_tot,
                 hbm_bytes_total=(2.0 * f_tot + w_tot) * 1024.0,
                 correction="FETCH_SIZE x2 (gfx950 wide-read under-count), WRITE_SIZE x1",
                 alg_note=rec.get("note", ""))
        if "alg_bytes_per_launch" in rec:   # constant-size launches, some of them no-ops
            fmax, wmax = max(fv), max(wv)
            fw = [x for x in fv if x >= 0.25 * fmax]
            ww = [x for x in wv if x >= 0.25 * wmax]
            per = (2.0 * sum(fw) / len(fw) + sum(ww) / len(ww)) * 1024.0
            e.update(basis="per_launch", working_dispatches=[len(fw), len(ww)], hbm_bytes_per_launch=per,
                     alg_bytes_per_launch=rec["alg_bytes_per_launch"], hbm_per_alg=per / rec["alg_bytes_per_launch"])
        else:
            e.update(basis="total", launches_reported=rec["launches"], alg_bytes_total=rec["alg_bytes"],
                     hbm_bytes_per_launch=e["hbm_bytes_total"] / len(fv),
                     hbm_per_alg=e["hbm_bytes_total"] / rec["alg_bytes"])
            if rec["launches"] != len(fv):
                e["dispatch_mismatch"] = f"bench reported {rec['launches']} launches, the fetch pass saw {len(fv)}"
        for k in ("units", "unit_name", "alg_bytes_per_unit"):
            if k in rec:
                e[k] = rec[k]
        if "units" in rec:
            e["hbm_bytes_per_unit"] = e["hbm_bytes_total"] / rec["units"]
        res[tpl] = e
        print(f"{tpl}: {e['hbm_bytes_per_launch'] / 1e6:.2f} MB per launch, {e['hbm_per_alg']:.3f} x algorithmic "
              f"({e['basis']})")
    doc = {"_about": ("rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py --pmc-pass (tools/prof_bench.sh, "
                      "tools/pmc_traffic.py); keyed by kernel template; bench.py uses an entry only while "
                      "its source_digest equals aiyagari_hark_amd.build.source_digest()"),
           "_stamp": stamp}
    doc.update(res)
    json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
