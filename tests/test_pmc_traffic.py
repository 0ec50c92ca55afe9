"""PMC traffic bookkeeping (host logic, no GPU): tools/pmc_traffic.py turns rocprofv3
FETCH_SIZE / WRITE_SIZE passes of ``bench.py --pmc-pass`` into per-template traffic stamped
with the library's source digest, and bench.py reports it only for the sources profiled."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(path, counter, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, k, v in rows:
            w.writerow(dict(Dispatch_Id=d, Kernel_Name=k, Counter_Name=counter, Counter_Value=v))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_pmc_summary_and_staleness(tmp_path, monkeypatch):
    k1 = "void aiy::ge_cluster_kernel<7, 7, 2, 512>(aiy::GeRun)"
    k2 = "void aiy::ge_cluster_kernel<7, 7, 1, 512>(aiy::GeRun)"
    ke = "void aiy::egm_cycle_kernel<32, 28, false, 2>(aiy::EgmArgs)"
    # FETCH in KB (doubled by the summary), WRITE in KB
    _csv(str(tmp_path / "f" / "run_counter_collection.csv"), "FETCH_SIZE",
         [(1, k1, 1000.0), (2, k2, 500.0), (3, ke, 100.0), (4, ke, 100.0), (5, ke, 1.0)])
    _csv(str(tmp_path / "w" / "run_counter_collection.csv"), "WRITE_SIZE",
         [(1, k1, 300.0), (2, k2, 200.0), (3, ke, 50.0), (4, ke, 50.0), (5, ke, 0.5)])
    log = tmp_path / "fetch.log"
    log.write_text("noise\n[bench-alg] " + json.dumps(dict(leg="table2", template="ge_cluster_kernel<7, 7, ",
                                                            launches=2, alg_bytes=3.5e6)) + "\n"
                   "[bench-alg] " + json.dumps(dict(leg="configs1", template="egm_cycle_kernel<32, 28, false, 2",
                                                    alg_bytes_per_launch=204800.0)) + "\n")
    from aiyagari_hark_amd import build
    stamp = tmp_path / "stamp.json"
    stamp.write_text(json.dumps(dict(source_digest=build.source_digest(), git_head="abc123")))
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), str(log), str(stamp), str(out)], check=True)
    doc = json.load(open(out))
    e = doc["ge_cluster_kernel<7, 7, "]
    assert e["dispatches"] == [2, 2] and e["basis"] == "total"
    assert abs(e["hbm_bytes_total"] - (2 * 1500 + 500) * 1024.0) < 1e-6
    assert abs(e["hbm_per_alg"] - (2 * 1500 + 500) * 1024.0 / 3.5e6) < 1e-12
    g = doc["egm_cycle_kernel<32, 28, false, 2"]
    assert g["basis"] == "per_launch" and g["working_dispatches"] == [2, 2]   # the no-op launch dropped
    assert abs(g["hbm_bytes_per_launch"] - (2 * 100 + 50) * 1024.0) < 1e-6

    b = _bench()
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    json.dump(doc, open(tmp_path / "profiles" / "pmc_traffic.json", "w"))
    t, info = b.pmc_traffic("ge_cluster_kernel<7, 7, ", 1.0e6)
    assert abs(t - e["hbm_per_alg"] * 1.0e6) < 1e-6 and info["traffic_pass"]["git_head"] == "abc123"
    t, info = b.pmc_traffic("hist_pull_kernel<32, 512", 1.0e6)   # never profiled
    assert t is None and "no PMC pass" in info["traffic_note"]
    doc["ge_cluster_kernel<7, 7, "]["source_digest"] = "0000000000000000"   # sources changed since
    json.dump(doc, open(tmp_path / "profiles" / "pmc_traffic.json", "w"))
    t, info = b.pmc_traffic("ge_cluster_kernel<7, 7, ", 1.0e6)
    assert t is None and info["traffic_note"].startswith("stale")
