"""tools/summarize_profile.py on a synthetic rocprofv3 output: a kernel
launched at two sizes (the c4 scan and the c4/8 shard's scan are both
KPirScanG<1,4>) keeps the counters and duration of its largest launches
apart, and bench.py's traffic lookup prefers them (CPU only)."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

SCAN = "void dpf_amd::KPirScanG<1, 4>(dpf_amd::ScanArgs)"
EXPAND = "void dpf_amd::KExpand<8, dpf_amd::EmitU32ModN64, false>(dpf_amd::ExpandArgs, dpf_amd::VtDev)"


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_ALL)
        w.writerow(header)
        w.writerows(rows)


def _fake_profile(root, tag):
    src = os.path.join(root, "gpurun_out", "prof_" + tag)
    # trace: 3 large scans (2.4 ms), 2 small (0.3 ms), one expansion
    launches = [(SCAN, 2400), (SCAN, 2450), (SCAN, 2500), (SCAN, 300), (SCAN, 320),
                (EXPAND, 150000)]
    rows, t = [], 1000
    for i, (k, us) in enumerate(launches):
        rows.append([i + 1, k, t, t + us * 1000])
        t += us * 1000 + 5000
    _write(os.path.join(src, "trace", "trace_kernel_trace.csv"),
           ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    avg = {SCAN: sum(u for k, u in launches if k == SCAN) / 5 * 1000, EXPAND: 150000 * 1000}
    _write(os.path.join(src, "trace", "trace_kernel_stats.csv"), ["Name", "Calls", "AverageNs"],
           [[SCAN, 5, avg[SCAN]], [EXPAND, 1, avg[EXPAND]]])
    # PMC pass: FETCH_SIZE in KiB (doubled by the summary), WRITE_SIZE in KiB
    pmc = []
    for i, (k, us) in enumerate(launches):
        big = us > 1000
        fetch = (8 << 20) if k == SCAN and big else (1 << 20) if k == SCAN else 100
        for c, v in (("FETCH_SIZE", fetch), ("WRITE_SIZE", 8 if k == SCAN else 64 << 20)):
            pmc.append([k, c, v, 0, us * 1000])
    _write(os.path.join(src, "pmc_fetch", "pmc_fetch_counter_collection.csv"),
           ["Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"],
           pmc)
    with open(os.path.join(src, "library.sha256"), "w") as f:
        f.write("ab" * 32 + "\n")


def test_largest_launches_kept_apart(tmp_path):
    import summarize_profile as S
    root = str(tmp_path)
    _fake_profile(root, "t1")
    S.main("t1", root=root)
    d = json.load(open(os.path.join(root, "profiles", "t1_pmc.json")))
    assert d["_meta"]["library_sha256"] == "ab" * 32
    scan = d[SCAN]
    big = scan["largest_launches"]
    assert big["launches"] == 3 and big["calls_in_trace"] == 3
    assert big["hbm_read_bytes"] == (8 << 20) * 1024 * 2
    assert abs(big["avg_duration_ns"] - 2450e3) < 1
    # the all-launch average mixes the sizes
    assert scan["hbm_read_bytes"] < big["hbm_read_bytes"]
    # a kernel of one size gets no separate entry
    assert "largest_launches" not in d[EXPAND]
    assert "largest launches" in open(os.path.join(root, "profiles", "t1_summary.md")).read()
