"""Summarise a tools/profile_gpu.sh run into profiles/.

Usage: python tools/summarize_profile.py <tag>

Reads gpurun_out/prof_<tag>/ (trace pass + PMC passes) and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.json           per-kernel, per-launch counter averages and
                                    corrected HBM bytes
  profiles/<tag>_summary.md         human-readable table

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("dpf_amd::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0] if "(" in name and "<" not in name.split("(")[0][-1:] else name[:80]


def main(tag, root=ROOT):
    src = os.path.join(root, "gpurun_out", "prof_" + tag)
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    kstats = {}
    if stats:
        shutil.copy(stats[0], os.path.join(dst, tag + "_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            kstats[r["Name"]] = r
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    # per pass and kernel: (duration, counter, value) of every dispatch, so that
    # a kernel launched at two sizes (the c4 scan and the c4/8 shard request
    # both run KPirScanG<1,4>) also gets the counters of its largest launches
    per_pass = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "dpf_amd" not in r["Kernel_Name"]:
                continue
            pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per_pass[(f, r["Kernel_Name"])].append((dur, r["Counter_Name"], float(r["Counter_Value"])))
    largest = collections.defaultdict(lambda: collections.defaultdict(list))
    partial = set()
    for (f, k), rows in per_pass.items():
        top = max(d for d, _, _ in rows)
        for d, c, v in rows:
            if d >= top // 2:
                largest[k][c].append(v)
            else:
                partial.add(k)
    trace_dur = collections.defaultdict(list)
    for tf in glob.glob(os.path.join(src, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(tf)):
            trace_dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    sha = os.path.join(src, "library.sha256")
    if os.path.exists(sha):
        # bench.py reports roofline.traffic only while this build is the one loaded
        out["_meta"] = {"library_sha256": open(sha).read().strip()}
    for k, d in pmc.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"counters_per_launch": avg, "launches": max(len(v) for v in d.values())}
        if "FETCH_SIZE" in avg:
            e["hbm_read_bytes"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            e["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if k in kstats:
            e["avg_duration_ns"] = float(kstats[k]["AverageNs"])
            e["calls_in_trace"] = int(kstats[k]["Calls"])
        if "SQ_INSTS_VALU" in avg and "SQ_INSTS_LDS" in avg:
            e["lds_per_valu"] = avg["SQ_INSTS_LDS"] / max(avg["SQ_INSTS_VALU"], 1)
        if k in partial:  # launches of several sizes: the largest ones alone too
            la = {c: sum(v) / len(v) for c, v in largest[k].items()}
            big = {"counters_per_launch": la, "launches": max(len(v) for v in largest[k].values())}
            if "FETCH_SIZE" in la:
                big["hbm_read_bytes"] = la["FETCH_SIZE"] * 1024 * 2
            if "WRITE_SIZE" in la:
                big["hbm_write_bytes"] = la["WRITE_SIZE"] * 1024
            if "FETCH_SIZE" in la and "WRITE_SIZE" in la:
                big["hbm_bytes"] = big["hbm_read_bytes"] + big["hbm_write_bytes"]
            td = trace_dur.get(k, [])
            if td:
                tl = [d for d in td if d >= max(td) // 2]
                big["avg_duration_ns"] = sum(tl) / len(tl)
                big["calls_in_trace"] = len(tl)
            e["largest_launches"] = big
        out[k] = e
    with open(os.path.join(dst, tag + "_pmc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    lines = ["# Profile %s" % tag, "",
             "Source: `bash tools/profile_gpu.sh %s` on one MI355X (trace pass "
             "`rocprofv3 --kernel-trace --stats`, then separate `--pmc` passes)." % tag, "",
             "| kernel | calls | avg ms | HBM read GB | HBM write GB | VALU wave-instr | LDS wave-instr | LDS bank conflicts |",
             "|---|---|---|---|---|---|---|---|"]
    kernels = {k: e for k, e in out.items() if k != "_meta"}
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1].get("avg_duration_ns", 0)):
        c = e["counters_per_launch"]
        lines.append("| `%s` | %s | %.3f | %.3f | %.3f | %.4g | %.4g | %.4g |" % (
            k[:90], e.get("calls_in_trace", "?"), e.get("avg_duration_ns", 0) / 1e6,
            e.get("hbm_read_bytes", 0) / 1e9, e.get("hbm_write_bytes", 0) / 1e9,
            c.get("SQ_INSTS_VALU", 0), c.get("SQ_INSTS_LDS", 0),
            c.get("SQ_LDS_BANK_CONFLICT", 0)))
    multi = [(k, e["largest_launches"]) for k, e in kernels.items() if "largest_launches" in e]
    if multi:
        lines += ["", "Kernels launched at several sizes — their largest launches alone "
                  "(dispatches of at least half the longest one's duration):", "",
                  "| kernel | calls | avg ms | HBM read GB | HBM write GB |", "|---|---|---|---|---|"]
        for k, b in multi:
            lines.append("| `%s` | %s | %.3f | %.3f | %.3f |" % (
                k[:90], b.get("calls_in_trace", "?"), b.get("avg_duration_ns", 0) / 1e6,
                b.get("hbm_read_bytes", 0) / 1e9, b.get("hbm_write_bytes", 0) / 1e9))
    with open(os.path.join(dst, tag + "_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
