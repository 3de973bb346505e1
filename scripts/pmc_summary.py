"""Summarise a scripts/profile.sh output directory: per-kernel average
duration (kernel trace) and per-launch counter values for the classify
kernel, plus HBM traffic per launch corrected as MI355X_MICROARCH.md's HBM
section prescribes (FETCH_SIZE reads 1/2 of wide coalesced streaming reads
on gfx950; the random 4-64 B lookups are reported as measured).

usage: python3 scripts/pmc_summary.py OUTDIR [kernel-substring] [--traffic HEADERS MODE STREAM_BYTES_PER_HDR LPM4_LAYOUT]

With --traffic, also writes profiles/pmc_traffic.json, which bench.py reports
as roofline.traffic when its batch size, mode and ipcache layout match: HBM-side bytes per
launch = FETCH_SIZE (x1 for the random lookups, +1x the streamed SoA input
bytes, which FETCH_SIZE counts at half on gfx950) + WRITE_SIZE.
"""
import csv
import glob
import re
import json
import os
import sys
from collections import defaultdict


def main(out, kname="k_classify_v4", traffic=None):
    res = {"kernels": {}, "counters": {}}
    ks = glob.glob(os.path.join(out, "kt", "*kernel_stats.csv"))
    if ks:
        for r in csv.DictReader(open(ks[0])):
            if "cfc" in r["Name"] or kname in r["Name"]:
                m = re.search(r"(k_\w+)", r["Name"])
                res["kernels"][m.group(1) if m else r["Name"].split("(")[0]] = {
                    "calls": int(r["Calls"]),
                    "avg_ms": float(r["AverageNs"]) / 1e6}
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(out, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        res["counters"][k] = sum(v) / len(v)
    c = res["counters"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res["hbm_fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
        res["hbm_write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                res[k + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        res["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if traffic and "hbm_fetch_bytes_per_launch" in res:
        n, mode, sb, layout = int(traffic[0]), traffic[1], float(traffic[2]), traffic[3]
        fix = 0.5 * n * sb
        res["hbm_bytes_per_launch"] = (res["hbm_fetch_bytes_per_launch"] + fix
                                       + res["hbm_write_bytes_per_launch"])
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        with open(os.path.join(root, "profiles", "pmc_traffic.json"), "w") as f:
            json.dump({"headers": n, "mode": mode, "lpm4_layout": layout,
                       "source": out,
                       "stream_read_bytes_per_header": sb,
                       "fetch_size_bytes": res["hbm_fetch_bytes_per_launch"],
                       "write_size_bytes": res["hbm_write_bytes_per_launch"],
                       "hbm_bytes_per_launch": res["hbm_bytes_per_launch"]},
                      f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    tr = None
    if "--traffic" in a:
        i = a.index("--traffic")
        tr = a[i + 1:i + 5]
        a = a[:i] + a[i + 5:]
    main(*a, traffic=tr)
