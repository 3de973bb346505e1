"""Summarise a scripts/profile.sh output directory: per-kernel average
duration (kernel trace) and per-launch counter values of every engine
kernel, with HBM traffic per launch corrected as MI355X_MICROARCH.md's HBM
section prescribes (FETCH_SIZE reads 1/2 of wide coalesced streaming reads
on gfx950; the random 4-64 B lookups are reported as measured).

usage: python3 scripts/pmc_summary.py OUTDIR [kernel-substring]
           [--skip N] [--save PROFILE_DIR]
           [--record WORKLOAD MODE LPM4_LAYOUT [variant=V] KERNEL:HEADERS:STREAM_BYTES ...]

--skip N leaves out each kernel's first N launches (the steady state: a
context's first apply sizes its sets from nothing).

--save copies the kernel statistics, the engine's rows of every counter pass
(cfc:: kernels only) and this summary into PROFILE_DIR (the committed
profiles/ tree).

--record adds (or replaces) this configuration's entry in
profiles/pmc_traffic.json, which bench.py reads for its roofline when the
workload, mode, ipcache layout, variant (lookup: classify only — the
default; ct_apply: classify + cfc_ct_apply + GC, whose classify kernel also
stores the CT bytes; notify) and per-kernel batch sizes match.  A spec
KERNEL:0:0 records a kernel without a batch size (the apply's and GC's, per
launch).  Per kernel
the L2 requests per launch (TCC_REQ_sum) and the HBM-side bytes per launch =
FETCH_SIZE + 1/2 x the streamed input bytes (HEADERS x STREAM_BYTES, which
FETCH_SIZE counts at half on gfx950) + WRITE_SIZE.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_name(full):
    m = re.search(r"(k_\w+)", full)
    return m.group(1) if m else full.split("(")[0]


def collect(out, skip=0):
    """skip: leave out each kernel's first `skip` launches (a context's first
    apply sizes its sets cold; the steady state is what the bench line
    describes), in the kernel trace's durations and in every counter pass"""
    res = {"kernels": {}, "counters": {}, "skipped_first_launches": skip}
    kt = glob.glob(os.path.join(out, "kt", "*kernel_trace.csv"))
    ks = glob.glob(os.path.join(out, "kt", "*kernel_stats.csv"))
    if kt:
        durs = defaultdict(list)
        for r in sorted(csv.DictReader(open(kt[0])), key=lambda r: int(r["Start_Timestamp"])):
            if "cfc::" in r["Kernel_Name"]:
                durs[kernel_name(r["Kernel_Name"])].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        for k, v in durs.items():
            v = v[skip:] if len(v) > skip else v
            res["kernels"][k] = {"calls": len(v), "avg_ms": sum(v) / len(v)}
    elif ks:
        for r in csv.DictReader(open(ks[0])):
            if "cfc::" in r["Name"]:
                res["kernels"][kernel_name(r["Name"])] = {
                    "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(out, "pmc*", "*counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if "cfc::" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        for r in rows:
            vals[kernel_name(r["Kernel_Name"])][r["Counter_Name"]].append(
                float(r["Counter_Value"]))
    for k, cs in vals.items():
        res["counters"][k] = {c: sum(v[skip:] if len(v) > skip else v) /
                              len(v[skip:] if len(v) > skip else v) for c, v in cs.items()}
    return res


def derived(c):
    d = {}
    if "FETCH_SIZE" in c:
        d["hbm_fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in c:
        d["hbm_write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                d[k + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    return d


def save(out, dst, res):
    import shutil
    os.makedirs(dst, exist_ok=True)
    ks = glob.glob(os.path.join(out, "kt", "*kernel_stats.csv"))
    if ks:
        shutil.copy(ks[0], os.path.join(dst, "kernel_stats.csv"))
    for f in sorted(glob.glob(os.path.join(out, "pmc*", "*counter_collection.csv"))):
        name = os.path.basename(os.path.dirname(f)) + ".csv"
        with open(f) as fi, open(os.path.join(dst, name), "w", newline="") as fo:
            r = csv.DictReader(fi)
            w = csv.DictWriter(fo, fieldnames=r.fieldnames)
            w.writeheader()
            for row in r:
                if "cfc::" in row["Kernel_Name"]:
                    w.writerow(row)
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(res, f, indent=1)


def record(res, workload, mode, layout, specs, source):
    """Write this configuration's per-kernel entry into profiles/pmc_traffic.json."""
    variant = "lookup"
    if specs and specs[0].startswith("variant="):
        variant = specs[0].split("=", 1)[1]
        specs = specs[1:]
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        db = json.load(open(path))
        entries = db.get("entries", [])
    except (OSError, ValueError):
        entries = []
    kern = {}
    for spec in specs:
        k, n, sb = spec.split(":")
        c = res["counters"].get(k)
        if c is None or "TCC_REQ_sum" not in c or k not in res["kernels"]:
            continue
        kern[k] = {
            "headers": int(n),
            "stream_read_bytes_per_header": float(sb),
            "l2_requests_per_launch": c["TCC_REQ_sum"],
            "l2_hits_per_launch": c.get("TCC_HIT_sum"),
            "l2_misses_per_launch": c.get("TCC_MISS_sum"),
            "hbm_bytes_per_launch": (c["FETCH_SIZE"] * 1024 + 0.5 * int(n) * float(sb)
                                     + c["WRITE_SIZE"] * 1024),
            "write_bytes_per_launch": c["WRITE_SIZE"] * 1024,
            "avg_ms": res["kernels"][k]["avg_ms"],
            "calls": res["kernels"][k]["calls"],
        }
    e = {"workload": workload, "mode": mode, "lpm4_layout": layout, "variant": variant,
         "source": source, "kernels": kern}
    entries = [x for x in entries
               if (x["workload"], x["mode"], x["lpm4_layout"], x.get("variant", "lookup")) !=
               (workload, mode, layout, variant)]
    entries.append(e)
    with open(path, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    return e


def main(argv):
    a = list(argv)
    rec = dst = None
    if "--record" in a:
        i = a.index("--record")
        rec = a[i + 1:]
        a = a[:i]
    if "--save" in a:
        i = a.index("--save")
        dst = a[i + 1]
        a = a[:i] + a[i + 2:]
    skip = 0
    if "--skip" in a:
        i = a.index("--skip")
        skip = int(a[i + 1])
        a = a[:i] + a[i + 2:]
    out = a[0]
    kname = a[1] if len(a) > 1 else "k_classify_v4"
    res = collect(out, skip)
    for k, c in res["counters"].items():
        res.setdefault("derived", {})[k] = derived(c)
    res["focus"] = kname
    if dst:
        save(out, dst, res)
    if rec:
        res["recorded"] = record(res, rec[0], rec[1], rec[2], rec[3:],
                                 os.path.relpath(dst or out, ROOT))
    print(json.dumps({"kernels": res["kernels"],
                      "counters": res["counters"].get(kname),
                      "derived": res.get("derived", {}).get(kname)}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
