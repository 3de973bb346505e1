"""One bench step's kernels in launch order from a rocprofv3 kernel trace:
start offset from the step's classify launch, duration, grid, and the idle
gap before each (host waits show as gaps).

usage: python3 scripts/step_timeline.py <kt dir> [step index from the end, default 1]
"""
import csv
import glob
import re
import sys


def short(name):
    """the kernel's own name out of a demangled signature"""
    m = re.search(r"\b(k_\w+)", name)
    if m:
        return m.group(1)
    m = re.search(r"(rocprim::[\w:]*?detail::\w+|__amd_\w+|hipcub::\w+)", name)
    return m.group(1) if m else name[:50]


def main(d, back=1):
    f = glob.glob(f"{d}/*kernel_trace.csv")[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith("k_classify")]
    a = starts[-back - 1] if back < len(starts) else starts[0]
    b = starts[-back] if back else len(rows)
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    tot = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = short(r["Kernel_Name"])
        grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:7.1f}"
              f"  grid {grid:>10}  {name}")
        tot += e - s
        prev_end = max(prev_end, e)
    print(f"step span {(prev_end - t0) / 1e3:.1f} us, kernels {tot / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
