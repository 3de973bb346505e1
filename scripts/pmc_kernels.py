"""Per-kernel averages of the PMC passes of scripts/gpu.sh (pmc step):
every counter per launch, for the kernels whose name matches a pattern.

    python scripts/pmc_kernels.py gpurun_out/r4q/c5ct 'k_ord_|k_cta_|k_ct_'
"""
import collections
import csv
import glob
import re
import sys


def main():
    d, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(f"{d}/pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)(<[^(]*>)?\(", r["Kernel_Name"])
            if not m or not pat.search(m.group(1)):
                continue
            key = m.group(1) + (m.group(2) or "")
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(key, r["Counter_Name"])] += 1
    for k in sorted(tot):
        print(k)
        for c, v in sorted(tot[k].items()):
            print(f"    {c:24s} {v / n[(k, c)]:16.4g}")


if __name__ == "__main__":
    main()
