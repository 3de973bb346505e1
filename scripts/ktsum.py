"""Per-kernel summary of a rocprofv3 --kernel-trace --stats directory:
name, calls, average and total ms (largest total first).

    python scripts/ktsum.py gpurun_out/r4m/c5ct/kt [N]
"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda x: -float(x["TotalDurationNs"]))
    for x in rows[:n]:
        print(f"{x['Name'][:72]:72s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e6:8.3f} "
              f"{float(x['TotalDurationNs']) / 1e6:9.2f}")


if __name__ == "__main__":
    main()
