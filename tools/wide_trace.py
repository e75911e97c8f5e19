"""Per-launch durations of the large-batch stage path from a rocprofv3
kernel-trace CSV: steps are cut at each sac_wide_gather dispatch and every
position of the step's launch sequence is averaged over the steps.
    python tools/wide_trace.py <kernel_trace.csv> [skip_steps]"""
import csv
import sys
from collections import defaultdict


def main(path, skip=10):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "sac_wide_gather" in name:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((name.split("(")[0][:48], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    steps = [s for s in steps[skip:-1] if len(s) == len(steps[skip])]
    if not steps:
        print("no complete steps")
        return
    n = len(steps[0])
    dur = defaultdict(float)
    gap = defaultdict(float)
    for s in steps:
        for i, (nm, a, b) in enumerate(s):
            dur[i] += (b - a) / 1e3
            if i:
                gap[i] += (a - s[i - 1][2]) / 1e3
    tot = sum((s[-1][2] - s[0][1]) / 1e3 for s in steps) / len(steps)
    print(f"{len(steps)} steps, {n} launches per step, step span {tot:.1f} us")
    for i in range(n):
        print(f"  {i:2d} {steps[0][i][0]:48s} {dur[i] / len(steps):8.2f} us  (gap before {gap[i] / len(steps):5.2f})")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
