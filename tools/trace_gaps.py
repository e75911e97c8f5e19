"""Kernel-trace timeline of a bench run (rocpd db): per-kernel average
duration and the idle gap before each kernel kind (start - previous end)."""
import collections
import glob
import sqlite3
import sys

db = sqlite3.connect(sorted(glob.glob(sys.argv[1] + "/**/*.db", recursive=True))[-1])
rows = list(db.execute("select name, start, end from kernels order by start"))
short = lambda n: n.split("(")[0].replace("void ", "")[:40]  # noqa: E731
rows = [(short(n), s, e) for n, s, e in rows if "sac_" in n]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i, (n, s, e) in enumerate(rows):
    dur[n].append((e - s) / 1e3)
    if i:
        gap[n].append((s - rows[i - 1][2]) / 1e3)
for n in dur:
    d, g = sorted(dur[n]), sorted(gap[n])
    print(f"{n:42s} n={len(d):5d} dur median {d[len(d) // 2]:7.2f} us   gap before median {g[len(g) // 2] if g else 0:6.2f} us")
span = (rows[-1][2] - rows[0][1]) / 1e3
print(f"span {span:.1f} us, sum of durations {sum(sum(v) for v in dur.values()):.1f} us over {len(rows)} kernels")
