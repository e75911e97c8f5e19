"""Per-kernel average of every counter in a tools/pmc_pass.sh database."""
import glob
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_summary import PHASE_KERNELS, short  # noqa: E402

for name in sys.argv[1:]:
    db = sqlite3.connect(sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc", name, "**", "*.db"),
                                          recursive=True))[-1])
    res = {}
    for k, c, n, v in db.execute("select kernel_name, counter_name, count(*), avg(value) from counters_collection "
                                 "group by kernel_name, counter_name"):
        if short(k) in PHASE_KERNELS:
            res.setdefault(short(k), {})[c] = v
    for k, d in res.items():
        print(name, k, {c: round(v) for c, v in sorted(d.items())})
