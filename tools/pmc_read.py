"""Per-kernel average of every counter in a tools/pmc_pass.sh database."""
import glob
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_summary import PHASE_KERNELS, short  # noqa: E402

# a NAME is a directory under gpurun_out/pmc, or a path to a rocprofv3 output directory
for name in sys.argv[1:]:
    d = name if os.path.isdir(name) else os.path.join(ROOT, "gpurun_out", "pmc", name)
    db = sqlite3.connect(sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))[-1])
    name = os.path.basename(os.path.normpath(name))
    res = {}
    for k, c, n, v in db.execute("select kernel_name, counter_name, count(*), avg(value) from counters_collection "
                                 "group by kernel_name, counter_name"):
        if short(k) in PHASE_KERNELS:
            res.setdefault(short(k), {})[c] = v
    for k, d in res.items():
        print(name, k, {c: round(v) for c, v in sorted(d.items())})
