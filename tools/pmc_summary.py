"""Condense a tools/profile_round.sh run (rocprofv3 rocpd databases under
gpurun_out/prof/) into committed per-round summaries:

    profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats (top_kernels view)
    profiles/<round>_pmc.json           per-kernel average HBM-side bytes per launch

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
collected in separate passes (they do not fit one TCC pass), are reported in
KiB, and on gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane)
coalesced reads, so it is doubled; WRITE_SIZE is taken as is.

    python tools/pmc_summary.py r01 [gpurun_out/prof]
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASE_KERNELS = ("sac_target_critic", "sac_critic_update", "sac_actor", "sac_actor_update",
                 "replay_gather_records_kernel", "replay_gather_kernel",
                 "replay_sample_kernel", "replay_push_kernel", "sac_policy_act_kernel",
                 "sac_wide_stage", "sac_wide_gather", "sac_wide_head")


def short(name: str) -> str:
    for k in PHASE_KERNELS:
        if k in name and not (k == "sac_actor" and "sac_actor_update" in name):
            return k
    return name[:80]


def one_db(pattern: str) -> sqlite3.Connection:
    dbs = sorted(glob.glob(pattern, recursive=True))
    if not dbs:
        raise SystemExit(f"no database matches {pattern}")
    return sqlite3.connect(dbs[-1])


def counter_avg(db: sqlite3.Connection, counter: str):
    out = {}
    for name, n, avg in db.execute(
            "select kernel_name, count(*), avg(value) from counters_collection where counter_name = ? "
            "group by kernel_name", (counter,)):
        out[short(name)] = (n, avg)
    return out


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("round", nargs="?", default="r01")
    ap.add_argument("src", nargs="?", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--tag", default="", help="suffix of the output files (e.g. _fp32, _gather)")
    ap.add_argument("--config", default="c2", help="bench config the profile ran (or 'gather')")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles"), help="output directory")
    a = ap.parse_args()
    rnd, src, tag = a.round, a.src, a.tag
    dst = a.dst
    os.makedirs(dst, exist_ok=True)

    kt = one_db(os.path.join(src, "kt", "**", "*.db"))
    rows = list(kt.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(os.path.join(dst, f"{rnd}_kernel_stats{tag}.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for name, calls, tot, avg, pct in rows:
            w.writerow([short(name), calls, round(tot, 3), round(avg, 3), round(pct, 3)])

    fetch = counter_avg(one_db(os.path.join(src, "fetch", "**", "*.db")), "FETCH_SIZE")
    write = counter_avg(one_db(os.path.join(src, "write", "**", "*.db")), "WRITE_SIZE")
    durations = {short(n): avg for n, _, _, avg, _ in rows}
    summary = {"config": a.config, "precision": a.precision,
               "source": "rocprofv3 --kernel-trace --stats; separate --pmc FETCH_SIZE / --pmc WRITE_SIZE passes",
               "correction": "fetch_bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950 wide-read undercount); "
                             "write_bytes = WRITE_SIZE KiB x 1024",
               "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if k not in PHASE_KERNELS:
            continue
        fb = 2.0 * fetch.get(k, (0, 0.0))[1] * 1024.0
        wb = write.get(k, (0, 0.0))[1] * 1024.0
        summary["kernels"][k] = {"launches_sampled": fetch.get(k, (0, 0))[0], "fetch_bytes": round(fb),
                                 "write_bytes": round(wb), "hbm_bytes_per_launch": round(fb + wb),
                                 "avg_us_kernel_trace": durations.get(k)}
    with open(os.path.join(dst, f"{rnd}_pmc{tag}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
