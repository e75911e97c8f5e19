"""MFMA utilisation and wait fractions per phase kernel from SQ counter passes
(tools/pmc_read.py output, one line per (pass, kernel) with per-launch
averages; passes named sq_<cfg>_<prec> (round 2: one pass) or sqa_/sqb_<cfg>_<prec>
(round 4: MFMA-busy + GRBM in one pass, wave / wait cycles in another; lines of
the same <cfg>_<prec> are merged):

    mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
        (MFMA-busy SIMD cycles over the SIMD cycles of the launch; GRBM_GUI_ACTIVE
         sums the 8 XCDs' busy cycles, MI355X_MICROARCH.md "DVFS give-back")
    wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked in s_waitcnt / barriers)

    python tools/sq_summary.py profiles/r04_sq_counters.txt > profiles/r04_mfma_busy.json
"""
import ast
import json
import sys

out = {"formula": __doc__.split("\n\n")[1].strip(), "kernels": {}}
merged = {}
for line in open(sys.argv[1]):
    name, kernel, rest = line.split(" ", 2)
    if "replay" in kernel:
        continue
    cfg = name.split("_", 1)[1]
    merged.setdefault(f"{cfg}/{kernel}", {}).update(ast.literal_eval(rest))
for key, d in merged.items():
    e = {"counters": d}
    if "GRBM_GUI_ACTIVE" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
        e["mfma_busy_frac"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
        e["wait_frac"] = round(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 3)
    out["kernels"][key] = e
print(json.dumps(out, indent=1))
