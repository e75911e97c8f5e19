"""MFMA utilisation and wait fractions per phase kernel from the SQ pass of
tools/profile_r02.sh (profiles/<round>_sq_counters.txt, one line per
(pass, kernel) with per-launch averages of the counters):

    mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
        (MFMA-busy SIMD cycles over the SIMD cycles of the launch; GRBM_GUI_ACTIVE
         sums the 8 XCDs' busy cycles, MI355X_MICROARCH.md "DVFS give-back")
    wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked in s_waitcnt / barriers)

    python tools/sq_summary.py profiles/r02_sq_counters.txt > profiles/r02_mfma_busy.json
"""
import ast
import json
import sys

out = {"formula": __doc__.split("\n\n")[1].strip(), "kernels": {}}
for line in open(sys.argv[1]):
    name, kernel, rest = line.split(" ", 2)
    if "replay" in kernel:
        continue
    d = ast.literal_eval(rest)
    simd_cycles = d["GRBM_GUI_ACTIVE"] / 8 * 1024
    out["kernels"][f"{name}/{kernel}"] = {
        "mfma_busy_frac": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles, 4),
        "wait_frac": round(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 3),
        "counters": d}
print(json.dumps(out, indent=1))
