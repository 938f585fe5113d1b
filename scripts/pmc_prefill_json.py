"""Summarise the prefill GEMM PMC passes (scripts/pmc_prefill.sh) into profiles/<round>/pmc_prefill.json.
Normalisation (MI355X_MICROARCH §rocprofv3, DVFS note): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
kernel cycles = GRBM_GUI_ACTIVE / 8; SQ_VALU_MFMA_BUSY_CYCLES sums the busy cycles of the 1024 SIMDs
(MFMA util = busy / (cycles x 1024)); SQ_LDS_IDX_ACTIVE sums LDS-array cycles of the 256 CUs.
usage: pmc_prefill_json.py gpurun_out/<tag> profiles/<round>/pmc_prefill.json"""
import collections
import csv
import glob
import json
import sys

root, out = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float)
for f in glob.glob(root + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gemm_x" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
cyc = agg["GRBM_GUI_ACTIVE"] / 8.0
res = {
    "kernel": "k_gemm_x (exact prefill GEMMs, all 18 layers + logits, one T=2048 pass)",
    "mfma_util": round(agg["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4),
    "lds_busy": round(agg["SQ_LDS_IDX_ACTIVE"] / (cyc * 256), 4),
    "lds_bank_conflict_frac": round(agg["SQ_LDS_BANK_CONFLICT"] / agg["SQ_LDS_IDX_ACTIVE"], 4),
    "valu_inst_per_wave_cycle": round(agg["SQ_ACTIVE_INST_VALU"] / agg["SQ_WAVE_CYCLES"], 4),
    "wait_any_frac": round(agg["SQ_WAIT_ANY"] / agg["SQ_WAVE_CYCLES"], 4),
    "raw": {k: v for k, v in sorted(agg.items())},
    "note": "MFMA util counts ISSUED MFMA cycles: the exact path's lane-masked f16 MFMAs carry 4x the useful "
            "products (3/4 of each A row is zero, DESIGN.md §5b)",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "raw"}))
