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
KERNELS = {
    "k_gemm_x4": "exact Q4_0 prefill GEMMs on v_mfma_f32_16x16x4_4b_f16 (all 18 layers + logits, one T=2048 pass): one "
                 "instruction block = one AVX2 lane, every product useful; 3 waves per SIMD (DESIGN.md §5b)",
    "k_gemm_x<": "exact Q4_0 prefill GEMMs (all 18 layers + logits, one T=2048 pass); MFMA util counts ISSUED "
                "MFMA cycles: the lane-masked f16 MFMAs carry 4x the useful products (DESIGN.md §5b)",
    "k_attn_rows": "exact prefill attention, row form (per row, v_fma_mix chains; GHIP_ATT_MX=0)",
    "k_attn_mx": "exact prefill attention on the f32 matrix cores (vec_dot_f16's 32 fmaf chains on "
                 "v_mfma_f32_16x16x4_f32, four K steps per MFMA; DESIGN.md §5b)",
    "k_gemm_kq": "exact K-quant prefill GEMMs (Q4_K_M layout, dense lane-major MFMA; Q6_K issues 2 MFMAs per "
                 "product, the even part and the low bit; DESIGN.md §5c)",
}
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(root + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for k in KERNELS:
            if k in r["Kernel_Name"].replace("ghip::(anonymous namespace)::", ""):
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
res = {}
for k, a in agg.items():
    cyc = a["GRBM_GUI_ACTIVE"] / 8.0
    e = {"kernel": k, "what": KERNELS[k]}
    if cyc > 0:
        e["mfma_util"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4)
        e["lds_busy"] = round(a["SQ_LDS_IDX_ACTIVE"] / (cyc * 256), 4)
    if a["SQ_LDS_IDX_ACTIVE"] > 0:
        e["lds_bank_conflict_frac"] = round(a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"], 4)
    if a["SQ_WAVE_CYCLES"] > 0:
        e["valu_inst_per_wave_cycle"] = round(a["SQ_ACTIVE_INST_VALU"] / a["SQ_WAVE_CYCLES"], 4)
        e["wait_any_frac"] = round(a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], 4)
        e["wait_inst_lds_frac"] = round(a["SQ_WAIT_INST_LDS"] / a["SQ_WAVE_CYCLES"], 4)
    e["raw"] = {c: v for c, v in sorted(a.items())}
    res[k] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: {x: y for x, y in v.items() if x != "raw"} for k, v in res.items()}, indent=1))
