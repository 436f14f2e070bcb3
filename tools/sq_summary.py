"""SQ counter ratios per kernel from tools/pmc_bench.sh output dirs -> one JSON (committed under profiles/).
Ratios are of SQ_WAVE_CYCLES (the cycles the kernel's waves were resident): VALU / LDS instruction issue,
waits on anything (s_waitcnt) and the part of them on LDS (lgkm); vm waits ~= wait_any - wait_lds.
Usage: python3 tools/sq_summary.py OUT.json gpurun_out/pmcb_fixed gpurun_out/pmcb_mixed ..."""
import csv
import glob
import json
import os
import sys


def load(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


out = {"note": __doc__.split("Usage")[0].strip(), "configs": {}}
for d in sys.argv[2:]:
    cfg = os.path.basename(d.rstrip("/")).replace("pmcb_", "")
    res = {}
    for k, c in load(d).items():
        wc = c.get("SQ_WAVE_CYCLES")
        if not wc:
            continue
        r = {"valu_issue": c["SQ_ACTIVE_INST_VALU"] / wc, "lds_issue": c["SQ_ACTIVE_INST_LDS"] / wc,
             "wait_any": c["SQ_WAIT_ANY"] / wc, "wait_lds": c["SQ_WAIT_INST_LDS"] / wc,
             "lds_bank_conflict_of_lds_active": c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"],
             "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
             "lds_insts_per_wave": c["SQ_INSTS_LDS"] / c["SQ_WAVES"]}
        r["wait_vm_approx"] = r["wait_any"] - r["wait_lds"]
        res[k] = {"ratios": {a: round(b, 4) for a, b in r.items()}, "raw": c}
    out["configs"][cfg] = res
json.dump(out, open(sys.argv[1], "w"), indent=1)
for cfg, res in out["configs"].items():
    for k, v in res.items():
        print(cfg, k, v["ratios"])
