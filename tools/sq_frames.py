"""SQ counter summary of the compressed-table scan's decoders (tools/pmc_tz.sh output: two --pmc passes) -> one JSON
under profiles/: per kernel the counters averaged over its dispatches, per wave, and -- for k_ts_decode -- per
frame (the bench table's 65,536 Snappy frames) and per frame element (106.5 elements a frame on average, measured
on the generator's frames). SQ cycle counters count in units of 4 cycles (quad-cycles) on gfx950.
Usage: python3 tools/sq_frames.py OUT.json gpurun_out/pmc/a gpurun_out/pmc/b"""
import csv
import glob
import json
import os
import sys

FRAMES = 65536
ELEMS_PER_FRAME = 106.5


def load(dirs):
    per = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("lcrc_dev::", "")
                per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main(out, *dirs):
    per = load(dirs)
    res = {"source": "tools/pmc_tz.sh (bench.py --config table --compression 1), rocprofv3 --pmc, two passes",
           "note": "instruction counts are per dispatch; *_per_frame divide k_ts_decode's by 65,536 frames",
           "kernels": {}}
    for k in ("k_ts_decode", "k_ts_open2"):
        c = per.get(k)
        if not c:
            continue
        waves = c.get("SQ_WAVES", 0) or 1
        e = {name: round(v) for name, v in c.items()}
        e["per_wave"] = {n: round(c[n] / waves, 1) for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                             "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY") if n in c}
        if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_ANY" in c:
            e["issue_fraction"] = round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3)
        if k == "k_ts_decode":
            e["per_frame"] = {n: round(c[n] / FRAMES, 1) for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS")
                              if n in c}
            e["per_element_per_frame"] = {n: round(v / ELEMS_PER_FRAME, 2) for n, v in e["per_frame"].items()}
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1)[:3000])


if __name__ == "__main__":
    main(*sys.argv[1:])
