"""Summarise rocprofv3 SQ counter passes (tools/gpu_round.sh sq) per kernel: per-launch averages and derived
ratios (issued VALU per wave, wait/active fractions of wave cycles)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "sq*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            k = k.split("<")[0] + ("<" + r["Kernel_Name"].split("<", 1)[1].split(">")[0] + ">" if "<" in r["Kernel_Name"] else "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(d):
    acc = load(d)
    out = {}
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        w = avg.get("SQ_WAVES", 0)
        wc = avg.get("SQ_WAVE_CYCLES", 0)
        der = {}
        if w:
            der["valu_insts_per_wave"] = avg.get("SQ_INSTS_VALU", 0) / w
            der["lds_insts_per_wave"] = avg.get("SQ_INSTS_LDS", 0) / w
            der["salu_insts_per_wave"] = avg.get("SQ_INSTS_SALU", 0) / w
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in avg:
                    der[c.lower() + "_frac_of_wave_cycles"] = avg[c] / wc
        out[k] = {"avg": avg, "derived": der, "launches": len(next(iter(cs.values())))}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
