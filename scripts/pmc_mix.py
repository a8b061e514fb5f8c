"""Instruction-mix / stall summary of a rocprofv3 --pmc csv pass (scripts/gpu_run.sh
pmcb5): per kernel, the counters averaged per dispatch and the fractions of the
waves' cycles that were waiting on memory / barriers (SQ_WAIT_ANY), stalled at
issue (SQ_WAIT_INST_ANY) and issuing VALU (SQ_ACTIVE_INST_VALU). Usage:
    python scripts/pmc_mix.py <rocprofv3 -d dir> [top]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:top]
    print("| kernel | dispatches | wave cycles / disp | wait (mem/barrier) | issue stall | VALU active | VALU insts / disp | LDS insts / disp |")
    print("|---|---|---|---|---|---|---|---|")
    for k, c in rows:
        n = len(disp[k])
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"| `{k[:60]}` | {n} | {wc / n:.3g} | {c.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f} | "
              f"{c.get('SQ_INSTS_VALU', 0) / n:.3g} | {c.get('SQ_INSTS_LDS', 0) / n:.3g} |")


if __name__ == "__main__":
    main()
