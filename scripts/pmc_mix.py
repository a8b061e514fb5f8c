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
    key = "SQ_WAVE_CYCLES" if any("SQ_WAVE_CYCLES" in c for c in acc.values()) else None
    if key is None:  # a pass without the SQ mix: every counter per dispatch
        rows = sorted(acc.items(), key=lambda kv: -sum(kv[1].values()))[:top]
        names = sorted({n for _, c in rows for n in c})
        print("| kernel | dispatches | " + " | ".join(f"{n} / disp" for n in names) + " | derived |")
        print("|---|---|" + "---|" * len(names) + "---|")
        for k, c in rows:
            n = len(disp[k])
            der = []
            if "FETCH_SIZE" in c:  # KiB per dispatch; gfx950 counts wide reads at half
                der.append(f"fetch x2 {2 * c['FETCH_SIZE'] / n / 1024:.2f} MB")
            if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
                der.append(f"LDS conflict {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
                der.append(f"MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * c['GRBM_GUI_ACTIVE'] / 8):.3f}")
            if "SQ_WAVES" in c and c.get("GRBM_GUI_ACTIVE"):
                der.append(f"waves {c['SQ_WAVES'] / n:.0f}")
            print(f"| `{k[:60]}` | {n} | " + " | ".join(f"{c.get(x, 0) / n:.4g}" for x in names)
                  + " | " + "; ".join(der) + " |")
        return
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
