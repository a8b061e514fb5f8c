"""Per-launch HBM traffic and MFMA busy of the benched kernels from rocprofv3
PMC csv passes (scripts/gpu_evidence_r2.sh: FETCH_SIZE, WRITE_SIZE and
SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE + SQ_WAVE_CYCLES,
each its own run, large-v3 bf16, 32 clips, 8 decode steps).

usage: python scripts/pmc_report.py <gpurun_out dir> <tag> [--md out.md] [--traffic-json f]

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE (KiB)
reports half the bytes of a wide coalesced (16 B/lane) read on gfx950, so it
is doubled (every kernel listed streams its operands with 16-B lane loads);
WRITE_SIZE (KiB) is taken as is. GRBM_GUI_ACTIVE is summed over the 8 XCDs:
chip cycles = GRBM_GUI_ACTIVE / 8. MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs x chip cycles) -- the fraction of the dispatch's cycles in which
an average SIMD's MFMA pipe was busy.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# kernel-name substring -> class; the first match wins
CLASSES = [
    ("dec_attn_kernelIDF16bLb0E", "dec_attn_cross"),
    ("dec_attn_kernelIDF16bLb1E", "dec_attn_self"),
    ("dec_xattn_kernel", "dec_xattn_grouped"),
    ("gemm_splitk", "gemm_splitk"),
    ("gemm_skinny", "gemm_skinny"),
    ("ln_dec_kernel", "ln_dec"),
    ("gemm_big", "gemm_big"),
    ("enc_attn_kernel", "enc_attn"),
]

# large-v3, 32 rows: algorithmic bytes per launch of the decode kernels whose
# shape the (class, grid) key identifies uniquely (weights + K/V streamed
# once; activations and split-K slabs are small beside them and not counted)
D, FF, T, ROWS, VOCAB = 1280, 5120, 1500, 32, 51866
ALGO = {
    "dec_attn_cross": 2 * ROWS * T * D * 2,  # K and V of every clip, f16
}


def classify(name):
    return next((c for k, c in CLASSES if k in name), None)


def load(path, counters):
    """{(class, grid, name): {counter: [values per dispatch]}, ...} plus durations."""
    vals = defaultdict(lambda: defaultdict(dict))
    dur = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            cls = classify(r["Kernel_Name"])
            if cls is None or r["Counter_Name"] not in counters:
                continue
            key = (cls, int(r["Grid_Size"]), r["Kernel_Name"])
            vals[key][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


def main():
    root, tag = sys.argv[1], sys.argv[2]
    def pdir(c):  # (round 2: pmc_<tag>_<c>; scripts/gpu_run.sh: <tag>_pmc_<c>)
        a = os.path.join(root, f"pmc_{tag}_{c}")
        return a if os.path.isdir(a) else os.path.join(root, f"{tag}_pmc_{c}")

    fetch, _ = load(pdir("FETCH_SIZE"), {"FETCH_SIZE"})
    write, _ = load(pdir("WRITE_SIZE"), {"WRITE_SIZE"})
    mf, mdur = load(pdir("MFMA"),
                    {"SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
                     "SQ_WAVE_CYCLES"})
    rows = []
    for key in sorted(set(fetch) | set(write) | set(mf), key=lambda k: (k[0], k[1])):
        cls, grid, name = key
        fd = fetch.get(key, {})
        wd = write.get(key, {})
        md = mf.get(key, {})
        n = max(len(fd), len(wd), len(md))
        fb = 2 * 1024 * sum(v["FETCH_SIZE"] for v in fd.values()) / max(1, len(fd))
        wb = 1024 * sum(v["WRITE_SIZE"] for v in wd.values()) / max(1, len(wd))
        busy = None
        clock = None
        if md and cls in ("gemm_big", "enc_attn"):
            mb = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for v in md.values())
            gu = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in md.values()) / 8
            ns = sum(mdur[d] for d in md)
            busy = mb / (1024 * gu) if gu else None
            clock = gu / ns if ns else None  # GHz (cycles per ns)
        rows.append({"class": cls, "grid": grid, "kernel": name[:80], "dispatches": n,
                     "fetch_bytes_x2": round(fb), "write_bytes": round(wb),
                     "bytes_per_launch": round(fb + wb), "algorithmic_bytes": ALGO.get(cls),
                     "mfma_busy": busy, "clock_ghz": clock})
    out = ["| class | grid | dispatches | FETCH_SIZE x2 MB | WRITE MB | algorithmic MB | "
           "traffic / algorithmic | MFMA busy | clock GHz |", "|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        a = r["algorithmic_bytes"]
        out.append(f"| {r['class']} | {r['grid']} | {r['dispatches']} | "
                   f"{r['fetch_bytes_x2'] / 1e6:.2f} | {r['write_bytes'] / 1e6:.3f} | "
                   f"{a / 1e6 if a else float('nan'):.1f} | "
                   f"{(r['bytes_per_launch'] / a) if a else float('nan'):.3f} | "
                   f"{r['mfma_busy'] if r['mfma_busy'] is not None else float('nan'):.3f} | "
                   f"{r['clock_ghz'] if r['clock_ghz'] is not None else float('nan'):.2f} |")
    text = "\n".join(out)
    print(text)
    if "--md" in sys.argv:
        open(sys.argv[sys.argv.index("--md") + 1], "w").write(text + "\n")
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    if "--traffic-json" in sys.argv:
        dst = sys.argv[sys.argv.index("--traffic-json") + 1]
        cur = json.load(open(dst)) if os.path.exists(dst) else {}
        for cls in ("dec_attn_cross", "dec_attn_self"):
            rs = [r for r in rows if r["class"] == cls]
            if rs:
                tot = sum(r["bytes_per_launch"] * r["dispatches"] for r in rs)
                cur[f"large-v3:{cls}:32"] = round(tot / sum(r["dispatches"] for r in rs))
        json.dump(cur, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
