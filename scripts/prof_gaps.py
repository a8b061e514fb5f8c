"""Per-kernel durations AND the idle gaps in front of each kernel from a
rocprofv3 kernel-trace database (rocpd SQLite): where the wall time of a
launch chain goes besides the kernels themselves. Usage:
    python scripts/prof_gaps.py <results.db> [steps]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    prev_end = None
    for name, st, en in rows:
        a = agg[name]
        a[0] += 1
        a[1] += en - st
        if prev_end is not None and st > prev_end:
            a[2] += st - prev_end
        prev_end = max(en, prev_end or en)
    tot_k = sum(a[1] for a in agg.values())
    tot_g = sum(a[2] for a in agg.values())
    print(f"wall {(rows[-1][2] - rows[0][1]) / 1e6 / steps:.2f} ms/step, kernels {tot_k / 1e6 / steps:.2f}, "
          f"gaps {tot_g / 1e6 / steps:.2f}, dispatches {len(rows) / steps:.0f}/step")
    print("| kernel | calls/step | avg us | gap-before avg us | kernel ms/step | gap ms/step |")
    print("|---|---|---|---|---|---|")
    for name, a in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:24]:
        print(f"| `{name[:70]}` | {a[0] / steps:.0f} | {a[1] / a[0] / 1e3:.2f} | {a[2] / a[0] / 1e3:.2f} | "
              f"{a[1] / 1e6 / steps:.2f} | {a[2] / 1e6 / steps:.2f} |")
    # the largest single idle gaps and where they fall: batch b = number of
    # mel_frames_kernel launches (one per batch) before the gap; batch 0 is
    # before the first batch's mel (start-up: weights, PCM synthesis, uploads)
    gaps = []
    batch = 0
    prev = None
    for name, st, en in rows:
        if prev is not None and st > prev[2]:
            gaps.append((st - prev[2], batch, prev[0], name, (prev[2] - rows[0][1]) / 1e6))
        if "mel_frames_kernel" in name:
            batch += 1
        if prev is None or en > prev[2]:
            prev = (name, st, en)
    print()
    print(f"largest single gaps ({batch} batches in the trace; 'mels before' = batches started "
          f"before the gap, 0 = start-up before the first batch):")
    print("| gap ms | at ms | mels before | kernel before | kernel after |")
    print("|---|---|---|---|---|")
    for g, b, pa, na, at in sorted(gaps, reverse=True)[:10]:
        print(f"| {g / 1e6:.2f} | {at:.1f} | {b} | `{pa[:48]}` | `{na[:48]}` |")


if __name__ == "__main__":
    main()
