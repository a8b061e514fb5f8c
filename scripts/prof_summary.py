"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel
stats table: calls, total ms, average us, share. Usage:
    python scripts/prof_summary.py <results.db> [out.md]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(grid_x), max(grid_y), max(workgroup_x), max(vgpr_count), max(scratch_size) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = ["| kernel | calls | total ms | avg us | min us | max us | share | vgpr | scratch |",
           "|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{r[0][:90]}` | {r[1]} | {r[2] / 1e6:.2f} | {r[3] / 1e3:.2f} | "
                   f"{r[4] / 1e3:.2f} | {r[5] / 1e3:.2f} | {100 * r[2] / tot:.1f}% | {r[9]} | {r[10]} |")
    out.append(f"\ntotal kernel time: {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} dispatches")
    text = "\n".join(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
