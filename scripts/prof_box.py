"""On the GPU box, after a rocprofv3 --kernel-trace run: summarise every
trace database under a directory into markdown next to it (per-kernel stats
as scripts/prof_summary.py, launch gaps as scripts/prof_gaps.py), then delete
the databases (they exceed what gpurun copies back). Usage:
    python scripts/prof_box.py <rocprofv3 -d dir> [steps]
"""
import contextlib
import glob
import io
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import prof_gaps  # noqa: E402
import prof_summary  # noqa: E402


def main():
    d = sys.argv[1]
    steps = sys.argv[2] if len(sys.argv) > 2 else "1"
    dbs = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
    if not dbs:
        print(f"prof_box: no trace database under {d}", file=sys.stderr)
        return 1
    for i, db in enumerate(dbs):
        base = d.rstrip("/") + (f"_{i}" if len(dbs) > 1 else "")
        sys.argv = ["prof_summary", db, base + "_kernel_stats.md"]
        prof_summary.main()
        buf = io.StringIO()
        sys.argv = ["prof_gaps", db, steps]
        with contextlib.redirect_stdout(buf):
            prof_gaps.main()
        open(base + "_gaps.md", "w").write(buf.getvalue())
        os.remove(db)
    return 0


if __name__ == "__main__":
    sys.exit(main())
