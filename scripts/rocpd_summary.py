"""Per-kernel summary of a rocprofv3 run written in its default rocpd (SQLite) format.

    rocprofv3 --kernel-trace -d gpurun_out/x -o run -- python3 scripts/fa_ab.py
    python scripts/rocpd_summary.py gpurun_out/x/run_results.db [name-regex [phase-marker-regex]]

Groups dispatches by (phase, kernel, grid size) and prints the count and the median / mean duration.
With a phase-marker regex, every run of marker kernels starts a new phase (e.g. ``distribution_``:
the random inputs scripts/fa_ab.py draws for each shape), so shapes with equal grids still come out
as separate rows.
"""

import re
import sqlite3
import statistics
import sys
from collections import defaultdict


def main() -> None:
    db = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    marker = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    con = sqlite3.connect(db)
    groups: dict[tuple[int, str, int], list[int]] = defaultdict(list)
    first: dict[tuple[int, str, int], int] = {}
    phase, inside = 0, False
    rows = con.execute("select name, grid_x, workgroup_x, duration, start from kernels order by start")
    for name, gx, wx, dur, start in rows:
        short = re.sub(r"\(.*", "", name)
        short = re.sub(r"^void ", "", short)
        if marker is not None and marker.search(name):
            if inside:
                phase, inside = phase + 1, False
            continue
        if not pat.search(short):
            continue
        inside = True
        key = (phase, short, gx // max(wx, 1))
        groups[key].append(dur)
        first.setdefault(key, start)
    print(f"{'phase':>5s} {'kernel':70s} {'wgs':>7s} {'n':>6s} {'median us':>10s} {'mean us':>9s}")
    for key in sorted(groups, key=lambda k: first[k]):
        v = groups[key]
        print(f"{key[0]:5d} {key[1][:70]:70s} {key[2]:7d} {len(v):6d} {statistics.median(v) / 1e3:10.1f} "
              f"{statistics.fmean(v) / 1e3:9.1f}")


if __name__ == "__main__":
    main()
