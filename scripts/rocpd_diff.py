"""Per-kernel total-time difference between two rocprofv3 runs (rocpd SQLite format): which kernels
one configuration adds or slows, summed over every dispatch of the run.

    python scripts/rocpd_diff.py gpurun_out/a/run_results.db gpurun_out/b/run_results.db [top]
"""
import collections
import re
import sqlite3
import sys


def totals(db):
    t, n = collections.defaultdict(float), collections.Counter()
    for name, dur in sqlite3.connect(db).execute("select name, duration from kernels"):
        s = re.sub(r"^void ", "", name)
        s = re.sub(r"\(.*", "", s) or name
        s = s.replace("(anonymous namespace)::", "")[:90]
        t[s] += dur / 1e6
        n[s] += 1
    return t, n


def main():
    (ta, na), (tb, nb) = totals(sys.argv[1]), totals(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    print(f"total kernel ms: a {sum(ta.values()):.1f}  b {sum(tb.values()):.1f}")
    for k in sorted(set(ta) | set(tb), key=lambda k: -abs(tb.get(k, 0) - ta.get(k, 0)))[:top]:
        print(f"{tb.get(k, 0) - ta.get(k, 0):+9.2f} ms  a {ta.get(k, 0):9.2f} ({na[k]:5d})  b {tb.get(k, 0):9.2f} ({nb[k]:5d})  {k}")


if __name__ == "__main__":
    main()
