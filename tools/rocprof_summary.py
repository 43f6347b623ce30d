"""Summarise a rocprofv3 --kernel-trace --stats run into the table kept under
profiles/ (per kernel: calls, total ms, average us, share).

  python -m tools.rocprof_summary <results.db | kernel_stats.csv> [--top N]

Reads either the rocpd SQLite database rocprofv3 writes by default or the
`*_kernel_stats.csv` of `--output-format csv`.
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3


def _short(name: str, width: int = 80) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name if len(name) <= width else name[: width - 3] + "..."


def load(path: str, last_ms: float = 0.0):
    rows = []
    if path.endswith(".db") and last_ms > 0:
        # only the last `last_ms` of the trace (the timed region of a bench run)
        c = sqlite3.connect(path)
        k = list(c.execute("select name, start, end from kernels"))
        t_end = max(e for _, _, e in k)
        agg = {}
        for n, s0, e in k:
            if s0 >= t_end - last_ms * 1e6:
                a = agg.setdefault(n, [0, 0.0])
                a[0] += 1
                a[1] += (e - s0) / 1e6
        tot = sum(v[1] for v in agg.values())
        rows = [(n, v[0], v[1], v[1] / v[0] * 1e3, 100 * v[1] / tot) for n, v in agg.items()]
    elif path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, calls, total, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            rows.append((name, int(calls), float(total) / 1e3, float(avg), float(pct)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                             float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return sorted(rows, key=lambda r: -r[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--last-ms", type=float, default=0.0,
                    help="only kernels that start in the last N ms of the trace")
    a = ap.parse_args()
    rows = load(a.path, a.last_ms)
    print(f"{'kernel':80s} {'calls':>6s} {'total ms':>9s} {'avg us':>9s} {'%':>6s}")
    for name, calls, total, avg, pct in rows[: a.top]:
        print(f"{_short(name):80s} {calls:6d} {total:9.2f} {avg:9.1f} {pct:6.2f}")


if __name__ == "__main__":
    main()
