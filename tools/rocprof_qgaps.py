"""Gaps of the busiest queue in a rocprofv3 kernel trace (diagnostic): every
idle interval of the main queue longer than --min-ms, the kernels around
it, and what the other queues ran inside it.

  python -m tools.rocprof_qgaps <results.db> --min-ms 2
"""
from __future__ import annotations

import argparse
import collections
import sqlite3

from tools.rocprof_summary import _short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-ms", type=float, default=2.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    busy = collections.Counter()
    for n, s, e, q in ks:
        busy[q] += e - s
    mq = busy.most_common(1)[0][0]
    main = [k for k in ks if k[3] == mq]
    print(f"main queue {mq}: {len(main)} kernels; queues {dict(busy)}")
    for prev, cur in zip(main, main[1:]):
        gap = (cur[1] - prev[2]) / 1e6
        if gap < a.min_ms:
            continue
        inside = [k for k in ks if k[3] != mq and k[2] > prev[2] and k[1] < cur[1]]
        occ = collections.Counter()
        for n, s, e, q in inside:
            occ[(q, _short(n, 40))] += (min(e, cur[1]) - max(s, prev[2])) / 1e6
        print(f"gap {gap:6.2f} ms after {_short(prev[0], 40)} before {_short(cur[0], 40)}; "
              f"other queues inside: {sum(occ.values()):.2f} ms")
        for (q, n), t in occ.most_common(6):
            print(f"    q{q} {n:40s} {t:6.2f} ms")


if __name__ == "__main__":
    main()
