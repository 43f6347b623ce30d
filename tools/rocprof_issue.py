"""Host issue vs device start on the main queue (diagnostic): from a
rocprofv3 --kernel-trace --hip-trace database, for the last `--last-ms` of
the trace, every idle gap of the busiest queue longer than `--min-gap-us`:
the kernel that ends it, the HIP API call that issued it (same correlation
id: its start relative to the gap's start, so a positive value = issued
after the queue went idle = a host-bound gap) and the slowest HIP API calls
the issuing thread made during the gap.

  python -m tools.rocprof_issue <results.db> --last-ms 40 --min-gap-us 30
"""
from __future__ import annotations

import argparse
import collections
import sqlite3

from tools.rocprof_summary import _short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-ms", type=float, default=40.0)
    ap.add_argument("--min-gap-us", type=float, default=30.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end, queue_id, corr_id from kernels order by start"))
    t_end = max(k[2] for k in ks)
    t0 = t_end - a.last_ms * 1e6
    ks = [k for k in ks if k[1] >= t0]
    busy = collections.Counter()
    for n, s, e, q, _ in ks:
        busy[q] += e - s
    mq = busy.most_common(1)[0][0]
    main = [k for k in ks if k[3] == mq]
    regs = list(c.execute("select name, tid, start, end, corr_id from regions "
                          "where start >= ? order by start", (t0 - 50e6,)))
    by_corr = {r[4]: r for r in regs if r[4]}
    by_tid = collections.defaultdict(list)
    for r in regs:
        by_tid[r[1]].append(r)
    print(f"main queue {mq}: {len(main)} kernels, busy {busy[mq] / 1e6:.2f} ms of {a.last_ms} ms")
    tot_gap, host_gap = 0.0, 0.0
    for prev, cur in zip(main, main[1:]):
        gap = (cur[1] - prev[2]) / 1e3
        if gap < a.min_gap_us:
            continue
        tot_gap += gap
        r = by_corr.get(cur[4])
        line = f"gap {gap:7.1f} us before {_short(cur[0], 50):50s}"
        if r is None:
            print(line + "  (issuing call not found)")
            continue
        iss = (r[2] - prev[2]) / 1e3
        if iss > 0:
            host_gap += min(gap, iss)
        line += f" issued by {r[0]} at gap{iss:+8.1f} us (tid {r[1]})"
        print(line)
        # what that thread did during the gap: its longest calls
        during = [x for x in by_tid[r[1]] if x[3] > prev[2] and x[2] < cur[1]]
        during.sort(key=lambda x: x[2] - x[3])
        for x in during[:4]:
            print(f"      {x[0]:32s} {(x[3] - x[2]) / 1e3:8.1f} us  at gap{(x[2] - prev[2]) / 1e3:+8.1f}")
    print(f"gaps >= {a.min_gap_us} us: {tot_gap:.1f} us total, of which issued after the queue "
          f"went idle: {host_gap:.1f} us")


if __name__ == "__main__":
    main()
