"""Per-queue kernel breakdown of the last `--last-ms` of a rocprofv3 kernel
trace (which stream spends its time where: the main stream's chain, the
encoder side stream, the aux stream).  Per queue: busy ms, then its kernels
by total time, with calls and time per frame (`--frames`).

  python -m tools.rocprof_queues <results.db> --last-ms 100 --frames 20
"""
from __future__ import annotations

import argparse
import sqlite3

from tools.rocprof_summary import _short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-ms", type=float, default=100.0)
    ap.add_argument("--frames", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    t_end = max(r[2] for r in rows)
    t0 = t_end - a.last_ms * 1e6
    win = [r for r in rows if r[1] >= t0]
    per_q = {}
    for n, s, e, q in win:
        d = per_q.setdefault(q, {})
        v = d.setdefault(n, [0, 0.0])
        v[0] += 1
        v[1] += (e - s) / 1e3
    f = a.frames
    for q, d in sorted(per_q.items(), key=lambda kv: -sum(v[1] for v in kv[1].values())):
        busy = sum(v[1] for v in d.values())
        print(f"== queue {q}: busy {busy / 1e3:.3f} ms in {a.last_ms:.0f} ms "
              f"({busy / 1e3 / f:.3f} ms per frame over {f:g} frames)")
        for n, (cnt, us) in sorted(d.items(), key=lambda kv: -kv[1][1])[:a.top]:
            print(f"  {_short(n, 78):78s} {cnt / f:6.1f}/fr {us / f:8.1f} us/fr  avg {us / cnt:7.1f} us")


if __name__ == "__main__":
    main()
