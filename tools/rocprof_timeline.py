"""Timeline view of a rocprofv3 kernel trace (tuning harness): per queue
busy time, the union of all queues (GPU busy), idle gaps, and the kernels
of a time window in start order.

  python -m tools.rocprof_timeline <results.db> [--last-ms 50] [--list 0]
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-ms", type=float, default=50.0)
    ap.add_argument("--skip-last-ms", type=float, default=0.0)
    ap.add_argument("--list", type=int, default=0)
    ap.add_argument("--gaps", type=int, default=0, help="print the N largest idle gaps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    t_end = max(r[2] for r in rows) - a.skip_last_ms * 1e6
    t0 = t_end - a.last_ms * 1e6
    win = [r for r in rows if r[1] >= t0 and r[2] <= t_end]
    per_q = {}
    for _, s, e, q in win:
        per_q[q] = per_q.get(q, 0) + (e - s)
    iv = sorted((s, e) for _, s, e, _ in win)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = (iv[-1][1] - iv[0][0]) if iv else 0
    print(f"window {span / 1e6:.2f} ms, {len(win)} kernels, GPU busy (union) {busy / 1e6:.2f} ms "
          f"({busy / max(span, 1):.1%}), idle gaps {sum(gaps) / 1e6:.2f} ms in {len(gaps)} gaps "
          f"(largest {max(gaps, default=0) / 1e3:.1f} us)")
    for q, t in sorted(per_q.items()):
        print(f"  queue {q}: kernel time {t / 1e6:.2f} ms")
    # queue segments: maximal runs of consecutive (by start) kernels on one queue
    seg = None
    for n, s, e, q in win:
        if seg is None or seg[0] != q:
            if seg is not None:
                print(f"  seg q{seg[0]} {(seg[1] - t0) / 1e3:9.1f} -> {(seg[2] - t0) / 1e3:9.1f} us"
                      f" ({seg[3]} kernels, first {seg[4]})")
            seg = [q, s, e, 0, re.sub(r"\(anonymous namespace\)::", "", n)[:40]]
        seg[2] = max(seg[2], e)
        seg[3] += 1
    if seg is not None:
        print(f"  seg q{seg[0]} {(seg[1] - t0) / 1e3:9.1f} -> {(seg[2] - t0) / 1e3:9.1f} us"
              f" ({seg[3]} kernels, first {seg[4]})")
    if a.gaps:
        # idle gaps of the union timeline with the kernels either side
        ends, gl = [], []
        cur_e, prev = None, None
        for n, s, e, q in win:
            if cur_e is not None and s > cur_e:
                gl.append((s - cur_e, (cur_e - t0) / 1e3, prev, n))
            if cur_e is None or e > cur_e:
                cur_e, prev = e, n
        gl.sort(reverse=True)
        short = lambda n: re.sub(r"\(anonymous namespace\)::", "", n)[:48]
        tot = {}
        for g, at, a0, b0 in gl:
            k = (short(a0), short(b0))
            tot[k] = tot.get(k, 0) + g
        print("  largest idle gaps (us, at us, after -> before):")
        for g, at, a0, b0 in gl[: a.gaps]:
            print(f"    {g / 1e3:7.1f} @ {at:9.1f}  {short(a0)} -> {short(b0)}")
        print("  idle time by (after -> before) pair:")
        for k, g in sorted(tot.items(), key=lambda kv: -kv[1])[: a.gaps]:
            print(f"    {g / 1e6:7.3f} ms  {k[0]} -> {k[1]}")
    for n, s, e, q in win[: a.list]:
        n = re.sub(r"\(anonymous namespace\)::", "", n)[:70]
        print(f"  q{q} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} us  {n}")


if __name__ == "__main__":
    main()
