"""Per-kernel means of the counters of rocprofv3 --pmc runs (diagnostic).

  python -m tools.pmc_kernels <dir> [<dir> ...] [--match REGEX]

Reads every *counter_collection.csv under the directories (one pass per
directory, each with its own counter set), sums each counter over the
dimensions of one dispatch, and prints, per kernel whose name matches, the
dispatch count and the mean of every counter per dispatch.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re

from tools.rocprof_summary import _short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default=".")
    a = ap.parse_args()
    # kernel -> counter -> [dispatch sums]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            disp = {}
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    if not re.search(a.match, r["Kernel_Name"]):
                        continue
                    key = (int(r["Dispatch_Id"]), r["Counter_Name"])
                    v = disp.setdefault(key, [r["Kernel_Name"], 0.0])
                    v[1] += float(r["Counter_Value"])
            for (_, cn), (kn, v) in disp.items():
                acc[kn][cn].append(v)
    for kn, cs in sorted(acc.items()):
        n = max(len(v) for v in cs.values())
        print(f"{_short(kn, 70)}  dispatches {n}")
        for cn, v in sorted(cs.items()):
            print(f"    {cn:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
