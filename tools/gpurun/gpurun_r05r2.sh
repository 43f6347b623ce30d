#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05r
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r05r/prof -o run -- python3 bench.py --steps 12 --warmup 4 $OFF > gpurun_out/r05r/prof.log 2>&1 || { tail -20 gpurun_out/r05r/prof.log; exit 1; }
python3 - > gpurun_out/r05r/corr.txt <<'PY'
import sqlite3, collections
c = sqlite3.connect('gpurun_out/r05r/prof/run_results.db')
print(list(c.execute("select name, corr_id, stream, queue from kernels order by start desc limit 8")))
names = collections.Counter(n for (n,) in c.execute("select name from regions where start > (select max(start) from regions) - 20000000"))
print(names.most_common(40))
print(list(c.execute("select name, corr_id, tid, start from regions where name like '%Launch%' order by start desc limit 8")))
print(list(c.execute("select name, corr_id, tid, start from regions where name like '%raph%' order by start desc limit 8")))
PY
rm -rf gpurun_out/r05r/prof
