#!/bin/bash
# rocprofv3 kernel + HIP API trace of a short bench run (host-side launch timing)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/hprof
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/hprof -o run -- python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-c3 --no-pairs --no-kprof > gpurun_out/bench_hprof.log 2>&1 || exit $?
python3 - <<'PY' > gpurun_out/hiptrace.txt 2>&1
import sqlite3, re
c = sqlite3.connect("gpurun_out/hprof/run_results.db")
names = [r[0] for r in c.execute("select name from sqlite_master where type='view'")]
print(names)
k = list(c.execute("select name, start, end, queue_id from kernels order by start"))
t_end = max(r[2] for r in k)
t0 = t_end - 25e6
cols = [d[0] for d in c.execute("select * from regions limit 1").description]
print(cols)
api = list(c.execute("select name, start, end, tid from regions order by start"))
ev = [("K q%d %s" % (q, re.sub(r'\(anonymous namespace\)::', '', n)[:50]), s, e) for n, s, e, q in k if s >= t0]
ev += [("A t%d %s" % (tid % 1000, n), s, e) for n, s, e, tid in api if s >= t0 and (e - s) > 20000]
ev.sort(key=lambda x: x[1])
for n, s, e in ev:
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {n}")
PY
rm -f gpurun_out/hprof/run_results.db
