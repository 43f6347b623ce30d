#!/bin/bash
# round 5: kernel trace of 80-frame runs, largest main-queue gaps with the other queues' work
set -o pipefail
D=gpurun_out/r05gapprof
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
for n in 1 2; do
  rm -rf $D/prof
  timeout -k 10 400 rocprofv3 --kernel-trace -d $D/prof -o run -- python3 bench.py --steps 80 --warmup 5 $OFF > $D/bench_$n.log 2>&1 || { tail -20 $D/bench_$n.log; exit 1; }
  grep '^{' $D/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $n', round(d['value'],1), d['critical_path']['big_gaps'])"
  python -m tools.rocprof_qgaps $D/prof/run_results.db --min-ms 2 > $D/qgaps_$n.txt 2>&1
  rm -f $D/prof/run_results.db
  head -30 $D/qgaps_$n.txt
done
