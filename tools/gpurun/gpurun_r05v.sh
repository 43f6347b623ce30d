#!/bin/bash
# round 5: contiguous read-back + hook-time delivery: SLAM tests, headline x3 with timeline
set -o pipefail
mkdir -p gpurun_out/r05v
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_slam.py > gpurun_out/r05v/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05v/tests.log; [ $rc -eq 0 ] || exit $rc
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
for n in 1 2 3; do
  for S in none; do
    S3_DIAG_SKIP=$S timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05v/one.log 2>&1 || { tail -20 gpurun_out/r05v/one.log; exit 1; }
    grep '^{' gpurun_out/r05v/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('skip=$S run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), c['big_gaps'])" | tee -a gpurun_out/r05v/ab.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05v/prof -o run -- python3 bench.py --steps 30 --warmup 5 $OFF > gpurun_out/r05v/prof.log 2>&1 || exit 1
python -m tools.rocprof_timeline gpurun_out/r05v/prof/run_results.db --last-ms 60 --gaps 15 > gpurun_out/r05v/timeline.txt 2>&1
rm -f gpurun_out/r05v/prof/run_results.db
