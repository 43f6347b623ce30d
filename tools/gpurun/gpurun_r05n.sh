#!/bin/bash
# round 5: parallel plan branches (k/v projection, MLP head): network / SLAM
# tests, then headline A/B (S3_PLAN_BRANCHES=0/1 alternating)
set -o pipefail
mkdir -p gpurun_out/r05n
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_net.py tests/test_n1.py tests/test_slam.py tests/test_pairs.py > gpurun_out/r05n/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05n/tests.log; [ $rc -eq 0 ] || exit $rc
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live"
for n in 1 2 3; do
  for B in 0 1; do
    S3_PLAN_BRANCHES=$B timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05n/one.log 2>&1 || { tail -20 gpurun_out/r05n/one.log; exit 1; }
    grep '^{' gpurun_out/r05n/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']
print('branches=$B run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3), 'gaps', c['big_gaps'])" | tee -a gpurun_out/r05n/ab.log
  done
done
