#!/bin/bash
# round 5: refine window-centre binning (parity + timing on captured tracker
# inputs), render read-back on the aux stream (SLAM tests + stall A/B runs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_matching.py tests/test_slam.py > gpurun_out/r05i_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05i_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m tools.bench_refine > gpurun_out/r05i_refine.log 2>&1
rc=$?; tail -20 gpurun_out/r05i_refine.log; [ $rc -eq 0 ] || exit $rc
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live"
: > gpurun_out/r05i_stall.log
for n in 1 2 3 4 5 6 7 8; do
  S3_STALL_TRACE=3 S3_HOST_PHASES=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05i_one.log 2> gpurun_out/r05i_err_$n.log || { tail -20 gpurun_out/r05i_err_$n.log; exit 1; }
  grep '^{' gpurun_out/r05i_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
h=c['host_step_ms']; k=max(range(len(h)), key=lambda i: h[i])
print('run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'big_gaps', c['big_gaps'], 'worst step', k, h[k])" | tee -a gpurun_out/r05i_stall.log
  echo "run $n stack dumps: $(grep -c 'most recent call first' gpurun_out/r05i_err_$n.log || true)" | tee -a gpurun_out/r05i_stall.log
done
