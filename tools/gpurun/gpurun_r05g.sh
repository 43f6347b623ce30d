#!/bin/bash
# round 5: tests for the GELU erf / tracker-view changes, then the host stall: AQL queue-limit
# warnings (AMD_LOG_LEVEL=2) in default runs vs a larger AQL queue (ROC_AQL_QUEUE_SIZE)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_net_ops.py tests/test_net.py tests/test_slam.py tests/test_n1.py > gpurun_out/r05g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05g_tests.log; [ $rc -eq 0 ] || exit $rc
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live"
: > gpurun_out/r05g_stall.log
for CFG in "AMD_LOG_LEVEL=2" "ROC_AQL_QUEUE_SIZE=65536" "AMD_LOG_LEVEL=2" "ROC_AQL_QUEUE_SIZE=65536" "AMD_LOG_LEVEL=2" "ROC_AQL_QUEUE_SIZE=65536" "AMD_LOG_LEVEL=2" "ROC_AQL_QUEUE_SIZE=65536"; do
  env $CFG S3_HOST_PHASES=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05g_one.log 2> gpurun_out/r05g_err.log || { tail -20 gpurun_out/r05g_err.log; exit 1; }
  nq=$(grep -c "AQL queue limit" gpurun_out/r05g_err.log || true)
  grep '^{' gpurun_out/r05g_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']
h=c['host_step_ms']; k=max(range(len(h)), key=lambda i: h[i])
print('$CFG', 'aql_limit_msgs', $nq, round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'max_gap', max(c['idle_gaps_ms']), 'attn_ms', round(r['trace_ms_per_frame'].get('s3n_attention', -1), 3), 'dense_ms', round(r['ms_per_frame'], 3), 'frac', round(r['frac'], 4), 'worst step', k, h[k], 'phases', c['host_phases_ms'].get(str(k)))" | tee -a gpurun_out/r05g_stall.log
done
