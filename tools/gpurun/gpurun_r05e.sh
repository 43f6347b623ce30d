#!/bin/bash
# round 5: attention after the bare v_exp_f32 (op tests + in-graph A/B), and the intermittent
# host stall: repeated headline runs with host-phase marks, default vs eager code-object loading
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_net_ops.py -k "attention" > gpurun_out/r05e_attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05e_attn_tests.log; [ $rc -eq 0 ] || exit $rc
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live"
: > gpurun_out/r05e_stall.log
for CFG in HIP_ENABLE_DEFERRED_LOADING=1 HIP_ENABLE_DEFERRED_LOADING=0 HIP_ENABLE_DEFERRED_LOADING=1 HIP_ENABLE_DEFERRED_LOADING=0 HIP_ENABLE_DEFERRED_LOADING=1 HIP_ENABLE_DEFERRED_LOADING=0; do
  t0=$(date +%s)
  env $CFG S3_HOST_PHASES=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05e_one.log 2>&1 || { tail -20 gpurun_out/r05e_one.log; exit 1; }
  t1=$(date +%s)
  grep '^{' gpurun_out/r05e_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']
h=c['host_step_ms']; k=max(range(len(h)), key=lambda i: h[i])
print('$CFG', 'wall_s', $t1-$t0, round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'max_gap', max(c['idle_gaps_ms']), 'attn_ms', round(r['trace_ms_per_frame'].get('s3n_attention', -1), 3), 'dense_ms', round(r['ms_per_frame'], 3), 'frac', round(r['frac'], 4), 'worst step', k, h[k], 'phases', c['host_phases_ms'].get(str(k)))" | tee -a gpurun_out/r05e_stall.log
done
