#!/bin/bash
# the pair plan's Gaussian DPTs on the aux stream (S3_GAUSS_AUX=1, default)
# vs on the main chain (=0): network / frontend / render GPU tests, then the
# headline A/B/A/B; the first run saves the tuner's choices (new 2-group
# DPT launch shapes)
set -o pipefail
O=gpurun_out/r06gx
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S3_GEMM_TUNE_DB_SAVE=$O/tune_new.json S3_GEMM_TUNE_LOG=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-c3 --no-pairs --no-map --no-cpu-baseline --no-backend --no-e2e --no-live --no-kprof --no-in-window > $O/tune.log 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
grep -c "gemm-tune" $O/tune.err || true
timeout -k 10 900 python3 -u -m pytest tests/test_net.py tests/test_slam.py tests/test_n1.py tests/test_gaussians.py -x -q --timeout 400 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
n=0
for cfg in "S3_GAUSS_AUX=1" "S3_GAUSS_AUX=0" "S3_GAUSS_AUX=1" "S3_GAUSS_AUX=0"; do
n=$((n+1))
env $cfg S3_GEMM_TUNE_DB=$O/tune_new.json timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-c3 --no-pairs --no-map --no-cpu-baseline --no-backend > $O/bench$n.log 2> $O/bench$n.err || { tail -20 $O/bench$n.err; exit 1; }
grep '^{' $O/bench$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('$cfg', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', c['big_gaps'], 'e2e', round(d.get('end_to_end_fps') or 0,1), 'live', round(d['live_camera']['frames_per_s'],1), 'rerender', d['frame_breakdown'].get('rerendered'), 'frac', round(d['roofline']['frac'],4))"
done
