#!/bin/bash
# speculative render on the aux stream (default) vs on the main stream
# (S3_RENDER_AUX=0): frontend GPU tests, then headline A/B/A/B
set -o pipefail
O=gpurun_out/r06ra
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python3 -u -m pytest tests/test_slam.py tests/test_n1.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
n=0
for cfg in "S3_RENDER_AUX=1" "S3_RENDER_AUX=0" "S3_RENDER_AUX=1" "S3_RENDER_AUX=0"; do
n=$((n+1))
env $cfg timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-c3 --no-pairs --no-map --no-cpu-baseline --no-backend > $O/bench$n.log 2> $O/bench$n.err || { tail -20 $O/bench$n.err; exit 1; }
grep '^{' $O/bench$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('$cfg', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', c['big_gaps'], 'e2e', round(d.get('end_to_end_fps') or 0,1), 'live', round(d['live_camera']['frames_per_s'],1), 'rerender', d['frame_breakdown'].get('rerendered'))"
done
