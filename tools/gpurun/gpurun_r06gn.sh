#!/bin/bash
# one-launch GN iteration + no match-info copies: tracker / SLAM / host-glue tests, two benches
set -o pipefail
O=gpurun_out/r06gn
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_tracker.py tests/test_host_glue.py tests/test_slam.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -25 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
grep '^{' $O/bench$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']
print('bench$i', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'gn_iters', d['frame_breakdown']['gn_iters_avg'], 'live', round(d['live_camera']['frames_per_s'],1), 'e2e', round(d['end_to_end_fps'],1))"
done
