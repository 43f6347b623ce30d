#!/bin/bash
# round 5 close: the driver's sequence on one box -- GPU tests, smoke, the bench command
set -o pipefail
mkdir -p gpurun_out/r05close
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05close/tests.log 2>&1 || { tail -30 gpurun_out/r05close/tests.log; exit 1; }
tail -1 gpurun_out/r05close/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05close/smoke.log 2>&1 || { tail -20 gpurun_out/r05close/smoke.log; exit 1; }
tail -1 gpurun_out/r05close/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05close/bench.log 2> gpurun_out/r05close/bench.err || { tail -20 gpurun_out/r05close/bench.err; exit 1; }
grep '^{' gpurun_out/r05close/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print(round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'c3', round(d['raster_c3']['fwd_ms'],3), 'frac', round(d['roofline']['frac'],4), 'live', round(d['live_camera']['frames_per_s'],1), 'e2e', round(d['end_to_end_fps'],1))"
