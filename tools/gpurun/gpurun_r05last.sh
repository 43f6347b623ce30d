#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05last
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_slam.py tests/test_bench_plan.py > gpurun_out/r05last/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05last/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05last/smoke.log 2>&1 || { tail -20 gpurun_out/r05last/smoke.log; exit 1; }
tail -1 gpurun_out/r05last/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05last/bench.log 2> gpurun_out/r05last/bench.err || { tail -20 gpurun_out/r05last/bench.err; exit 1; }
grep '^{' gpurun_out/r05last/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print(round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'c3', round(d['raster_c3']['fwd_ms'],3), 'frac', round(d['roofline']['frac'],4), 'live', round(d['live_camera']['frames_per_s'],1))"
