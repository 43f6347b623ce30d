#!/bin/bash
# round 5: decode-ahead against the tracked frame when it is likely to become a keyframe:
# frontend tests, then the headline over 20 / 40 / 80-frame windows
set -o pipefail
D=gpurun_out/r05da
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_slam.py > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
for st in 20 40 80 20; do
  timeout -k 10 300 python3 bench.py --steps $st --warmup 5 $OFF > $D/one.log 2>&1 || { tail -20 $D/one.log; exit 1; }
  grep '^{' $D/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; f=d['frame_breakdown']
print('steps $st', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'kf', f['keyframes'], 'da', f['decode_ahead'], 'big', c['big_gaps'])" | tee -a $D/ab.log
done
