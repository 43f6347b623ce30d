#!/bin/bash
# whole GPU suite, then headline A/B of the lookahead configurations (device path only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
rm -f gpurun_out/ab.log
for args in "" "--enc-batch 8 --enc-ahead 9" "--no-decode-ahead" "--enc-batch 1 --enc-ahead 0 --no-decode-ahead" ""; do
  echo "== $args" >> gpurun_out/ab.log
  timeout -k 10 300 python -u bench.py $Q $args 2>&1 | grep '^{' >> gpurun_out/ab.log || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/ab.log"):
    if l.startswith("=="): print(l.strip()); continue
    d=json.loads(l); fb=d["frame_breakdown"]
    print(f"  {d['value']:.1f} fps  kf_rate {fb['keyframe_rate']:.2f} ahead {fb.get('decode_ahead')}")
PY
