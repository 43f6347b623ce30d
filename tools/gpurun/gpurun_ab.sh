#!/bin/bash
# headline A/B over $CONFIGS (';'-separated bench argument sets), device path only
set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
rm -f gpurun_out/ab.log
IFS=';' read -ra CFG <<< "$CONFIGS"
for args in "${CFG[@]}"; do
  echo "== $args" >> gpurun_out/ab.log
  timeout -k 10 300 python -u bench.py $Q $args > gpurun_out/ab_run.log 2>&1 || { tail -30 gpurun_out/ab_run.log; exit 1; }
  grep '^{' gpurun_out/ab_run.log >> gpurun_out/ab.log || { tail -30 gpurun_out/ab_run.log; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/ab.log"):
    if l.startswith("=="): print(l.strip()); continue
    d=json.loads(l); fb=d["frame_breakdown"]
    print(f"  {d['value']:.1f} fps  kf_rate {fb['keyframe_rate']:.2f} ahead {fb.get('decode_ahead')}")
PY
