#!/bin/bash
# kernel trace + timeline of the default bench frame loop, and the no-decode-ahead loop
set -o pipefail
mkdir -p gpurun_out
STEPS=24 WIN_MS=60 GAPS=20 bash tools/gpurun/gpurun_prof.sh || exit 1
cp gpurun_out/timeline.txt gpurun_out/timeline_da.txt; cp gpurun_out/prof_summary_timed.txt gpurun_out/prof_timed_da.txt
STEPS=24 WIN_MS=60 GAPS=20 BENCH_ARGS="--no-decode-ahead" bash tools/gpurun/gpurun_prof.sh || exit 1
cp gpurun_out/timeline.txt gpurun_out/timeline_noda.txt; cp gpurun_out/prof_summary_timed.txt gpurun_out/prof_timed_noda.txt
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
rm -f gpurun_out/ab.log
for args in "" "--enc-batch 8 --enc-ahead 8" "--no-decode-ahead" "--enc-batch 8 --enc-ahead 8 --no-decode-ahead"; do
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
