#!/bin/bash
# round 4: live-camera leg A/B (deferred render on/off) + kernel trace
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof"
for args in "" "--no-deferred-render"; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF $args > gpurun_out/r04d_one.log 2>&1 || { tail -20 gpurun_out/r04d_one.log; exit 1; }
  python3 - "$args" <<'PY'
import json, sys
for line in open("gpurun_out/r04d_one.log"):
    if line.startswith("{"):
        d = json.loads(line)
print(repr(sys.argv[1]), round(d["value"], 1), d["live_camera"]["frames_per_s"], d["live_camera"]["latency_ms"]["p50"])
PY
done
rm -rf gpurun_out/prof4d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4d -o run -- python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04d_prof.log 2>&1 || { tail -20 gpurun_out/r04d_prof.log; exit 1; }
python -m tools.rocprof_timeline gpurun_out/prof4d/run_results.db --last-ms 120 --gaps 15 > gpurun_out/r04d_timeline.txt 2>&1
python -m tools.rocprof_summary gpurun_out/prof4d/run_results.db --last-ms 120 > gpurun_out/r04d_summary_last.txt 2>&1
rm -f gpurun_out/prof4d/run_results.db
head -40 gpurun_out/r04d_timeline.txt
head -40 gpurun_out/r04d_summary_last.txt
