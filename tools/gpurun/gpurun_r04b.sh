#!/bin/bash
# round 4: headline A/B (spans, deferred render, steps, lookahead)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-live --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof"
: > gpurun_out/r04b_ab.log
for args in "--steps 20" "--steps 20 --no-spans" "--steps 20 --no-deferred-render" "--steps 20 --no-spans --no-deferred-render" "--steps 120" "--steps 120 --no-spans" "--steps 20 --main-priority 0" "--steps 20 --enc-batch 1 --enc-ahead 0 --no-decode-ahead"; do
  timeout -k 10 300 python3 bench.py $args --warmup 5 $OFF > gpurun_out/r04b_one.log 2>&1 || { tail -20 gpurun_out/r04b_one.log; exit 1; }
  python3 - "$args" >> gpurun_out/r04b_ab.log <<'PY'
import json, sys
for line in open("gpurun_out/r04b_one.log"):
    if line.startswith("{"):
        d = json.loads(line)
        cp = d.get("critical_path") or {}
        print(f"{sys.argv[1]:60s} {d['value']:7.1f} fps  {d['ms_per_step']:6.2f} ms  idle {cp.get('main_idle_ms', float('nan')):5.2f}  net {cp.get('main_network_ms', float('nan')):5.2f} other {cp.get('main_other_ms', float('nan')):5.2f} kf {d['frame_breakdown']['keyframes']} da {d['frame_breakdown']['decode_ahead']}")
PY
  tail -1 gpurun_out/r04b_ab.log
done
timeout -k 10 300 python -u -m tools.gemm_ceiling --tiles 32,36,63,68 > gpurun_out/r04b_gemm_ceiling.log 2>&1 || { tail -20 gpurun_out/r04b_gemm_ceiling.log; exit 1; }
grep -v "^  t" gpurun_out/r04b_gemm_ceiling.log
