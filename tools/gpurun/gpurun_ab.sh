#!/bin/bash
# A/B of launch options on the C2 bench (no CPU / C3 / pairs legs).
# Usage: gpurun_ab.sh TAG=ENV[,ENV...] ...   e.g. v0=S3_ATTN_VARIANT=0
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=${1%%=*} envs=${1#*=}
  env ${envs//,/ } timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-c3 --no-pairs > gpurun_out/ab_$tag.log 2>&1 || { tail -20 gpurun_out/ab_$tag.log; exit 1; }
  python3 - gpurun_out/ab_$tag.log "$tag" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
r = d["roofline"]
print(sys.argv[2], "fps", round(d["value"], 2), "ms/step", round(d["ms_per_step"], 3),
      "gemm frac", round(r["frac"], 4),
      "trace", {k: round(v, 3) for k, v in r.get("trace_ms_per_frame", {}).items()})
EOF
}
for a in "$@"; do run "$a" || exit 1; done
