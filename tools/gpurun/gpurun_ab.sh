#!/bin/bash
# A/B of GEMM tuning modes on the C2 bench (no CPU / C3 / pairs legs):
# warm back-to-back timing (default) vs cold per-launch timing
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-c3 --no-pairs > gpurun_out/ab_$tag.log 2>&1 || { tail -20 gpurun_out/ab_$tag.log; exit 1; }
  python3 - gpurun_out/ab_$tag.log "$tag" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
r = d["roofline"]
print(sys.argv[2], "fps", round(d["value"], 2), "ms/step", round(d["ms_per_step"], 3),
      "gemm frac", round(r["frac"], 4), "net ms/frame", r.get("ms_per_frame"),
      "trace", r.get("trace_ms_per_frame"), "network_ms", d["frame_breakdown"]["network_ms"])
EOF
}
run warm S3_GEMM_TUNE_COLD=0
run cold S3_GEMM_TUNE_COLD=1
run warm2 S3_GEMM_TUNE_COLD=0
run cold2 S3_GEMM_TUNE_COLD=1
