#!/bin/bash
# round 4: regenerate the GEMM tuning database (new tiles 63/65/68) with a
# full bench run, then the driver's command loading it
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
T0=$(date +%s)
S3_GEMM_TUNE_DB="" S3_GEMM_TUNE_DB_SAVE=gpurun_out/tune_gfx950.json S3_GEMM_TUNE_LOG=1 timeout -k 10 900 python3 bench.py --steps 120 --warmup 5 > gpurun_out/r04c_tune_bench.log 2>&1 || { tail -30 gpurun_out/r04c_tune_bench.log; exit 1; }
echo "tuning bench wall $(( $(date +%s) - T0 )) s"
grep -c "gemm-tune" gpurun_out/r04c_tune_bench.log
python3 -c "import json; d=json.load(open('gpurun_out/tune_gfx950.json')); print(len(d['entries']), 'entries')"
cp gpurun_out/tune_gfx950.json splatt3r-slam_amd/splatt3r_amd/tune_gfx950.json
T0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04c_bench.log 2> gpurun_out/r04c_bench.err || { tail -30 gpurun_out/r04c_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - T0 )) s"
python3 - <<'PY'
import json
for line in open("gpurun_out/r04c_bench.log"):
    if line.startswith("{"):
        d = json.loads(line)
print("value", d["value"], "e2e", d.get("end_to_end_fps"), "live", d["live_camera"]["frames_per_s"], d["live_camera"]["latency_ms"])
print("crit", d["critical_path"])
r = d["roofline"]; print("roofline", r["frac"], r["ms_per_frame"], r["trace_ms_per_frame"])
print("c3", d["raster_c3"]["fwd_ms"], d["raster_c3"]["bwd_ms"], "kf", d["frame_breakdown"]["keyframes"])
PY
