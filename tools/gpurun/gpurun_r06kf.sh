#!/bin/bash
# keyframe sequence of the headline's synthetic pan (seed 0, 2 px per frame)
set -o pipefail
mkdir -p gpurun_out/r06kf
timeout -k 10 300 python3 -u -m tools.kf_stats --frames 48 --step 2.0 > gpurun_out/r06kf/kf.log 2>&1 || { tail -20 gpurun_out/r06kf/kf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06kf/kf.log | tail -60
