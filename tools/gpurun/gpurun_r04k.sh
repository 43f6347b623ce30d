#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -m tools.live_ab > gpurun_out/r04k_live_ab.log 2>&1 || { tail -20 gpurun_out/r04k_live_ab.log; exit 1; }
grep -E "live|end_to_end" gpurun_out/r04k_live_ab.log
