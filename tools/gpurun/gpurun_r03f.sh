#!/bin/bash
# per-launch network profiles (Bp 1/2, encoder batch 1/4), keyframe statistics of the synthetic pan, GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m tools.profile_net > gpurun_out/profile_net_eb1.log 2>&1 || { tail -20 gpurun_out/profile_net_eb1.log; exit 1; }
timeout -k 10 200 python -u -m tools.profile_net --EB 4 > gpurun_out/profile_net_eb4.log 2>&1 || { tail -20 gpurun_out/profile_net_eb4.log; exit 1; }
timeout -k 10 200 python -u -m tools.profile_net --Bp 2 > gpurun_out/profile_net_bp2.log 2>&1 || { tail -20 gpurun_out/profile_net_bp2.log; exit 1; }
timeout -k 10 300 python -u -m tools.kf_stats > gpurun_out/kf_stats.log 2>&1 || { tail -20 gpurun_out/kf_stats.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
