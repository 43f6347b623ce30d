#!/bin/bash
# decode-ahead kb=2 mismatch bisection: graphs off, B-direct off, live tuning log
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
K="decode_ahead_frontend_matches_sequential"
n=0
for cfg in "S3_GRAPHS=0" "S3_GEMM_BDIRECT=0" "S3_GEMM_TUNE_LOG=1" "S3_GEMM_TUNE_DB=" ; do
n=$((n+1))
env $cfg timeout -k 10 400 python -u -m pytest tests/test_slam.py -q -x -s --timeout 380 --timeout-method thread -k "$K" > $O/slam_$n.log 2>&1; echo "$cfg: $(tail -1 $O/slam_$n.log)"; grep -E "pose differences" $O/slam_$n.log | cut -c1-200
done
grep -c "gemm-tune" $O/slam_3.log
