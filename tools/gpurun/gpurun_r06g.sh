#!/bin/bash
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_net.py -q --timeout 500 --timeout-method thread -k "every_tile_of_a_reduction_class" > $O/cls.log 2>&1; grep -E "passed|failed|assert|AssertionError" $O/cls.log | head -30
K="decode_ahead_frontend_matches_sequential"
for cfg in "X=1" "X=2" "S3_SYNC_DEBUG=1" "S3_GEMM_BDIRECT=0" "S3_REFINE_LANES=16"; do
env $cfg timeout -k 10 400 python -u -m pytest tests/test_slam.py -q -x -s --timeout 380 --timeout-method thread -k "$K" > $O/slam_${cfg%%=*}_${cfg##*=}.log 2>&1; echo "$cfg: $(tail -1 $O/slam_${cfg%%=*}_${cfg##*=}.log)"; grep -E "pose differences|kb=" $O/slam_${cfg%%=*}_${cfg##*=}.log | cut -c1-220
done
