#!/bin/bash
# round 5: bisect the decode-ahead mismatch with plan branches
set -o pipefail
mkdir -p gpurun_out/r05p
T="tests/test_slam.py::test_decode_ahead_dropped_slots_match_sequential"
for B in 0 1 1 dec head; do
  S3_PLAN_BRANCHES=$B timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu $T > gpurun_out/r05p/t_$B.log 2>&1
  echo "branches=$B rc=$? $(tail -1 gpurun_out/r05p/t_$B.log)"
done
