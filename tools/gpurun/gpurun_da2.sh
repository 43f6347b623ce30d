#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_net.py::test_encoder_is_batch_invariant tests/test_net.py::test_tracker_pair_plan_is_batch_invariant tests/test_slam.py::test_decode_ahead_frontend_matches_sequential -v -s --timeout 300 --timeout-method thread > gpurun_out/da2_tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 gpurun_out/da2_tests.log; exit 1; }
grep -E "^(FAILED|PASSED|E  )|ahead|passed|failed" gpurun_out/da2_tests.log | head -30
