#!/bin/bash
# decode-ahead: batch-invariance + frontend equality tests, then headline A/B (device path only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_net.py::test_tracker_pair_plan_is_batch_invariant tests/test_net.py::test_encoder_is_batch_invariant tests/test_net.py::test_pair_batch_bp2_matches_bp1_and_golden tests/test_slam.py::test_decode_ahead_frontend_matches_sequential tests/test_slam.py::test_pipelined_frontend_matches_sequential -x -v --timeout 300 --timeout-method thread > gpurun_out/da_tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 gpurun_out/da_tests.log; exit 1; }
grep -E "^(FAILED|E  )" gpurun_out/da_tests.log | head -20
tail -5 gpurun_out/da_tests.log
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
for args in "" "--decode-ahead --enc-batch 2 --enc-ahead 3" "--decode-ahead --enc-batch 4 --enc-ahead 5" "--decode-ahead --enc-batch 4 --enc-ahead 4" "--enc-batch 4" "--decode-ahead"; do
  echo "== $args" >> gpurun_out/da_bench.log
  timeout -k 10 300 python -u bench.py $Q $args 2>&1 | grep '^{' >> gpurun_out/da_bench.log || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/da_bench.log"):
    if l.startswith("=="): print(l.strip()); continue
    d=json.loads(l); fb=d["frame_breakdown"]
    print(f"  {d['value']:.1f} fps  kf_rate {fb['keyframe_rate']:.2f} ahead {fb.get('decode_ahead')} tracked {fb['tracked']}")
PY
