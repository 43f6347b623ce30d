#!/bin/bash
# net_ops kernel changes (gauss_post, upsample2x): op + network parity tests, kernel time in the frame loop, bench x2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_net_ops.py tests/test_net.py tests/test_n1.py > gpurun_out/post_tests.log 2>&1 || { tail -30 gpurun_out/post_tests.log; exit 1; }
tail -2 gpurun_out/post_tests.log
STEPS=24 WIN_MS=60 bash tools/gpurun/gpurun_prof.sh || exit 1
grep -E 'k_gauss_post|k_upsample2x' gpurun_out/prof_summary.txt gpurun_out/prof_summary_timed.txt
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/pb$i.log 2>&1 || { tail -20 gpurun_out/pb$i.log; exit 1; }
  grep '^{' gpurun_out/pb$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fps', d['value'])"
done
