#!/bin/bash
# halo variant tests + decomposition, end-to-end thread A/B, host profile of the frame loop
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py -k "halo" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/halo_tests.log 2>&1 || { tail -30 gpurun_out/halo_tests.log; exit 1; }
tail -1 gpurun_out/halo_tests.log
timeout -k 10 300 python -u -m tools.bench_conv_parts --tiles 3,46,47,48,49,50 --B 2 > gpurun_out/conv_parts2.log 2>&1 || { tail -20 gpurun_out/conv_parts2.log; exit 1; }
grep conv gpurun_out/conv_parts2.log
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-kprof"
rm -f gpurun_out/e2e_ab.log
for args in "--e2e-loaders 4 --e2e-writers 3" "--e2e-loaders 8 --e2e-writers 4" "--e2e-loaders 12 --e2e-writers 6"; do
  echo "== $args" >> gpurun_out/e2e_ab.log
  timeout -k 10 400 python -u bench.py $Q $args > gpurun_out/e2e_run.log 2>&1 || { tail -30 gpurun_out/e2e_run.log; exit 1; }
  grep '^{' gpurun_out/e2e_run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('  device', round(d['value'],1), 'e2e', round(d['end_to_end_fps'],1))" >> gpurun_out/e2e_ab.log
done
cat gpurun_out/e2e_ab.log
timeout -k 10 300 python -u -m tools.host_profile > gpurun_out/host_profile.log 2>&1 || { tail -20 gpurun_out/host_profile.log; exit 1; }
head -45 gpurun_out/host_profile.log
