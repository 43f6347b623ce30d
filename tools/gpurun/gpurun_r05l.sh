#!/bin/bash
# round 5: per-tile binning v2 (large binning workgroups, run tie fixup) and
# order-free radix counts: raster tests, C3 A/B, kernel stats of both binnings
set -o pipefail
mkdir -p gpurun_out/r05l
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_raster.py > gpurun_out/r05l/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05l/tests.log; [ $rc -eq 0 ] || exit $rc
for B in tile global; do
  timeout -k 10 200 python -u -m tools.bench_raster --iters 10 --binning $B > gpurun_out/r05l/c3_$B.log 2>&1 || { tail -5 gpurun_out/r05l/c3_$B.log; exit 1; }
  grep '^{' gpurun_out/r05l/c3_$B.log
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05l/prof_$B -o run -- python3 -m tools.bench_raster --iters 5 --no-backward --binning $B > gpurun_out/r05l/prof_$B.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r05l/prof_$B/run_kernel_stats.csv')):
    if 'k_' in r['Name']: print('$B', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
