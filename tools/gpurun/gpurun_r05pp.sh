#!/bin/bash
# round 5: raster tests, C3 bench, and per-kernel counters of the C3 forward+backward
set -o pipefail
D=gpurun_out/r05pp
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_raster.py tests/test_n1.py > $D/tests.log 2>&1
rc=$?; tail -2 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m tools.bench_raster --iters 10 > $D/c3.log 2>&1 || { tail -5 $D/c3.log; exit 1; }
grep '^{' $D/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('fwd_ms','fwd_deferred_ms','deferred_equal','bwd_ms','phases_ms')})"
rm -rf $D/p1 $D/p2 $D/p3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $D/p1 -o run -- python3 -m tools.pmc_traffic run --workload raster > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr --kernel-trace --output-format csv -d $D/p2 -o run -- python3 -m tools.pmc_traffic run --workload raster > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $D/p3 -o run -- python3 -m tools.pmc_traffic run --workload raster > $D/p3.log 2>&1 || { tail -5 $D/p3.log; exit 1; }
python -m tools.pmc_kernels $D/p1 $D/p2 $D/p3 > $D/pmc.txt 2>&1
find $D -name '*.csv' -size +2M -delete
cat $D/pmc.txt | head -150
