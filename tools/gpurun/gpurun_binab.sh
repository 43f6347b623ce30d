#!/bin/bash
# single-pass tile binning A/B: segment size, debug phase skips, radix path; then parity
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
: > gpurun_out/binab.log
run() {  # label, env..., -- args
  local label=$1; shift
  echo "== $label" >> gpurun_out/binab.log
  env "$@" timeout -k 10 120 python -u -m tools.bench_raster --P 4194304 --iters 10 --no-backward $BARGS >> gpurun_out/binab.log 2>&1 || return 1
}
run default S3_X=0 && run ranks2048 S3_RASTER_BIN_RANKS=2048 && run dbg1 S3_RASTER_BIN_DBG=1 \
 && run dbg2 S3_RASTER_BIN_DBG=2 && run dbg4 S3_RASTER_BIN_DBG=4 && run dbg8 S3_RASTER_BIN_DBG=8 \
 && run dbg12 S3_RASTER_BIN_DBG=12 \
 && BARGS="--binning 1" run radix S3_X=0 || { tail -20 gpurun_out/binab.log; exit 1; }
grep -o '^== .*\|"binning": [0-9.]*\|"fwd_ms": [0-9.]*' gpurun_out/binab.log
timeout -k 10 300 python -u -m pytest tests/test_raster.py -m gpu -x -q -k "binning or c3_full" --timeout 200 --timeout-method thread > gpurun_out/rt1.log 2>&1 || { tail -30 gpurun_out/rt1.log; exit 1; }
tail -1 gpurun_out/rt1.log
S3_RASTER_BIN_RANKS=2048 timeout -k 10 300 python -u -m pytest tests/test_raster.py -m gpu -x -q -k "binning or c3_full" --timeout 200 --timeout-method thread > gpurun_out/rt2.log 2>&1 || { tail -30 gpurun_out/rt2.log; exit 1; }
tail -1 gpurun_out/rt2.log
