#!/bin/bash
# write the GEMM tuning database from a full bench run, then two bench runs that load it
set -o pipefail
mkdir -p gpurun_out
S3_GEMM_TUNE_DB= S3_GEMM_TUNE_DB_SAVE=gpurun_out/tune_gfx950.json timeout -k 10 700 python -u bench.py > gpurun_out/db_bench0.log 2>&1 || { tail -20 gpurun_out/db_bench0.log; exit 1; }
ls -la gpurun_out/tune_gfx950.json
grep '^{' gpurun_out/db_bench0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('writer fps', d['value'], 'frac', d['roofline']['frac'])"
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
for i in 1 2 3; do
  S3_GEMM_TUNE_DB=gpurun_out/tune_gfx950.json S3_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u bench.py $Q > gpurun_out/db_b$i.log 2>&1 || { tail -20 gpurun_out/db_b$i.log; exit 1; }
  echo "tuned shapes not in the database: $(grep -c '^\[gemm-tune\] [0-9]' gpurun_out/db_b$i.log)"
  grep '^{' gpurun_out/db_b$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('db fps', d['value'])"
done
