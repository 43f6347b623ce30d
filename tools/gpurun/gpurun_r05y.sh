#!/bin/bash
# round 5: regenerate the GEMM tuning database on the current kernels, then
# headline A/B old DB vs new DB
set -o pipefail
mkdir -p gpurun_out/r05y
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
T0=$(date +%s)
S3_GEMM_TUNE_DB="" S3_GEMM_TUNE_DB_SAVE=gpurun_out/r05y/tune_gfx950.json timeout -k 10 900 python3 -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-live > gpurun_out/r05y/tune_bench.log 2>&1 || { tail -30 gpurun_out/r05y/tune_bench.log; exit 1; }
echo "tuning bench wall $(( $(date +%s) - T0 )) s"
python3 -c "import json; d=json.load(open('gpurun_out/r05y/tune_gfx950.json')); print(len(d['entries']), 'entries', d.get('abi'))"
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
for n in 1 2 3; do
  for DB in old new; do
    if [ $DB = new ]; then export S3_GEMM_TUNE_DB=gpurun_out/r05y/tune_gfx950.json; else unset S3_GEMM_TUNE_DB; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05y/one.log 2>&1 || { tail -20 gpurun_out/r05y/one.log; exit 1; }
    grep '^{' gpurun_out/r05y/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('db=$DB run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), c['big_gaps'])" | tee -a gpurun_out/r05y/ab.log
  done
done
