#!/bin/bash
# headline A/B on one box: this tree vs the round-2 python tree (same .so)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-kprof"
: > gpurun_out/abr02.log
for i in 1 2; do
  echo "== new $i" >> gpurun_out/abr02.log
  timeout -k 10 200 python -u bench.py $ARGS --no-e2e > gpurun_out/ab_new.log 2>&1 || { tail -20 gpurun_out/ab_new.log; exit 1; }
  grep '^{"metric"' gpurun_out/ab_new.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],3))" >> gpurun_out/abr02.log
  echo "== r02 $i" >> gpurun_out/abr02.log
  (cd ab_r02 && timeout -k 10 200 python -u bench.py $ARGS > ../gpurun_out/ab_old.log 2>&1) || { tail -20 gpurun_out/ab_old.log; exit 1; }
  grep '^{"metric"' gpurun_out/ab_old.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],3))" >> gpurun_out/abr02.log
done
cat gpurun_out/abr02.log
