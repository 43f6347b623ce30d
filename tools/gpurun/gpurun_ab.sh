#!/bin/bash
# A/B of frontend scheduling options on the C2 bench (no CPU / C3 / pairs legs)
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-c3 --no-pairs --no-kprof "$@" > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "$* : $(grep -o '"value": [0-9.]*' gpurun_out/ab.log | head -1)"
}
run
run --late-prefetch
run
run --late-prefetch
run --late-prefetch --enc-batch 3
run --enc-batch 3
