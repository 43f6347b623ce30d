#!/bin/bash
# frame-loop device copies by call site on the round-6 tree
set -o pipefail
mkdir -p gpurun_out/r06cs
timeout -k 10 400 python3 -u -m tools.copy_sites --steps 20 > gpurun_out/r06cs/sites.log 2>&1 || { tail -5 gpurun_out/r06cs/sites.log; exit 1; }
grep -v "^\[" gpurun_out/r06cs/sites.log | tail -40
