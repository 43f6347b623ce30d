#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05cs
timeout -k 10 400 python3 -u -m tools.copy_sites --steps 20 > gpurun_out/r05cs/sites.log 2>&1 || { tail -5 gpurun_out/r05cs/sites.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05cs/sites.log
