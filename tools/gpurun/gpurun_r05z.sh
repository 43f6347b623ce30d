#!/bin/bash
# round 5: where the DPT halo convs spend their time (current tree)
set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 300 python3 -u -m tools.bench_conv_parts --tiles 51,52,48 --B 1 > gpurun_out/r05z/conv_parts_b1.log 2>&1 || { tail -5 gpurun_out/r05z/conv_parts_b1.log; exit 1; }
cat gpurun_out/r05z/conv_parts_b1.log
