#!/bin/bash
# round 5: refine counters (which bound: VALU issue, memory wait, L1/L2)
set -o pipefail
mkdir -p gpurun_out/r05j
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rocprofv3 -L > gpurun_out/r05j/counters_all.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
P2="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
RX="--kernel-include-regex k_refine"
timeout -k 10 300 rocprofv3 --kernel-trace --stats $RX -d gpurun_out/r05j/trace -o run --output-format csv -- python3 -m tools.refine_pmc > gpurun_out/r05j/trace.log 2>&1 || { tail -5 gpurun_out/r05j/trace.log; exit 1; }
k=0
for P in "$P1" "$P2"; do
  k=$((k+1))
  timeout -s KILL 240 rocprofv3 --pmc $P $RX -d gpurun_out/r05j/pmc$k -o run --output-format csv -- python3 -m tools.refine_pmc > gpurun_out/r05j/pmc$k.log 2>&1 || { tail -5 gpurun_out/r05j/pmc$k.log; exit 1; }
done
find gpurun_out/r05j -type f ! -name "*.csv" ! -name "*.txt" ! -name "*.log" -delete
du -sh gpurun_out/r05j; find gpurun_out/r05j -name "*.csv" | head -20
