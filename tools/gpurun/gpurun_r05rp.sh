#!/bin/bash
# round 5: counters of the refine kernels on one captured tracker call
set -o pipefail
D=gpurun_out/r05rp
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf $D/p1 $D/p2
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $D/p1 -o run -- python3 -m tools.refine_pmc > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU TA_BUSY_avr FETCH_SIZE --kernel-trace --output-format csv -d $D/p2 -o run -- python3 -m tools.refine_pmc > $D/p2.log 2>&1 || { tail -5 $D/p2.log; exit 1; }
python -m tools.pmc_kernels $D/p1 $D/p2 --match refine > $D/pmc.txt 2>&1
find $D -name '*.csv' -size +2M -delete
cat $D/pmc.txt
