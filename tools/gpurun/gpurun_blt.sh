set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/blt -o blt -- python3 -u tools/hipblaslt_probe.py > gpurun_out/blt.log 2>&1
find gpurun_out/blt -name "*kernel_stats.csv" | head -3
