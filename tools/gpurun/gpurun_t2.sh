set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pairs.py tests/test_slam.py tests/test_dataio.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/t2.log 2>&1; tail -15 gpurun_out/t2.log
