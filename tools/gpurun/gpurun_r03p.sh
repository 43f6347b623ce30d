#!/bin/bash
# attention kernel variants at the batched frame composition (encoder 8 images, Bp = 2 pairs)
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 3 4 0; do
  echo "== S3_ATTN_VARIANT=$v"
  S3_ATTN_VARIANT=$v CONFIGS=" " bash tools/gpurun/gpurun_ab.sh | grep fps || exit 1
done
