#!/bin/bash
set -o pipefail
tag=${1:-st}
mkdir -p gpurun_out/$tag
timeout -k 10 120 ./tools/op_stamps 64 > gpurun_out/$tag/op_stamps.txt 2>&1 || { cat gpurun_out/$tag/op_stamps.txt; exit 1; }
cat gpurun_out/$tag/op_stamps.txt
