#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw15
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/sw15/tests.log 2>&1 || { tail -40 gpurun_out/sw15/tests.log; exit 1; }
tail -2 gpurun_out/sw15/tests.log
tools/sweep.sh gpurun_out/sw15 \
 ";--steps 3 --warmup 1" \
 ";--steps 3 --warmup 1 --workload small --map-records 1048576 --group-maps 16"
cat gpurun_out/sw15/sweep.txt
