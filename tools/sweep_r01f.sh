#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw6
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/sw6/tests.log 2>&1 || { tail -30 gpurun_out/sw6/tests.log; exit 1; }
tail -2 gpurun_out/sw6/tests.log
tools/sweep.sh gpurun_out/sw6 \
 ";--steps 3 --warmup 1 --reserve-cus 32" \
 ";--steps 3 --warmup 1 --reserve-cus 64" \
 ";--steps 3 --warmup 1 --workload zipf" \
 ";--steps 3 --warmup 1 --workload small --map-records 1048576 --group-maps 16"
cat gpurun_out/sw6/sweep.txt
