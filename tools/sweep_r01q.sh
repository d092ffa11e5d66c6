#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw17
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sw17/tests.log 2>&1 || { tail -40 gpurun_out/sw17/tests.log; exit 1; }
tail -2 gpurun_out/sw17/tests.log
tools/sweep.sh gpurun_out/sw17 \
 ";--steps 3 --warmup 1 --workload small" \
 ";--steps 3 --warmup 1"
cat gpurun_out/sw17/sweep.txt
