#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw16
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -x -v --timeout 120 --timeout-method thread -k "small or max_partitions or golden or record_sizes" > gpurun_out/sw16/tests.log 2>&1 || { tail -40 gpurun_out/sw16/tests.log; exit 1; }
tail -3 gpurun_out/sw16/tests.log
tools/sweep.sh gpurun_out/sw16 \
 ";--steps 3 --warmup 1 --workload small --map-records 1048576 --group-maps 16" \
 ";--steps 3 --warmup 1 --workload small --map-records 1048576 --group-maps 8" \
 ";--steps 3 --warmup 1 --workload small --map-records 1048576 --group-maps 32"
cat gpurun_out/sw16/sweep.txt
