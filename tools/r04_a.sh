#!/bin/bash
# round 4: the IPC import-pattern probe, then resolve-vs-spill, bench.py's self-launched ranks
# and the rehearsals
set -o pipefail
mkdir -p gpurun_out/r04_a
timeout -k 5 120 python -u tools/ipc_stress_probe.py 8 1 > gpurun_out/r04_a/ipc_patterns.txt 2>&1
echo "probe rc=$?" >> gpurun_out/r04_a/ipc_patterns.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_exchange_maps.py > gpurun_out/r04_a/maps.txt 2>&1 &&
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_rehearsal.py tests/test_gpu_ipc_reuse.py tests/test_gpu_shuffle_exchange.py \
  > gpurun_out/r04_a/rehearsal.txt 2>&1
