#!/bin/bash
# round 4, first GPU call: the IPC double-export probe, then bench.py's self-launched ranks
set -o pipefail
mkdir -p gpurun_out/r04_a
timeout -k 10 120 python -u tools/ipc_race_probe.py > gpurun_out/r04_a/ipc_race_probe.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_rehearsal.py -k "own_ranks or two_ranks" > gpurun_out/r04_a/rehearsal.txt 2>&1
