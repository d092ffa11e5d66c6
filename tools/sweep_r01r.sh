#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw18
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_host_mirror.py -x -v --timeout 200 --timeout-method thread > gpurun_out/sw18/tests.log 2>&1 || { tail -60 gpurun_out/sw18/tests.log; exit 1; }
tail -20 gpurun_out/sw18/tests.log
