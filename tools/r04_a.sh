#!/bin/bash
# round 4, first GPU call: the JVM group formation / large maps through the JNI harness,
# resolve-vs-spill, bench.py's self-launched ranks and the rehearsals, then the IPC stress probe
set -o pipefail
mkdir -p gpurun_out/r04_a
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_host_mirror.py tests/test_gpu_exchange_maps.py \
  > gpurun_out/r04_a/jni_and_maps.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_rehearsal.py tests/test_gpu_ipc_reuse.py tests/test_gpu_shuffle_exchange.py \
  > gpurun_out/r04_a/rehearsal.txt 2>&1
rc=$?
timeout -k 5 150 python -u tools/ipc_stress_probe.py 8 10 > gpurun_out/r04_a/ipc_stress_probe.txt 2>&1
echo "stress probe rc=$?" >> gpurun_out/r04_a/ipc_stress_probe.txt
exit $rc
