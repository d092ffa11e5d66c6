set -o pipefail
mkdir -p gpurun_out/s3a
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -m gpu -x -v --timeout 120 --timeout-method thread -k "exchange" > gpurun_out/s3a/tests.log 2>&1 || { tail -40 gpurun_out/s3a/tests.log; exit 1; }
tail -3 gpurun_out/s3a/tests.log
timeout -k 10 300 python -u bench.py --rccl-at-one --records 268435456 --steps 3 --warmup 1 > gpurun_out/s3a/bench_rccl1.json 2> gpurun_out/s3a/bench_rccl1.err || { tail -30 gpurun_out/s3a/bench_rccl1.err; exit 1; }
cat gpurun_out/s3a/bench_rccl1.json
