#!/bin/bash
# One GPU call: one-pass parity tests, then the full map-side suite, then a bench line.
set -o pipefail
tag=${1:-op1}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_onepass.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests_onepass.log 2>&1 || { tail -40 $out/tests_onepass.log; exit 1; }
tail -3 $out/tests_onepass.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_partition.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests_partition.log 2>&1 || { tail -40 $out/tests_partition.log; exit 1; }
tail -3 $out/tests_partition.log
timeout -k 10 300 python -u bench.py --map-records 131072 --group-maps 256 --steps 5 --warmup 2 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 > $out/bench_op.json 2> $out/bench_op.err || { tail -30 $out/bench_op.err; exit 1; }
cat $out/bench_op.json
SUX_ONEPASS=0 timeout -k 10 300 python -u bench.py --map-records 131072 --group-maps 256 --steps 5 --warmup 2 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 > $out/bench_3k.json 2> $out/bench_3k.err || { tail -30 $out/bench_3k.err; exit 1; }
cat $out/bench_3k.json
