#!/bin/bash
# One GPU call: variable-length parity tests, then the bench's varlen leg with varlen_kernel 2 and 3.
set -o pipefail
tag=${1:-varlen}; out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
legs="--steps 1 --warmup 1 --no-cpu-baseline --reduce-sort-records 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --self-check 0"
for k in 3; do
  timeout -k 10 300 python -u bench.py $legs --tuning varlen_kernel=$k > $out/bench_v$k.json 2> $out/bench_v$k.err || { tail -30 $out/bench_v$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_v$k.json')); print('varlen_kernel=$k', d['varlen'])"
done
