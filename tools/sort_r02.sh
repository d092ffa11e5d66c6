#!/bin/bash
# One GPU call: sort parity tests, then the bench's reduce-side sort legs with the MSD finish
# (default) and with LSD passes only (sort_msd=2).
set -o pipefail
tag=${1:-sort}; out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
legs="--steps 1 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --self-check 0"
for t in 1; do
  timeout -k 10 300 python -u bench.py $legs --tuning sort_msd=$t > $out/bench_msd$t.json 2> $out/bench_msd$t.err || { tail -30 $out/bench_msd$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_msd$t.json')); print('sort_msd=$t', d['reduce_sort'], d['reduce_sort_long'])"
done
