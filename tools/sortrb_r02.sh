#!/bin/bash
# One GPU call: sort + exchange + fetch tests, then the bench's sort legs (pinned read-backs).
set -o pipefail
out=gpurun_out/${1:-sortrb}; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_shuffle_exchange.py tests/test_gpu_host_mirror.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --self-check 0 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['reduce_sort'], d['reduce_sort_long']); print(d['plugin']['fetch_one_reducer'])"
