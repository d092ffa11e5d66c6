#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sw19
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_partition.py -x -q --timeout 200 --timeout-method thread -k "sort or small or max_part or golden or terasort_keys" > gpurun_out/sw19/tests.log 2>&1 || { tail -60 gpurun_out/sw19/tests.log; exit 1; }
tail -2 gpurun_out/sw19/tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sw19/b.json 2> gpurun_out/sw19/b.err || { tail gpurun_out/sw19/b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/sw19/b.json')); print(d['value'], d['reduce_sort'])"
tools/sweep.sh gpurun_out/sw19 ";--steps 3 --warmup 1 --workload small"
cat gpurun_out/sw19/sweep.txt
