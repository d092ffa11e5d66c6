#!/bin/bash
# round 4: large-bucket launches on a side stream: sort tests, timing (random / range-partition
# keys), the bench's reduce_sort on a real partition
set -o pipefail
O=gpurun_out/r04_sort2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py > $O/sort_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/timing.txt 2>&1 || exit 1
  SORT_PROF_INPUT=partition timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/timing.txt 2>&1 || exit 1
  SORT_PROF_INPUT=partition timeout -k 10 60 python3 tools/sort_prof.py 30 sort_msd=3 >> $O/timing.txt 2>&1 || exit 1
done
timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 > $O/bench.json 2> $O/bench.err && echo bench ok
