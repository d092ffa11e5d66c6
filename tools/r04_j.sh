#!/bin/bash
# round 4: sort tests after the per-bucket lower-bound starts, timing, and the bench (its sort
# leg now sorts a real reduce partition)
set -o pipefail
O=gpurun_out/r04_j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py > $O/sort_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/sort_timing.txt 2>&1 || exit 1
  timeout -k 10 60 python3 tools/sort_prof.py 30 sort_msd=3 >> $O/sort_timing.txt 2>&1 || exit 1
done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err && echo bench ok || exit 1
timeout -k 10 600 python3 bench.py --tuning sort_msd=3 --maps-2e27 0 --plugin-groups 0 --plugin-host-maps 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 > $O/bench_msd3.json 2> $O/bench_msd3.err && echo bench3 ok
