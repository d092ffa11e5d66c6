#!/bin/bash
# round 4: the sort with the chunked top pass: parity tests, timing (chunked vs one-pass top
# digit), kernel trace of the chunked run
set -o pipefail
O=gpurun_out/r04_sort; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sort.py > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/timing.txt 2>&1 || exit 1
  timeout -k 10 60 python3 tools/sort_prof.py 30 sort_msd=3 >> $O/timing.txt 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 tools/sort_prof.py 20 > $O/prof.txt 2>&1
