#!/bin/bash
# round 4 checkpoint 2: every GPU test, smoke, sort timing (chunked vs one-pass) + its kernel
# trace, then the default bench and its headline-only kernel stats
set -o pipefail
O=gpurun_out/r04_i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo smoke ok || exit 1
for i in 1 2; do
  timeout -k 10 60 python3 tools/sort_prof.py 30 >> $O/sort_timing.txt 2>&1 || exit 1
  timeout -k 10 60 python3 tools/sort_prof.py 30 sort_msd=3 >> $O/sort_timing.txt 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/sortprof -o run -- python3 tools/sort_prof.py 20 > $O/sortprof.txt 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err && echo bench ok
