#!/bin/bash
# round 4 final checkpoint: every GPU test, smoke, the default bench
set -o pipefail
O=gpurun_out/${OUT:-r04_final}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo smoke ok || exit 1
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err && echo bench ok
