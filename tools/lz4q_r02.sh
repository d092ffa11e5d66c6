#!/bin/bash
# One GPU call: the LZ4 parity tests under a short limit (progress per test), then the compress legs.
set -o pipefail
out=gpurun_out/${1:-lz4q}; mkdir -p $out
echo "start $(date +%s)"
timeout -k 10 100 python -u -m pytest tests/test_gpu_lz4.py -m gpu -x -v --timeout 60 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 150 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --reduce-sort-records 0 --file-maps 0 --plugin-groups 0 --self-check 0 > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -30 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print('compress', d['compress']); print('varlen compress', d['varlen']['compress'])"
