#!/bin/bash
# One GPU call: LZ4 parity (liblz4 bit-exact), then the compress legs of the bench.
set -o pipefail
tag=${1:-lz4}; out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --reduce-sort-records 0 --file-maps 0 --plugin-groups 0 --self-check 0 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print('compress', d['compress']); print('varlen compress', d['varlen']['compress'])"
