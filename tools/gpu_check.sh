#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprofv3 kernel-trace summary.  Stops at the first failure.
# usage: tools/gpu_check.sh TAG [extra bench args]
set -o pipefail
tag=${1:-r01}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== tests" && timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
echo "== smoke" && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -30 $out/smoke.log; exit 1; }
echo "== bench" && timeout -k 10 400 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
echo "== rocprof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $out/prof.json 2> $out/prof.err || { tail -30 $out/prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
head -12 $out/kernel_stats.csv
echo "== sort A/B" && timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --self-check 0 --tuning small_kernel=1 > $out/bench_sort_turn.json 2> $out/bench_sort_turn.err || { tail -20 $out/bench_sort_turn.err; exit 1; }
python3 -c "import json; a=json.load(open('$out/bench.json')); b=json.load(open('$out/bench_sort_turn.json')); print('sort sorted-chunk', a['reduce_sort'], a['reduce_sort_long']); print('sort turn       ', b['reduce_sort'], b['reduce_sort_long'])"
