#!/bin/bash
# Round 2: full-size runs of every BASELINE.json config that fits one GPU (+ the N>1 rehearsal).
set -o pipefail
out=gpurun_out/configs_r02
mkdir -p $out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -20 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['value'], d['unit'], d['ms_per_step'], d['config']['workload'][:90], d.get('reduce_sort', {}).get('GB/s'))"
}
legs="--varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --reduce-sort-records 0"
run c2_terasort_100GB --steps 3 --warmup 1
run c2_terasort_maps2e27 --steps 2 --warmup 1 --map-records 134217728 --group-maps 1 $legs
run c4_zipf_100GB --steps 3 --warmup 1 --workload zipf $legs
run c5_small_17GB --steps 3 --warmup 1 --workload small $legs
run c5_small_maps64k --steps 3 --warmup 1 --workload small --map-records 65536 --group-maps 256 $legs
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_rehearsal.py -q --timeout 250 --timeout-method thread > $out/rehearsal.log 2>&1 || { tail -30 $out/rehearsal.log; exit 1; }
tail -1 $out/rehearsal.log
