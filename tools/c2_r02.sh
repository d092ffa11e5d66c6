#!/bin/bash
# BASELINE configs that fit one GPU, full size, default (pipelined) map side, self-checked.
set -o pipefail
out=gpurun_out/${1:-r02_configs}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 "$@" > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -20 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('%-24s %8.1f GB/s  ms/step %7.2f  k3 %s %.3f  map %.3f  check %s  %s' % ('$name', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline_map_side']['frac'], d.get('self_check',{}).get('ok'), d['config']['workload'][:80]))"
}
run c2_terasort_100GB --steps 3 --warmup 1
run c2_terasort_maps2e27 --steps 3 --warmup 1 --map-records 134217728
run c4_zipf_100GB --steps 3 --warmup 1 --workload zipf
run c5_small_17GB --steps 3 --warmup 1 --workload small
run c5_small_maps64k --steps 3 --warmup 1 --workload small --map-records 65536
