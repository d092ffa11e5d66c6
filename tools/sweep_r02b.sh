#!/bin/bash
# Map-side launch-overlap sweep through the node tuning table (sux_tuning), every line
# self-checked (bench.py --self-check: index offsets, record multiset, partition grouping).
# usage: tools/sweep_r02b.sh TAG
set -o pipefail
out=gpurun_out/${1:-r02_sw_b}
mkdir -p $out
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 \
    --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 "$@" \
    > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); m=d['roofline_map_side']; print('%-24s %8.1f GB/s  ms/step %7.2f  hist %6.1f  scatter %6.1f  k3 frac %.3f  check %s' % ('$name', d['value'], d['ms_per_step'], m['kernels_ms']['hist']/d['steps'], m['kernels_ms']['scatter']/d['steps'], d['roofline']['frac'], d['self_check']['ok']))"
}
run base --map-pipeline 0
run base_s2 --map-pipeline 0 --streams 2
run pipe_co --map-pipeline 1
run pipe_co_h1 --map-pipeline 1 --tuning hist_wgs_per_cu=1
run pipe_co_h2 --map-pipeline 1 --tuning hist_wgs_per_cu=2
run pipe_co_d2 --map-pipeline 1 --tuning scatter_depth=2
run pipe_noco --map-pipeline 1 --tuning coresident=-1
run pipe_noco_h1 --map-pipeline 1 --tuning coresident=-1,hist_wgs_per_cu=1
