#!/bin/bash
# One GPU call: MSD small-record parity tests, then C5 bench A/B (sorted chunks vs two-level MSD,
# isolated launch groups and pipelined) and a rocprofv3 kernel summary.  Stops at the first failure.
# usage: tools/msd_r02.sh TAG
set -o pipefail
tag=${1:-msd}; out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
legs="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --no-cpu-baseline"
echo "== tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py -m gpu -x -v --timeout 120 --timeout-method thread -k "msd or small_record or sorted_chunk" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
run() {  # name, extra args
  timeout -k 10 300 python -u bench.py --workload small --steps 5 --warmup 2 $legs "${@:2}" > $out/bench_$1.json 2> $out/bench_$1.err || { tail -30 $out/bench_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$1.json')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], {k: round(v/5,2) for k,v in d['roofline_map_side']['kernels_ms'].items()}, d.get('self_check',{}).get('ok'))"
}
echo "== bench"
run k4iso --map-pipeline 0 --tuning small_kernel=4
run k4 --tuning small_kernel=4
#run k4w1 --tuning small_kernel=4,small_wgs_per_cu=1
#run k4w1iso --map-pipeline 0 --tuning small_kernel=4,small_wgs_per_cu=1
echo "== stamps" && timeout -k 10 120 ./tools/msd_stamps 200 > $out/stamps.txt 2>&1 || { cat $out/stamps.txt; exit 1; }; cat $out/stamps.txt
