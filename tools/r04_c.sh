#!/bin/bash
# round 4: the headline bench (full default line), a headline-only rocprof kernel trace + stats
# (every k_scatter8 launch in it is a headline launch), and the PMC passes for terasort, zipf and
# small (profiles/collect_pmc.py).  Run from the repo root on the GPU box.
set -o pipefail
O=gpurun_out/r04_c; mkdir -p $O
export TMPDIR=/tmp
HEAD="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --self-check 0 --no-cpu-baseline"
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_headline -o run -- python3 bench.py --steps 5 --warmup 2 $HEAD > $O/prof_headline.json 2> $O/prof_headline.err &&
for w in terasort zipf small; do
  timeout -k 10 500 python3 profiles/collect_pmc.py --out $O/pmc --workload $w > $O/pmc_$w.log 2>&1 || exit 1
done
