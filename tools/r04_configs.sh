#!/bin/bash
# round 4: the other BASELINE configs at N = 1 with the round-4 PMC traffic (C4 Zipf, C5 small)
set -o pipefail
O=gpurun_out/r04_configs; mkdir -p $O
L="--varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0"
timeout -k 10 400 python3 bench.py --workload zipf $L > $O/c4_zipf.json 2> $O/c4_zipf.err || exit 1
timeout -k 10 400 python3 bench.py --workload small $L > $O/c5_small.json 2> $O/c5_small.err && echo ok
