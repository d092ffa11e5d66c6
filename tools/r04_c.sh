#!/bin/bash
# round 4: MSD scan rewrite parity + C5 lines, the IPC pattern probe (fixed), the headline bench,
# a headline-only rocprof kernel trace + stats, PMC passes
set -o pipefail
O=gpurun_out/r04_c; mkdir -p $O
export TMPDIR=/tmp
LEGS="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipelined.py -k "msd16 or small" > $O/msd_tests.txt 2>&1 &&
timeout -k 10 240 python -u bench.py --workload small --steps 5 --warmup 2 $LEGS > $O/c5.json 2> $O/c5.err &&
timeout -k 10 240 python -u bench.py --workload small --map-records 65536 --steps 5 --warmup 2 $LEGS > $O/c5_m64k.json 2> $O/c5_m64k.err &&
timeout -k 5 150 python -u tools/ipc_stress_probe.py 8 3 > $O/ipc_patterns.txt 2>&1
echo "probe rc=$?" >> $O/ipc_patterns.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_headline -o run -- python3 bench.py --steps 5 --warmup 2 $LEGS --self-check 0 > $O/prof_headline.json 2> $O/prof_headline.err
