#!/bin/bash
# round 4: C5 direct-store variants (parity + bench), the one-read probe
set -o pipefail
O=gpurun_out/r04_b; mkdir -p $O
timeout -k 5 150 python -u tools/ipc_stress_probe.py 8 1 > $O/ipc_ptracer.txt 2>&1
echo "probe rc=$?" >> $O/ipc_ptracer.txt
LEGS="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipelined.py -k "msd16" > $O/msd_tests.txt 2>&1 &&
for d in 0 1 2 3; do
  timeout -k 10 240 python -u bench.py --workload small --steps 5 --warmup 2 $LEGS --tuning msd_direct=$d > $O/c5_direct$d.json 2> $O/c5_direct$d.err || exit 1
done &&
for d in 0 3; do
  timeout -k 10 240 python -u bench.py --workload small --map-records 65536 --steps 5 --warmup 2 $LEGS --tuning msd_direct=$d > $O/c5_m64k_direct$d.json 2> $O/c5_m64k_direct$d.err || exit 1
done &&
timeout -k 10 120 tools/onemap_probe_2048 32 > $O/onemap_2048.txt 2>&1 &&
timeout -k 10 120 tools/onemap_probe_4096 32 > $O/onemap_4096.txt 2>&1
