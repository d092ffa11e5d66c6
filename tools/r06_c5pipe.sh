set -e
mkdir -p gpurun_out/r06_o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipelined.py -k "msd16" > gpurun_out/r06_o/tests.txt 2>&1
LEG="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0"
for t in 24 56 24 56; do
  timeout -k 10 300 python -u bench.py $LEG --tuning msd_direct=$t > gpurun_out/r06_o/c5_$t.json 2>> gpurun_out/r06_o/c5.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06_o/c5_$t.json').read().strip().splitlines()[-1]); rm=d['roofline_map_side']; print('msd_direct=$t', d['value'], d['ms_per_step'], rm['kernels_ms'], d['self_check'] if 'self_check' in d else '')" >> gpurun_out/r06_o/summary.txt
  timeout -k 10 300 python -u bench.py $LEG --map-pipeline 0 --tuning msd_direct=$t > gpurun_out/r06_o/c5s_$t.json 2>> gpurun_out/r06_o/c5.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06_o/c5s_$t.json').read().strip().splitlines()[-1]); rm=d['roofline_map_side']; print('serial msd_direct=$t', d['value'], d['ms_per_step'], rm['kernels_ms'])" >> gpurun_out/r06_o/summary.txt
done
