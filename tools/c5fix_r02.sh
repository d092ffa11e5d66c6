set -o pipefail
mkdir -p gpurun_out/c5fix
legs="--varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --reduce-sort-records 0 --no-cpu-baseline"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_partition.py -m gpu -x -q --timeout 200 --timeout-method thread -k "small or msd or sorted_chunk" > gpurun_out/c5fix/tests.log 2>&1 || { tail -20 gpurun_out/c5fix/tests.log; exit 1; }
tail -1 gpurun_out/c5fix/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workload small --map-records 65536 --group-maps 256 $legs > gpurun_out/c5fix/maps64k.json 2> gpurun_out/c5fix/maps64k.err && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --workload small $legs > gpurun_out/c5fix/small.json 2> gpurun_out/c5fix/small.err && python3 -c "
import json
for f in ['maps64k','small']:
    d=json.load(open('gpurun_out/c5fix/'+f+'.json')); print(f, d['value'], d['roofline']['kernel'], d['self_check']['ok'])"
