set -o pipefail
mkdir -p gpurun_out/k3ab
legs="--reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $legs --map-pipeline 0 > gpurun_out/k3ab/iso.json 2>gpurun_out/k3ab/iso.err && timeout -k 10 200 python -u bench.py $legs > gpurun_out/k3ab/pipe.json 2>gpurun_out/k3ab/pipe.err && python3 -c "
import json
for f in ['iso','pipe']:
    d=json.load(open('gpurun_out/k3ab/'+f+'.json')); print(f, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['self_check']['ok'])"
