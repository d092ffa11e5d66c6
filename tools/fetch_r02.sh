set -o pipefail
out=gpurun_out/fetch1; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_mirror.py tests/test_gpu_shuffle_exchange.py tests/test_gpu_sort.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --reduce-sort-records 0 --file-maps 0 --compress-maps 0 --varlen-rows 0 --self-check 0 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['plugin'])"
