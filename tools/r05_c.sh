set -o pipefail
O=gpurun_out/r05_c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29555 bench.py --gpus 8 --rehearse-one-gpu --workload terasort --records 100000 --map-records 20000 --group-maps 2 --steps 1 --warmup 0 --verify > $O/w8.json 2> $O/w8.err; echo "w8 rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_host_mirror.py tests/test_gpu_exchange_maps.py tests/test_gpu_bench_rehearsal.py > $O/tests.txt 2>&1; echo "tests rc=$?"
