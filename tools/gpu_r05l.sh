set -o pipefail
O=gpurun_out/r05_l; mkdir -p $O
export TMPDIR=/tmp
LEGS="--workload small --steps 3 --warmup 1 --no-cpu-baseline --reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0 --self-check 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one -o run -- python3 bench.py $LEGS --map-pipeline 0 > $O/one.json 2> $O/one.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/two -o run -- python3 bench.py $LEGS > $O/two.json 2> $O/two.err || exit 1
echo done
