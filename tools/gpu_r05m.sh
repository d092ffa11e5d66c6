set -o pipefail
O=gpurun_out/r05_m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort.py > $O/sort_tests.txt 2>&1; rc=$?; echo "sort tests rc=$rc"; tail -2 $O/sort_tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_random_$i.txt 2>&1 || exit 1
SORT_PROF_INPUT=partition timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_partition_$i.txt 2>&1 || exit 1
done
tail -qn 1 $O/sort_random_*.txt $O/sort_partition_*.txt
LEGS="--workload small --steps 3 --warmup 1 --no-cpu-baseline --reduce-sort-records 0 --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0 --self-check 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one -o run -- python3 bench.py $LEGS --map-pipeline 0 > $O/one.json 2> $O/one.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/two -o run -- python3 bench.py $LEGS > $O/two.json 2> $O/two.err || exit 1
echo done
