set -o pipefail
O=gpurun_out/r05_h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/diag_hip.py > $O/diag.txt 2>&1; echo "diag rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_pipelined.py -k "sort or msd16" > $O/sort_msd_tests.txt 2>&1; rc=$?; echo "sort/msd tests rc=$rc"; tail -3 $O/sort_msd_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_random.txt 2>&1 || exit 1
SORT_PROF_INPUT=partition timeout -k 10 120 python3 tools/sort_prof.py 20 > $O/sort_partition.txt 2>&1 || exit 1
tail -1 $O/sort_random.txt $O/sort_partition.txt
L="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0"
for i in 1 2; do
for t in 0 8 16 24; do
timeout -k 10 200 python3 bench.py $L --tuning msd_direct=$t > $O/c5_t${t}_$i.json 2> $O/c5_t${t}_$i.err || exit 1
done
echo "round $i done"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py -k "owned or peer_major or tickets or export_cache or single_rank" tests/test_gpu_bench_rehearsal.py > $O/own_tests.txt 2>&1; echo "own tests rc=$?"; tail -3 $O/own_tests.txt
