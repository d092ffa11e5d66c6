set -e
mkdir -p gpurun_out/r06_n
timeout -k 10 800 python -u bench.py > gpurun_out/r06_n/bench.json 2> gpurun_out/r06_n/bench.err
LEG="--workload small --steps 3 --warmup 1 --no-cpu-baseline --varlen-rows 0 --compress-maps 0 --file-maps 0 --reduce-sort-records 0 --plugin-groups 0 --plugin-host-maps 0 --maps-2e27 0 --c4-steps 0 --c5-steps 0"
timeout -k 10 300 python -u bench.py $LEG --map-pipeline 0 > gpurun_out/r06_n/c5_serial.json 2> gpurun_out/r06_n/c5_serial.err
timeout -k 10 300 python -u bench.py $LEG > gpurun_out/r06_n/c5_pipe.json 2> gpurun_out/r06_n/c5_pipe.err
