#!/bin/bash
# plugin-leg shapes on one GPU (bench.py --rehearse-one-gpu): which fail the device check
out=gpurun_out/r03t; mkdir -p $out
run() { tag=$1; w=$2; shift 2
  timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=$w --master-addr=127.0.0.1 --master-port=$((29500 + RANDOM % 400)) bench.py --gpus $w --rehearse-one-gpu --steps 1 --warmup 0 --self-check 0 "$@" > $out/$tag.json 2> $out/$tag.err
  rc=$?; echo "$tag rc=$rc $(grep -h -m1 'RuntimeError: ' $out/$tag.err)" | tee -a $out/summary.txt
  [ $rc -ge 124 ] && exit $rc; return 0; }
run w8_m19_g2_p4 8 --records 4194304 --map-records 524288 --group-maps 2 --plugin-groups 4
run w8_m19_g2_p4_0 8 --records 4194304 --map-records 524288 --group-maps 2 --plugin-groups 4 --steps 0
