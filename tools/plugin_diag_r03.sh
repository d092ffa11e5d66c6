#!/bin/bash
# plugin-path diagnostic shapes (tools/plugin_diag.py), one GPU, 8 ranks
out=gpurun_out/r03s; mkdir -p $out
d() { tag=$1; shift
  timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=$((29500 + RANDOM % 400)) tools/plugin_diag.py "$@" > $out/$tag.log 2>&1
  rc=$?; echo "== $tag rc=$rc"; grep -h "maps differ\|batched\|map_output_index\|pid check" $out/$tag.log | sort | head -8
  [ $rc -ge 124 ] && exit $rc; return 0; }
d m19g2 524288 2 4


