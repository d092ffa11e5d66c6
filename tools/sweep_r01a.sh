tools/sweep.sh gpurun_out/sw1 \
 ";--steps 3 --warmup 1 --group-maps 8" \
 ";--steps 3 --warmup 1 --group-maps 1" \
 "SUX_TILE_RECS=256;--steps 3 --warmup 1 --group-maps 1" \
 "SUX_TILE_RECS=512;--steps 3 --warmup 1 --group-maps 2" \
 "SUX_TILE_RECS=256;--steps 3 --warmup 1 --group-maps 2 --map-records 524288" \
 "SUX_TILE_RECS=512;--steps 3 --warmup 1 --group-maps 8 --streams 2" \
 "SUX_TILE_RECS=256;--steps 3 --warmup 1 --group-maps 1 --streams 2"
cat gpurun_out/sw1/sweep.txt
