#!/bin/bash
# Diagnostic builds of the library for VERDICT r05 #2 (k_msd16a's LDS bank conflicts): the same
# library with sux_small.hip compiled under SUX_MSD_WHATIF=LEVEL (pass A's output is then NOT
# bucket-sorted — time it with --self-check 0 only):
#   1  the stage store at a conflict-free slot, no bucket-start read (the ds_write_b128 scatter's
#      conflicts gone)
#   2  1 + the wave ranking's counter accesses at conflict-free digits
# Output: tools/whatif<LEVEL>/libsparkucx_amd.so (run on the GPU with tools/gpujob.sh ab).
#   usage: tools/msd_whatif.sh LEVEL...   (from the repo root, after make -C sparkucx_amd/csrc)
set -e
ROCM=${ROCM:-/opt/rocm}
C=sparkucx_amd/csrc
for L in "$@"; do
  D=tools/whatif$L
  mkdir -p $D
  $ROCM/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall \
    -Wno-unused-result -I$ROCM/include -Iinclude -DSUX_MSD_WHATIF=$L -c $C/sux_small.hip -o $D/sux_small.o
  objs=$(ls $C/build/*.o | grep -v -e sux_small.hip.o -e _loop -e loopback_rccl)
  $ROCM/bin/hipcc --offload-arch=gfx950 $objs $D/sux_small.o -shared -L$ROCM/lib \
    -Wl,-rpath,$ROCM/lib -lrccl -lamdhip64 -o $D/libsparkucx_amd.so
  rm -f $D/sux_small.o
  echo "built $D/libsparkucx_amd.so"
done
