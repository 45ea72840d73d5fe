#!/bin/bash
# A timing variant of p2p_sched.hip only (not parity-checked; never shipped): the scratch copy
# ggrs_amd/exp/src_<name>/p2p_sched.hip (edit it, or pass -D macros) compiled with the product's
# flags and linked with the product's other objects into ggrs_amd/exp/libggrs_amd_<name>.so.
#   bash tools/exp_sched_variant.sh <name> [-DMACRO ...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
SRC=ggrs_amd/exp/src_$NAME/p2p_sched.hip
[ -f "$SRC" ] || { mkdir -p "$(dirname $SRC)"; cp ggrs_amd/csrc/p2p_sched.hip "$SRC"; }
FLAGS=$(python3 -c "from ggrs_amd import build as b; print(' '.join([*b.FLAGS, *b.UNIT_FLAGS['p2p_sched.hip']]))")
OBJ=ggrs_amd/exp/p2p_sched_$NAME.o
/opt/rocm/bin/hipcc $FLAGS "$@" -I include -I ggrs_amd/csrc -c -o $OBJ $SRC
OTHERS=$(ls ggrs_amd/_obj/*.o | grep -v p2p_sched.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ggrs_amd/exp/libggrs_amd_$NAME.so $OTHERS $OBJ
echo ggrs_amd/exp/libggrs_amd_$NAME.so
