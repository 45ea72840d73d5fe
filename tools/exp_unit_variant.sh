#!/bin/bash
# A timing variant of one source unit (not parity-checked; never shipped): the scratch copy
# ggrs_amd/exp/src_<name>/<unit> compiled with the product's flags for that unit and linked with the
# product's other objects into ggrs_amd/exp/libggrs_amd_<name>.so.
#   bash tools/exp_unit_variant.sh <unit, e.g. codec.hip> <name> [-DMACRO ...]
set -e
cd "$(dirname "$0")/.."
UNIT=$1; NAME=$2; shift 2
SRC=ggrs_amd/exp/src_$NAME/$UNIT
[ -f "$SRC" ] || { mkdir -p "$(dirname $SRC)"; cp ggrs_amd/csrc/$UNIT "$SRC"; }
FLAGS=$(python3 -c "from ggrs_amd import build as b; print(' '.join([*b.FLAGS, *b.UNIT_FLAGS.get('$UNIT', [])]))")
OBJ=ggrs_amd/exp/${UNIT%.hip}_$NAME.o
/opt/rocm/bin/hipcc $FLAGS "$@" -I include -I ggrs_amd/csrc -c -o $OBJ $SRC
OTHERS=$(ls ggrs_amd/_obj/*.o | grep -v "/$UNIT.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ggrs_amd/exp/libggrs_amd_$NAME.so $OTHERS $OBJ
echo ggrs_amd/exp/libggrs_amd_$NAME.so
