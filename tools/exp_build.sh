#!/bin/bash
# Timing-experiment variants of the engine library (results NOT parity-checked; never shipped):
#   bash tools/exp_build.sh <name> -DMACRO ...   ->  ggrs_amd/exp/libggrs_amd_<name>.so
# Same units and flags as the product build (ggrs_amd/build.py), plus the given ones; objects in
# ggrs_amd/exp/libggrs_amd_<name>.so.obj.  Select one at run time with
# GGRS_AMD_EXP_LIB=libggrs_amd_<name>.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ggrs_amd/exp
python3 - "$NAME" "$@" <<'PY'
import sys
from ggrs_amd import build
name, extra = sys.argv[1], sys.argv[2:]
print(build.build(force=True, out=f"ggrs_amd/exp/libggrs_amd_{name}.so", extra=extra))
PY
