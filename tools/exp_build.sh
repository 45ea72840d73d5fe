#!/bin/bash
# Timing-experiment variants of the engine library (results NOT parity-checked; never shipped):
#   bash tools/exp_build.sh <name> -DMACRO ...   ->  ggrs_amd/exp/libggrs_amd_<name>.so
# The product sources carry no experiment switches: this copies ggrs_amd/csrc to a scratch
# directory, applies tools/exp/*.patch there (the hooks: GGRS_EXP_STAMPS phase stamps,
# GGRS_EXP_NOCLAMP, GGRS_EXP_PIN) and builds it with the product's units and flags plus the given
# ones; objects in ggrs_amd/exp/libggrs_amd_<name>.so.obj.  Select one at run time with
# GGRS_AMD_EXP_LIB=libggrs_amd_<name>.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ggrs_amd/exp
SCRATCH=ggrs_amd/exp/src_$NAME
rm -rf "$SCRATCH" && cp -r ggrs_amd/csrc "$SCRATCH"
for p in tools/exp/*.patch; do patch -s -d "$SCRATCH" -p1 < "$p"; done
python3 - "$NAME" "$SCRATCH" "$@" <<'PY'
import os, sys
from ggrs_amd import build
name, src, extra = sys.argv[1], os.path.abspath(sys.argv[2]), sys.argv[3:]
print(build.build(force=True, out=f"ggrs_amd/exp/libggrs_amd_{name}.so", extra=extra, csrc=src))
PY
