#!/bin/bash
# Timing-experiment variants of the engine library (results NOT parity-checked; never shipped):
#   bash tools/exp_build.sh <name> -DMACRO ...   ->  ggrs_amd/exp/libggrs_amd_<name>.so
# select one at run time with GGRS_AMD_EXP_LIB=libggrs_amd_<name>.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ggrs_amd/exp
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -Wno-unused-function \
  "$@" -I include -I ggrs_amd/csrc -o ggrs_amd/exp/libggrs_amd_$NAME.so \
  ggrs_amd/csrc/engine.hip ggrs_amd/csrc/branch.hip ggrs_amd/csrc/particles.hip ggrs_amd/csrc/p2p.hip ggrs_amd/csrc/codec.hip
echo ggrs_amd/exp/libggrs_amd_$NAME.so
