#!/bin/bash
# Round 4 probe: particle parity under max-ilp with particles.h's two inline-asm 24-bit multiply-adds
# written as __umul24 / __mul24 (ggrs_amd/exp/libggrs_amd_noasm.so) -- does the r04r failure follow
# the inline asm?
set -u
TAG=${1:-r04v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
GGRS_AMD_EXP_LIB=libggrs_amd_noasm.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_particles.py > gpurun_out/pytest_${TAG}_noasm.log 2>&1; echo "noasm rc=$?"; tail -4 gpurun_out/pytest_${TAG}_noasm.log
echo $TAG done
