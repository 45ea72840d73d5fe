#!/bin/bash
# Round 4 probe: the all-units max-ilp experiment library halted every config-5 session (r04q);
# run the particle GPU parity tests against it (and against the product library) to see whether
# the particle kernel's results change with the machine scheduler.
set -u
TAG=${1:-r04r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_particles.py \
  > gpurun_out/pytest_${TAG}_prod.log 2>&1; echo "prod rc=$?"; tail -3 gpurun_out/pytest_${TAG}_prod.log
GGRS_AMD_EXP_LIB=libggrs_amd_allilp.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_particles.py > gpurun_out/pytest_${TAG}_allilp.log 2>&1; echo "allilp rc=$?"; tail -15 gpurun_out/pytest_${TAG}_allilp.log
echo $TAG done
