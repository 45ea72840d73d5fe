#!/bin/bash
# Round 4: branch / desync tests (lane-pair trunk split, canonical desync history), config 3 line +
# phase stamps + rocprof, then the config-3 PMC profile.
set -u
TAG=${1:-r04b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_branch.py tests/test_gpu_desync.py tests/test_gpu_exchange.py \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
bash tools/rounds/r04_c3.sh ${TAG}_c3 || exit 11
bash tools/profile.sh ${TAG}_pc3 --config 3 || exit 12
echo r04b done
