#!/bin/bash
# Round 4 (ran against commit 64e156e, reverted after): v5 at 32 threads per block (two waves per SIMD at 4096 sessions) against 64: parity of
# the SyncTest GPU tests under GGRS_V5_THREADS=32, then config 2 bench lines of both forms.
set -u
TAG=${1:-r04d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
GGRS_V5_THREADS=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_synctest.py > gpurun_out/pytest_${TAG}_32.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}_32.log; exit 10; }
tail -2 gpurun_out/pytest_${TAG}_32.log
for kw in 64 32 64 32; do
  GGRS_V5_THREADS=$kw timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$kw.json \
    2> gpurun_out/bench_${TAG}_$kw.err || { tail -20 gpurun_out/bench_${TAG}_$kw.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2 kw', sys.argv[2], '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_$kw.json $kw
done
echo $TAG done
