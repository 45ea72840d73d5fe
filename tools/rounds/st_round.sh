#!/bin/bash
# SyncTest iteration on the GPU box: SyncTest parity tests, default bench (v5) and the v4 path,
# then the profile of the default bench.  usage: bash tools/st_round.sh <tag> [noprof]
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG}_st tests/test_gpu_synctest.py tests/test_gpu_sincosf.py || exit 10
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 11; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --path chains > gpurun_out/bench_${TAG}_v4.json 2> gpurun_out/bench_${TAG}_v4.err || exit 12
[ "${2:-}" = "noprof" ] && exit 0
bash tools/profile.sh $TAG --steps 10 || exit 13
echo st_round done
