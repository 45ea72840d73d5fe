#!/bin/bash
# P2P iteration on the GPU box: P2P + desync parity tests, the P2P bench (default and HBM-ring flat
# form), optionally the profile.  usage: bash tools/p2p_round.sh <tag> [prof]
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG}_p2p tests/test_gpu_p2p.py tests/test_gpu_desync.py || exit 10
timeout -k 10 300 python -u bench.py --workload p2p --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 11; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python -u bench.py --workload p2p --no-cpu-baseline --p2p-form flat > gpurun_out/bench_${TAG}_hbm.json 2> gpurun_out/bench_${TAG}_hbm.err || exit 12
[ "${2:-}" = "prof" ] || exit 0
bash tools/profile.sh $TAG --workload p2p --steps 10 || exit 13
echo p2p_round done
