#!/bin/bash
# Every workload on one box: GPU tests, default bench + profile (tools/round.sh), config-5 profile,
# then the bench line of configs 3, 4, 5, P2P and the codec.  usage: bash tools/all_workloads.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/round.sh $TAG || exit $?
bash tools/profile.sh ${TAG}_c5 --config 5 --steps 10 || exit 20
bash tools/gpu_bench.sh ${TAG}_w "--config 3" "--config 4" "--config 5" "--workload p2p" "--workload codec" || exit 21
echo all done
