#!/bin/bash
# Round 4: PMC profiles (tools/profile.sh: kernel trace, FETCH/WRITE, SQ, GRBM passes) of config 2
# on the current tree, the P2P config-2 shape (chains form) and the 65,536-session P2P default
# (canonical flat kernel).
set -u
TAG=${1:-r04c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/profile.sh ${TAG}_c2 || exit 11
bash tools/profile.sh ${TAG}_p2pc2 --workload p2p --sessions 4096 --latency 8 --max-prediction 9 || exit 12
bash tools/profile.sh ${TAG}_p2p --workload p2p || exit 13
echo r04c done
