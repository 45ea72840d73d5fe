#!/bin/bash
# The scheduled P2P bench lines with their CPU baselines, then a trace + PMC profile of one of them.
#   bash tools/evidence_lines.sh <tag> "<bench args of the profiled line>"
set -e
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1
mkdir -p gpurun_out/$TAG
for a in "p2p_jitter4096:--workload p2p --arrivals jitter --sessions 4096 --max-prediction 9" "p2p_stall:--workload p2p --arrivals stall" "p2p_jitter:--workload p2p --arrivals jitter"; do
  name=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/$TAG/lines_${TAG}_$name.json 2> gpurun_out/$TAG/$name.err
  echo "$name done"
done
bash tools/profile.sh ${TAG}_prof $2
