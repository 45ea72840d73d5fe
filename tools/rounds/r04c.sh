#!/bin/bash
# Round 4: PMC profiles (tools/profile.sh: kernel trace, FETCH/WRITE, SQ, GRBM passes) of config 2
# on the current tree, the P2P config-2 shape (chains form) and the 65,536-session P2P default
# (canonical flat kernel).
set -u
TAG=${1:-r04c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  tests/test_gpu_branch.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench.py --workload p2p --sessions 4096 --latency 8 --max-prediction 9 --no-cpu-baseline \
  > gpurun_out/bench_${TAG}_p2pc2.json 2> gpurun_out/bench_${TAG}_p2pc2.err || { tail -20 gpurun_out/bench_${TAG}_p2pc2.err; exit 11; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('p2p c2', '%.4g' % d['value'], d['roofline']['avg_launch_ms'])" gpurun_out/bench_${TAG}_p2pc2.json
bash tools/profile.sh ${TAG}_c2 || exit 11
bash tools/profile.sh ${TAG}_p2pc2 --workload p2p --sessions 4096 --latency 8 --max-prediction 9 || exit 12
bash tools/profile.sh ${TAG}_p2p --workload p2p || exit 13
echo r04c done
