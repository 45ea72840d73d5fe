#!/bin/bash
# Round 4: canonical flat kernel with the ring copy trimmed to the cells a launch reads / saves:
# P2P + desync GPU tests, the 65,536-session P2P bench line (twice), its kernel trace + PMC.
set -u
TAG=${1:-r04g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  tests/test_gpu_desync.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload p2p --no-cpu-baseline \
  > gpurun_out/bench_${TAG}_p2p_$i.json 2> gpurun_out/bench_${TAG}_p2p_$i.err || { tail -20 gpurun_out/bench_${TAG}_p2p_$i.err; exit 11; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('p2p', '%.4g' % d['value'], d['roofline']['avg_launch_ms'])" gpurun_out/bench_${TAG}_p2p_$i.json
done
bash tools/profile.sh ${TAG}_p2p --workload p2p || exit 12
echo $TAG done
