#!/bin/bash
# Round 4: prefix kernel with write-through ring saves (config 3), canonical flat kernel with its
# sin/cos constants in VGPRs, chains kernel write-through A/B (GGRS_EXP_WT, experiment toggle):
# branch + P2P GPU tests, bench lines, config-3 trace + PMC.
set -u
TAG=${1:-r04i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_branch.py \
  tests/test_gpu_p2p.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_$name.json $name
}
for i in 1 2; do
  run c3_$i --config 3
  run p2p_$i --workload p2p
  unset GGRS_EXP_WT; run p2pc2_wt0_$i --workload p2p --sessions 4096 --latency 8 --max-prediction 9
  export GGRS_EXP_WT=1; run p2pc2_wt1_$i --workload p2p --sessions 4096 --latency 8 --max-prediction 9
  unset GGRS_EXP_WT
done
bash tools/profile.sh ${TAG}_c3 --config 3 || exit 12
echo $TAG done
