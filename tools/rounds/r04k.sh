#!/bin/bash
# Round 4 experiment (toggle removed after: not adopted): rounds_kernel ring saves write-through (GGRS_EXP_WT=1) against the default
# policy on config 4 and config 3's general form (A/B twice), branch GPU tests under the toggle;
# the chains kernel with its prologue loads hoisted (config-2 P2P shape, twice).
set -u
TAG=${1:-r04k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
GGRS_EXP_WT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_branch.py \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 11; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], c.get('general_form_frames_per_s', ''))" gpurun_out/bench_${TAG}_$name.json $name
}
for i in 1 2; do
  for wt in 0 1; do
    if [ $wt = 1 ]; then export GGRS_EXP_WT=1; else unset GGRS_EXP_WT; fi
    run c4_wt${wt}_$i --config 4
    run c3_wt${wt}_$i --config 3
  done
  unset GGRS_EXP_WT
  run p2pc2_$i --workload p2p --sessions 4096 --latency 8 --max-prediction 9
done
echo $TAG done
