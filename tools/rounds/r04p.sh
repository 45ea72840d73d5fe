#!/bin/bash
# Round 4: branch.hip on the default machine scheduler: branch + exchange GPU tests, config 3 (and its
# general form) and config 4 bench lines twice, config-3 kernel trace + PMC.
set -u
TAG=${1:-r04p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_branch.py \
  tests/test_gpu_exchange.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], c.get('general_form_frames_per_s', ''))" gpurun_out/bench_${TAG}_$name.json $name
}
for i in 1 2; do
  run c3_$i --config 3
  run c4_$i --config 4
done
bash tools/profile.sh ${TAG}_c3 --config 3 || exit 13
echo $TAG done
