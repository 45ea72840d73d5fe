#!/bin/bash
# Round 4: particles.h without inline asm (product build, default scheduler): particle GPU tests and
# the config-5 bench line (twice).
set -u
TAG=${1:-r04y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_particles.py \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_c5_$i.json 2> gpurun_out/bench_${TAG}_c5_$i.err \
    || { tail -20 gpurun_out/bench_${TAG}_c5_$i.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', '%.4g' % d['value'], d['ms_per_step'], d.get('halted_lanes'), d.get('parity'))" gpurun_out/bench_${TAG}_c5_$i.json
done
echo $TAG done
