#!/bin/bash
# Round 4: the canonical sparse-saving kernel: P2P + desync GPU tests, the sparse P2P bench line
# (twice), its kernel trace + PMC.
set -u
TAG=${1:-r04s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  tests/test_gpu_desync.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 10; }
tail -2 gpurun_out/pytest_$TAG.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" gpurun_out/bench_${TAG}_$name.json $name
}
run sparse_1 --workload p2p --sparse
run sparse_2 --workload p2p --sparse
run p2p_1 --workload p2p
bash tools/profile.sh ${TAG}_sparse --workload p2p --sparse || exit 13
echo $TAG done
