#!/bin/bash
# Round 4 experiment: the engine library built with LLVM's default AMDGPU scheduler
# (ggrs_amd/exp/libggrs_amd_noilp.so, tools/exp_build.sh noilp -mllvm -amdgpu-sched-strategy=max-occupancy)
# against the product build (max-ilp), A/B twice on configs 2 and 3 and the two P2P shapes.
set -u
TAG=${1:-r04o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" gpurun_out/bench_${TAG}_$name.json $name
}
for i in 1 2; do
  for v in ilp noilp; do
    if [ $v = noilp ]; then export GGRS_AMD_EXP_LIB=libggrs_amd_noilp.so; else unset GGRS_AMD_EXP_LIB; fi
    run c2_${v}_$i
    run c3_${v}_$i --config 3
    run p2p_${v}_$i --workload p2p
    run p2pc2_${v}_$i --workload p2p --sessions 4096 --latency 8 --max-prediction 9
  done
done
unset GGRS_AMD_EXP_LIB
echo $TAG done
