#!/bin/bash
# Round 4 experiment: another LLVM AMDGPU machine-scheduler strategy on every unit
# (ggrs_amd/exp/libggrs_amd_memclause.so: max-memory-clause; iterative-ilp did not build)
# against the product build, on config 2, config 3 and config 2's P2P shape; A/B twice.
set -u
TAG=${1:-r04w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], (d.get('parity') or {}).get('trace_equal', ''))" gpurun_out/bench_${TAG}_$name.json $name
}
for i in 1 2; do
  for v in prod memclause; do
    if [ $v = prod ]; then unset GGRS_AMD_EXP_LIB; else export GGRS_AMD_EXP_LIB=libggrs_amd_$v.so; fi
    run c2_${v}_$i
    run c3_${v}_$i --config 3
    run p2pc2_${v}_$i --workload p2p --sessions 4096 --latency 8 --max-prediction 9
  done
done
unset GGRS_AMD_EXP_LIB
echo $TAG done
