#!/bin/bash
# Round 4 experiment: the library with max-ilp on every unit (ggrs_amd/exp/libggrs_amd_allilp.so) against
# the product build on the units that compile with the default scheduler: codec, config 5
# (particles), the request boundary (requests.hip); A/B twice.
set -u
TAG=${1:-r04q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err \
    || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 12; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['ms_per_step'], r.get('avg_launch_ms'))" gpurun_out/bench_${TAG}_$name.json $name
}
for i in 1 2; do
  for v in prod allilp; do
    if [ $v = allilp ]; then export GGRS_AMD_EXP_LIB=libggrs_amd_allilp.so; else unset GGRS_AMD_EXP_LIB; fi
    run codec_${v}_$i --workload codec
    run c5_${v}_$i --config 5 --steps 5
    run req_${v}_$i --workload requests
  done
done
unset GGRS_AMD_EXP_LIB
echo $TAG done
