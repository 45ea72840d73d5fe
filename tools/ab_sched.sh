#!/bin/bash
# A/B of scheduled-P2P library variants on the GPU box (timing only):
#   bash tools/ab_sched.sh "<bench args>" lib1 lib2 ...   (libN: ggrs_amd/exp/libggrs_amd_<libN>.so)
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
ARGS=$1; shift
for rep in 1 2; do
for lib in "$@"; do
  GGRS_AMD_EXP_LIB=libggrs_amd_$lib.so timeout -k 10 200 python -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab_${lib}_$rep.json 2>/dev/null || { echo "$lib failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_${lib}_$rep.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['roofline']['avg_launch_ms'], d['parity'].get('every_session_bit_exact'))"
done
done
