#!/bin/bash
# Time config 2 under experiment libraries: bash tools/exp_sweep.sh "<lanes...>" <lib names...>  (base = shipped lib)
LANES=$1; shift
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for lib in "$@"; do
  for l in $LANES; do
    if [ "$lib" = base ]; then unset GGRS_AMD_EXP_LIB; else export GGRS_AMD_EXP_LIB=libggrs_amd_$lib.so; fi
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --lanes $l --steps 10 > gpurun_out/exp_${lib}_$l.json 2> gpurun_out/exp_${lib}_$l.err || { echo "$lib $l failed"; tail -5 gpurun_out/exp_${lib}_$l.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/exp_${lib}_$l.json').read().strip().splitlines()[-1]); print('$lib', $l, d['value'], d['roofline'].get('avg_launch_ms'))"
  done
done
