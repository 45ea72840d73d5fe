#!/bin/bash
# time config 3 under experiment libraries (timing only, no parity): bash tools/r03_exp_c3.sh <libs...> (base = shipped)
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = base ]; then unset GGRS_AMD_EXP_LIB; else export GGRS_AMD_EXP_LIB=libggrs_amd_$lib.so; fi
  timeout -k 10 120 python -u bench.py --config 3 --no-cpu-baseline --steps 30 > gpurun_out/expc3_$lib.json 2> gpurun_out/expc3_$lib.err || { echo "$lib failed"; tail -5 gpurun_out/expc3_$lib.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/expc3_$lib.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['roofline']['avg_kernel_ms_per_round'], d['ms_per_step'])"
done
