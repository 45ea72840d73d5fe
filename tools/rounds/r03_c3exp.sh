#!/bin/bash
# Round 3: config 3 under timing builds (ggrs_amd/exp/libggrs_amd_<name>.so; no parity), 16 rounds per launch.
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for lib in base "$@"; do
  if [ "$lib" = base ]; then L=""; else L=libggrs_amd_$lib.so; fi
  GGRS_AMD_EXP_LIB=$L timeout -k 10 120 python -u bench.py --config 3 --no-cpu-baseline --steps 30 > gpurun_out/b.json 2> gpurun_out/b.err || { echo "$lib failed"; tail -5 gpurun_out/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print('$lib', '%.4g'%d['value'], d['roofline']['avg_kernel_ms_per_round'], d['ms_per_step'])" | tee -a gpurun_out/summary_c3exp.txt
done
