#!/bin/bash
# Round 3: config-3 phase stamps (timing build ggrs_amd/exp/libggrs_amd_stamps.so)
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for n in 4 16 64; do
GGRS_AMD_EXP_LIB=libggrs_amd_stamps.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 3 --rounds-per-step $n --steps 3 --warmup 2 > gpurun_out/pstamps_$n.txt 2> gpurun_out/pstamps_$n.err || { tail -20 gpurun_out/pstamps_$n.err; exit 11; }
echo "rounds $n"; grep PSTAMPS gpurun_out/pstamps_$n.txt | tail -8
done
