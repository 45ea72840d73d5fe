#!/bin/bash
# Round 3: v5 phase stamps (timing build ggrs_amd/exp/libggrs_amd_stamps.so; printf from two blocks)
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for n in 8 512; do
GGRS_AMD_EXP_LIB=libggrs_amd_stamps.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --frames-per-step $n --steps 4 --warmup 2 > gpurun_out/stamps_$n.txt 2> gpurun_out/stamps_$n.err || { tail -20 gpurun_out/stamps_$n.err; exit 11; }
grep STAMPS gpurun_out/stamps_$n.txt | tail -6
done
