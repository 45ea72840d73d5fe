#!/bin/bash
# Round 4: config 3 -- the bench line (with the general form), phase stamps of one launch at 4, 16
# and 64 rounds (timing build ggrs_amd/exp/libggrs_amd_stamps.so), rocprof kernel stats.
set -u
TAG=${1:-r04c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 11; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%.4g' % d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms_per_round'], d.get('general_form'))" gpurun_out/bench_${TAG}.json
for n in 4 16 64; do
GGRS_AMD_EXP_LIB=libggrs_amd_stamps.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 3 --rounds-per-step $n --steps 3 --warmup 2 > gpurun_out/pstamps_${TAG}_$n.txt 2> gpurun_out/pstamps_${TAG}_$n.err || { tail -20 gpurun_out/pstamps_${TAG}_$n.err; exit 12; }
echo "rounds $n"; grep PSTAMPS gpurun_out/pstamps_${TAG}_$n.txt | tail -8
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run -- python3 $R/bench.py --config 3 --no-cpu-baseline > $R/gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 $R/gpurun_out/prof_${TAG}.log; exit 13; }
find $R/gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1 | xargs head -8
echo r04c3 done
