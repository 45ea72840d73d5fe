# configs 3/4: exchange GPU tests, bench lines (1 GPU fused, 1-rank RCCL exchange, gloo 2-rank
# rehearsal), then a kernel-trace + PMC profile of each
set -u
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_branch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_ex.log 2>&1 || { tail -30 gpurun_out/pt_ex.log; exit 10; }
tail -2 gpurun_out/pt_ex.log
bash tools/gpu_bench.sh r02a "--config 3" "--config 4" || exit 11
GGRS_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_r02a_dist1.json 2> gpurun_out/bench_r02a_dist1.err || { tail -20 gpurun_out/bench_r02a_dist1.err; exit 12; }
cat gpurun_out/bench_r02a_dist1.json
GGRS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config 4 --peers --steps 5 > gpurun_out/bench_r02a_gloo2.json 2> gpurun_out/bench_r02a_gloo2.err || { tail -20 gpurun_out/bench_r02a_gloo2.err; exit 13; }
cat gpurun_out/bench_r02a_gloo2.json
bash tools/profile.sh r02_c3 --config 3 --steps 10 || exit 14
bash tools/profile.sh r02_c4 --config 4 --steps 10 || exit 15
echo done
