set -u
cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
i=0
for a in "--no-lane-server" "" ; do
  GGRS_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29800 + i)) bench.py --workload requests $a --gpus 1 --no-cpu-baseline > gpurun_out/rd_$i.json 2> gpurun_out/rd_$i.err || exit 10
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['config']['us_per_call'])" gpurun_out/rd_$i.json "dist [$a]"
  i=$((i+1))
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29850 bench.py --workload requests --gpus 1 --no-cpu-baseline > gpurun_out/rd_x.json 2> gpurun_out/rd_x.err || exit 11
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('torchrun, no group', d['config']['us_per_call'])" gpurun_out/rd_x.json
