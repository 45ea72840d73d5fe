# every workload's bench line (CPU baselines included) + PMC profiles of codec and requests
set -u
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out
bash tools/gpu_bench.sh r02b "" "--config 5" "--workload p2p" "--workload codec" "--workload requests" "--workload requests --lanes 16384" || exit 11
bash tools/profile.sh r02_codec --workload codec --steps 10 || exit 14
bash tools/profile.sh r02_req --workload requests --no-lane-server --steps 4 || exit 15
echo done
