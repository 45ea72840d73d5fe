set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r06_fe
for a in "p2p_jitter4096:--workload p2p --arrivals jitter --sessions 4096 --max-prediction 9" "p2p_stall:--workload p2p --arrivals stall" "p2p_jitter:--workload p2p --arrivals jitter"; do
  name=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/r06_fe/lines_r06fe_$name.json 2> gpurun_out/r06_fe/$name.err
  echo "$name done"
done
bash tools/profile.sh r06_fe_j4096 --workload p2p --arrivals jitter --sessions 4096 --max-prediction 9
