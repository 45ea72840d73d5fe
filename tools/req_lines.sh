cd ${GRAFT_REPO_ROOT:-.} && mkdir -p gpurun_out
for spec in "req:--workload requests" "reqp2p:--workload requests --req-form p2p --lanes 4096 --req-threads 16 --req-deferred"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/lines_r06final_$name.json 2> gpurun_out/lines_r06final_$name.err || { echo "$name failed"; tail -5 gpurun_out/lines_r06final_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['cpu_baseline'])" gpurun_out/lines_r06final_$name.json $name
done
