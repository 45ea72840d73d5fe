# P2P timing + traffic experiments: bash tools/exp_p2p.sh <variant>...
set -u
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --no-cpu-baseline --workload p2p > gpurun_out/p2p_base.json 2>/dev/null || exit 11
for v in "$@"; do
  GGRS_AMD_EXP_LIB=libggrs_amd_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --workload p2p > gpurun_out/p2p_$v.json 2>/dev/null || exit 12
  GGRS_AMD_EXP_LIB=libggrs_amd_$v.so bash tools/profile.sh p2p_$v --workload p2p --steps 10 || exit 13
done
bash tools/profile.sh p2p_base --workload p2p --steps 10 || exit 14
for f in gpurun_out/p2p_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['roofline']['avg_launch_ms'],d['parity'])"; done
