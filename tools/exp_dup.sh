# timing experiments: bash tools/exp_dup.sh <variant>...  (ggrs_amd/exp/libggrs_amd_<variant>.so)
set -u
cd ${GRAFT_REPO_ROOT}
mkdir -p gpurun_out
for L in 3072 4096; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --lanes $L > gpurun_out/exp_base_$L.json 2>/dev/null || exit 11
  for v in "$@"; do
    GGRS_AMD_EXP_LIB=libggrs_amd_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --lanes $L > gpurun_out/exp_${v}_$L.json 2>/dev/null || exit 12
  done
done
for f in gpurun_out/exp_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['roofline']['avg_launch_ms'],d['parity'])"; done
