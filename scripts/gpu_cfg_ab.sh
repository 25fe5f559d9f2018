# Config lines (bench_configs.py) under several reduce-kernel env settings, one
# process per setting, back to back on one box: CFG_VARIANTS="A=1,B=2 A=0".
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/cfg_ab.jsonl
for v in ${CFG_VARIANTS:-MIPX_RMFMA=0 MIPX_RMFMA=}; do
    env $(echo "$v" | tr ',' ' ') timeout -k 10 300 python3 -u bench_configs.py --configs ${CONFIGS:-C3,C4,C5} > gpurun_out/cfg_ab.log 2>&1 || { tail -20 gpurun_out/cfg_ab.log; exit 1; }
    grep '^{' gpurun_out/cfg_ab.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/cfg_ab.jsonl
done
cut -c1-220 gpurun_out/cfg_ab.jsonl
