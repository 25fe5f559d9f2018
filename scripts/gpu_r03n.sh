# r03 checkpoint: k_rcol row-piece stores + k_bmf fp32 rounding / flip-once (defaults):
# full GPU suite, A/Bs, configs, C2 under the centre convention, op survey
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/blur_ab.py "MIPX_BMF=1,MIPX_BMF_FP=1,MIPX_BMF_X1=1" "MIPX_BMF=1,MIPX_BMF_FP=0,MIPX_BMF_X1=1" "MIPX_BMF=1,MIPX_BMF_FP=1,MIPX_BMF_X1=0" "MIPX_BMF=1,MIPX_BMF_FP=0,MIPX_BMF_X1=0" "MIPX_BMF=,MIPX_BMF_FP=1,MIPX_BMF_X1=1" > $O/blur_ab.jsonl 2> $O/blur_ab.err || { tail $O/blur_ab.err; exit 1; }
cat $O/blur_ab.jsonl
VARIANTS='MIPX_RCOL_WST=1;MIPX_RCOL_WST=0;MIPX_RCOL=0' timeout -k 10 400 python3 -u scripts/ab_rcol.py > $O/ab_rcol.jsonl 2> $O/ab_rcol.err || { tail $O/ab_rcol.err; exit 1; }
cat $O/ab_rcol.jsonl
timeout -k 10 300 python3 -u bench_configs.py --configs C3,C4,C5 --steps 10 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail $O/configs.err; exit 1; }
cut -c1-300 $O/configs.jsonl
MIPX_REDUCE_CENTRE=1 timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --no-cpu > $O/bench_centre.json 2> $O/bench_centre.err || { tail $O/bench_centre.err; exit 1; }
cut -c1-400 $O/bench_centre.json
bash scripts/op_survey.sh > $O/op_survey.txt 2>&1; rc=$?; cp gpurun_out/op_survey.jsonl $O/; cat $O/op_survey.txt; exit $rc
