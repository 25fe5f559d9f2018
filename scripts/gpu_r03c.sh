set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_affine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_rcol.log 2>&1; rc=$?; tail -5 $O/pytest_rcol.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/ab_rcol.py > $O/ab_rcol.jsonl 2> $O/ab_rcol.err || { tail $O/ab_rcol.err; exit 1; }
cat $O/ab_rcol.jsonl
timeout -k 10 300 python3 -u scripts/rot_ab.py "MIPX_ROT_T=64,MIPX_ROT_ORDER=0" "MIPX_ROT_T=128,MIPX_ROT_ORDER=0" "MIPX_ROT_T=64,MIPX_ROT_ORDER=1" "MIPX_ROT_T=128,MIPX_ROT_ORDER=1" "MIPX_ROT_T=128,MIPX_ROT_ORDER=1,MIPX_ROT_XCD=0" > $O/rot_ab.jsonl 2> $O/rot_ab.err || { tail $O/rot_ab.err; exit 1; }
cat $O/rot_ab.jsonl
for a in "affine --w 1920 --h 1080 --b 3 --n 16 --s 2" "affine --w 550 --h 740 --b 3 --n 64 --s 2" "affine --w 1024 --h 768 --b 4 --n 16 --s 1.5"; do
  MIPX_AFFINE_SEP=1 timeout -k 5 60 python3 scripts/op_bench.py $a --iters 20 2>/dev/null | grep '^{' >> $O/affine.jsonl || exit 1
  MIPX_AFFINE_SEP=0 timeout -k 5 60 python3 scripts/op_bench.py $a --iters 20 2>/dev/null | grep '^{' >> $O/affine.jsonl || exit 1
done
cat $O/affine.jsonl
