# row-staged zoom + 16-byte affine staging: parity + op timing
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03u; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_affine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "zoom or affine or plan or fuzz" > $O/pytest_zoom.log 2>&1; rc=$?; tail -3 $O/pytest_zoom.log; [ $rc -eq 0 ] || exit $rc
: > $O/ops.jsonl
for a in "zoom --w 1920 --h 1080 --b 3 --n 16 --s 2" "zoom --w 1024 --h 768 --b 4 --n 16 --s 3" "zoom --w 640 --h 480 --b 3 --n 64 --s 4" "affine --w 1920 --h 1080 --b 3 --n 16 --s 2" "affine --w 550 --h 740 --b 3 --n 64 --s 2" "affine --w 1024 --h 768 --b 4 --n 16 --s 1.5"; do
  timeout -k 5 60 python3 scripts/op_bench.py $a --iters 20 2>/dev/null | grep '^{' >> $O/ops.jsonl || exit 1
done
cat $O/ops.jsonl
