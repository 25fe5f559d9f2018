# k_bmf parity (-k "blur or gauss") then blur timings with MIPX_BMF=1 / 0 (k_blur2d)
# per shape, one op_bench process each.
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_pipeline.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "blur or gauss or c3" > gpurun_out/pytest_bmf.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_bmf.log; [ $rc -eq 0 ] || { grep -m5 -B5 "Error\|assert" gpurun_out/pytest_bmf.log | head -40; exit $rc; }
fi
: > gpurun_out/blur_ab.jsonl
for sh in "768 512 4 512 5" "1920 1080 3 32 1" "1920 1080 3 32 3" "1920 1080 3 32 5" "3840 2160 3 8 3" "1024 1024 4 64 2"; do
  set -- $sh
  for v in ${BMF_VARIANTS:-1 0}; do
    MIPX_BMF=$v timeout -k 10 60 python3 scripts/op_bench.py blur --w $1 --h $2 --b $3 --n $4 --s $5 --iters 20 > gpurun_out/ob.txt 2>&1 || { cat gpurun_out/ob.txt; exit 1; }
    echo "{\"bmf\": $v, \"shape\": \"$sh\", \"out\": $(grep '^{' gpurun_out/ob.txt | tail -1)}" >> gpurun_out/blur_ab.jsonl
  done
done
cut -c1-200 gpurun_out/blur_ab.jsonl
