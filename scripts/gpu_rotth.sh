# rot 90/270 with 64 or 128 input rows per tile: parity, then the A/B
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_rotth.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_rotth.log; [ $rc -ne 0 ] && exit $rc
F=gpurun_out/rotth_ab.jsonl; : > $F
for p in 64 128 64 128; do
  for args in "rot --w 3840 --h 2160 --b 3 --n 32 --s 90" "rot --w 3840 --h 2160 --b 4 --n 32 --s 270" "rot --w 1920 --h 1080 --b 3 --n 64 --s 270"; do
    echo -n "{\"th\": $p, \"r\": " >> $F
    MIPX_ROT_TH=$p timeout -k 5 60 python3 scripts/op_bench.py $args 2>/dev/null | grep '^{' | tr -d '\n' >> $F || exit 1
    echo "}" >> $F
  done
done
cut -c1-220 $F
