# packed RGB stores in k_hpass: parity (pack3 on/off + the whole hpass/blur/fuzz set), then the RGB reduceh A/B
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_pack3.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_pack3.log; [ $rc -ne 0 ] && exit $rc
F=gpurun_out/pack3_ab.jsonl; : > $F
for p in 0 1 0 1; do
  for args in "reduceh --w 1920 --h 675 --b 3 --n 64 --s 1.6 --iters 20" "reduceh --w 1920 --h 450 --b 3 --n 64 --s 2.4 --iters 20" "blur --w 1920 --h 1080 --b 3 --n 32 --s 3"; do
    echo -n "{\"pack3\": $p, \"r\": " >> $F
    MIPX_HP_PACK3=$p MIPX_BLUR2D=0 timeout -k 5 60 python3 scripts/op_bench.py $args 2>/dev/null | grep '^{' | tr -d '\n' >> $F || exit 1
    echo "}" >> $F
  done
done
cut -c1-220 $F
