set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
F=gpurun_out/pass_split.jsonl; : > $F
for args in "reducev --w 1920 --h 1080 --b 3 --n 64 --s 1.6" "reduceh --w 1920 --h 675 --b 3 --n 64 --s 1.6" "reducev --w 1920 --h 1080 --b 4 --n 64 --s 1.6" "reduceh --w 1920 --h 675 --b 4 --n 64 --s 1.6" "reducev --w 1920 --h 1080 --b 3 --n 64 --s 2.4" "reduceh --w 1920 --h 450 --b 3 --n 64 --s 2.4" "reduceh --w 1920 --h 675 --b 3 --n 64 --s 1.6 --iters 20"; do
  MIPX_HP_REPACK=1 timeout -k 5 60 python3 scripts/op_bench.py $args 2>/dev/null | grep '^{' >> $F || exit 1
done
MIPX_HP_REPACK=0 timeout -k 5 60 python3 scripts/op_bench.py reduceh --w 1920 --h 675 --b 3 --n 64 --s 1.6 2>/dev/null | grep '^{' >> $F || exit 1
cut -c1-200 $F
