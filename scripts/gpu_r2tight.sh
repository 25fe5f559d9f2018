set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r2ab; mkdir -p $O; export TMPDIR=/tmp
VARIANTS=66,322,323 BANDS=3 BATCH=256 ROUNDS=5 timeout -k 10 200 python3 scripts/ab_reduce.py > $O/rgb_tight.jsonl 2> $O/rgb_tight.err || { tail -3 $O/rgb_tight.err; exit 1; }
cat $O/rgb_tight.jsonl
VARIANTS=66,322,323 BANDS=4 BATCH=192 ROUNDS=5 timeout -k 10 200 python3 scripts/ab_reduce.py > $O/rgba_tight.jsonl 2> $O/rgba_tight.err || { tail -3 $O/rgba_tight.err; exit 1; }
cat $O/rgba_tight.jsonl
