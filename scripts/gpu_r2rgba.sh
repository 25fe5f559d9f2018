set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r2ab; mkdir -p $O; export TMPDIR=/tmp
for bnd in 2 1 3; do
  MIPX_R2_BAND=$bnd VARIANTS=66,2,130,67 BANDS=4 BATCH=192 ROUNDS=3 timeout -k 10 200 python3 scripts/ab_reduce.py > $O/rgba_band$bnd.jsonl 2> $O/rgba_band$bnd.err || { tail -3 $O/rgba_band$bnd.err; exit 1; }
  echo "band $bnd"; cat $O/rgba_band$bnd.jsonl
done
