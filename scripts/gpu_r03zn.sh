# k_bcol launch geometry (MIPX_BCOL_DBG) for the RGB strip variants
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zn; mkdir -p $O; export TMPDIR=/tmp
for v in 1 0; do
MIPX_BCOL_DBG=1 MIPX_BCOL_RGB192=$v timeout -k 10 60 python3 -u scripts/op_bench.py blur --w 1920 --h 1080 --b 3 --n 64 --s 1 --warm-ms 0 --iters 1 2>&1 | sort | uniq -c | tail -3
MIPX_BCOL_DBG=1 MIPX_BCOL_RGB192=$v timeout -k 10 60 python3 -u scripts/op_bench.py blur --w 1920 --h 1080 --b 3 --n 64 --s 5 --warm-ms 0 --iters 1 2>&1 | sort | uniq -c | tail -3
done
