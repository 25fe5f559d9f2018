# HBM traffic of C3's kernels with demand-driven regions on and off (FETCH_SIZE / WRITE_SIZE
# in separate passes, counters + kernel trace only); summarised with scripts/traffic_json.py
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/pmc_c3; mkdir -p $O; export TMPDIR=/tmp
for d in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MIPX_DEMAND=$d timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/d$d/$c -o run -- python3 bench_configs.py --configs C3 --steps 2 --warmup 1 > $O/d${d}_$c.log 2>&1 || { tail -5 $O/d${d}_$c.log; exit 1; }
  done
done
echo done
