# kernel breakdown of C3 and C5 after k_rot90_px (rocprofv3 kernel stats of bench_configs)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zc; mkdir -p $O; export TMPDIR=/tmp
for c in C3 C5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench_configs.py --configs $c --steps 10 --warmup 2 > $O/$c.log 2>&1 || { tail $O/$c.log; exit 1; }
find $O/prof_$c -name "*kernel_stats.csv" -exec cp {} $O/${c}_kernel_stats.csv \;
grep images_per_sec $O/$c.log | cut -c1-250
done
for c in C3 C5; do python3 - $O/${c}_kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    n=r["Name"].replace("(anonymous namespace)::","").replace("void mipx::","").split("(")[0][:60]
    print(f'{n:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f} %')
PY
done
