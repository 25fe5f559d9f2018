# demand tests with junk-filled workspaces + request-path reuse; blur-geometry memory probe; r03 PMC traffic of C2
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03r; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_demand_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_demand.log 2>&1; rc=$?; tail -3 $O/pytest_demand.log; [ $rc -eq 0 ] || exit $rc
PROBE_BLUR=1 timeout -k 10 120 ./scripts/strip_probe > $O/probe.jsonl 2>&1 || { cat $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
PMC_LIST='FETCH_SIZE
WRITE_SIZE' TAG=r03 STEPS=3 timeout -k 10 400 bash scripts/pmc.sh > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 scripts/traffic_json.py gpurun_out/pmc_r03 "k_reduce2x2<3, 66>" $O/traffic_r03.json "C2 bench.py --steps 3, 256 x 4K RGB -> 1080p" && cat $O/traffic_r03.json
