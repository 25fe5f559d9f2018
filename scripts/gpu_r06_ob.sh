#!/bin/bash
# r06: k_rcol one-barrier steps (MIPX_RCOL_1B): rcol parity tests, then same-process A/Bs
# at the small-reduce survey shapes and C3's window reduce, then C3 both ways
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_ob}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_chain_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_rcol.log" 2>&1
tail -2 "$O/pytest_rcol.log"
while read -r args; do
  [ -z "$args" ] && continue
  run 120 python3 scripts/op_bench.py $args --iters 20 --ab MIPX_RCOL_1B=0,1 >> "$O/ob_ab.jsonl" 2>> "$O/ob_ab.err"
done <<LIST
reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333
reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747
reduce --w 500 --h 375 --b 3 --n 128 --s 1.46484375
reduce --w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667
reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6
LIST
for v in 0 1; do
  MIPX_RCOL_1B=$v run 300 python3 -u bench_configs.py --configs C3,C5 --steps 10 --warmup 2 >> "$O/configs_ob$v.jsonl" 2>> "$O/configs.err"
done
python3 - "$O" <<'PY'
import json, sys, glob
for l in open(sys.argv[1] + "/ob_ab.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(l.strip()[:300])
for f in sorted(glob.glob(sys.argv[1] + "/configs_ob*.jsonl")):
    for l in open(f):
        d = json.loads(l); print(f[-12:], d["config"], d["ms_per_step"], d["device_ms_per_step"], d["hbm_frac"], d["verified_vs_oracle"])
PY
