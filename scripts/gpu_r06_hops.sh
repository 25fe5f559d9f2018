#!/bin/bash
# r06: k_rcol's specialised builds with host-built operands (device_rcol_hops) against the
# argument-driven builds (MIPX_RCOL_SPEC=0), the 4-wave builds forced (MIPX_RCOL_W4=1), the rcol
# tests, then C3 / C4 / C5
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_hops}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 600 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_chain_gpu.py tests/test_parity_gpu.py tests/test_configs_gpu.py \
  -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_hops.log" 2>&1
tail -1 "$O/pytest_hops.log"
MIPX_RCOL_W4=1 run 600 python3 -u -m pytest tests/test_rcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$O/pytest_hops_w4.log" 2>&1
tail -1 "$O/pytest_hops_w4.log"
ab() { run 150 python3 scripts/op_bench.py "$@" --iters 20 >> "$O/ab.jsonl" 2>> "$O/ab.err"; }
for a in "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
    "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667" "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" \
    "--w 1920 --h 1080 --b 3 --n 64 --s 2.4" "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333" \
    "--w 364 --h 273 --b 3 --n 128 --s 1.421875"; do
  ab reduce $a --ab MIPX_RCOL_SPEC=0,1
  ab reduce $a --ab MIPX_RCOL_W4=0,1
done
for v in 0 1 0 1; do
  MIPX_RCOL_SPEC=$v timeout -k 10 300 python3 -u bench_configs.py --configs C3,C4,C5 --steps 10 --warmup 2 \
    | sed "s/^{/{\"spec\": $v, /" >> "$O/configs.jsonl" 2>> "$O/configs.err" || { echo "configs failed"; exit 1; }
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/ab.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        knob = [k for k in d if k.startswith("MIPX_")][0]
        print(f'{d["op"]} {d["w"]}x{d["h"]}x{d["b"]} s{d["s"]:.4g} {knob}={d[knob]} r{d["round"]} {d["ms"]:.4f} ms {d["alg_GBps"]/8000:.1%} same={d["same_as_first"]}')
for l in open(O + "/configs.jsonl"):
    d = json.loads(l); print(d["spec"], d["config"], d["ms_per_step"], d["hbm_frac"], d["verified_vs_oracle"])
PY
