#!/bin/bash
# r06: k_bcol with the settled switches, wst2 and sd != 0 compiled in (MIPX_BCOL_SPEC): the blur
# tests on the default (specialised) builds, same-process A/Bs on the survey's blur shapes,
# then C3 / C5 off / on
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_bspec}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 600 python3 -u -m pytest tests/test_bcol_gpu.py tests/test_pipeline.py tests/test_demand_gpu.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$O/pytest_bspec.log" 2>&1
tail -1 "$O/pytest_bspec.log"
ab() { run 150 python3 scripts/op_bench.py "$@" --iters 20 >> "$O/ab.jsonl" 2>> "$O/ab.err"; }
for a in "--w 768 --h 512 --b 4 --n 512 --s 5" "--w 1920 --h 1080 --b 3 --n 64 --s 1" "--w 1920 --h 1080 --b 3 --n 64 --s 3" \
    "--w 3840 --h 2160 --b 3 --n 16 --s 5" "--w 1920 --h 1080 --b 4 --n 64 --s 2"; do
  ab blur $a --ab MIPX_BCOL_SPEC=0,1
done
for v in 0 1 0 1; do
  MIPX_BCOL_SPEC=$v timeout -k 10 300 python3 -u bench_configs.py --configs C3,C5 --steps 10 --warmup 2 \
    | sed "s/^{/{\"bspec\": $v, /" >> "$O/configs.jsonl" 2>> "$O/configs.err" || { echo "configs failed"; exit 1; }
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/ab.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(f'{d["op"]} {d["w"]}x{d["h"]}x{d["b"]} s{d["s"]:.4g} spec={d["MIPX_BCOL_SPEC"]} r{d["round"]} {d["ms"]:.4f} ms {d["alg_GBps"]/8000:.1%} same={d["same_as_first"]}')
for l in open(O + "/configs.jsonl"):
    d = json.loads(l); print(d["bspec"], d["config"], d["ms_per_step"], d["hbm_frac"], d["verified_vs_oracle"])
PY
