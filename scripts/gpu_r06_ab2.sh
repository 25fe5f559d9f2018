#!/bin/bash
# r06 A/B runner 2: k_rcol set-up latency (early tap loads, pipelined prime), conflict-free
# tile read-back lanes (k_rcol RGBA, k_bcol, k_enlm), then C3 / C5 with the new knobs on / off
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_ab2}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
if [ "${TESTS:-1}" = 1 ]; then
  run 600 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_bcol_gpu.py tests/test_affine_gpu.py tests/test_chain_gpu.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_ab.log" 2>&1
  tail -2 "$O/pytest_ab.log"
fi
ab() { run 150 python3 scripts/op_bench.py "$@" --iters 20 >> "$O/ab.jsonl" 2>> "$O/ab.err"; }
for a in "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
    "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667" "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" \
    "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333"; do
  ab reduce $a --ab MIPX_RCOL_TEARLY=0,1
  ab reduce $a --ab MIPX_RCOL_PPIPE=0,1
done
ab reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333 --ab MIPX_RCOL_TRL=0,1
for a in "--w 768 --h 512 --b 4 --n 512 --s 5" "--w 1920 --h 1080 --b 3 --n 64 --s 3"; do
  ab blur $a --ab MIPX_BCOL_WSW=0,1
done
for a in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" \
    "--w 1024 --h 768 --b 4 --n 16 --s 1.5" "--w 1280 --h 720 --b 3 --n 16 --s 3"; do
  ab affine $a --ab MIPX_ENLM_OSW=0,1
done
OFF="MIPX_RCOL_TEARLY=0 MIPX_RCOL_PPIPE=0 MIPX_RCOL_TRL=0 MIPX_BCOL_VPERM=0 MIPX_BCOL_WSW=0"
for v in off on off on; do
  if [ $v = off ]; then E="$OFF"; else E=""; fi
  env $E timeout -k 10 300 python3 -u bench_configs.py --configs C3,C5 --steps 10 --warmup 2 \
    | sed "s/^{/{\"knobs\": \"$v\", /" >> "$O/configs.jsonl" 2>> "$O/configs.err" || { echo "configs failed"; exit 1; }
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
    d = json.loads(l); print(d["knobs"], d["config"], d["sampling"], d["ms_per_step"], d["hbm_frac"], d["verified_vs_oracle"])
PY
