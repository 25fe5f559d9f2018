#!/bin/bash
# k_enlm timing probes (MIPX_ENLM_DBG: 1 no staging loads, 2 no stores, 3 neither) and band heights
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05s}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/dbg_ab.jsonl"; : > "$O/br_ab.jsonl"
export MIPX_ENLM=2
for args in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5"; do
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_DBG=0,1,2,3 >> "$O/dbg_ab.jsonl"
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_BR=0,64,96,128,176,240 >> "$O/br_ab.jsonl"
done
python3 - "$O/dbg_ab.jsonl" "$O/br_ab.jsonl" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        k = [x for x in d if x.startswith("MIPX_")][0]
        if d["round"] == 0: print(d["w"], d["h"], d["b"], d["s"], k, d[k], d["ms"], round(d["alg_GBps"] / 8000, 3))
PY
