#!/bin/bash
# r06 fusion probe: does k_rcol on C3's window shape absorb more work per step?
# MIPX_RCOL_DBG (PROBES library): 2 = a third barrier + the horizontal pass twice,
# 3 = the vertical pass twice, 4 = both
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_fprobe}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
export MIPX_LIB_PATH=imaginary_amd/libmipx_probes.so
run 200 python3 scripts/op_bench.py reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333 --iters 20 \
  --ab MIPX_RCOL_DBG=0,2,3,4 >> "$O/ab.jsonl" 2>> "$O/err.log"
run 200 python3 scripts/op_bench.py reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747 --iters 20 \
  --ab MIPX_RCOL_DBG=0,2,3,4 >> "$O/ab.jsonl" 2>> "$O/err.log"
run 200 python3 scripts/op_bench.py blur --w 768 --h 512 --b 4 --n 512 --s 5 --iters 20 >> "$O/ab.jsonl" 2>> "$O/err.log"
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/ab.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["op"], d["w"], d["h"], d["b"], d.get("MIPX_RCOL_DBG"), d.get("round"), round(d["ms"], 4), d.get("same_as_first"))
PY
