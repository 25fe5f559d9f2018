#!/bin/bash
# k_reduce2m fine band sweep (MIPX_R2M_BAND 6-11) and k_reduce2x2 bands (MIPX_R2_BAND 1-3), same-process A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05band2}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/r2m_band_ab.jsonl"
run 200 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --sampling centre --iters 20 --ab MIPX_R2M_BAND=6,7,8,9,10,11,8 >> "$O/r2m_band_ab.jsonl"
run 200 python3 scripts/op_bench.py reduce --w 2048 --h 2048 --b 4 --n 512 --s 2 --sampling centre --iters 20 --ab MIPX_R2M_BAND=12,14,16,18,20,16 >> "$O/r2m_band_ab.jsonl"
run 200 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2_BAND=1,2,3,2 > "$O/r2_band_ab.jsonl"
python3 - "$O/r2m_band_ab.jsonl" "$O/r2_band_ab.jsonl" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        k = [x for x in d if x.startswith("MIPX_")][0]
        print(d["w"], d["b"], d.get("sampling"), k, d[k], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 4), d["same_as_first"])
PY
