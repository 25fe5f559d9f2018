#!/bin/bash
# k_enlm: realignment dwords from the neighbour lane (MIPX_ENLM_SHF) — affine parity, the
# realignment loads' share (MIPX_ENLM_DBG=4 with SHF=0), same-process A/B; k_reduce2m parity
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05z}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_affine.log" 2>&1
tail -2 "$O/pytest_affine.log"
run 400 python3 -u -m pytest tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduce2x2_variants or 4k_to_1080p" > "$O/pytest_r2.log" 2>&1
tail -2 "$O/pytest_r2.log"
: > "$O/dbg4_ab.jsonl"; : > "$O/shf_ab.jsonl"
export MIPX_ENLM=2
for args in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5"; do
  MIPX_ENLM_SHF=0 run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_DBG=0,4,1 >> "$O/dbg4_ab.jsonl"
done
for args in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5" \
            "--w 1280 --h 720 --b 3 --n 16 --s 3" "--w 960 --h 540 --b 3 --n 16 --s 4" "--w 1024 --h 768 --b 4 --n 16 --s 2"; do
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_SHF=0,1 >> "$O/shf_ab.jsonl"
done
python3 - "$O/dbg4_ab.jsonl" "$O/shf_ab.jsonl" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l); k = [x for x in d if x.startswith("MIPX_")][0]
        print(d["w"], d["h"], d["b"], d["s"], k, d[k], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
