#!/bin/bash
# k_reduce2m: odd bands walk up (MIPX_R2M_ALT) — 2x2 parity under both conventions, same-process
# A/B on the survey 2x2 shapes at the centre convention, band heights under it, HBM fetch PMC
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05w}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduce2x2_variants or 4k_to_1080p" > "$O/pytest_r2.log" 2>&1
tail -2 "$O/pytest_r2.log"
: > "$O/alt_ab.jsonl"; : > "$O/band_ab.jsonl"
for args in "--w 3840 --h 2160 --b 3 --n 256 --s 2" "--w 2048 --h 2048 --b 4 --n 512 --s 2"; do
  run 150 python3 scripts/op_bench.py reduce $args --sampling centre --iters 20 --ab MIPX_R2M_ALT=0,1 >> "$O/alt_ab.jsonl"
  run 200 python3 scripts/op_bench.py reduce $args --sampling centre --iters 20 --ab MIPX_R2M_BAND=4,8,12,16 >> "$O/band_ab.jsonl"
done
python3 - "$O/alt_ab.jsonl" "$O/band_ab.jsonl" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l); k = [x for x in d if x.startswith("MIPX_")][0]
        print(d["w"], d["h"], d["b"], k, d[k], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 4), d["same_as_first"])
PY
for alt in 0 1; do
  MIPX_R2M_ALT=$alt TAG=r2m_alt$alt OP_ARGS="reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --sampling centre" PMC_LIST="FETCH_SIZE
WRITE_SIZE" run 300 bash scripts/pmc_op.sh > "$O/pmc_alt$alt.txt"
  cat "$O/pmc_alt$alt.txt"
done
