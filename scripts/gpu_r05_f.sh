#!/bin/bash
# chain W3 A/B + k_rcol prime-overlap A/B on the small survey shapes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05f}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 300 python3 -u -m pytest tests/test_chain_gpu.py tests/test_rcol_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
MIPX_CHAIN=1 run 300 python3 scripts/cfg_ab.py --config C3 --ab MIPX_CHAIN_W3=0,1 --rounds 2 > "$O/c3_w3_ab.jsonl"
cat "$O/c3_w3_ab.jsonl"
for args in "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
            "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333" \
            "--w 364 --h 273 --b 3 --n 128 --s 1.421875"; do
  run 120 python3 scripts/op_bench.py reduce $args --iters 20 --ab MIPX_RCOL_PRIME=0,1 >> "$O/prime_ab.jsonl"
done
python3 - "$O/prime_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["w"], d["h"], d["b"], d["s"], "prime", d["MIPX_RCOL_PRIME"], "r", d["round"], d["ms"], d["alg_GBps"], d["same_as_first"])
PY
