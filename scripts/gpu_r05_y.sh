#!/bin/bash
# small-image reduces: time against batch size (latency- or throughput-bound?) and the
# k_enlm timing probes / band heights (gpu_r05_s.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05y}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/small_n.jsonl"
for n in 64 128 256 512 1024; do
  run 100 python3 scripts/op_bench.py reduce --w 480 --h 270 --b 3 --n $n --s 1.6 --iters 20 >> "$O/small_n.jsonl"
done
for n in 64 128 256 512; do
  run 100 python3 scripts/op_bench.py reduce --w 500 --h 375 --b 3 --n $n --s 1.465 --iters 20 >> "$O/small_n.jsonl"
done
for n in 24 48 96 192; do
  run 100 python3 scripts/op_bench.py reduce --w 1333 --h 1000 --b 3 --n $n --s 1.6666666666666667 --iters 20 >> "$O/small_n.jsonl"
done
python3 - "$O/small_n.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["w"], d["h"], d["n"], d["s"], d["ms"], round(d["alg_GBps"] / 8000, 4))
PY
OUT=${OUT:-r05y} run 600 bash scripts/gpu_r05_s.sh
