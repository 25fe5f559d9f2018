#!/bin/bash
# r06: how much of a small-image k_rcol launch is the block set-up (operand tables, seeds,
# the prime)?  MIPX_RCOL_DBG=1 (PROBES library only) returns after the set-up and prime.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_setup}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
for a in "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
    "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667" "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" \
    "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333"; do
  MIPX_LIB_PATH=imaginary_amd/libmipx_probes.so run 150 python3 scripts/op_bench.py reduce $a --iters 20 --ab MIPX_RCOL_DBG=0,1 >> "$O/setup_ab.jsonl" 2>> "$O/err.log"
  run 150 python3 scripts/op_bench.py reduce $a --iters 20 --ab MIPX_RCOL_W4=0,1 >> "$O/w4_ab.jsonl" 2>> "$O/err.log"
  run 150 python3 scripts/op_bench.py reduce $a --iters 20 --ab MIPX_RCOL_1B=0,1 >> "$O/ob_ab.jsonl" 2>> "$O/err.log"
done
# k_reduce2x2 with non-temporal loads / stores (variants 82 / 98 / 114)
run 200 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 50 --ab MIPX_R2_VARIANT=66,82,98,114 >> "$O/nt_ab.jsonl" 2>> "$O/err.log"
python3 - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); knob = [k for k in d if k.startswith("MIPX_")][0]
            print(f'{f.split("/")[-1][:8]} {d["w"]}x{d["h"]}x{d["b"]} s{d["s"]:.4g} {knob}={d[knob]} r{d["round"]} {d["ms"]:.4f} ms {d["alg_GBps"]/8000:.1%}')
PY
