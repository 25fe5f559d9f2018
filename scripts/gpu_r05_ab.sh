#!/bin/bash
# r05 same-process A/Bs (each step under its own limit, stop at the first failure)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05ab}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
for s in ${AB:-c3chain r2d walk}; do
  echo "== $s $(date +%T)"
  case $s in
    c3chain) run 300 python3 scripts/cfg_ab.py --config C3 --ab MIPX_CHAIN=0,1 --rounds 3 > "$O/c3_chain_ab.jsonl"
             run 300 python3 scripts/cfg_ab.py --config C3 --ab MIPX_CHAIN=0,1 --rounds 3 --sampling centre >> "$O/c3_chain_ab.jsonl"
             cat "$O/c3_chain_ab.jsonl" ;;
    r2d) run 300 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2D=0,1 > "$O/r2d_ab.jsonl"
         run 300 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2D=0,1 --sampling centre >> "$O/r2d_ab.jsonl"
         run 300 python3 scripts/op_bench.py reduce --w 2048 --h 2048 --b 4 --n 512 --s 2 --iters 10 --ab MIPX_R2D=0,1 >> "$O/r2d_ab.jsonl"
         cat "$O/r2d_ab.jsonl" ;;
    walk) run 300 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2_WALK=1,2,4,12 > "$O/walk_ab.jsonl"
          cat "$O/walk_ab.jsonl" ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
