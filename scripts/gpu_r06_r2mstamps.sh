#!/bin/bash
# r06: k_reduce2m per-step phase stamps (make PROBES=1, MIPX_R2M_DBG=8), centre convention
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_r2mstamps}"; mkdir -p "$O"
export MIPX_LIB_PATH=imaginary_amd/libmipx_probes.so
for a in "--w 3840 --h 2160 --b 3 --n 256 --s 2" "--w 2048 --h 2048 --b 4 --n 512 --s 2"; do
  MIPX_R2M_DBG=8 timeout -k 10 120 python3 scripts/op_bench.py reduce $a --sampling centre --iters 2 --warm-ms 0 \
    >> "$O/ab.jsonl" 2>> "$O/stamps.log" || { echo "failed: $a"; exit 1; }
done
grep r2m_stamps "$O/stamps.log" | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    ph = ['barrier1','vertical','barrier2','ring_store','loads','edge','horizontal','store']
    tot = sum(d[p] for p in ph)
    print(d['w'], d['h'], d['b'], 'blocks', d['blocks'], 'block', round(d['block_mean']), 'step', round(tot), ' '.join(f'{p}={d[p]:.0f}({d[p]/tot:.0%})' for p in ph))
"
