#!/bin/bash
# r06: k_rcol per-step phase stamps (make PROBES=1, MIPX_RCOL_DBG=8): where a step's time goes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_stamps}"; mkdir -p "$O"
export MIPX_LIB_PATH=imaginary_amd/libmipx_probes.so
for a in "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
    "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333"; do
  MIPX_RCOL_DBG=8 timeout -k 10 120 python3 scripts/op_bench.py reduce $a --iters 2 --warm-ms 0 >> "$O/ab.jsonl" 2>> "$O/stamps.log" \
    || { echo "failed: $a"; exit 1; }
done
grep rcol_stamps "$O/stamps.log" | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    ph = ['ring_write','barrier1','vertical','issue','barrier2','horizontal','store']
    tot = sum(d[p] for p in ph)
    print(d['ow'], d['oh'], d['n'], 'blocks', d['blocks'], 'block', round(d['block_mean']), 'setup', {k[6:]: round(v) for k, v in d.items() if k.startswith('setup_')},
          'step', round(tot), ' '.join(f'{p}={d[p]:.0f}({d[p]/tot:.0%})' for p in ph))
"
