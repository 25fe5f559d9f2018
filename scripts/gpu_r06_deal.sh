#!/bin/bash
# r06: C4 / C5 plan groups dealt to the streams least-loaded by bytes (default) against the
# r05 round-robin (MIPX_BENCH_DEAL=rr), alternating processes; then 4 / 6 / 8 streams
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_deal}"; mkdir -p "$O"
cfg() { local tag=$1; shift; timeout -k 10 300 "$@" | sed "s/^{/{\"ab\": \"$tag\", /" >> "$O/configs.jsonl" 2>> "$O/configs.err" || { echo "configs failed"; exit 1; }; }
for rep in 1 2 3; do
  MIPX_BENCH_DEAL=rr cfg rr python3 -u bench_configs.py --configs C4,C5 --steps 10 --warmup 2
  cfg lpt python3 -u bench_configs.py --configs C4,C5 --steps 10 --warmup 2
done
for st in 6 8; do cfg "lpt_s$st" python3 -u bench_configs.py --configs C5 --steps 10 --warmup 2 --streams $st; done
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/configs.jsonl"):
    d = json.loads(l); print(d["ab"], d["config"], d["ms_per_step"], d["hbm_frac"], d["images_per_sec"], d["verified_vs_oracle"])
PY
