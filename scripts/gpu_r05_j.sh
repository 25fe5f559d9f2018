#!/bin/bash
# k_rcol conflict-free horizontal reads (MIPX_RCOL_SWZ) parity + A/B; k_enlm PMC
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05j}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
tail -2 "$O/pytest.log"
: > "$O/swz_ab.jsonl"
for args in "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
            "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333"; do
  run 120 python3 scripts/op_bench.py reduce $args --iters 20 --ab MIPX_RCOL_SWZ=0,1 >> "$O/swz_ab.jsonl"
done
python3 - "$O/swz_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["w"], d["h"], d["b"], d["s"], "swz", d["MIPX_RCOL_SWZ"], "r", d["round"], d["ms"], d["alg_GBps"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
export MIPX_ENLM=2
TAG=enlm_1080p OP_ARGS="affine --w 1920 --h 1080 --b 3 --n 16 --s 2" PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE" run 300 bash scripts/pmc_op.sh > "$O/pmc_enlm_1080p.txt" 2>&1
cat "$O/pmc_enlm_1080p.txt"
