#!/bin/bash
# PMC of k_rcol on the C1 shape against the 1080p row at the same shrink
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05pmcs}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
TAG=rcol_c1 OP_ARGS="reduce --w 480 --h 270 --b 3 --n 256 --s 1.6" run 400 bash scripts/pmc_op.sh > "$O/pmc_rcol_480x270.txt"
TAG=rcol_1080 OP_ARGS="reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6" run 400 bash scripts/pmc_op.sh > "$O/pmc_rcol_1080p.txt"
paste "$O/pmc_rcol_480x270.txt" "$O/pmc_rcol_1080p.txt" | awk '{print $1, $2, $3, $6}'
