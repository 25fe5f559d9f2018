#!/bin/bash
# A/B one op_bench case over a list of env settings: ENVS="A=1 B=2;A=2" OP="reducev --w ..."
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
IFS=';' read -ra SETS <<< "$ENVS"
for rnd in 1 2; do
  for e in "${SETS[@]}"; do
    out=$(env $e timeout -k 5 60 python3 scripts/op_bench.py $OP 2>/dev/null | grep '^{') || exit 1
    echo "{\"env\": \"$e\", \"round\": $rnd, \"r\": $out}"
  done
done
