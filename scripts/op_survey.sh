#!/bin/bash
# Per-op survey: every engine op at the config shapes, device-resident, HIP-event timed
# (scripts/op_bench.py), as algorithmic GB/s = fraction of the 8 TB/s HBM peak.
# One JSON line per case into gpurun_out/op_survey.jsonl.  Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
F="$OUT/op_survey.jsonl"; : > "$F"
while read -r args; do
  [ -z "$args" ] && continue
  timeout -k 5 60 python3 scripts/op_bench.py $args --iters 20 2>/dev/null | grep '^{' >> "$F" || { echo "failed: $args"; exit 1; }
done <<LIST
reduce --w 3840 --h 2160 --b 3 --n 256 --s 2
reduce --w 2048 --h 2048 --b 4 --n 512 --s 2
reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333
reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6
reduce --w 1920 --h 1080 --b 3 --n 64 --s 2.4
reduce --w 500 --h 375 --b 3 --n 128 --s 1.46484375
reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747
reducev --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333
reduceh --w 1024 --h 768 --b 4 --n 512 --s 1.3333333333333333
shrink --w 4000 --h 3000 --b 3 --n 64 --s 8
shrink --w 4000 --h 3000 --b 3 --n 64 --s 11
shrink --w 3840 --h 2160 --b 3 --n 64 --s 4
shrink --w 1920 --h 1080 --b 3 --n 64 --s 3
shrink --w 3840 --h 2160 --b 3 --n 32 --s 2
shrink --w 4000 --h 3000 --b 3 --n 32 --s 3
reduce --w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667
blur --w 768 --h 512 --b 4 --n 512 --s 5
blur --w 1920 --h 1080 --b 3 --n 64 --s 1
blur --w 1920 --h 1080 --b 3 --n 64 --s 3
blur --w 3840 --h 2160 --b 3 --n 16 --s 5
embed --w 3840 --h 2160 --b 3 --n 32 --ow 3840 --oh 3840 --extend 1
embed --w 3840 --h 2160 --b 3 --n 32 --ow 3840 --oh 3840 --extend 0
embed --w 3840 --h 2160 --b 3 --n 32 --ow 3840 --oh 3840 --extend 3
extract --w 3840 --h 2160 --b 3 --n 32 --ow 2000 --oh 1500
rot --w 3840 --h 2160 --b 3 --n 32 --s 90
rot --w 3840 --h 2160 --b 3 --n 32 --s 180
rot --w 3840 --h 2160 --b 4 --n 32 --s 270
flip --w 3840 --h 2160 --b 3 --n 32 --s 0
flip --w 3840 --h 2160 --b 3 --n 32 --s 1
affine --w 1920 --h 1080 --b 3 --n 16 --s 2
affine --w 550 --h 740 --b 3 --n 64 --s 2
affine --w 1024 --h 768 --b 4 --n 16 --s 1.5
affine --w 1280 --h 720 --b 3 --n 16 --s 3
affine --w 960 --h 540 --b 3 --n 16 --s 4
zoom --w 1920 --h 1080 --b 3 --n 16 --s 2
LIST
python3 - "$F" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f'{d["op"]:8s} {d["w"]}x{d["h"]}x{d["b"]} n{d["n"]:<4} s={d["s"]:<7.4g} -> {d["out"][0]}x{d["out"][1]}  {d["ms"]:8.4f} ms  {d["alg_GBps"]:7.1f} GB/s  {d["alg_GBps"]/8000:6.1%}')
PY
