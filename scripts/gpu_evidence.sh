#!/bin/bash
# The round's evidence runner (replaces the one-off scripts/gpu_r0*.sh recipes): each
# step under its own time limit, stopping at the first failure.
#   OUT=r04x STEPS="tests smoke bench configs stats pmc_c2 pmc_c3 survey" bash scripts/gpu_evidence.sh
# tests   full -m gpu suite                 -> $O/pytest_gpu.log
# smoke   __graft_entry__.smoke()            -> $O/smoke.log
# bench   bench.py (N=1, driver launch path) -> $O/bench.json (+ bench_centre.json)
# configs bench_configs.py C3 C4 C5          -> $O/configs.jsonl
# stats   rocprofv3 --kernel-trace --stats of bench.py and of each config -> $O/stats_*/
# pmc_c2  FETCH_SIZE / WRITE_SIZE passes of bench.py at both samplings -> $O/traffic.json
# pmc_c3  the same over the C3 config, per kernel  -> $O/traffic_c3.json
# survey  scripts/op_survey.sh                   -> $O/op_survey.jsonl
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-evidence}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
pmc2() {  # pmc2 <dir> <cmd...>: FETCH_SIZE and WRITE_SIZE in separate passes (gfx950 counter limits)
  local d=$1; shift
  run 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$d/p1" -o run -- "$@" > "$d.p1.log" 2>&1
  run 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$d/p2" -o run -- "$@" > "$d.p2.log" 2>&1
}
for s in ${STEPS:-tests smoke bench configs}; do
  echo "== $s $(date +%T)"
  case $s in
    tests) run 1000 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
             > "$O/pytest_gpu.log" 2>&1; tail -2 "$O/pytest_gpu.log" ;;
    smoke) run 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; tail -2 "$O/smoke.log" ;;
    bench) run 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
             --master-port 29512 bench.py --gpus 1 --steps 100 --warmup 20 > "$O/bench.json" 2> "$O/bench.err"
           run 300 python3 bench.py --steps 100 --warmup 20 --no-cpu --sampling centre > "$O/bench_centre.json" 2>> "$O/bench.err"
           cut -c1-240 "$O/bench.json" "$O/bench_centre.json" ;;
    configs) run 600 python3 -u bench_configs.py --configs C3,C4,C5 --steps 10 --warmup 2 > "$O/configs.jsonl" 2> "$O/configs.err"
             run 300 python3 -u bench_configs.py --configs C3 --steps 10 --warmup 2 --sampling centre \
               >> "$O/configs.jsonl" 2>> "$O/configs.err"; cut -c1-200 "$O/configs.jsonl" ;;
    stats) run 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_c2" -o run -- \
             python3 bench.py --steps 100 --warmup 20 --no-cpu > "$O/stats_c2.log" 2>&1
           run 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_c2_centre" -o run -- \
             python3 bench.py --steps 100 --warmup 20 --no-cpu --sampling centre > "$O/stats_c2_centre.log" 2>&1
           for c in C3 C4 C5; do
             run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_$c" -o run -- \
               python3 bench_configs.py --configs $c --steps 10 --warmup 2 > "$O/stats_$c.log" 2>&1
           done ;;
    pmc_c2) for smp in corner centre; do
              pmc2 "$O/pmc_c2_$smp" python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify --sampling $smp
            done
            ALG_BYTES=7962624000 run 60 python3 scripts/traffic_json.py "$O/pmc_c2_corner" "k_reduce2x2<3, 66>" "$O/traffic.json" \
              "C2 bench.py --steps 3, 256 x 4K RGB -> 1080p, corner sampling"
            ALG_BYTES=7962624000 run 60 python3 scripts/traffic_json.py "$O/pmc_c2_centre" "k_reduce2m<3>" "$O/traffic.json" \
              "C2 bench.py --steps 3 --sampling centre, 256 x 4K RGB -> 1080p" ;;
    pmc_c3) pmc2 "$O/pmc_c3" python3 bench_configs.py --configs C3 --steps 3 --warmup 1 --warm-ms 0
            run 60 python3 scripts/traffic_json.py "$O/pmc_c3" "" "$O/traffic_c3.json" "C3 bench_configs.py --steps 3: every kernel" --per-kernel ;;
    survey) run 900 bash scripts/op_survey.sh > "$O/op_survey.txt" 2>&1; cp gpurun_out/op_survey.jsonl "$O/" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
