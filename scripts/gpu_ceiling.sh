set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ceiling > gpurun_out/ceiling_r02.jsonl 2>&1; rc=$?; cat gpurun_out/ceiling_r02.jsonl; exit $rc
