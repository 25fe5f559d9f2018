set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r02h; export TMPDIR=/tmp
timeout -k 10 600 bash scripts/op_survey.sh > gpurun_out/r02h/op_survey.log 2>&1 || exit $?
cp gpurun_out/op_survey.jsonl gpurun_out/r02h/op_survey.jsonl; echo done
