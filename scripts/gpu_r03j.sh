# memory-only ceilings of the generic reduce's strip walk (scripts/strip_probe.hip)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03j; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 ./scripts/strip_probe > $O/strip_probe.jsonl 2>&1; rc=$?; cat $O/strip_probe.jsonl; exit $rc
