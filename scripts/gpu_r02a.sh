# round 2: smoke + new GPU suites (configs C4/C5, request path, fuzz) + full suite
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail=15 --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu.log; exit $rc
