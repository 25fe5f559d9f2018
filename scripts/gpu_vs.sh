set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py tests/test_rstrip_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduce or rstrip or shrink" > gpurun_out/pytest_vs.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_vs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_VP_SHARE=1 MIPX_VP_SHARE=0 > gpurun_out/vs_ab.jsonl 2>gpurun_out/vs_ab.err; rc=$?; cut -c1-170 gpurun_out/vs_ab.jsonl; tail -3 gpurun_out/vs_ab.err; exit $rc
