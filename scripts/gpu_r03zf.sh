# embed / flip row kernels: parity, then the store-policy A/B (scripts/nt_ab.py)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "embed or flip or rot" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/nt_ab.py > $O/nt_ab.jsonl 2>&1 || { tail $O/nt_ab.jsonl; exit 1; }
cat $O/nt_ab.jsonl
