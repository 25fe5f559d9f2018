set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vsprof -o run -- python3 scripts/rs_ab.py MIPX_VP_SHARE=1 MIPX_VP_SHARE=0 > gpurun_out/vs_ab2.jsonl 2>gpurun_out/vs_ab2.err; rc=$?
find gpurun_out/vsprof -name "*stats*" | head; exit $rc
