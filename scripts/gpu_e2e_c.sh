# request-path throughput from C (tests/c/mipx_e2e.c): thread / in-flight / queue sweep
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
gcc -O2 -std=c11 -D_DEFAULT_SOURCE -I include tests/c/mipx_e2e.c -L imaginary_amd -lmipx -lpthread \
    -Wl,-rpath,$GRAFT_REPO_ROOT/imaginary_amd -o /tmp/mipx_e2e || exit 1
: > gpurun_out/e2e_c.jsonl
for cfg in "16 32 1 2 8" "16 32 2 2 8" "8 64 1 4 8" "32 16 1 2 8" "16 32 1 2 16" "4 128 1 8 8"; do
  timeout -k 10 120 /tmp/mipx_e2e $cfg >> gpurun_out/e2e_c.jsonl || exit $?
done
cut -c1-330 gpurun_out/e2e_c.jsonl
