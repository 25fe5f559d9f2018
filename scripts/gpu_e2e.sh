set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/e2e_q.jsonl
for q in 1 2 3 1 2 3; do
  for t in 16 32; do
    timeout -k 10 120 python3 -u bench_configs.py --configs E2E --e2e-queues $q --e2e-threads $t --e2e-requests 512 2>>gpurun_out/e2e_q.err | grep '^{' >> gpurun_out/e2e_q.jsonl || exit 1
  done
done
cut -c1-400 gpurun_out/e2e_q.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['queues'], d['requests']//1, d['images_per_sec'], d['host_link_gbs'], d['mean_batch'], d.get('requests_per_queue'))"
