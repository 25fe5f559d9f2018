# k_bcol with 16-byte-aligned horizontal operands (ds_read_b128): parity, A/B, PMC
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zj; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_bcol_gpu.py tests/test_demand_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 120 python3 -u scripts/op_bench.py"
{ $A blur --w 1920 --h 1080 --b 3 --n 64 --s 1 --ab MIPX_BCOL_A16=0,1 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 3 --ab MIPX_BCOL_A16=0,1 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 5 --ab MIPX_BCOL_A16=0,1 &&
  $A blur --w 3840 --h 2160 --b 3 --n 16 --s 5 --ab MIPX_BCOL_A16=0,1 &&
  $A blur --w 4000 --h 3000 --b 3 --n 16 --s 3 --ab MIPX_BCOL_A16=0,1 &&
  $A blur --w 768 --h 512 --b 4 --n 512 --s 5 --ab MIPX_BCOL_A16=0,1 &&
  $A blur --w 1920 --h 1080 --b 4 --n 32 --s 2 --ab MIPX_BCOL_A16=0,1; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    print(d["op"], d["w"], d["h"], d["b"], d["s"], k, d[k], d["round"], d["ms"], d["alg_GBps"], d["same_as_first"])
PY
PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVES" TAG=b5a OP_ARGS="blur --w 1920 --h 1080 --b 3 --n 64 --s 5" timeout -k 10 200 bash scripts/pmc_op.sh > $O/pmc_bcol_a16_rgb_s5.txt 2>&1 || { tail $O/pmc_bcol_a16_rgb_s5.txt; exit 1; }
cat $O/pmc_bcol_a16_rgb_s5.txt
