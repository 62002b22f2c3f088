#!/bin/bash
# round-6 start: baseline on this box; native RCCL path vs HW queue count (hypothesis: a 5th+ HIP stream makes the
# compute and side streams share a hardware queue at GPU_MAX_HW_QUEUES=4); comm_cus pricing at a forced comm world
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_01
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {
  local n=$1; shift
  local m=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model $m --no-plain-run --no-extra-configs --diag-steps 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
timeout -k 10 400 python3 bench.py --no-extra-configs > $O/base.json 2> $O/base.err || { tail -20 $O/base.err; exit 1; }
cat $O/base.json
run pg_q8 resnet50 GPU_MAX_HW_QUEUES=8 &&
run nat resnet50 PDNN_DDP_NATIVE_COMM=1 &&
run nat_q8 resnet50 PDNN_DDP_NATIVE_COMM=1 GPU_MAX_HW_QUEUES=8 &&
run pg resnet50 PDNN_TUNE=side_wgrad=1 &&
run cw8_cus16 resnet50 PDNN_BENCH_COMM_WORLD=8 &&
run cw8_cus8 resnet50 PDNN_BENCH_COMM_WORLD=8 PDNN_TUNE=comm_cus=8 &&
run cw8_cus0 resnet50 PDNN_BENCH_COMM_WORLD=8 PDNN_TUNE=comm_cus=0 &&
run g_pg gpt2_small PDNN_TUNE=side_wgrad=1 &&
run g_cw8_cus16 gpt2_small PDNN_BENCH_COMM_WORLD=8 &&
run g_cw8_cus8 gpt2_small PDNN_BENCH_COMM_WORLD=8 PDNN_TUNE=comm_cus=8 &&
run g_pg2 gpt2_small PDNN_TUNE=side_wgrad=1 || exit 1
echo done
