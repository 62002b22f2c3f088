#!/bin/bash
# new defaults (s2_halo=3 with measured routing, ds_sub=1, comm_cus=0, split tied GPT-2 embedding, no native RCCL):
# GPU tests of the touched paths, ResNet-50 / GPT-2 A/B, one kernel trace of the ResNet-50 plain step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_03
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_s2_gpu.py tests/test_ddp_gpu.py tests/test_transformer_gpu.py tests/test_fused_blocks_gpu.py tests/test_tuning_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {
  local n=$1; shift
  local m=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --model $m --no-plain-run --no-extra-configs --diag-steps 3 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
run r_def resnet50 PDNN_TUNE=ds_sub=1 && run r_ds0 resnet50 PDNN_TUNE=ds_sub=0 && run r_def2 resnet50 PDNN_TUNE=ds_sub=1 && run r_ds0b resnet50 PDNN_TUNE=ds_sub=0 || exit 1
run g_split gpt2_small PDNN_DDP_SPLIT_TIED=1 && run g_nosplit gpt2_small PDNN_DDP_SPLIT_TIED=0 && run g_split2 gpt2_small PDNN_DDP_SPLIT_TIED=1 || exit 1
python3 -c "import json;d=json.load(open('$O/g_split.json'));c=d['comm'];print('split bucket_mb',c['bucket_mb'],'ready',c['fp32']['bucket_ready_ms'],'bwd_end',c['fp32']['backward_end_ms'])"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -d /tmp/q4 -o q4 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --plain > $O/q4.log 2>&1 || exit $?
find /tmp/q4 -name "*kernel_trace.csv" -exec cp {} $O/q4_trace.csv \;
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $O/q4_trace.csv --steps 3 --by-grid --top 80 > $O/grid_summary.txt 2>&1
head -3 $O/grid_summary.txt
echo done
