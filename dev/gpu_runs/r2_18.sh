#!/bin/bash
# pp engine on 1x1 convs: epilogue drain on/off vs the 128-row kernel; GPT-2 shapes drain on/off
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_18
mkdir -p $O
cd $GRAFT_REPO_ROOT
L=1,3,4,5,7,9,11,13,15,17,19,21
timeout -k 10 120 env PDNN_PP_CONV_MINN=100000 python -u tools/bench_conv.py --no-ref --layers $L --json $O/c_reg.json > $O/c_reg.log 2>&1
timeout -k 10 120 env PDNN_PP_CONV_FWD_K=0 PDNN_PP_CONV_DGRAD_K=0 PDNN_PP_DRAIN=0 python -u tools/bench_conv.py --no-ref --layers $L --json $O/c_pp0.json > $O/c_pp0.log 2>&1
timeout -k 10 120 env PDNN_PP_CONV_FWD_K=0 PDNN_PP_CONV_DGRAD_K=0 PDNN_PP_DRAIN=1 python -u tools/bench_conv.py --no-ref --layers $L --json $O/c_pp1.json > $O/c_pp1.log 2>&1
timeout -k 10 120 env PDNN_PP_DRAIN=0 python -u tools/pp_check.py --perf-only --json $O/g_d0.json > $O/g_d0.log 2>&1
timeout -k 10 120 env PDNN_PP_DRAIN=1 python -u tools/pp_check.py --perf-only --json $O/g_d1.json > $O/g_d1.log 2>&1
echo done
