#!/bin/bash
# 4-wave form with 64-deep slices (N = 768 GEMMs): numerics + per-GEMM timings vs the 8-wave 64-deep form
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_19
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "pp_narrow" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in fc2_fwd fc_dgrad qkv_dgrad proj_dgrad proj_fwd; do
  PDNN_TUNE=pp_w4=1 timeout -k 10 120 python3 dev/probes/gpt2_gemms.py $g > $O/w4_$g.json 2>> $O/err.log || exit 1
  timeout -k 10 120 python3 dev/probes/gpt2_gemms.py $g > $O/w8_$g.json 2>> $O/err.log || exit 1
  python3 -c "import json;a=json.load(open('$O/w4_$g.json'));b=json.load(open('$O/w8_$g.json'));print('$g w4', a['auto'], 'w8', b['auto'], 'torch', b['torch'])"
done
