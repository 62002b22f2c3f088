#!/bin/bash
# batched slab reduce: pp wgrad tests, 1x1 wgrad engine table, pp pixel threshold A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_38
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_wgrad1x1.py > $O/wgrad1x1.log 2>&1 || { tail -20 $O/wgrad1x1.log; exit 1; }
grep -v amdgpu.ids $O/wgrad1x1.log | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['H'], r['conv'], 'reg', r['reg_us'], 'pp', r['pp_best'], 'auto', r['pp_auto_splits'], r.get('pp_s%d_us' % r['pp_auto_splits']))"
i=0
for T in "" "wgrad1x1_pp_pix=200704" "" "wgrad1x1_pp_pix=200704"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
timeout -k 10 300 python -u bench.py --model gpt2_small --steps 20 --no-ddp-rehearsal > $O/gpt2.log 2>&1 || exit 1
echo "[gpt2] $(grep -o '"value": [0-9.]*' $O/gpt2.log)"
echo done
