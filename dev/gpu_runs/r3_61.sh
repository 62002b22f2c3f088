#!/bin/bash
# fork through write/wait value (light_events=2) vs fence-free events (1): tests + plain and DDP-path A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_61
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PDNN_TUNE="light_events=2" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_blocks_gpu.py tests/test_models_gpu.py tests/test_ddp_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for T in "" "light_events=2" "" "light_events=2"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
export PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1
i=0
for T in "" "light_events=2" "" "light_events=2"; do
  i=$((i+1))
  MASTER_PORT=$((29711+i)) PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --ddp-rehearsal > $O/d$i.log 2>&1 || { tail -20 $O/d$i.log; exit 1; }
  echo "[ddp $T] $(grep -o '"value": [0-9.]*' $O/d$i.log | head -1)"
done
echo done
