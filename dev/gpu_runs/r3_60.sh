#!/bin/bash
# fork_merge / wprep / join_once A/B; DDP-path light_events A/B + trace; cost of one cross-stream fork on the compute stream: torch wait_stream vs fence-free event vs write/wait value
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_60
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/fork_cost.py > $O/fork.log 2>&1 || { tail -20 $O/fork.log; exit 1; }
cat $O/fork.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_blocks_gpu.py tests/test_models_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for T in "" "fork_merge=1" "wprep=0" "join_once=0" "" "fork_merge=1" "wprep=0" "join_once=0"; do
  i=$((i+1))
  PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --no-ddp-rehearsal > $O/b$i.log 2>&1 || exit 1
  echo "[$T] $(grep -o '"value": [0-9.]*' $O/b$i.log)"
done
# DDP path at world 1 (1-rank RCCL group): light_events A/B through the bucket launches, and a kernel trace
export PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1
i=0
for T in "" "light_events=0" "" "light_events=0"; do
  i=$((i+1))
  MASTER_PORT=$((29611+i)) PDNN_TUNE="$T" timeout -k 10 200 python -u bench.py --steps 30 --ddp-rehearsal > $O/d$i.log 2>&1 || { tail -20 $O/d$i.log; exit 1; }
  echo "[ddp $T] $(grep -o '"value": [0-9.]*' $O/d$i.log | head -1)"
done
export MASTER_PORT=29631
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ddp --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 3 --ddp-rehearsal > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }

echo done
