#!/bin/bash
# PMC of the halo 3x3 conv (stage 1 fwd / dgrad) and the 1x1 panel kernel, + k-of-n throttle re-measure
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_10
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for k in fwd dgrad panel; do
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d /tmp/p_$k -o p --output-format csv -- python3 $R/tools/c3_probe.py --kind $k > $O/p_$k.log 2>&1 || exit 1
find /tmp/p_$k -name "*counter_collection.csv" -exec cp {} $O/pmc_$k.csv \;
done
cd $R
R2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
PDNN_FORCE_PG=1 PDNN_DDP_FORCE_COMM=1 timeout -k 10 300 $R2 --master-port 29612 bench.py --gpus 1 --steps 30 --warmup 8 --num-aggregate 1 > $O/bench_kofn1.log 2>&1 && tail -n 1 $O/bench_kofn1.log | cut -c1-150 || exit 1
echo done
