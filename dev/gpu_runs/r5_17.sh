#!/bin/bash
# ping-pong phase traces: where a 2-round N = 3072 / K = 768 GEMM and a 1-round N = 768 GEMM spend time
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5_17
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R
for args in "8192 3072 768 --bn 192" "8192 3072 1536 --bn 192" "8192 3072 768 --bn 256" "8192 768 3072 --bn 96" "8192 768 768 --bn 96" "8192 2304 768 --bn 288"; do
  PDNN_TUNE=pp_w4=1 timeout -k 10 120 python3 dev/probes/pp_one.py $args --trace >> $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
  PDNN_TUNE=pp_w4=0 timeout -k 10 120 python3 dev/probes/pp_one.py $args --trace >> $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
done
grep -v amdgpu.ids $O/trace.txt
export TMPDIR=/tmp
cd /tmp
P="TCC_HIT TCC_MISS TCC_REQ TCC_EA0_RDREQ TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TOTAL_ACCESSES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"
Q="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_MFMA"
for v in 1 0; do
  PDNN_TUNE=pp_w4=$v timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $P -d /tmp/p$v -o p$v --output-format csv -- python3 $R/dev/probes/n768_gemm.py both fc2 > $O/p$v.log 2>&1 || exit 1
  find /tmp/p$v -name "*counter_collection.csv" -exec cp {} $O/pmc_a_w4$v.csv \;
  PDNN_TUNE=pp_w4=$v timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $Q -d /tmp/q$v -o q$v --output-format csv -- python3 $R/dev/probes/n768_gemm.py both fc2 > $O/q$v.log 2>&1 || exit 1
  find /tmp/q$v -name "*counter_collection.csv" -exec cp {} $O/pmc_b_w4$v.csv \;
done
echo done
