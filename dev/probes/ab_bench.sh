#!/bin/bash
# Same-box A/B of bench.py: alternate two PDNN_TUNE settings N times (bench noise across boxes is ~1%).
#   bash dev/probes/ab_bench.sh OUTDIR "A_TUNE" "B_TUNE" [pairs] [extra bench args]
O=$1; A=$2; B=$3; N=${4:-3}; shift 4; X="$@"
mkdir -p $O
for i in $(seq 1 $N); do
  for v in "$A" "$B"; do
    PDNN_TUNE="$v" timeout -k 10 300 python -u bench.py --no-ddp-rehearsal $X > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
    echo "[$v] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  done
done
