#!/bin/bash
# Same-box A/B of bench.py between the in-tree kernel library (B) and a base build (A, dev/probes/build_base.py).
#   bash dev/probes/ab_lib.sh OUTDIR BASE.so [pairs] [extra bench args]
O=$1; BASE=$2; N=${3:-3}; shift 3; X="$@"
mkdir -p $O
for i in $(seq 1 $N); do
  PDNN_KERNEL_LIB=$BASE timeout -k 10 300 python -u bench.py --no-ddp-rehearsal $X > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  echo "[base] $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
  timeout -k 10 300 python -u bench.py --no-ddp-rehearsal $X > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  echo "[new]  $(grep -o '"value": [0-9.]*' $O/ab.log)" | tee -a $O/ab_summary.txt
done
