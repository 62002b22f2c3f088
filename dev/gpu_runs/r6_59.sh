#!/bin/bash
# host enqueue vs GPU completion per phase of one step (is the start of the backward launch-bound?)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_59
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python3 dev/probes/host_phase.py --model resnet50 > $O/r50.txt 2>&1 || { tail -20 $O/r50.txt; exit 1; }
timeout -k 10 240 python3 dev/probes/host_phase.py --model gpt2_small > $O/gpt2.txt 2>&1 || { tail -20 $O/gpt2.txt; exit 1; }
cat $O/r50.txt $O/gpt2.txt | grep host
echo done
