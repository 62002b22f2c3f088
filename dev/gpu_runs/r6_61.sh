#!/bin/bash
# end of round 6: N > 1 rehearsal on the one-GPU box: bench.py's multi-rank branch with 2 ranks sharing cuda:0 over gloo
# (RCCL needs one GPU per rank); ResNet-50 and GPT-2, short runs.  Checks the JSON line, MAX timing, comm block.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_61
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PDNN_BENCH_BACKEND=gloo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --diag-steps 1 > $O/r50_n2.json 2> $O/r50_n2.err || { tail -30 $O/r50_n2.err; exit 1; }
cut -c1-600 $O/r50_n2.json
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --model gpt2_small --gpus 2 --steps 3 --warmup 2 --diag-steps 1 > $O/gpt2_n2.json 2> $O/gpt2_n2.err || { tail -30 $O/gpt2_n2.err; exit 1; }
cut -c1-600 $O/gpt2_n2.json
echo done
