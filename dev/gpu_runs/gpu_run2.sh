#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/run2
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_conv.py --batch 256 --json gpurun_out/run2/bench_conv.json > gpurun_out/run2/bench_conv.log 2>&1
