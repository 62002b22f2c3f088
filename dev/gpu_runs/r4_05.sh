#!/bin/bash
# wide kernel v1 routed to its winning shapes: numerics; flagship trajectory vs fp32; per-layer 1x1 timings
# (default and glds-forced); world-1 RCCL AVG sweep (device-event timing); flagship bench + DDP rehearsal comm block
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4_05
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_conv1x1_wide_gpu.py tests/test_trajectory_gpu.py tests/test_tuning_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -le 1 ] || exit $rc        # test failures are reported, a crash / timeout ends the run
timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_default.log 2>&1 || { tail -20 $O/c1_default.log; exit 1; }
PDNN_TUNE=glds=2 timeout -k 10 200 python -u tools/bench_conv1x1.py > $O/c1_glds.log 2>&1 || { tail -20 $O/c1_glds.log; exit 1; }
tail -n 1 $O/c1_default.log $O/c1_glds.log
PDNN_FORCE_PG=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 tools/bench_allreduce.py --ops all_reduce,broadcast --dtypes float32,bfloat16 > $O/allreduce_w1.log 2>&1 || { tail -20 $O/allreduce_w1.log; exit 1; }
grep -c '"op"' $O/allreduce_w1.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-250

timeout -k 10 300 python -u bench.py --graph on --no-ddp-rehearsal > $O/bench_graph.log 2>&1 || { tail -20 $O/bench_graph.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench_graph.log
timeout -k 10 300 python -u -m cProfile -o $O/bench.cprof bench.py --steps 10 --warmup 5 --no-ddp-rehearsal --diag-steps 0 > $O/cprof_bench.log 2>&1 || { tail -20 $O/cprof_bench.log; exit 1; }
python -c "import pstats; p = pstats.Stats('$O/bench.cprof'); p.sort_stats('tottime').print_stats(45)" > $O/cprof_tottime.txt 2>&1
python -c "import pstats; p = pstats.Stats('$O/bench.cprof'); p.sort_stats('cumulative').print_stats(60)" > $O/cprof_cum.txt 2>&1
echo profiled
echo done
