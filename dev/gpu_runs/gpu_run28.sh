#!/bin/bash
# Diagnose a host segfault at hipGraph capture_end: the failing test alone, then the others alone.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run28
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
P="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 200 $P tests/test_graphs_gpu.py::test_trainer_graph_mode > $O/t_trainer.log 2>&1 || exit $?
$T 200 $P tests/test_graphs_gpu.py::test_graph_step_shape_change_runs_eager > $O/t_shape.log 2>&1 || exit $?
