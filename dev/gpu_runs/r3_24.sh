#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py 2>&1 | tail -20
