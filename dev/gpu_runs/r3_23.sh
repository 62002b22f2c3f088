#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python -u dev/stem_ab.py 2>&1 | head -60
