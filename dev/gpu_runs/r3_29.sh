#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/host_timing.py --steps 10 --cpu-profile 2>&1 | tail -45
