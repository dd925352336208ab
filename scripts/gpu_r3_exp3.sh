#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/varlen_c3.py 192 32 4 2>&1 | tail -3 || exit 1
timeout -k 10 300 python3 scripts/varlen_c3.py 192 32 8 2>&1 | tail -2 || exit 1
