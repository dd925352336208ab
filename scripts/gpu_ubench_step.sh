#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MODES:-hbm fused}; do timeout -k 5 120 ./scripts/ubench/decode_step $m || exit 1; done
