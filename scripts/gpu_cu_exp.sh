#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
F=ffffffff; Z=00000000
run() { timeout -k 10 180 python3 scripts/exp_cu_partition.py "$1" "$2" 2>&1 | tail -1; }
run - - || exit 1
run $F,$F,$F,$F,$Z,$Z,$Z,$Z $Z,$Z,$Z,$Z,$F,$F,$F,$F || exit 1
run 55555555,55555555,55555555,55555555,55555555,55555555,55555555,55555555 aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa,aaaaaaaa || exit 1
run $F,$F,$Z,$Z,$Z,$Z,$Z,$Z $Z,$Z,$F,$F,$F,$F,$F,$F || exit 1
run 0000ffff,0000ffff,0000ffff,0000ffff,0000ffff,0000ffff,0000ffff,0000ffff ffff0000,ffff0000,ffff0000,ffff0000,ffff0000,ffff0000,ffff0000,ffff0000 || exit 1
