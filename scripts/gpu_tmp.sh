cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 0 16 32 64; do timeout -k 5 120 ./scripts/ubench/gemm_f32_bench $p | grep -v check || exit 1; done
