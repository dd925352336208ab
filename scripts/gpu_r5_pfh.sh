#!/bin/bash
# After the f16-MFMA prefill tiles (row-local forwards included) and the 1.5 * 2^23 MFMA start in the tiled prefill GEMM
# only: the GPU suite, the batch-32 step and prefill vs lib/diag/mg_old.so (previous commit), then the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=fun-asr-gguf_amd/lib/libfunasr_hip.so; O=fun-asr-gguf_amd/lib/diag/mg_old.so
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pfh_tests.log 2>&1 || { tail -40 gpurun_out/pfh_tests.log; exit 1; }
tail -2 gpurun_out/pfh_tests.log
pf() { FUNASR_HIP_LIB=$2 timeout -k 10 200 python -u scripts/prof_batch_prefill.py $3 204 5 2>&1 | sed "s/^/$1 B=$3 /" | tee -a gpurun_out/pfh_ab.log; }
dec() { FUNASR_HIP_LIB=$2 AB_M=$3 timeout -k 10 200 python -u scripts/prof_decode_ab.py 128 - 2>&1 | sed "s/^/$1 /" | tee -a gpurun_out/pfh_ab.log; }
dec new $L 32 && dec old $O 32 && dec new $L 32 && dec old $O 32 || exit 1
for b in 1 6 32; do pf new $L $b && pf old $O $b || exit 1; done
timeout -k 10 600 python -u bench.py > gpurun_out/bench_pfh.json 2> gpurun_out/bench_pfh.err || { tail -20 gpurun_out/bench_pfh.err; exit 1; }
cut -c1-300 gpurun_out/bench_pfh.json
