set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m "gpu" -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -40 gpurun_out/gpu_tests.log
exit $rc
