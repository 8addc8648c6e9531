set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/g1/tests.log 2>&1; rc=$?; tail -3 gpurun_out/g1/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/g1/cfg4.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams 1 > gpurun_out/g1/cfg4_1s.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/g1/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams 1 > $GRAFT_REPO_ROOT/gpurun_out/g1/prof.log 2>&1 || exit $?
echo done
