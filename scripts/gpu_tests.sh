set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
echo "rc=$?"
tail -30 gpurun_out/t1.log
