set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
WGCS_GSO_SLACK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k gso > gpurun_out/gsosw_ts.log 2>&1; echo "tests slack rc=$? $(tail -1 gpurun_out/gsosw_ts.log)"
for rep in 1 2 3; do
for sl in 0 1; do
  for st in 1 2; do
    WGCS_GSO_SLACK=$sl timeout -k 10 120 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams $st > gpurun_out/gsosw_b${sl}_$st.log 2>&1 || exit 1
    echo "slack=$sl streams=$st $(python -c "import json;d=json.loads(open('gpurun_out/gsosw_b${sl}_$st.log').read().splitlines()[-1]);r=d['roofline'];print(d['value'],r['kernel_ms'],r['frac'],r.get('kernel_ms_one_stream'))")"
  done
done
done
