set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for nb in 0 1; do
  WGCS_GSO_NB2=$nb timeout -k 10 300 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_fullsize.py tests/test_golden.py tests/test_gpu_stager.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gsosw_t$nb.log 2>&1; rc=$?
  echo "tests nb2=$nb rc=$rc $(tail -1 gpurun_out/gsosw_t$nb.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
for rep in 1 2 3; do
for nb in 0 1; do
  for st in 1 2; do
    WGCS_GSO_NB2=$nb timeout -k 10 120 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams $st > gpurun_out/gsosw_b${nb}_$st.log 2>&1 || exit 1
    echo "nb2=$nb streams=$st $(python -c "import json;d=json.loads(open('gpurun_out/gsosw_b${nb}_$st.log').read().splitlines()[-1]);r=d['roofline'];print(d['value'],r['kernel_ms'],r['frac'],r.get('kernel_ms_one_stream'))")"
  done
done
done
