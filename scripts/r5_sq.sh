set -u
cd $GRAFT_REPO_ROOT
TAG=r5_sc1 LIBS="libwgcsum.so scripts/probe_so/libwgcsum_sc1.so" timeout -k 10 500 bash scripts/r5_gso_ab.sh 2 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5_sq; mkdir -p $OUT
export TMPDIR=/tmp
for k in lds rows; do
  if [ $k = rows ]; then export WGCS_GSO_KERNEL=rows; fi
  (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/$k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/$k.log 2>&1) || { echo "FAIL $k"; tail -5 $OUT/$k.log; exit 1; }
  python3 scripts/pmc_summary.py $OUT/$k | grep -A10 gso_
done
