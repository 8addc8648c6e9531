# Rehearse the N=2 bench on a 1-GPU box: 2 ranks share cuda:0 over gloo (the driver runs RCCL, one GPU per rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export WGCS_DIST_BACKEND=gloo
for cfg in cfg2 cfg5 cfg4 cfg1 udp_split gro_device gro_staged; do
  echo "== $cfg"
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config $cfg --steps 50 --warmup 5 > gpurun_out/${TAG:-r1}.rehearse_$cfg.log 2>&1 || { echo "FAIL $cfg rc=$?"; tail -20 gpurun_out/${TAG:-r1}.rehearse_$cfg.log; exit 1; }
  grep '^{' gpurun_out/${TAG:-r1}.rehearse_$cfg.log | cut -c1-300
done
