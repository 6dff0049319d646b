# Two ranks on ONE GPU over gloo: exercises bench.py's multi-process path
# (rendezvous, per-rank seeding, advantage statistics, gradient bucket
# all-reduce, max-over-ranks timing) on a single-GPU box.
cd /root/repo && mkdir -p gpurun_out
MARLMAZE_DP_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mazes 8192 --steps 2 --warmup 1 \
  > gpurun_out/dp_rehearsal.log 2>&1
echo "dp rehearsal rc=$?"; tail -2 gpurun_out/dp_rehearsal.log | cut -c1-400
