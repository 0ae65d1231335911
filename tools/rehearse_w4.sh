# N = 4 rehearsal of the bench's multi-rank path on ONE GPU (gloo, every rank on cuda:0):
# query all-gather, 4 DB shards of 250k rows (Q = 512 per shard search), top-k all-gather + merge,
# max-over-ranks timing.  Throughput is not meaningful (4 ranks share one GPU).
set -e
mkdir -p gpurun_out/w4
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --one-device --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 \
  > gpurun_out/w4/bench.json 2> gpurun_out/w4/bench.err
tail -1 gpurun_out/w4/bench.json
