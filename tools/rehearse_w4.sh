# N = 2 and N = 4 rehearsal of the bench's multi-rank path on ONE GPU (gloo, every rank on cuda:0):
# each rank extracts its own images; the queued descriptors of 8 steps are all-gathered and
# searched (certified) against the rank's DB shard, the last partial batch flushed; top-k +
# certificate flags all-gathered + merged; max-over-ranks timing.  Throughput is not
# meaningful (the ranks share one GPU).
set -e
mkdir -p gpurun_out/w4
for N in 2 4; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29530 + N)) bench.py --gpus $N --steps 10 --warmup 2 --alt-steps 0 --dist-backend gloo --one-device \
    --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 \
    > gpurun_out/w4/bench_w$N.json 2> gpurun_out/w4/bench_w$N.err
  python3 -c "
import json
d=json.loads(open('gpurun_out/w4/bench_w$N.json').read().strip().splitlines()[-1])
print('N=$N', d['value'], d['ms_per_step'], 'searches', d['searches'], 'requeried', d['requeried'], 'query_batch', d['config']['query_batch'], 'comm', d['comm'] and {k: v for k, v in d['comm'].items() if k.endswith('_ms')}, 'knn', d['knn']['ms_per_batch'], d['knn']['requeried'])"
done
