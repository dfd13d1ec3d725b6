# RCCL inside the captured step: one-rank nccl process group through the point-sharded path
# (all_gather / all_reduce captured in the hipGraph), graph vs eager, then the plain N=1 bench.
set -e
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --dist --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dist1.log 2>&1 \
  || { tail -30 gpurun_out/dist1.log; exit 1; }
grep -h "execution\|metric" gpurun_out/dist1.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 1 --dist --eager --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dist1e.log 2>&1 \
  || { tail -30 gpurun_out/dist1e.log; exit 1; }
grep -h "metric" gpurun_out/dist1e.log | cut -c1-300
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b1.log 2>&1 || { tail -30 gpurun_out/b1.log; exit 1; }
grep -h "metric" gpurun_out/b1.log
