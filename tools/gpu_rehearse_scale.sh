# N > 1 bench paths rehearsed on ONE GPU (the driver form: torch.distributed.run, one rank per process, gloo and the
# host all-reduce instead of RCCL): N = 2 (replicas + cfg4 sharded companion) and N = 8 (replicas + cfg5 world-8
# sharded companion).  usage: bash tools/gpu_rehearse_scale.sh  ->  gpurun_out/r05rh/n{2,8}.json
set -e
O=gpurun_out/r05rh
mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 30 --warmup 5 --rehearse --sharded-steps 30 > $O/n2.json 2> $O/n2.err
cat $O/n2.json
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8 --steps 10 --warmup 5 --rehearse --sharded-steps 10 > $O/n8.json 2> $O/n8.err
cat $O/n8.json
