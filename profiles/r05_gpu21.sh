#!/bin/bash
# Round 5: the N>1 bench path (one process per rank, torch.distributed launch) on the one GPU
# of the box with the shared-memory transport: N=2 cfg2 weak scaling and N=4 cfg3 strong.
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --transport shm --ranks-per-gpu 2 --no-cpu-baseline > gpurun_out/bench_n2_shm.json 2> gpurun_out/bench_n2_shm.err
echo "n2 rc=$?"; grep '^{' gpurun_out/bench_n2_shm.json | head -c 700; echo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --workload cfg3 --steps 4 --warmup 2 --transport shm --ranks-per-gpu 4 --no-cpu-baseline > gpurun_out/bench_n4_shm.json 2> gpurun_out/bench_n4_shm.err
echo "n4 rc=$?"; grep '^{' gpurun_out/bench_n4_shm.json | head -c 700; echo
