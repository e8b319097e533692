#!/bin/bash
# Round 5: the N>1 bench path (2 processes on the box's one GPU, shared-memory transport),
# round-4 final build (scratch/r04, its own bench.py and bindings) vs this round's, alternating.
mkdir -p gpurun_out
run() {  # $1 bench.py path, $2 tag, $3 port
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $3 $1 --gpus 2 --steps 20 --warmup 3 --transport shm --ranks-per-gpu 2 --no-cpu-baseline --no-cfg3 > gpurun_out/n2_$2.json 2> gpurun_out/n2_$2.err || return $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/n2_$2.json') if l.startswith('{')][-1]);print('$2', round(d['ms_per_step'],3), d['phase_ms_per_call'])"
}
run scratch/r04/bench.py r04a 29521 && run bench.py r05a 29522 && run scratch/r04/bench.py r04b 29523 && run bench.py r05b 29524
