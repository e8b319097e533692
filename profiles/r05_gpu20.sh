#!/bin/bash
# Round 5: rocprofv3 kernel trace of the cfg3 8-slab split in the full-step turns mode (every
# kernel of a slab's step alone on the GPU): per-slab kernel breakdown of a step.
mkdir -p gpurun_out/r05_turns2_trace
export TMPDIR=/tmp
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05_turns2_trace/kt -o run -- python3 profiles/slab_turns.py --slabs 8 --repeat 1 --steps 4 --warmup 2 --modes inplace > gpurun_out/r05_turns2_trace/run.log 2>&1 || exit $?
ls -la gpurun_out/r05_turns2_trace/kt/* | head
