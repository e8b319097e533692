#!/bin/bash
# Round 5: slab pack scan with its loads batched — full GPU suite, then the
# full-step turns trace of the cfg3 8-slab split (per-slab kernel breakdown).
mkdir -p gpurun_out/r05_turns2_trace_c
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r05x.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputest_r05x.log | tail -12
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05_turns2_trace_c/kt -o run -- python3 profiles/slab_turns.py --slabs 8 --repeat 1 --steps 4 --warmup 2 --modes inplace > gpurun_out/r05_turns2_trace_c/run.log 2>&1 || exit $?
grep -o '"slab_kernels_ms_per_step": [^]]*]' gpurun_out/r05_turns2_trace_c/run.log | tail -1
