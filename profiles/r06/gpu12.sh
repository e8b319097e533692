#!/bin/bash
# Round 6: the fused update at one particle per thread (blocks of 1024): divide / slab / motion
# GPU tests, cfg2 A/B against the separate launches, the cfg3 8 y-slab turns run and its trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_divide_inc.py tests/test_gpu_items.py tests/test_gpu_slab.py tests/test_gpu_slab_y.py tests/test_motion.py tests/test_gpu_parity.py tests/test_symmetry.py tests/test_ext.py tests/test_developed.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06/test12.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test12.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash profiles/ab.sh 3 main:SPH_CLS_SPLIT=1 main -- --steps 40 --warmup 5 > gpurun_out/r06/ab12.log 2>&1 || exit $?
cat gpurun_out/r06/ab12.log
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace,overlap > gpurun_out/r06/turns8_y12.log 2>&1 || exit $?
tail -c 1200 gpurun_out/r06/turns8_y12.log
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y12" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y12.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y12 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y12_breakdown.json | tail -3
rm -rf gpurun_out/r06/trace_y12
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06/cfg3_single12.json 2> gpurun_out/r06/cfg3_single12.err || exit $?
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/cfg3_single12.json') if l.startswith('{')][-1])
print('cfg3 single', d['ms_per_step'], d['phase_ms_per_call'])"
