#!/bin/bash
# Round 6: kernel trace of the cfg3 8 y-slab turns run (ghosts in place) with the fused update,
# per-slab kernel breakdown; cfg3 single domain on the same box (the T8 denominator).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y11" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y11.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y11 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y11_breakdown.json | tail -3
rm -rf gpurun_out/r06/trace_y11
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06/cfg3_single11.json 2> gpurun_out/r06/cfg3_single11.err || exit $?
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06/cfg3_single11.json') if l.startswith('{')][-1])
print('cfg3 single', d['ms_per_step'], d['phase_ms_per_call'])"
