#!/bin/bash
# Round 5 final: the 8-slab cfg3 split's bound weight measured in the full-step turns mode,
# then the full GPU suite, smoke(), the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for w in 0.1 0.2 0.3 0.5; do
  SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --slabs 8 --repeat 1 --steps 6 --modes inplace --bound-weight $w > "$R/gpurun_out/turns_bw${w}.log" 2>&1 || exit $?
  echo "bw $w"; grep -o '"bounds": [^]]*]' "$R/gpurun_out/turns_bw${w}.log" | head -1; grep -o '"slab_kernels_ms_per_step": [^]]*]' "$R/gpurun_out/turns_bw${w}.log" | tail -1; grep -o '"wall_ms_per_step": [0-9.]*' "$R/gpurun_out/turns_bw${w}.log" | tail -1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$R/gpurun_out/gputest_r05z.log" 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$R/gpurun_out/gputest_r05z.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$R/gpurun_out/smoke_r05z.log" 2>&1; echo "smoke rc=$?"; tail -2 "$R/gpurun_out/smoke_r05z.log"
timeout -k 10 400 python -u bench.py > "$R/gpurun_out/bench_r05z.json" 2> "$R/gpurun_out/bench_r05z.err"
echo "bench rc=$?"; head -c 600 "$R/gpurun_out/bench_r05z.json"
