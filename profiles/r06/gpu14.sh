#!/bin/bash
# Round 6: where the fused update's time goes — kernel stats of cfg2 with the fused update and
# with the separate launches (SPH_CLS_SPLIT=1), and the cfg3 8 y-slab turns trace with the
# separate launches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
for v in fused split; do
  e=""; [ $v = split ] && e="SPH_CLS_SPLIT=1"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r06/ks14_$v" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > "$R/gpurun_out/r06/ks14_$v.log" 2>&1 || exit $?
  f=$(find gpurun_out/r06/ks14_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/r06/ks14_${v}_stats.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if any(k in n for k in ('k_update','k_inc_classify','k_inc_push','k_inc_boxes','k_items_place','k_dt','k_pack')):
        print('$v', n.split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
  rm -rf gpurun_out/r06/ks14_$v
done
SPH_CLS_SPLIT=1 SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y14" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y14.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y14 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y14_breakdown.json | tail -8
rm -rf gpurun_out/r06/trace_y14
# the fused update's block shape: the previous commit's library (base: 1024 threads, dcell /
# code reloaded), this one (1024 threads, one load phase, registers), 512 threads x 2 particles
for v in gpurun_var/base main gpurun_var/u512; do
  lib=$R/$v/libsphcore.so; [ $v = main ] && lib=$R/dualsphysics_multilayer_amd/lib/libsphcore.so
  SPH_LIB=$lib SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 1 --modes inplace > gpurun_out/r06/turns14_$(basename $v).log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06/turns14_$(basename $v).log').read().strip().splitlines()[-1])['summary_min_over_repeats']['inplace']
print('$v', 'wall', d['wall_ms_per_step'], 'update', d['update_ms'], 'divide', d['divide_ms'], 'kern', d['slab_kernels_ms_per_step'])"
done
timeout -k 10 500 bash profiles/ab.sh 2 gpurun_var/base main gpurun_var/u512 -- --steps 40 --warmup 5 > gpurun_out/r06/ab14.log 2>&1 || exit $?
cat gpurun_out/r06/ab14.log
