#!/bin/bash
# Round 5: 4 waves/SIMD for every k_fluid_tiled + grids of resident blocks only; bench cfg2 / cfg3,
# the launch-tail diagnostic, the 8-slab full-step turns, the parity tests of the tiled kernel.
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/b14_cfg2.json 2> gpurun_out/b14_cfg2.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/b14_cfg2.json').read().strip().splitlines()[-1]);print('cfg2',d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/b14_cfg3.json 2> gpurun_out/b14_cfg3.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/b14_cfg3.json').read().strip().splitlines()[-1]);print('cfg3',d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 10 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/b14_cfg5.json 2> gpurun_out/b14_cfg5.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/b14_cfg5.json').read().strip().splitlines()[-1]);print('cfg5',d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
L=$(pwd)/scratch/tail/libsphcore.so
SPH_LIB=$L timeout -k 10 200 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail3_cfg2.json 2> gpurun_out/tail3_cfg2.err || exit $?
grep TAIL gpurun_out/tail3_cfg2.err | tail -4
SPH_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg3 --steps 6 --warmup 2 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail3_cfg3.json 2> gpurun_out/tail3_cfg3.err || exit $?
grep TAIL gpurun_out/tail3_cfg3.err | tail -4
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --slabs 8 --repeat 1 --steps 6 --modes inplace > gpurun_out/turns8_r05l.log 2>&1 || exit $?
grep -o '"summary_min_over_repeats".*' gpurun_out/turns8_r05l.log | cut -c1-900
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize.py tests/test_nn.py tests/test_gpu_items.py tests/test_ext.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_r05l.log 2>&1
echo "parity rc=$?"; tail -3 gpurun_out/parity_r05l.log
