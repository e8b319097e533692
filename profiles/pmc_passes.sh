#!/bin/bash
# PMC diagnostic passes (one counter group per rocprofv3 run, MI355X_MICROARCH.md §rocprofv3).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${1:-$R/gpurun_out/pmc}
ARGS=${BENCH_ARGS:-"--steps 6 --warmup 2 --no-cpu-baseline --developed-presteps 0"}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM_RD" \
  "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum" \
  "SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1
done
echo pmc-done
