#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/mdbcprof
export TMPDIR=/tmp
mkdir -p $OUT
A="--boundary mdbc --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/bench.py $A > $OUT/kt.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py $A > $OUT/p1.log 2>&1
echo done
