#!/bin/bash
# Round 6: diagnose the 512 x 2 fused update (gpurun_var/u512) against the per-particle kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
SPH_LIB=$R/gpurun_var/u512/libsphcore.so timeout -k 10 300 python3 profiles/r06/dbg_upd512.py > gpurun_out/r06/dbg18.log 2>&1; rc=$?
cat gpurun_out/r06/dbg18.log | tail -20
exit $rc
