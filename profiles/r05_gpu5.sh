#!/bin/bash
# Round 5: the mDBC slab face diagnostics (every slab's face sizes and counts).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "tests/test_mdbc.py::test_gpu_mdbc_on_slabs_matches_reference" "tests/test_2d.py::test_gpu_mdbc_2d_slabs_match_reference" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/mdbcdiag.log 2>&1
echo "diag rc=$?"; grep -E "SphError|passed|failed" gpurun_out/mdbcdiag.log | head -8
