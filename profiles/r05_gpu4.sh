#!/bin/bash
# Round 5: the mDBC slab face diagnostics, the full GPU suite, the default bench.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "tests/test_mdbc.py::test_gpu_mdbc_on_slabs_matches_reference" -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/mdbcdiag.log 2>&1
echo "diag rc=$?"; grep -E "SphError|passed|failed" gpurun_out/mdbcdiag.log | head -8
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r05e.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/gputest_r05e.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r05e.json 2> gpurun_out/bench_r05e.err
echo "bench rc=$?"; cat gpurun_out/bench_r05e.json | head -c 1500
