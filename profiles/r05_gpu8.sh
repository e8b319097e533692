#!/bin/bash
# Round 5: the slab body tests after the floating-normal face fix.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bodies.py tests/test_mdbc.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/bodies_r05h.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/bodies_r05h.log | tail -20
exit $rc
