#!/bin/bash
# Round 5: slab / mDBC / body tests, then the three-mode turns measurement and a trace.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r05d.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|^E  " gpurun_out/gputest_r05d.log | sort | uniq -c | sort -rn | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export SPH_SLAB_TURNS=1
timeout -k 10 400 python -u profiles/slab_turns.py --repeat 2 > gpurun_out/turns_r05d.log 2>&1 || exit $?
tail -c 1200 gpurun_out/turns_r05d.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_turns2 -o run \
  -- python3 profiles/slab_turns.py --repeat 1 --only overlap --steps 4 --warmup 2 > gpurun_out/prof_turns2.log 2>&1
echo "rocprof rc=$?"
