#!/bin/bash
# Alternating A/B of libsphcore variants on one box: profiles/ab.sh <rounds> <lib-or-"main"> ... -- [bench args]
# Prints one line per run: variant, ms/step, interaction ms (HIP events).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:?rounds}; shift
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" = "--" ] && shift
ARGS=${*:-"--steps 40 --warmup 5"}
for i in $(seq 1 $N); do
  for v in "${V[@]}"; do
    # "main:VAR=value" = the in-tree library with a test-hook environment variable
    envs=""; name=${v%%:*}; [ "$name" != "$v" ] && envs=${v#*:}
    if [ "$name" = main ]; then lib=$R/dualsphysics_multilayer_amd/lib/libsphcore.so; else lib=$R/$name/libsphcore.so; fi
    env $envs SPH_LIB=$lib timeout -k 10 200 python3 "$R/bench.py" $ARGS --no-cpu-baseline --no-cfg3 > /tmp/ab.json 2>/tmp/ab.err || { cat /tmp/ab.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('/tmp/ab.json') if l.startswith('{')][-1])
print('%-28s %8.4f ms/step  inter %8.4f ms  div %7.4f  frac %.4f' % ('$v', d['ms_per_step'], d['phase_ms_per_call']['interaction'], d['phase_ms_per_call']['divide'], d['roofline']['frac']))"
  done
done
