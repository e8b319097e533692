for i in 1 2 3; do
  for m in 15 1; do
    SPH_TIMING_PHASES=$m timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-cfg3 > /tmp/b.json 2>/tmp/b.err || { cat /tmp/b.err; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('/tmp/b.json') if l.startswith('{')][-1])
print('mask $m  %.4f ms/step  inter %.4f  value %.4g' % (d['ms_per_step'], d['phase_ms_per_call']['interaction'], d['value']))"
  done
done
