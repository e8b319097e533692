export TMPDIR=/tmp; T=$1; shift
mkdir -p gpurun_out/$T && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/$T/log.txt 2>&1
