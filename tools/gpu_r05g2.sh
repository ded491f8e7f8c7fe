set -u
export PYTHONUNBUFFERED=1
RATES="3.91,3.0 3.91,3.05 3.91,3.1 3.91,3.15 3.91,3.2" BENCH_ARGS="--model geneing-wavernn --mode BITS --bits 10" TAGS=.gen2 bash tools/rot_tune.sh
