# rotation balance A/B + a rocprof kernel trace of the rotated C2 call
set -o pipefail
bash tools/rot_tune.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_c2r
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2r -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_c2r/bench.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof_c2r -name "*kernel_stats.csv" | head -3
