# round 5, first pass: the whole -m gpu suite (sweep lines into $OUT/sweep.jsonl), then the
# default bench line
set -o pipefail
OUT=${OUT:-gpurun_out/r05a}
mkdir -p $OUT
WRNN_SWEEP_OUT=$OUT/sweep.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -3
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
brc=$?
tail -c 3000 $OUT/bench.log
echo "bench rc=$brc"
exit $rc
