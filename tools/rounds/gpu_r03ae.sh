# Round 3ae: closing bench lines on the final tree (c4 default, c3, c5, c1img).  -> gpurun_out/r03ae/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 > $O/bench_c5.log 2>&1
timeout -k 10 400 python -u bench.py --config c1img > $O/bench_c1img.log 2>&1
for f in c4 c3 c5 c1img; do tail -1 $O/bench_$f.log | cut -c1-200; done
