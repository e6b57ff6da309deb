# r06b: (1) the GPU suite on the current tree (sampler flags bit-packed, several-GPU group);
# (1b) distance-kernel event/stagger variants (tools/knn_ab.py, C3 shape); (2) C4 bench A/B, two interleaved rounds: prev (HEAD before the bit-pack) / cur / bw8 (512-iteration
# bound blocks), isolated kernel times from the bench line; (3) the round profile of cur on C4 (kernel
# trace + HBM counters); (4) kernel trace of single c1img scenes (tools/scene_timeline.py).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
V=$PWD/computervision_objectdetection_featurematching_amd/lib/variants
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || rc=$?
tail -3 $O/pytest_gpu.log
# a fault, abort or time limit ends the call here; plain test failures do not stop the measurements
case $rc in 124|134|137|139) echo "pytest rc $rc: stopping"; exit 1;; esac
# distance kernel: keyed insertion events (ev), waves 4-7 staggered (stg), both; parity vs base
MIM_LIB=$V/libmim_base.so timeout -k 10 300 python3 -u tools/knn_ab.py --tag base --save --steps 10 > $O/ab_base_full.json 2> $O/ab_base_full.err
for v in ev stg evstg; do
  MIM_LIB=$V/libmim_$v.so timeout -k 10 300 python3 -u tools/knn_ab.py --tag $v --steps 10 > $O/ab_${v}_full.json 2> $O/ab_${v}_full.err
done
for i in 1 2; do
  for v in base ev stg evstg; do
    MIM_LIB=$V/libmim_$v.so timeout -k 10 200 python3 -u tools/knn_ab.py --tag $v --c3-only --steps 20 > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err
  done
done
for i in 1 2; do
  for v in prev cur bw8; do
    L=$V/libmim_$v.so
    [ $v = cur ] && L=$PWD/computervision_objectdetection_featurematching_amd/lib/libmim.so
    MIM_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 30 --cpu-sample 0 > $O/bench_${v}_$i.log 2>&1
    tail -1 $O/bench_${v}_$i.log | cut -c1-120
  done
done
timeout -k 10 900 bash tools/prof_round.sh c4 > $O/prof_round_c4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1img -o run -- \
  python3 bench.py --config c1img --inflight 1 --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 > $O/c1img_bench.log 2>&1 < /dev/null
python3 tools/scene_timeline.py $O/c1img/run_kernel_trace.csv 4 > $O/c1img_timeline.txt
echo done
