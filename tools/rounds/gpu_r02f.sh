# Round-2 closing GPU run with 16 hardware queues and 12 batches in flight: bench lines C3 (default),
# C1 surrogate, C1 on the reference's images, C5, the rocprofv3 kernel trace + stats of the default
# bench (prof_bench.sh, with the HIP-event cross-check) and the reference-data run.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02f
for C in c3 c1 c1img c5; do
  timeout -k 10 300 python -u bench.py --config $C > gpurun_out/r02f/bench_$C.log 2>&1 || { echo "bench $C rc=$?"; exit 1; }
  echo "bench $C ok"; tail -n 1 gpurun_out/r02f/bench_$C.log | cut -c 1-300
done
timeout -k 10 200 python -u bench.py --config c1img --inflight 1 --cpu-sample 0 > gpurun_out/r02f/bench_c1img_i1.log 2>&1 || { echo "bench c1img i1 failed"; exit 1; }
tail -n 1 gpurun_out/r02f/bench_c1img_i1.log | cut -c 1-300
bash tools/prof_bench.sh || { echo "prof_bench failed"; exit 1; }
echo prof-done
timeout -k 10 200 python -u tools/run_dataset.py > gpurun_out/r02f/dataset_run.json 2>gpurun_out/r02f/dataset_run.err || { echo "dataset failed"; exit 1; }
echo all-done
