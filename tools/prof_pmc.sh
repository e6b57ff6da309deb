# HBM traffic of the distance kernel (separate --pmc passes, MI355X_MICROARCH.md "HBM").
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv --kernel-include-regex 'knn2_bf16|ransac_score|ransac_hypo' \
     -d gpurun_out/pmc/$C -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-timing > gpurun_out/pmc/$C.log 2>&1
done
