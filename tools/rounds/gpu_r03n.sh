# Round 3n: distance kernel with the four A fragments of a 32-row block read before its first MFMA
# (ld4: one LDS wait per block instead of three) vs default: isolated kernels + parity (knn_ab), C3
# pipelined line of each.  -> gpurun_out/r03n/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
V=computervision_objectdetection_featurematching_amd/lib/variants
timeout -k 10 240 python -u tools/knn_ab.py --tag default --save > $O/ab.log 2> $O/ab.err
MIM_LIB=$PWD/$V/libmim_ld4.so timeout -k 10 200 python -u tools/knn_ab.py --tag ld4 >> $O/ab.log 2>> $O/ab.err
timeout -k 10 200 python -u tools/knn_ab.py --tag default2 >> $O/ab.log 2>> $O/ab.err
MIM_LIB=$PWD/$V/libmim_ld4.so timeout -k 10 200 python -u tools/knn_ab.py --tag ld4b >> $O/ab.log 2>> $O/ab.err
cut -c1-200 $O/ab.log; grep -o '"parity": "[^"]*"' $O/ab.log | cut -c1-60
timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > $O/bench_c3.log 2>&1
tail -1 $O/bench_c3.log | cut -c1-150
MIM_LIB=$PWD/$V/libmim_ld4.so timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 > $O/bench_c3_ld4.log 2>&1
tail -1 $O/bench_c3_ld4.log | cut -c1-150
