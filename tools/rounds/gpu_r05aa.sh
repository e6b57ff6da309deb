# Round 5aa: the SIFT descriptor kernel at 6 waves per SIMD (VGPRs capped at 80 with 56 B of spills;
# LDS 29 -> 22 KiB per block: histogram aliased onto the batch buffer, the per-word pixel ranks summed at
# the scatter, 16-bit row tables) against HEAD (4 waves: 105 VGPRs) and the new LDS layout at 4 waves
# (variants/libmim_occ4.so): SIFT / pipeline / dataset GPU tests first, then descriptor launch times and
# the c1img and dataset lines, two rounds.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sift or pipeline or dataset or c1" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("single_scene_ms"), d.get("sift_640x480_ms"))'; }
for i in 1 2; do
  for v in new prev occ4; do
    if [ $v = new ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --config c1img --cpu-sample 0 --parity-sample 0 > $O/c1img_${v}_$i.log 2>&1; echo "c1img $v $(show $O/c1img_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config dataset --cpu-sample 0 --parity-sample 0 > $O/dataset_${v}_$i.log 2>&1; echo "dataset $v $(show $O/dataset_${v}_$i.log)"
  done
done
for v in new prev occ4; do
  if [ $v = new ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$v -o run --output-format csv -- \
    python3 bench.py --config c1img --steps 3 --warmup 1 --iso-steps 3 --cpu-sample 0 --parity-sample 0 --inflight 1 > $O/tr_$v.log 2>&1 || true
  python3 -c "
import csv
d=sorted(((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3, int(r['Grid_Size_Y'])) for r in csv.DictReader(open('$O/tr_$v/run_kernel_trace.csv')) if 'descr_kernel' in r['Kernel_Name'])
b=[round(x) for x,y in d if y>1]; print('$v descr 5-scale launches (us):', b)
"
done
