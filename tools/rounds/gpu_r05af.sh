# Round 5af: the exact kernel's register footprint (its waves hold their VGPRs for a Jacobi's duration
# while the distance kernel needs whole VGPR files, r05ad): launch bounds sized for 4 waves per SIMD (116
# VGPRs, no spill) and 6 (80 VGPRs, 140 B of spills) against the default (134): RANSAC GPU tests on the
# 6-wave build, then C4 and C3 lines and isolated exact time, two interleaved rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05af
mkdir -p $O
MIM_LIB=$PWD/variants/libmim_eocc6.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ransac or filtered or bound or configs or c3_full" > $O/pytest_eocc6.log 2>&1 || { tail -30 $O/pytest_eocc6.log; exit 1; }
tail -1 $O/pytest_eocc6.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "exact", r["exact"], "score", r["score"])'; }
for i in 1 2; do
  for v in base eocc4 eocc6; do
    if [ $v = base ]; then unset MIM_LIB; else export MIM_LIB=$PWD/variants/libmim_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --parity-sample 2 --iso-steps 2 > $O/c4_${v}_$i.log 2>&1; echo "c4 $v $(show $O/c4_${v}_$i.log)"
    timeout -k 10 300 python -u bench.py --config c3 --cpu-sample 0 --parity-sample 2 --iso-steps 2 > $O/c3_${v}_$i.log 2>&1; echo "c3 $v $(show $O/c3_${v}_$i.log)"
  done
done
