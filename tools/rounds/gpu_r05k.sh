# Round 5k: the SIFT descriptor over the compacted patch (window rows only): SIFT, pipeline and dataset
# tests, then c1img (one scene alone and 12 in flight) and a kernel trace, A/B against HEAD's sift.hip.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 120 ./tools/issue_probe > $O/issue_probe.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_sift_gpu.py tests/test_sift_limits_gpu.py tests/test_pipeline_gpu.py tests/test_dataset_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "scene", d.get("single_scene_ms"), "sift", d.get("sift_640x480_ms"))'; }
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export MIM_LIB=$PWD/variants/libmim_prev.so; else unset MIM_LIB; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --config c1img > $O/c1img_${v}_$i.log 2>&1; echo "c1img $v $(show $O/c1img_${v}_$i.log)"
  done
done
unset MIM_LIB
timeout -k 10 600 bash tools/prof_round.sh c1img
grep -E "descr|blur|refine|small|exact" gpurun_out/prof_c1img/trace/*stats.csv | cut -c1-160 | head -8
