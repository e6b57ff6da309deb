# Round 3ad: the dynamic distance schedule as the default for batches with >= one sweep per resident
# block: pytest -m gpu as the driver runs it, smoke, fresh C3 / C4 profiles (isolated traces + HBM
# counters).  -> gpurun_out/r03ad/, gpurun_out/prof_c3, prof_c4
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
set +e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
set -e
echo "pytest rc $rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit 1; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for C in c3 c4; do
  bash tools/prof_round.sh $C > $O/prof_$C.log 2>&1
  echo "prof $C done"
done
