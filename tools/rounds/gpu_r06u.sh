# Round 6 u: the sampler grids' floor (MIM_SAMPLER_MIN_BLOCKS, default 4096 blocks in all) on the 8-GPU
# shard (bench.py --shard-of 8, 32 problems per step, batches in flight), interleaved, two rounds
# -> profiles/r06u_sampler_min_blocks_ab.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
show() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["roofline"]["kernel_ms_per_step_isolated"]; print(d["value"], d["ms_per_step"], "attempt", k.get("attempt"), "check", k.get("check"))'; }
for i in 1 2; do
  for mb in 4096 0 1024; do
    MIM_SAMPLER_MIN_BLOCKS=$mb timeout -k 10 300 python -u bench.py --shard-of 8 --cpu-sample 0 > $O/shard_mb${mb}_$i.log 2>&1
    echo "mb=$mb run $i: $(show $O/shard_mb${mb}_$i.log)" | tee -a $O/summary.txt
  done
done
