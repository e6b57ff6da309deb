# same-box A/B: hardware queues x batches in flight x HIP-event timing (C3 and C1 surrogate)
set -e
mkdir -p gpurun_out
run() {
  echo "$*" >> gpurun_out/exp4.log
  timeout -k 10 120 env GPU_MAX_HW_QUEUES=$Q python -u bench.py --cpu-sample 0 "$@" 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/exp4.log
}
for rep in 1 2; do
Q=4 run --inflight 3
Q=16 run --inflight 3
Q=16 run --inflight 12
Q=4 run --inflight 3 --no-timing
Q=16 run --inflight 12 --no-timing
Q=16 run --inflight 3 --no-timing
done
Q=4 run --inflight 3 --config c1
Q=16 run --inflight 3 --config c1
Q=16 run --inflight 2 --config c1
