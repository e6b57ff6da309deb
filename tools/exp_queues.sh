# same-box sweep: --hw-queues x --inflight (C3, no CPU baseline), two repeats of the current default
set -e
mkdir -p gpurun_out
run() {
  echo "$*" >> gpurun_out/exp5.log
  timeout -k 10 120 python -u bench.py --cpu-sample 0 "$@" 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/exp5.log
}
run --hw-queues 16 --inflight 12
run --hw-queues 24 --inflight 16
run --hw-queues 24 --inflight 20
run --hw-queues 32 --inflight 24
run --hw-queues 16 --inflight 12 --steps 40
run --hw-queues 24 --inflight 16 --steps 40
run --hw-queues 16 --inflight 12
