#!/bin/bash
# Point-to-point microbenchmark sweep on one GPU (hosts/bandwidth_benchmark,
# hosts/latency_benchmark): ranks as host threads over the in-process
# transport, then two processes over RCCL launched by torchrun --no-python
# with --fake-host.  Every step under its own time limit; the first failure
# ends the script.  usage: tools/p2p_sweep.sh <out dir>
set -o pipefail
O=${1:-gpurun_out/p2p}
mkdir -p $O
B=hosts/_build
export HSA_ENABLE_IPC_MODE_LEGACY=0 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
step() {  # step <log name> <command...>
  local name=$1; shift
  timeout -k 10 120 "$@" > $O/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED $name rc=$rc"; tail -20 $O/$name.log; exit $rc; fi
  echo "== $name"; grep -E "Average|One-way|Conf interval 99:" $O/$name.log
}
for kb in 1 64 1024 16384 262144; do
  step bw_threads_bulk_$kb $B/bandwidth_benchmark -k $kb -r 1 -i 10 -p 2
done
step bw_threads_element_1024 $B/bandwidth_benchmark -k 1024 -r 1 -i 5 -p 2 -m element
step lat_threads_element $B/latency_benchmark -n 2000 -r 1 -i 10 -p 2
step lat_threads_bulk $B/latency_benchmark -n 2000 -r 1 -i 10 -p 2 -m bulk
port=$((29500 + RANDOM % 2000))
trstep() {  # trstep <log name> <host> <args...>: two processes under torchrun
  local name=$1; shift
  port=$((port + 1))
  step $name python -m torch.distributed.run --no-python --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port "$@" --fake-host
}
for kb in 1 64 1024 16384 262144; do
  trstep bw_procs_bulk_$kb $B/bandwidth_benchmark -k $kb -r 1 -i 10
done
trstep bw_procs_element_1024 $B/bandwidth_benchmark -k 1024 -r 1 -i 5 -m element
trstep lat_procs_element $B/latency_benchmark -n 500 -r 1 -i 5
trstep lat_procs_bulk $B/latency_benchmark -n 500 -r 1 -i 5 -m bulk
echo done
