#!/bin/bash
# Rehearse the N-rank bench path on a one-GPU box: every rank on device 0,
# gloo instead of RCCL, the exchanged frames checked bit for bit against
# single-rank renders, for both scaling modes (weak: frame batch + all-to-all,
# strong: one frame + gather).  (The real N-GPU runs use --dist-backend nccl,
# one rank per GPU, and are launched by the driver.)
set -o pipefail
mkdir -p gpurun_out
for mode in weak strong; do
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 1 --warmup 0 --spp 16 --cpu-baseline 0 \
    --dist-backend gloo --verify-gather --scaling $mode > gpurun_out/rehearse_${mode}_$n.log 2>&1 || { echo "$mode N=$n FAILED"; tail -20 gpurun_out/rehearse_${mode}_$n.log; exit 1; }
  grep '"metric"' gpurun_out/rehearse_${mode}_$n.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["scaling"], "N=%d"%d["n_gpus"], d["value"], d["unit"], "verified:", d.get("gather_verified"), d["config"]["parallelism"], d["config"]["workload"])'
done
done
