#!/usr/bin/env bash
# bench.py at world 2 with both ranks SHARING ONE GPU (JLA_SINGLE_DEVICE=1; gloo for the host-side collectives, the
# custom xGMI kernels for the tensor-parallel ones): the multi-GPU bench flow end to end -- the headline at a reduced
# layer count (marked -DEBUG in its config), then the tp_points phase (Llama-2-13B at MP 2, all layers) with the litmus
# result. Functional evidence for the driver's 8-GPU run, not a TP speed number. Output: gpurun_out/tp2/.
set -o pipefail
mkdir -p gpurun_out/tp2
export JLA_SINGLE_DEVICE=1 JLA_DIST_BACKEND=gloo
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --layers 4 --batch 256 --latency-batches 1 \
  --no-sampled --ttft-len 0 --no-calibration --tp-batches 1 32 256 ${EXTRA:-} \
  --json-out gpurun_out/tp2/bench_tp2.json > gpurun_out/tp2/bench_tp2.log 2>&1
rc=$?
tail -5 gpurun_out/tp2/bench_tp2.log
exit $rc
