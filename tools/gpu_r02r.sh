#!/bin/bash
# Round-2 re-entry pass: the end-of-session check (parity tests, smoke, bench,
# stream bench + stats), then the multi-rank launch paths on the one GPU:
#  - torch.distributed.run at one rank: the RCCL group, barrier, all-reduce
#    and all-gather around the HIP modem;
#  - bench.py --gpus 2 --backend gloo: the self-launcher with two ranks
#    sharing the card (weak scaling, n_gpus 2).
export TMPDIR=/tmp
bash tools/final_check.sh || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
    --master-port=29511 bench.py --gpus 1 --no-cpu-baseline > gpurun_out/bench_rccl1.json 2> gpurun_out/bench_rccl1.err || exit 1
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --no-cpu-baseline > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || exit 1
