#!/bin/bash
# Round 4: two-rank rehearsal of the N > 1 bench path on one GPU (gloo for the
# collectives: both ranks share device 0), with a short e2e leg over two shards.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
VAFC_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --e2e-reads 20000000 > $O/r04w_dist2.json 2> $O/r04w_dist2.err || { echo DIST2_FAILED; tail -30 $O/r04w_dist2.err; exit 1; }
cut -c1-600 $O/r04w_dist2.json
