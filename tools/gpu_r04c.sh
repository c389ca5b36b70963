#!/bin/bash
set -o pipefail
R=$(pwd); O=$R/gpurun_out
bash tools/abl_pmc.sh || exit 1
timeout -k 10 600 python tools/n8_projection.py --shards 8 --runs 3 > $O/r04c_n8.json 2> $O/r04c_n8.err || { echo N8_FAILED; tail -20 $O/r04c_n8.err; exit 1; }
cat $O/r04c_n8.json
