#!/bin/bash
# Piece-size A/B of the in-process file pass at several file sizes (the
# per-rank share of an N-GPU pass): bench.py --reads R with VAFC_INGEST_PIECE
# set, alternating, two rounds.   tools/piece_ab.sh TAG "READS..." "PIECES..."
set -o pipefail
TAG=${1:?tag}
READS=${2:-12500000}
PIECES=${3:-"16777216 33554432"}
mkdir -p gpurun_out
for r in 1 2; do
for n in $READS; do
for p in $PIECES; do
  o=gpurun_out/${TAG}_${n}_${p}_$r
  VAFC_INGEST_PIECE=$p timeout -k 10 400 python bench.py --reads $n --no-cli --no-cpu --no-parity --steps 8 --warmup 2 \
    --kernel-steps 2 > $o.json 2> $o.err || exit 1
  python3 -c "
import json
d=json.loads(open('$o.json').read().strip().splitlines()[-1])
print('reads $n piece $p round $r', d['value'], d['e2e']['step_ms'])"
done
done
done
