#!/bin/bash
# Reader-thread A/B of the in-process file pass (C2, 100M reads): bench.py with
# VAFC_BENCH_THREADS set, alternating, two rounds.   tools/thread_ab.sh TAG "THREADS..."
set -o pipefail
TAG=${1:?tag}
TS=${2:-"8 12 16"}
mkdir -p gpurun_out
for r in 1 2; do
for t in $TS; do
  o=gpurun_out/${TAG}_t${t}_$r
  VAFC_BENCH_THREADS=$t timeout -k 10 400 python bench.py --no-cli --no-cpu --no-parity --steps 8 --warmup 2 \
    --kernel-steps 2 > $o.json 2> $o.err || exit 1
  python3 -c "
import json
d=json.loads(open('$o.json').read().strip().splitlines()[-1])
print('threads $t round $r', d['value'], d['e2e']['step_ms'])"
done
done
