#!/bin/bash
# ThreadSanitizer run of the host readers (host code only, no GPU; the round-6
# held shares resume a decoder whose threads outlive the scan):
#   tools/tsan_gz.cpp     the parallel inflater (vafc_gzip.cpp): whole stream,
#                         two-pass and held shares of five gzip shapes vs zlib;
#   tools/tsan_ingest.cpp the parallel FASTQ reader over them (vafc_ingest.cpp):
#                         the plain file whole and in byte ranges, the gzip file
#                         in two-pass and held shares, vs the sequential reader.
# Any report fails the run.
#   tools/tsan_gz.sh [threads] [chunk_bytes]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=${1:-4}
CH=${2:-16384}
mkdir -p "$ROOT/tools/bin"
BIN=$ROOT/tools/bin/tsan_gz
CS=$ROOT/kmer-cnt_amd/csrc
TS="-std=c++17 -O1 -g -fsanitize=thread -fno-omit-frame-pointer -pthread -I$ROOT/include -I$CS"
g++ $TS "$ROOT/tools/tsan_gz.cpp" "$CS/vafc_gzip.cpp" -lz -o "$BIN"
g++ $TS "$ROOT/tools/tsan_ingest.cpp" "$CS/vafc_ingest.cpp" "$CS/vafc_gzip.cpp" "$CS/vafc_fastq.cpp" -lz \
    -o "$ROOT/tools/bin/tsan_ingest"
D=$(mktemp -d)
trap 'rm -rf "$D"' EXIT
python3 - "$D" <<'PY'
import os, random, struct, sys, zlib
d = sys.argv[1]
rng = random.Random(5)
recs = []
for i in range(12000):
    s = "".join(rng.choice("ACGT") for _ in range(150))
    q = "".join(rng.choice("FGHI#") for _ in range(150))
    recs.append("@r%d\n%s\n+\n%s\n" % (i, s, q))
text = "".join(recs).encode()

def member(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    body = c.compress(data) + c.flush()
    return b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03" + body + struct.pack("<II", zlib.crc32(data), len(data))

c = zlib.compressobj(1, zlib.DEFLATED, -15)
pig = b"".join(c.compress(text[a:a + 60000]) + c.flush(zlib.Z_SYNC_FLUSH) for a in range(0, len(text), 60000)) + c.flush()
cut = [0, len(text) // 3 + 11, 2 * len(text) // 3 + 5, len(text)]
shapes = {
    "one": member(text, 1),
    "six": member(text, 6),
    "pigz": b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x04\x03" + pig + struct.pack("<II", zlib.crc32(text), len(text)),
    "multi": b"".join(member(text[a:b], 1) for a, b in zip(cut, cut[1:])),
    "fixed": member(text, 1, zlib.Z_FIXED),
}
for k, v in shapes.items():
    open(os.path.join(d, k + ".fq.gz"), "wb").write(v)
open(os.path.join(d, "t.fq"), "wb").write(text)
PY
export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1"
for f in one six pigz multi fixed; do
  for w in 2 3; do
    "$BIN" "$D/$f.fq.gz" "$T" "$CH" "$w"
  done
done
for f in one pigz multi; do
  VAFC_INGEST_PIECE=65536 VAFC_GZ_CHUNK=16384 "$ROOT/tools/bin/tsan_ingest" "$D/t.fq" "$D/$f.fq.gz" "$T" 3
done
echo "tsan_gz: all clean"
