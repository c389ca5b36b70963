#!/bin/bash
# Host sanitizer run (the reference's `make asan=1`,
# Makefile:10-13): libvafc.so rebuilt with AddressSanitizer + UBSan on all host
# code (kmer-cnt_amd/lib_asan), then the CPU tests of the untrusted-input
# parsers -- the gzip inflater, the FASTA/FASTQ readers, the parallel ingest,
# the .vaf loader -- run against it.  Any report aborts the run.
#   tools/asan_tests.sh [pytest args...]     (CPU only; no GPU needed)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -j8 -C "$ROOT/kmer-cnt_amd/csrc" asan=1 ../lib_asan/libvafc.so ../lib_asan/vaf-counter
make -s -j8 -C "$ROOT/oracle"
RT=$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
cd "$ROOT"
env LD_PRELOAD="$RT" \
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    VAFC_LIB="$ROOT/kmer-cnt_amd/lib_asan/libvafc.so" VAFC_NO_TORCH=1 VAFC_SKIP_BUILD=1 \
    python -m pytest tests/test_gzip.py tests/test_reader.py tests/test_ingest_parallel.py tests/test_corr.py \
        tests/test_abi.py -m "not gpu" -q -p no:cacheprovider "$@"
