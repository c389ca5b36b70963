#!/usr/bin/env python3
"""Reference-side binding test infrastructure: applies the
documented patch to the reference's own main() in memory and compiles the
result against libvafc.so.

    python oracle/bind_reference.py [--ref /root/reference] [--out oracle/_ref/vaf-counter-vafc]

The reference source is read from where it lies and the patched text is
written only to a temporary directory; the one output is the binary (under
oracle/_ref/, git-ignored like the other reference builds).  The patch keeps
the reference's loader, its khashl map and its writer, and replaces only the
counting seam (count_fastq_kmers, vaf-counter.c:550/647-650): the map's
(key, value) pairs are uploaded to the device (vc_create), each input file is
counted by vc_count_file, and the device counts are copied back into the
reference's pattern_t counters before its writer runs (vaf-counter.c:653-681).

Each edit is (anchor line in vaf-counter.c, code inserted before/after it or
replacing it); the anchors are single statements of the reference's main()
(vaf-counter.c:633, 649, 651, 734).  Exits 1 if an anchor is not found.
"""
import argparse
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

HEADER = '#include "vafc.h"   /* libvafc.so: the MI355X counting seam */\n'

# vaf-counter.c:633 -- after the reference builds its map, upload it
AFTER_MAP = r'''
	/* [vafc] the reference's own map (first insert already won) becomes the
	 * device table: its (key, value) pairs, value = (i << 1) | is_alt */
	vc_ctx *vctx = NULL;
	if (kmer_map) {
		khint_t it, nk = 0;
		uint64_t *vkeys = (uint64_t*)malloc((kh_size(kmer_map) + 1) * sizeof(uint64_t));
		uint32_t *vvals = (uint32_t*)malloc((kh_size(kmer_map) + 1) * sizeof(uint32_t));
		const char *vdev = getenv("VAFC_DEVICE");
		for (it = 0; it < kh_end(kmer_map); ++it)
			if (kh_exist(kmer_map, it)) vkeys[nk] = kh_key(kmer_map, it), vvals[nk++] = kh_val(kmer_map, it);
		if (vc_create(&vctx, k, vkeys, vvals, nk, (uint32_t)db->n, vdev ? atoi(vdev) : 0) != VC_OK) {
			fprintf(stderr, "Error: failed to create k-mer map\n");
			return 1;
		}
		free(vkeys); free(vvals);
	}
'''

# vaf-counter.c:649 -- the per-file call
COUNT_CALL = r'''		{   /* [vafc] count_fastq_kmers on the GPU; an unopenable file is skipped, as :557 */
			vc_file_stats vst;
			if (vc_count_file(vctx, argv[i], block_size, n_thread, &vst) == VC_OK) {
				g_perf_stats.total_bases_processed += vst.bases;
				g_perf_stats.total_sequences_processed += vst.seqs;
			}
		}
'''

# vaf-counter.c:651 -- before the counting timer stops: counts back into pattern_t
BEFORE_TIMER = r'''	{   /* [vafc] device counts -> the reference's counters; its writer runs unchanged */
		uint32_t *vcnt = (uint32_t*)calloc(2 * (size_t)db->n + 2, sizeof(uint32_t));
		uint64_t vkm = 0;
		if (vc_finish(vctx, vcnt, &vkm) != VC_OK) {
			fprintf(stderr, "Error: counting failed\n");
			return 1;
		}
		for (i = 0; i < db->n; ++i) db->a[i].ref_count = vcnt[2 * i], db->a[i].alt_count = vcnt[2 * i + 1];
		g_perf_stats.total_kmers_extracted = vkm;
		free(vcnt);
	}
'''

# vaf-counter.c:734
AFTER_DESTROY = '\tvc_destroy(vctx);\n'

EDITS = [
    ("\tkmer_map = create_combined_kmer_map(db, k);\n", "after", AFTER_MAP),
    ("\t\tcount_fastq_kmers(argv[i], k, n_thread, block_size, kmer_map, db);\n", "replace", COUNT_CALL),
    ("\tg_perf_stats.time_kmer_counting = get_time() - t_end;\n", "before", BEFORE_TIMER),
    ("\tkmer_cnt_destroy(kmer_map);\n", "after", AFTER_DESTROY),
]


def patch(text):
    out = HEADER + text
    for anchor, how, code in EDITS:
        if out.count(anchor) != 1:
            raise SystemExit("bind_reference: anchor not found exactly once: %r" % anchor)
        new = {"after": anchor + code, "before": code + anchor, "replace": code}[how]
        out = out.replace(anchor, new)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "_ref", "vaf-counter-vafc"))
    ap.add_argument("--cc", default=os.environ.get("CC", "gcc"))
    a = ap.parse_args()
    src = os.path.join(a.ref, "vaf-counter.c")
    lib = os.path.join(ROOT, "kmer-cnt_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libvafc.so")):
        sys.exit("bind_reference: build libvafc.so first (make -C kmer-cnt_amd/csrc)")
    with open(src) as f:
        text = patch(f.read())
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "vaf-counter-vafc.c")
        with open(p, "w") as f:
            f.write(text)
        rpath = os.path.relpath(lib, os.path.dirname(os.path.abspath(a.out)))
        # the reference's own flags (Makefile:44) plus the include path and libvafc.so
        cmd = [a.cc, "-g", "-Wall", "-O2", "-mssse3", "-msse4.1", "-I" + a.ref, "-I" + os.path.join(ROOT, "include"),
               "-o", a.out, p, os.path.join(a.ref, "kthread.c"), "-L" + lib, "-lvafc",
               "-Wl,-rpath,$ORIGIN/" + rpath, "-lz", "-lpthread"]
        subprocess.run(cmd, check=True)


if __name__ == "__main__":
    main()
