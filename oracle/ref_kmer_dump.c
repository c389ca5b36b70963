/*
 * ref_kmer_dump.c -- TEST INFRASTRUCTURE ONLY (golden-vector generator).
 *
 * Compiles the reference's own vaf-counter.c (where it lies under
 * /root/reference, never copied) with its main() renamed, and exposes its
 * static extract_kmers_to_buf() (vaf-counter.c:349-427) so the per-read
 * canonical k-mer lists of the REAL reference can be dumped as fixtures.
 *
 * stdin : repeated records  <u32 len><len raw bytes>
 * stdout: repeated records  <u32 n><n x u64 canonical k-mers>
 * argv[1] = k
 * Output goes only to oracle/_ref/ (see oracle/Makefile).
 */
#define main vaf_counter_reference_main
#include VAF_REF_SRC
#undef main

int main(int argc, char *argv[])
{
	int k = argc > 1 ? atoi(argv[1]) : 21;
	uint32_t len;
	while (fread(&len, 4, 1, stdin) == 1) {
		char *s = (char*)malloc(len ? len : 1);
		kmer_buf_t buf = {0, 0, 0};
		uint32_t n;
		if (len && fread(s, 1, len, stdin) != len) { free(s); return 1; }
		extract_kmers_to_buf(&buf, k, (int)len, s);
		n = (uint32_t)buf.n;
		fwrite(&n, 4, 1, stdout);
		if (n) fwrite(buf.a, 8, n, stdout);
		free(buf.a);
		free(s);
	}
	return 0;
}
