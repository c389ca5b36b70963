/*
 * spg_oracle.c -- CPU restatement of the reference snp-pattern-gen
 * (candidate k-mer counting over a genome).
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/ and the spg CPU-baseline leg of tools/spg_bench.py may run
 *   anything built from this file, and only as the CHECKER.  The product
 *   (libvafc.so, the HIP snp-pattern-gen CLI) never links it.
 *
 * Parity pinning: checked byte-for-byte (output file, stderr, exit code)
 * against the real reference binary oracle/_ref/snp-pattern-gen, compiled
 * from /root/reference/snp-pattern-gen.c by oracle/Makefile, on the fixtures
 * of tests/golden/spg/ (tests/golden/make_golden_spg.py).
 *
 * A literal, scalar statement of the reference program:
 *
 *   genome            kseq_read loop, name + sequence   snp-pattern-gen.c:67-103
 *   chromosome lookup first name match                  snp-pattern-gen.c:118-126
 *   key encoding      seq_nt4_table, canonical          snp-pattern-gen.c:129-157
 *   SNP k-mers        k/2 flank, N check, alt at centre snp-pattern-gen.c:192-217
 *   candidates        BED pass 1, ref + alt keys        snp-pattern-gen.c:259-296
 *   genome counting   rolling canonical k-mers, +1 on   snp-pattern-gen.c:159-190
 *                     candidate keys (u32)
 *   selection/output  ref count 1, alt count 0          snp-pattern-gen.c:306-355
 *
 * It reuses the kseq reader, the nt4 table and the open-addressing key table
 * of vafc_oracle.c (included below, without its main).
 */
#include "vafc_oracle.c"

typedef struct {
	char *name;
	char *seq;
	int len;
} sseq_t;

typedef struct {
	int n, m;
	sseq_t *a;
} sgenome_t;

/* load_fasta: every record until kseq_read < 0; the sequence is kept as a C
 * string (strdup in the reference: a NUL byte would end it early, but len
 * stays kseq's length) */
static sgenome_t *sg_load(const char *fn)
{
	oreader_t r;
	sgenome_t *g;
	if (rd_open(&r, fn) != 0) return 0;
	g = (sgenome_t*)calloc(1, sizeof(*g));
	while (rd_record(&r) >= 0) {
		if (g->n == g->m) {
			g->m = g->m ? g->m << 1 : 16;
			g->a = (sseq_t*)realloc(g->a, g->m * sizeof(sseq_t));
		}
		g->a[g->n].name = (char*)malloc(r.name.l + 1);
		memcpy(g->a[g->n].name, r.name.s ? r.name.s : "", r.name.l);
		g->a[g->n].name[r.name.l] = 0;
		g->a[g->n].seq = (char*)malloc(r.seq.l + 1);
		if (r.seq.l) memcpy(g->a[g->n].seq, r.seq.s, r.seq.l);
		g->a[g->n].seq[r.seq.l] = 0;
		g->a[g->n].len = (int)r.seq.l;
		++g->n;
	}
	rd_close(&r);
	return g;
}

static sseq_t *sg_find(sgenome_t *g, const char *chr)
{
	int i;
	for (i = 0; i < g->n; ++i)
		if (strcmp(g->a[i].name, chr) == 0) return &g->a[i];
	return 0;
}

static uint64_t sg_encode(const char *s, int k)
{
	int i;
	uint64_t x = 0;
	for (i = 0; i < k; ++i) {
		int c = g_nt4[(unsigned char)s[i]];
		if (c >= 4) return UINT64_MAX;
		x = (x << 2) | (uint64_t)c;
	}
	return x;
}

static int sg_snp_kmers(sseq_t *s, int pos, char alt, int k, char *ref_kmer, char *alt_kmer)
{
	int flank = k / 2, start = pos - flank, i;
	if (start < 0 || start + k > s->len) return 0;
	for (i = 0; i < k; ++i)
		if (g_nt4[(unsigned char)s->seq[start + i]] >= 4) return 0;
	memcpy(ref_kmer, s->seq + start, k);
	ref_kmer[k] = 0;
	memcpy(alt_kmer, s->seq + start, k);
	alt_kmer[flank] = alt;
	alt_kmer[k] = 0;
	return 1;
}

/* candidate table: key -> slot in cnt[] */
typedef struct {
	otable_t *t;
	uint32_t *cnt;
	uint32_t n, m;
} scand_t;

static void sc_put(scand_t *c, uint64_t key, int *n_candidate)
{
	uint32_t v;
	if (otable_get(c->t, key, &v)) return;
	if (c->n == c->m) {
		c->m = c->m ? c->m << 1 : 1024;
		c->cnt = (uint32_t*)realloc(c->cnt, c->m * sizeof(uint32_t));
	}
	otable_put(c->t, key, c->n);
	c->cnt[c->n++] = 0;
	++*n_candidate;
}

/* count_candidate_kmers (snp-pattern-gen.c:159-190) */
static void sg_count(sgenome_t *g, int k, scand_t *c)
{
	int i, j, l;
	uint64_t x0, x1, mask = (1ULL << k * 2) - 1, shift = (uint64_t)(k - 1) * 2;
	for (i = 0; i < g->n; ++i) {
		const char *seq = g->a[i].seq;
		int len = g->a[i].len;
		for (j = l = 0, x0 = x1 = 0; j < len; ++j) {
			int b = g_nt4[(unsigned char)seq[j]];
			if (b < 4) {
				x0 = (x0 << 2 | (uint64_t)b) & mask;
				x1 = x1 >> 2 | (uint64_t)(3 - b) << shift;
				if (++l >= k) {
					uint64_t y = x0 < x1 ? x0 : x1;
					uint32_t v;
					if (otable_get(c->t, y, &v)) ++c->cnt[v];
				}
			} else {
				l = 0;
				x0 = x1 = 0;
			}
		}
	}
}

typedef struct {
	char chr[256];
	int start, end;
	char rsid[256];
	char ref, alt;
} ssnp_t;

#define SG_SCAN(fp, s) fscanf(fp, "%254s%d%d%254s %c %c", (s).chr, &(s).start, &(s).end, (s).rsid, &(s).ref, &(s).alt)

int main(int argc, char *argv[])
{
	int c, k = 21, n_total = 0, n_unique = 0, n_candidate = 0;
	char *bed_fn = 0, *fasta_fn = 0, *out_fn = 0;
	char ref_kmer[128], alt_kmer[128];
	FILE *bed_fp, *out_fp;
	sgenome_t *g;
	scand_t cand = {0, 0, 0, 0};
	ssnp_t snp;

	opterr = 0;
	while ((c = getopt(argc, argv, "k:b:f:o:")) >= 0) {
		if (c == 'k') k = atoi(optarg);
		else if (c == 'b') bed_fn = optarg;
		else if (c == 'f') fasta_fn = optarg;
		else if (c == 'o') out_fn = optarg;
	}
	if (k % 2 == 0) {
		fprintf(stderr, "Error: k must be odd\n");
		return 1;
	}
	if (!bed_fn || !fasta_fn || !out_fn) {
		fprintf(stderr, "Usage: snp-pattern-gen -k %d -b <snps.bed> -f <ref.fa> -o <patterns.txt>\n", k);
		fprintf(stderr, "Options:\n");
		fprintf(stderr, "  -k INT    k-mer length (must be odd) [%d]\n", k);
		fprintf(stderr, "  -b FILE   input BED file with SNPs\n");
		fprintf(stderr, "  -f FILE   input reference genome FASTA file\n");
		fprintf(stderr, "  -o FILE   output pattern file\n");
		return 1;
	}
	init_tables();
	fprintf(stderr, "[M::%s] Loading reference genome...\n", "main");
	g = sg_load(fasta_fn);
	if (!g) {
		fprintf(stderr, "Error: failed to load FASTA file\n");
		return 1;
	}
	fprintf(stderr, "[M::%s] Loaded %d sequences\n", "main", g->n);
	fprintf(stderr, "[M::%s] Generating candidate k-mers from BED file...\n", "main");
	bed_fp = fopen(bed_fn, "r");
	if (!bed_fp) {
		fprintf(stderr, "Error: failed to open BED file\n");
		return 1;
	}
	{   /* the oracle's key table does not grow: size it for two keys per row */
		int rows = 0;
		while (SG_SCAN(bed_fp, snp) == 6) ++rows;
		rewind(bed_fp);
		cand.t = otable_new(2 * (uint64_t)rows + 16);
	}
	while (SG_SCAN(bed_fp, snp) == 6) {
		sseq_t *s = sg_find(g, snp.chr);
		if (!s) continue;
		if (sg_snp_kmers(s, snp.start, snp.alt, k, ref_kmer, alt_kmer)) {
			uint64_t re = sg_encode(ref_kmer, k), ae = sg_encode(alt_kmer, k);
			if (re == UINT64_MAX || ae == UINT64_MAX) continue;
			sc_put(&cand, canonical_of(re, k), &n_candidate);
			sc_put(&cand, canonical_of(ae, k), &n_candidate);
		}
	}
	fclose(bed_fp);
	fprintf(stderr, "[M::%s] Generated %d candidate k-mers\n", "main", n_candidate);
	fprintf(stderr, "[M::%s] Counting candidate k-mers in genome...\n", "main");
	sg_count(g, k, &cand);
	fprintf(stderr, "[M::%s] Finished counting k-mers\n", "main");
	bed_fp = fopen(bed_fn, "r");
	if (!bed_fp) {
		fprintf(stderr, "Error: failed to open BED file\n");
		return 1;
	}
	out_fp = fopen(out_fn, "w");
	if (!out_fp) {
		fprintf(stderr, "Error: failed to open output file\n");
		return 1;
	}
	fprintf(stderr, "[M::%s] Processing SNPs...\n", "main");
	while (SG_SCAN(bed_fp, snp) == 6) {
		sseq_t *s = sg_find(g, snp.chr);
		++n_total;
		if (!s) {
			fprintf(stderr, "Warning: chromosome %s not found\n", snp.chr);
			continue;
		}
		if (sg_snp_kmers(s, snp.start, snp.alt, k, ref_kmer, alt_kmer)) {
			uint64_t re = sg_encode(ref_kmer, k), ae = sg_encode(alt_kmer, k);
			uint32_t rv, av;
			if (re == UINT64_MAX || ae == UINT64_MAX) continue;
			if (otable_get(cand.t, canonical_of(re, k), &rv) && cand.cnt[rv] == 1 &&
			    otable_get(cand.t, canonical_of(ae, k), &av) && cand.cnt[av] == 0) {
				fprintf(out_fp, "%s\t%d\t%d\t%s\t%c\t%c\t%s\t%s\n", snp.chr, snp.start, snp.end, snp.rsid,
				        snp.ref, snp.alt, ref_kmer, alt_kmer);
				++n_unique;
			}
		}
	}
	fprintf(stderr, "[M::%s] Total SNPs: %d, Unique k-mer pairs: %d\n", "main", n_total, n_unique);
	fclose(bed_fp);
	fclose(out_fp);
	return 0;
}
