/*
 * corr_oracle.c -- CPU restatement of the reference correlation-matrix
 * (depth-aware Pearson between .vaf files + UPGMA).
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/ and the CPU-baseline leg of tools/corr_bench.py may run
 *   anything built from this file, and only as the CHECKER.  The product
 *   (libvafc.so, the HIP correlation-matrix CLI) never links it.
 *
 * Parity pinning: checked byte-for-byte (.corr, .tree, stderr, exit code)
 * against the real reference binary oracle/_ref/correlation-matrix, compiled
 * from /root/reference/correlation-matrix.c by oracle/Makefile, on the
 * fixtures of tests/golden/corr/ (tests/golden/make_golden_corr.py).
 *
 * What it restates, in the reference's order of operations (every double
 * operation separately rounded, no fused multiply-add -- the reference is
 * built for x86-64 without -mfma):
 *
 *   options        o:tm:d:M:, presets, usage text     correlation-matrix.c:268-316
 *   .vaf loader    fgets(4096) lines, '#'/"CHR" skip,   correlation-matrix.c:25-90
 *                  9-field sscanf, 100000-row cap,
 *                  name = basename cut at ".vaf"
 *   one pair       count valid rows, means, centred    correlation-matrix.c:94-143
 *                  sums, epsilon branch
 *   matrix         i < j with n = rows of sample i     correlation-matrix.c:146-162
 *   .corr writer   "%.6f" cells                        correlation-matrix.c:350-366
 *   tree           1 - r, first strict minimum,        correlation-matrix.c:190-257
 *                  average linkage, "%.4f" halves
 *
 * Rows of sample j past its own count are read as vaf 0.0, depth 0: the
 * reference reads its per-sample arrays (malloc'd 100000 entries, fresh
 * zero pages from mmap at that size) up to sample i's count.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <getopt.h>

#define CO_CAP 100000     /* correlation-matrix.c:8 MAX_SNPS */
#define CO_LINE 4096      /* correlation-matrix.c:9 MAX_LINE */

typedef struct {
	char name[256];
	double *x;            /* CO_CAP entries, zero past n */
	int *d;
	int n;
} co_sample;

/* correlation-matrix.c:25-90 */
static int co_load(const char *path, co_sample *s)
{
	FILE *f = fopen(path, "r");
	if (!f) return -1;
	const char *slash = strrchr(path, '/');
	snprintf(s->name, sizeof s->name, "%s", slash ? slash + 1 : path);
	char *cut = strstr(s->name, ".vaf");
	if (cut) *cut = 0;
	s->x = (double*)calloc(CO_CAP, sizeof(double));
	s->d = (int*)calloc(CO_CAP, sizeof(int));
	s->n = 0;
	char buf[CO_LINE];
	while (fgets(buf, sizeof buf, f)) {
		if (buf[0] == '#' || strncmp(buf, "CHR", 3) == 0) continue;
		char c1[256], c3[256], a1, a2;
		int pos, rc, ac, tot;
		double v;
		if (sscanf(buf, "%255s\t%d\t%255s\t%c\t%c\t%d\t%d\t%d\t%lf", c1, &pos, c3, &a1, &a2, &rc, &ac, &tot, &v) != 9)
			continue;
		if (s->n >= CO_CAP) {
			fprintf(stderr, "Warning: too many SNPs (max %d), truncating\n", CO_CAP);
			break;
		}
		s->x[s->n] = v;
		s->d[s->n] = tot;
		s->n++;
	}
	fclose(f);
	return 0;
}

/* correlation-matrix.c:94-143, three passes over rows [0, n) */
static double co_pair(const co_sample *a, const co_sample *b, int n, int min_snps, int min_depth)
{
	int cnt = 0;
	for (int i = 0; i < n; ++i) cnt += a->d[i] >= min_depth && b->d[i] >= min_depth;
	if (cnt < min_snps) return 0.0;
	double sa = 0, sb = 0;
	for (int i = 0; i < n; ++i)
		if (a->d[i] >= min_depth && b->d[i] >= min_depth) { sa += a->x[i]; sb += b->x[i]; }
	const double ma = sa / cnt, mb = sb / cnt;
	double sab = 0, saa = 0, sbb = 0;
	for (int i = 0; i < n; ++i) {
		if (!(a->d[i] >= min_depth && b->d[i] >= min_depth)) continue;
		const double u = a->x[i] - ma, w = b->x[i] - mb;
		const double uw = u * w, uu = u * u, ww = w * w;
		sab += uw;
		saa += uu;
		sbb += ww;
	}
	const double ra = sqrt(saa), rb = sqrt(sbb);
	if (ra < 1e-10 || rb < 1e-10) return sab / (sqrt(saa * sbb) + 0.00001);
	return sab / (ra * rb);
}

/* correlation-matrix.c:190-257 */
static void co_tree(const co_sample *s, int n, double *const *r, FILE *fp)
{
	double *dist = (double*)malloc((size_t)n * n * sizeof(double));
	char *on = (char*)malloc(n);
	for (int i = 0; i < n; ++i) {
		on[i] = 1;
		for (int j = 0; j < n; ++j) dist[(size_t)i * n + j] = 1.0 - r[i][j];
	}
	fputs("# Simple dendrogram (UPGMA-like clustering)\n# Format: (Sample1:distance, Sample2:distance)\n", fp);
	for (int left = n; left > 1; --left) {
		int bi = -1, bj = -1;
		double best = 1e10;
		for (int i = 0; i < n; ++i) {
			if (!on[i]) continue;
			for (int j = i + 1; j < n; ++j)
				if (on[j] && dist[(size_t)i * n + j] < best) { best = dist[(size_t)i * n + j]; bi = i; bj = j; }
		}
		if (bi < 0) break;
		fprintf(fp, "Cluster: %s (%.4f) <-> %s (%.4f)\n", s[bi].name, best / 2, s[bj].name, best / 2);
		for (int k = 0; k < n; ++k) {
			if (k == bi || k == bj || !on[k]) continue;
			const double m = (dist[(size_t)bi * n + k] + dist[(size_t)bj * n + k]) / 2.0;
			dist[(size_t)bi * n + k] = dist[(size_t)k * n + bi] = m;
		}
		on[bj] = 0;
	}
	free(dist);
	free(on);
}

static void co_usage(int min_snps, int min_depth)
{
	fprintf(stderr, "Usage: correlation-matrix -o <output.corr> [-t] [-M MODE] [-m INT] [-d INT] <sample1.vaf> <sample2.vaf> [sample3.vaf ...]\n"
	                "Options:\n"
	                "  -o FILE    output correlation matrix file\n"
	                "  -t         build tree/dendrogram (outputs to <output.tree>)\n"
	                "  -M MODE    preset mode: 'matched' (same individual, depth\xe2\x89\xa5" "5, SNPs\xe2\x89\xa5" "10),\n"
	                "                          'unmatched' (related/unrelated, depth\xe2\x89\xa5" "1, SNPs\xe2\x89\xa5" "20),\n"
	                "                          'strict' (high confidence, depth\xe2\x89\xa5" "10, SNPs\xe2\x89\xa5" "30)\n");
	fprintf(stderr, "  -m INT     minimum SNPs with sufficient depth required [%d]\n", min_snps);
	fprintf(stderr, "  -d INT     minimum depth per SNP [%d]\n", min_depth);
	fprintf(stderr, "\nNote: -m and -d override preset mode values\n");
}

int main(int argc, char **argv)
{
	const char *out = NULL, *mode = NULL;
	int tree = 0, min_snps = 20, min_depth = 1, set_m = 0, set_d = 0, c;
	opterr = 0;
	while ((c = getopt(argc, argv, "o:tm:d:M:")) >= 0) {
		if (c == 'o') out = optarg;
		else if (c == 't') tree = 1;
		else if (c == 'm') min_snps = atoi(optarg), set_m = 1;
		else if (c == 'd') min_depth = atoi(optarg), set_d = 1;
		else if (c == 'M') mode = optarg;
	}
	/* presets, correlation-matrix.c:282-306: {name, depth, snps} */
	static const struct { const char *name, *label; int depth, snps; } presets[] = {
		{"matched", "matched", 5, 10}, {"unmatched", "unmatched", 1, 20},
		{"default", "unmatched", 1, 20}, {"strict", "strict", 10, 30}};
	if (mode) {
		int p = -1;
		for (int i = 0; i < 4; ++i)
			if (strcmp(mode, presets[i].name) == 0) { p = i; break; }
		if (p < 0) {
			fprintf(stderr, "Error: unknown mode '%s'. Valid modes: matched, unmatched, strict\n", mode);
			return 1;
		}
		if (!set_d) min_depth = presets[p].depth;
		if (!set_m) min_snps = presets[p].snps;
		fprintf(stderr, "[M::main] Using '%s' mode: min_depth=%d, min_snps=%d\n", presets[p].label, min_depth, min_snps);
	}
	const int n = argc - optind;
	if (!out || n < 2) {
		co_usage(min_snps, min_depth);
		return 1;
	}
	fprintf(stderr, "[M::main] Loading %d VAF files...\n", n);
	co_sample *s = (co_sample*)calloc(n, sizeof(co_sample));
	for (int i = 0; i < n; ++i) {
		if (co_load(argv[optind + i], &s[i]) != 0) {
			fprintf(stderr, "Error: failed to load %s\n", argv[optind + i]);
			return 1;
		}
		fprintf(stderr, "[M::main] Loaded %s: %d SNPs\n", s[i].name, s[i].n);
	}
	fprintf(stderr, "[M::main] Computing correlation matrix...\n");
	double **r = (double**)malloc(n * sizeof(double*));
	for (int i = 0; i < n; ++i) r[i] = (double*)malloc(n * sizeof(double));
	for (int i = 0; i < n; ++i) {
		r[i][i] = 1.0;
		for (int j = i + 1; j < n; ++j) r[i][j] = r[j][i] = co_pair(&s[i], &s[j], s[i].n, min_snps, min_depth);
	}
	fprintf(stderr, "[M::main] Writing correlation matrix...\n");
	FILE *fp = fopen(out, "w");
	if (!fp) {
		fprintf(stderr, "Error: failed to open output file\n");
		return 1;
	}
	fputs("Sample", fp);
	for (int i = 0; i < n; ++i) fprintf(fp, "\t%s", s[i].name);
	fputc('\n', fp);
	for (int i = 0; i < n; ++i) {
		fputs(s[i].name, fp);
		for (int j = 0; j < n; ++j) fprintf(fp, "\t%.6f", r[i][j]);
		fputc('\n', fp);
	}
	fclose(fp);
	fprintf(stderr, "[M::main] Correlation matrix written to %s\n", out);
	if (tree) {
		char tn[512];
		snprintf(tn, sizeof tn, "%s", out);
		char *e = strstr(tn, ".corr");
		if (e) strcpy(e, ".tree");
		else strcat(tn, ".tree");
		fprintf(stderr, "[M::main] Building dendrogram...\n");
		FILE *tf = fopen(tn, "w");
		if (tf) {
			co_tree(s, n, r, tf);
			fclose(tf);
			fprintf(stderr, "[M::main] Dendrogram written to %s\n", tn);
		}
	}
	for (int i = 0; i < n; ++i) free(s[i].x), free(s[i].d), free(r[i]);
	free(r);
	free(s);
	return 0;
}
