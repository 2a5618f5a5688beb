/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (see oracle/README.md).
 *
 * A thin driver linked against the reference sources compiled in place from
 * /root/reference by oracle/Makefile (outputs go to oracle/_ref/ only).  It
 * is used to (1) produce golden fixtures in this container and (2) time the
 * reference CPU path as bench.py's `cpu_baseline` (kind "reference").
 * Nothing in the shipped product links or loads this file.
 *
 * Commands mirror main.cpp:45-59 for the two commands we need:
 *   ibwa_ref index [-a is|bwtsw] <in.fa>   -> bwa_index   (bwtindex.c:42)
 *   ibwa_ref aln [opts] <prefix> <in.fq>   -> bwa_aln     (bwtaln.c:243)
 *   ibwa_ref occ4 <prefix.bwt> k...        -> bwt_occ4    (bwt.c:157)  (KAT)
 *   ibwa_ref sw <ref_seq> <read_seq>       -> aln_local_core (stdaln.c:529)
 *   ibwa_ref swf <pairs.tsv>               -> aln_local_core over a file of pairs
 *   ibwa_ref sa <prefix> <rows.tsv>        -> bwt_sa (bwt.c:69) over bwt_restore_sa (bwtio.c:29)
 *   ibwa_ref samse|sampe ...               -> bwa_sai2sam_se / bwa_sai2sam_pe (bwase.c:710, bwape.c)
 *   ibwa_ref gswf <pairs.tsv>              -> aln_global_core (stdaln.c:345) + bwa_aln_path2cigar
 *                                             with aln_param_bwa, as refine_gapped_core calls it
 *   ibwa_ref psw <prefix> <pairs.tsv> <type> <avg> <std> <ap_prior>
 *                                          -> bwa_paired_sw (bwasw.c:270) on pairs read from a file
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "bwt.h"
#include "bwtaln.h"
#include "stdaln.h"
#include "dbset.h"
#include "bwasw.h"

int bwa_index(int argc, char *argv[]);
int bwa_sai2sam_se(int argc, char *argv[]);
int bwa_sai2sam_pe(int argc, char *argv[]);

/* This harness takes the place of the reference's main.cpp (which needs the cmake-generated
 * version.h): besides main() that file defines only the @PG printer samse/sampe call
 * (main.cpp:31-34).  Here it names the harness instead of a version string. */
void bwa_print_sam_PG(void)
{
	printf("@PG\tID:bwa\tPN:bwa\tVN:ibwa_ref-harness\n");
}
int bwa_aln(int argc, char *argv[]);
extern unsigned char nst_nt4_table[256];

static int cmd_occ4(int argc, char *argv[])
{
	int i;
	bwt_t *bwt;
	if (argc < 3) return 1;
	bwt = bwt_restore_bwt(argv[1]);
	for (i = 2; i < argc; ++i) {
		bwtint_t k = (bwtint_t)strtoul(argv[i], 0, 0), c4[4];
		bwt_occ4(bwt, k, c4);
		printf("%u\t%u\t%u\t%u\t%u\n", k, c4[0], c4[1], c4[2], c4[3]);
	}
	bwt_destroy(bwt);
	return 0;
}

/* sw <ref> <read> : both as ACGTN strings; prints score, path_len and the path */
static int cmd_sw(int argc, char *argv[])
{
	int l1, l2, i, path_len = 0, score, n_cigar = 0;
	unsigned char *s1, *s2;
	path_t *path;
	uint32_t *cigar;
	AlnParam ap = aln_param_bwa;
	if (argc < 3) return 1;
	l1 = strlen(argv[1]); l2 = strlen(argv[2]);
	s1 = (unsigned char*)malloc(l1 + 1); s2 = (unsigned char*)malloc(l2 + 1);
	for (i = 0; i < l1; ++i) s1[i] = nst_nt4_table[(int)argv[1][i]];
	for (i = 0; i < l2; ++i) s2[i] = nst_nt4_table[(int)argv[2][i]];
	path = (path_t*)calloc(l1 + l2 + 2, sizeof(path_t));
	score = aln_local_core(s1, l1, s2, l2, &ap, path, &path_len, 1, 0);
	printf("%d\t%d", score, path_len);
	if (score >= 0 && path_len > 0) {
		cigar = aln_path2cigar32(path, path_len, &n_cigar);
		printf("\t%d,%d\t%d,%d\t", path[path_len-1].i, path[path_len-1].j, path[0].i, path[0].j);
		for (i = 0; i < n_cigar; ++i) printf("%u%c", cigar[i]>>4, "MIDS"[cigar[i]&0xf]);
		free(cigar);
	}
	printf("\n");
	free(path); free(s1); free(s2);
	return 0;
}

/* swf <pairs.tsv> : one "ref<TAB>read" (ACGTN strings) per line; prints one line of
 * score, path_len, start i,j, end i,j, CIGAR per input line (empty fields when no path) */
static int cmd_swf(int argc, char *argv[])
{
	static char line[1 << 16];
	FILE *fp;
	AlnParam ap = aln_param_bwa;
	if (argc < 2 || !(fp = fopen(argv[1], "r"))) return 1;
	while (fgets(line, sizeof line, fp)) {
		char *t = strchr(line, '\t'), *r2;
		int l1, l2, i, path_len = 0, score, n_cigar = 0;
		unsigned char *s1, *s2;
		path_t *path;
		if (!t) continue;
		*t = 0; r2 = t + 1;
		r2[strcspn(r2, "\r\n")] = 0;
		l1 = strlen(line); l2 = strlen(r2);
		s1 = (unsigned char*)malloc(l1 + 1); s2 = (unsigned char*)malloc(l2 + 1);
		for (i = 0; i < l1; ++i) s1[i] = nst_nt4_table[(int)line[i]];
		for (i = 0; i < l2; ++i) s2[i] = nst_nt4_table[(int)r2[i]];
		path = (path_t*)calloc(l1 + l2 + 2, sizeof(path_t));
		score = aln_local_core(s1, l1, s2, l2, &ap, path, &path_len, 1, 0);
		printf("%d\t%d", score, path_len);
		if (score >= 0 && path_len > 0) {
			uint32_t *cigar = aln_path2cigar32(path, path_len, &n_cigar);
			printf("\t%d,%d\t%d,%d\t", path[path_len-1].i, path[path_len-1].j, path[0].i, path[0].j);
			for (i = 0; i < n_cigar; ++i) printf("%u%c", cigar[i]>>4, "MIDS"[cigar[i]&0xf]);
			free(cigar);
		} else printf("\t\t\t");
		printf("\n");
		free(path); free(s1); free(s2);
	}
	fclose(fp);
	return 0;
}

/* sa <prefix> <rows.tsv> : one "strand<TAB>k<TAB>len" per line; prints the line plus the
 * bwt_sa value of row k on the strand's index and the position bwtdb_sa2seq computes from it
 * (dbset.c:240-246 with db->offset = 0: strand 1 -> bwt_sa(bwt[0], k); strand 0 ->
 * bwt[1]->seq_len - (bwt_sa(bwt[1], k) + len), in bwtint_t arithmetic).  dbset.c itself is not
 * compiled here (it pulls in the remap / cache layers); its three lines are restated. */
static int cmd_sa(int argc, char *argv[])
{
	char fn[4096];
	bwt_t *bwt[2];
	FILE *fp;
	unsigned strand, k, len;
	if (argc < 3) return 1;
	snprintf(fn, sizeof fn, "%s.bwt", argv[1]); bwt[0] = bwt_restore_bwt(fn);
	snprintf(fn, sizeof fn, "%s.sa", argv[1]); bwt_restore_sa(fn, bwt[0]);
	snprintf(fn, sizeof fn, "%s.rbwt", argv[1]); bwt[1] = bwt_restore_bwt(fn);
	snprintf(fn, sizeof fn, "%s.rsa", argv[1]); bwt_restore_sa(fn, bwt[1]);
	if (!(fp = fopen(argv[2], "r"))) return 1;
	while (fscanf(fp, "%u %u %u", &strand, &k, &len) == 3) {
		bwtint_t sa = bwt_sa(bwt[strand ? 0 : 1], k);
		/* bwtdb_sa2seq (dbset.c:244): u64 offset + u32 seq_len - u32 (sa + len), i.e. u64 arithmetic */
		uint64_t pos = strand ? (uint64_t)sa : (uint64_t)0 + bwt[1]->seq_len - (bwtint_t)(sa + len);
		printf("%u\t%u\t%u\t%u\t%llu\n", strand, k, len, sa, (unsigned long long)pos);
	}
	fclose(fp);
	bwt_destroy(bwt[0]); bwt_destroy(bwt[1]);
	return 0;
}

/* gswf <pairs.tsv> : one "ref<TAB>read" per line; prints score, path_len and the CIGAR of
 * aln_global_core(ref, read, &aln_param_bwa) as refine_gapped_core (bwase.c:196-198) runs it */
static int cmd_gswf(int argc, char *argv[])
{
	static char line[1 << 16];
	FILE *fp;
	AlnParam ap = aln_param_bwa;
	if (argc < 2 || !(fp = fopen(argv[1], "r"))) return 1;
	while (fgets(line, sizeof line, fp)) {
		char *t = strchr(line, '\t'), *r2;
		int l1, l2, i, path_len = 0, score, n_cigar = 0;
		unsigned char *s1, *s2;
		path_t *path;
		bwa_cigar_t *cigar;
		if (!t) continue;
		*t = 0; r2 = t + 1;
		r2[strcspn(r2, "\r\n")] = 0;
		l1 = strlen(line); l2 = strlen(r2);
		s1 = (unsigned char*)malloc(l1 + 1); s2 = (unsigned char*)malloc(l2 + 1);
		for (i = 0; i < l1; ++i) s1[i] = nst_nt4_table[(int)line[i]];
		for (i = 0; i < l2; ++i) s2[i] = nst_nt4_table[(int)r2[i]];
		path = (path_t*)calloc(l1 + l2 + 2, sizeof(path_t));
		score = aln_global_core(s1, l1, s2, l2, &ap, path, &path_len);
		printf("%d\t%d\t", score, path_len);
		if (path_len > 0) {
			cigar = bwa_aln_path2cigar(path, path_len, &n_cigar);
			for (i = 0; i < n_cigar; ++i) printf("%u%c", __cigar_len(cigar[i]), "MIDS"[__cigar_op(cigar[i])]);
			free(cigar);
		}
		printf("\n");
		free(path); free(s1); free(s2);
	}
	fclose(fp);
	return 0;
}

/* psw: bwa_paired_sw (bwasw.c:270-304) over mate pairs described one per line as
 *   <end 0 fields> <TAB> <end 1 fields>, each end = read(ACGTN) strand type mapQ seQ extra_flag
 *   n_mm n_gapo n_gape pos   (space separated)
 * The bwa_seq_t are set up as bwa_read_seq does (bwaseqio.c:180-192: seq = the read reversed,
 * rseq = its reverse complement); remapped_pos = pos.  Prints per end the fields bwa_paired_sw
 * may change and the CIGAR, then the four counters of its stderr summary. */
pe_opt_t *bwa_init_pe_opt(void); /* bwape.c:72, not declared in a header */
static void psw_end(bwa_seq_t *p, char *f)
{
	char rd[4096];
	unsigned strand, type, mapQ, seQ, xf, mm, go, ge;
	unsigned long long pos;
	int i, l;
	sscanf(f, "%4095s %u %u %u %u %u %u %u %u %llu", rd, &strand, &type, &mapQ, &seQ, &xf, &mm, &go, &ge, &pos);
	l = strlen(rd);
	memset(p, 0, sizeof(*p));
	p->len = p->full_len = p->clip_len = l;
	p->seq = (ubyte_t*)calloc(l, 1);
	p->rseq = (ubyte_t*)calloc(l, 1);
	for (i = 0; i < l; ++i) p->seq[i] = nst_nt4_table[(int)rd[i]];
	memcpy(p->rseq, p->seq, l);
	seq_reverse(l, p->seq, 0);
	seq_reverse(l, p->rseq, 1);
	p->strand = strand; p->type = type; p->mapQ = mapQ; p->seQ = seQ; p->extra_flag = xf;
	p->n_mm = mm; p->n_gapo = go; p->n_gape = ge;
	p->pos = p->remapped_pos = pos;
}

static int cmd_psw(int argc, char *argv[])
{
	static char line[1 << 14];
	const char *prefix[1];
	dbset_t *dbs;
	pe_opt_t *popt;
	isize_info_t ii;
	bwa_seq_t *seqs[2];
	int n = 0, m = 1024, i, k, j;
	FILE *fp;
	if (argc < 7) return 1;
	prefix[0] = argv[1];
	dbs = dbset_restore(1, prefix, BWA_MODE_GAPE | BWA_MODE_COMPREAD, 0, 0);
	popt = bwa_init_pe_opt();
	popt->type = atoi(argv[3]);
	popt->n_threads = 1;
	memset(&ii, 0, sizeof ii);
	ii.avg = atof(argv[4]); ii.std = atof(argv[5]); ii.ap_prior = atof(argv[6]);
	seqs[0] = (bwa_seq_t*)calloc(m, sizeof(bwa_seq_t));
	seqs[1] = (bwa_seq_t*)calloc(m, sizeof(bwa_seq_t));
	if (!(fp = fopen(argv[2], "r"))) return 1;
	while (fgets(line, sizeof line, fp)) {
		char *t = strchr(line, '\t');
		if (!t) continue;
		*t = 0;
		if (n == m) {
			m <<= 1;
			seqs[0] = (bwa_seq_t*)realloc(seqs[0], m * sizeof(bwa_seq_t));
			seqs[1] = (bwa_seq_t*)realloc(seqs[1], m * sizeof(bwa_seq_t));
		}
		psw_end(seqs[0] + n, line);
		psw_end(seqs[1] + n, t + 1);
		++n;
	}
	fclose(fp);
	bwa_paired_sw(dbs, n, seqs, popt, &ii);
	for (i = 0; i < n; ++i) {
		for (k = 0; k < 2; ++k) {
			bwa_seq_t *p = seqs[k] + i;
			printf("%s%u %u %llu %llu %u %u %u %u %u %u %u %u %d ", k ? "\t" : "", p->type, p->strand,
			       (unsigned long long)p->pos, (unsigned long long)p->remapped_pos, p->dbidx, p->remapped_dbidx,
			       p->mapQ, (unsigned)p->seQ, p->n_mm, p->n_gapo, p->n_gape, p->extra_flag, p->n_cigar);
			if (!p->n_cigar) printf("*");
			for (j = 0; j < p->n_cigar; ++j) printf("%u%c", __cigar_len(p->cigar[j]), "MIDS"[__cigar_op(p->cigar[j])]);
			free(p->seq); free(p->rseq); free(p->cigar);
		}
		printf("\n");
	}
	free(seqs[0]); free(seqs[1]); free(popt);
	dbset_destroy(dbs);
	return 0;
}

int main(int argc, char *argv[])
{
	if (argc < 2) {
		fprintf(stderr, "usage: ibwa_ref index|aln|occ4|sw ...\n");
		return 1;
	}
	if (strcmp(argv[1], "index") == 0) return bwa_index(argc - 1, argv + 1);
	if (strcmp(argv[1], "aln") == 0) return bwa_aln(argc - 1, argv + 1);
	if (strcmp(argv[1], "occ4") == 0) return cmd_occ4(argc - 1, argv + 1);
	if (strcmp(argv[1], "sw") == 0) return cmd_sw(argc - 1, argv + 1);
	if (strcmp(argv[1], "swf") == 0) return cmd_swf(argc - 1, argv + 1);
	if (strcmp(argv[1], "sa") == 0) return cmd_sa(argc - 1, argv + 1);
	if (strcmp(argv[1], "gswf") == 0) return cmd_gswf(argc - 1, argv + 1);
	if (strcmp(argv[1], "psw") == 0) return cmd_psw(argc - 1, argv + 1);
	if (strcmp(argv[1], "samse") == 0) return bwa_sai2sam_se(argc - 1, argv + 1);
	if (strcmp(argv[1], "sampe") == 0) return bwa_sai2sam_pe(argc - 1, argv + 1);
	fprintf(stderr, "unknown command %s\n", argv[1]);
	return 1;
}
