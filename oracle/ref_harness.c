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
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "bwt.h"
#include "bwtaln.h"
#include "stdaln.h"

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
		uint64_t pos = strand ? (uint64_t)sa : (uint64_t)(bwtint_t)(bwt[1]->seq_len - (bwtint_t)(sa + len));
		printf("%u\t%u\t%u\t%u\t%llu\n", strand, k, len, sa, (unsigned long long)pos);
	}
	fclose(fp);
	bwt_destroy(bwt[0]); bwt_destroy(bwt[1]);
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
	if (strcmp(argv[1], "samse") == 0) return bwa_sai2sam_se(argc - 1, argv + 1);
	if (strcmp(argv[1], "sampe") == 0) return bwa_sai2sam_pe(argc - 1, argv + 1);
	fprintf(stderr, "unknown command %s\n", argv[1]);
	return 1;
}
