/*
 * ibwa_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference `ibwa aln` hot path (BWA 0.5.9 fork):
 *   bwt.c      bwt_occ / bwt_2occ / bwt_occ4 / bwt_2occ4 / bwt_match_exact_alt
 *   bwtio.c    bwt_restore_bwt
 *   bwtaln.c   gap_init_opt, bwa_cal_maxdiff, bwt_cal_width, bwa_cal_sa_reg_gap
 *   bwtgap.c   gap stack, gap_shadow, bwt_match_gap
 *   stdaln.c   aln_global_core, aln_local_core (row a11/a12 of SURVEY §8a)
 *   bwt.c      bwt_sa, bwtio.c bwt_restore_sa, dbset.c bwtdb_sa2seq
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this
 * library, and only as the checker or the CPU baseline -- never as a product
 * fallback.  Pinned against golden vectors produced by the compiled
 * reference (tests/golden/, tools/make_golden.py).
 */
#ifndef IBWA_ORACLE_H
#define IBWA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* bwt.h:42-54, without the SA part (not on the aln path) */
typedef struct {
	uint32_t primary;
	uint32_t L2[5];
	uint32_t seq_len;
	uint32_t bwt_size;  /* in uint32 words, incl. interleaved Occ counts */
	uint32_t *bwt;
	int owns;
} or_bwt_t;

/* bwtaln.h:105-115: serialised raw as the 64-byte .sai header */
typedef struct {
	int s_mm, s_gapo, s_gape;
	int mode;
	int indel_end_skip, max_del_occ, max_entries;
	float fnr;
	int max_diff, max_gapo, max_gape;
	int max_seed_diff, seed_len;
	int n_threads;
	int max_top2;
	int trim_qual;
} or_gap_opt_t;

/* bwtaln.h:34-38 (16 bytes) */
typedef struct {
	uint32_t n_mm:8, n_gapo:8, n_gape:8, a:1;
	uint32_t k, l;
	int score;
} or_aln1_t;

#define OR_MODE_GAPE     0x01
#define OR_MODE_COMPREAD 0x02
#define OR_MODE_LOGGAP   0x04
#define OR_MODE_NONSTOP  0x10

or_bwt_t *or_bwt_load(const char *fn);
or_bwt_t *or_bwt_wrap(uint32_t primary, const uint32_t L2_1to4[4], uint32_t *words, uint64_t n_words);
void or_bwt_free(or_bwt_t *b);

uint32_t or_occ(const or_bwt_t *b, uint32_t k, int c);
void or_occ4(const or_bwt_t *b, uint32_t k, uint32_t cnt[4]);
void or_2occ4(const or_bwt_t *b, uint32_t k, uint32_t l, uint32_t ck[4], uint32_t cl[4]);

void or_gap_init_opt(or_gap_opt_t *o);
int or_cal_maxdiff(int l, double err, double thres);

/*
 * Batch driver, restating bwa_cal_sa_reg_gap (bwtaln.c:80-140) over
 * flat arrays.  seq: concatenated bwa_seq_t.seq arrays (the read reversed,
 * codes 0..4; bwaseqio.c:191); rseq is derived per read (bwaseqio.c:192).
 * Outputs: n_aln[i]; *alns_out = malloc'd concatenation of all hits in read
 * order (free with or_free).  touches_out (optional) receives the number of
 * Occ-interval touches per read.  Returns the total hit count.
 */
int64_t or_cal_sa_reg_gap(const or_bwt_t *bwt0, const or_bwt_t *bwt1, int64_t n_seqs,
                          const uint8_t *seq, const uint64_t *off, const uint32_t *len,
                          const or_gap_opt_t *opt, int n_threads,
                          int32_t *n_aln, or_aln1_t **alns_out, uint32_t *touches_out);
void or_free(void *p);
/* next or_cal_sa_reg_gap only: per read a pop count p (0: none) -> touches[r] = the touches counted
 * before pop p + 1 (the read's total when p is 0 or never reached) */
void or_set_touch_split(const uint32_t *pops, uint32_t *touches);
void or_exact_touches(const or_bwt_t *bwt0, const or_bwt_t *bwt1, int64_t n_seqs, const uint8_t *seq,
                      const uint64_t *off, const uint32_t *len, int mode, int K, int jump, uint32_t *touches);

/* stdaln.c:529 restated: local SW + banded global path fill (aln_param_bwa) */
typedef struct { int i, j; unsigned char ctype; } or_path_t;
int or_aln_local_core(const uint8_t *seq1, int len1, const uint8_t *seq2, int len2,
                      or_path_t *path, int *path_len, int thres, int *subo);
int or_aln_global_core(const uint8_t *seq1, int len1, const uint8_t *seq2, int len2,
                       int band_width, int gap_end, or_path_t *path, int *path_len);
int or_path2cigar32(const or_path_t *path, int path_len, uint32_t *cigar);

/* SA -> coordinate: bwt_restore_sa (bwtio.c:29), bwt_sa (bwt.c:69), bwtdb_sa2seq (dbset.c:240) */
void or_bwt_info(const or_bwt_t *b, uint32_t *primary, uint32_t *seq_len);
uint32_t *or_sa_load(const char *fn, const or_bwt_t *b, uint32_t *intv, uint64_t *n_sa);
uint32_t or_bwt_sa(const or_bwt_t *b, const uint32_t *sa, uint32_t intv, uint32_t k, uint32_t *steps);
void or_sa2seq_batch(const or_bwt_t *b0, const uint32_t *sa0, const or_bwt_t *b1, const uint32_t *sa1,
                     uint32_t intv, int64_t n, const uint8_t *strand, const uint32_t *k, const uint32_t *len,
                     uint64_t *pos, uint32_t *steps);

#ifdef __cplusplus
}
#endif
#endif
