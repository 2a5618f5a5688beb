/*
 * ibwa_bwa_compat.h -- the drop-in boundary in the reference's own types.
 *
 * A reference build links libibwa_amd.so in place of bwtaln.c's
 * bwa_cal_sa_reg_gap.  The structs below are layout mirrors of
 * the reference's bwt_t (bwt.h:41-53) and bwa_seq_t (bwtaln.h:62-93) on the
 * x86-64 SysV ABI -- same member types, order and bit-fields -- so the
 * reference's pointers can be passed straight through; tests/test_compat.py
 * checks every offset against the reference headers where they exist.
 * gap_opt_t is ibwa_gap_opt_t (ibwa_aln.h), bwt_aln1_t is ibwa_aln1_t.
 *
 * Failure behaviour: the reference function returns void and crashes on
 * allocation failure; this one prints the HIP/engine error to stderr and
 * abort()s.  It never computes on the CPU.
 */
#ifndef IBWA_BWA_COMPAT_H
#define IBWA_BWA_COMPAT_H
#include <stdint.h>
#include <stdio.h>

#include "ibwa_aln.h"

#ifdef __cplusplus
extern "C" {
#endif

/* bwt_t (bwt.h:41-53) */
typedef struct {
	uint32_t primary;       /* row of the $ suffix */
	uint32_t L2[5];         /* cumulative symbol counts, L2[4] = seq_len */
	uint32_t seq_len;
	uint32_t bwt_size;      /* words at .bwt */
	uint32_t *bwt;          /* interleaved [4 counts][8 BWT words] per 128 rows */
	uint32_t cnt_table[256];
	int sa_intv;
	uint32_t n_sa;
	uint32_t *sa;
} ibwa_ref_bwt_t;

/* bwt_multi1_t (bwtaln.h:51-60) -- only its size matters here */
typedef struct {
	uint64_t pos, remapped_pos;
	uint32_t dbidx, remapped_dbidx;
	int32_t remapped_seqid;
	int remap_identical;
	uint32_t n_cigar:15, gap:8, mm:8, strand:1;
	uint32_t *cigar;
} ibwa_ref_multi1_t;

/* bwa_seq_t (bwtaln.h:62-93) */
typedef struct {
	char *name;
	uint8_t *seq, *rseq, *qual;       /* seq: the read reversed (bwaseqio.c:191) */
	uint32_t len:20, strand:1, type:2, dummy:1, extra_flag:8;
	uint32_t n_mm:8, n_gapo:8, n_gape:8, mapQ:8;
	int score;
	int clip_len;
	int n_aln;                        /* out */
	ibwa_aln1_t *aln;                 /* out, malloc'd (freed by bwa_free_read_seq) */
	int n_multi;
	ibwa_ref_multi1_t *multi;
	uint32_t sa;
	uint64_t pos;
	uint64_t remapped_pos;
	uint32_t dbidx, remapped_dbidx;
	int32_t remapped_seqid;
	int remap_identical;
	uint64_t c1:28, c2:28, seQ:8;
	int n_cigar;
	uint32_t *cigar;
	int tid;
	char bc[16];
	uint32_t full_len:20, nm:12;
	char *md;
} ibwa_ref_seq_t;

#define IBWA_TYPE_NO_MATCH 0 /* BWA_TYPE_NO_MATCH, bwtaln.h:7 */
#define IBWA_TYPE_MATESW 3   /* BWA_TYPE_MATESW, bwtaln.h:10 */
#define IBWA_SAM_FPP 2       /* SAM_FPP, bwtaln.h:13 */
#define IBWA_PET_STD 1       /* BWA_PET_STD, bwtaln.h:117 */
#define IBWA_PET_SOLID 2     /* BWA_PET_SOLID, bwtaln.h:118 */

/* pe_opt_t (bwtaln.h:120-128) */
typedef struct {
	int max_isize, force_isize;
	int max_occ;
	int n_multi, N_multi;
	int n_threads;
	int type, is_sw, is_preload;
	int remapping;
	double ap_prior;
} ibwa_ref_pe_opt_t;

/* isize_info_t (bwapair.h:8-11) */
typedef struct {
	double avg, std, ap_prior;
	uint32_t low, high, high_bayesian;
} ibwa_ref_isize_info_t;

/* bntann1_t / bntamb1_t / bntseq_t (bntseq.h:40-62) */
typedef struct {
	int64_t offset;
	int32_t len;
	int32_t n_ambs;
	uint32_t gi;
	char *name, *anno;
} ibwa_ref_bntann1_t;
typedef struct {
	int64_t offset;
	int32_t len;
	char amb;
} ibwa_ref_bntamb1_t;
typedef struct {
	int64_t l_pac;
	int32_t n_seqs;
	uint32_t seed;
	ibwa_ref_bntann1_t *anns;
	int32_t n_holes;
	ibwa_ref_bntamb1_t *ambs;
	FILE *fp_pac;                  /* the .pac, read by seq_load_pac (dbset.c:103-108) */
} ibwa_ref_bntseq_t;

/* seq_t (bwaremap.h:24-29): one reference's metadata, its packed sequence once loaded, and the
 * compound-sequence remappings (opaque here) */
typedef struct {
	ibwa_ref_bntseq_t *bns;
	uint8_t *data;                 /* l_pac / 4 + 1 bytes (dbset_load_pac), or NULL */
	int remap;
	void **mappings;               /* bnsremap_t ** */
} ibwa_ref_seqt_t;

/* bwtdb_t (dbset.h:12-19) */
typedef struct {
	const char *prefix;
	ibwa_ref_bwt_t *bwt[2];
	void *bwtcache;                /* bwtcache_t * */
	uint64_t offset;               /* of this reference in the concatenated coordinates */
	ibwa_ref_seqt_t *bns;
	ibwa_ref_seqt_t *ntbns;
} ibwa_ref_bwtdb_t;

/* dbset_t (dbset.h:21-30): the primary reference and the alternates of `sampe`, concatenated */
typedef struct {
	int count;
	int color_space;
	int preload;
	ibwa_ref_bwtdb_t **db;
	ibwa_ref_seqt_t **bns;
	ibwa_ref_seqt_t **ntbns;
	uint64_t l_pac;                /* sum of every reference's l_pac */
	uint64_t total_bwt_seq_len[2];
} ibwa_ref_dbset_t;

/*
 * Bring the index of a running `aln` onto the GPUs (called by
 * bwa_aln_core after bwt_restore_bwt, bwtaln.c:189).  n_gpus <= 0: every
 * visible device.  The first device receives the arrays over PCIe, the rest
 * by device-to-device copies.  Returns 0, or an IBWA_E* code.
 */
int ibwa_gpu_init(ibwa_ref_bwt_t *const bwt[2], int n_gpus);
/* As ibwa_gpu_init, with slices_per_gpu engines on every GPU (a batch is split into
 * n_gpus * slices_per_gpu contiguous slices, the slices of one GPU running concurrently) and a
 * batch split only into slices of at least min_reads_per_slice reads (ibwa_gpu_init: 1 and
 * 1024, the reference's THREAD_BLOCK_SIZE claim, bwtaln.c:16). */
int ibwa_gpu_init_ex(ibwa_ref_bwt_t *const bwt[2], int n_gpus, int slices_per_gpu, int min_reads_per_slice);
/* Release the engines (before bwt_destroy, bwtaln.c:239). */
void ibwa_gpu_destroy(void);

/*
 * bwa_cal_sa_reg_gap (bwtaln.h:148, bwtaln.c:80-140), same signature and
 * effects: for every read, aln/n_aln computed exactly as the reference
 * does; sa = 0, type = NO_MATCH, c1 = c2 = 0; name/seq/rseq/qual freed and
 * set to NULL.  `tid` is ignored (one call per batch, from the n_threads <= 1
 * branch); the batch is split in contiguous slices over the GPUs with the
 * batch-level options of bwtaln.c:89-93.  Without ibwa_gpu_init the first
 * call initialises one GPU from `bwt`.  (Inside a reference build bwtaln.h
 * already declares it with the reference's layout-identical types.)
 */
#ifndef BWTALN_H
void bwa_cal_sa_reg_gap(int tid, ibwa_ref_bwt_t *const bwt[2], int n_seqs, ibwa_ref_seq_t *seqs,
                        const ibwa_gap_opt_t *opt);
#endif

/*
 * bwa_sw_core (bwasw.c:29-112) for n mate rescues at once -- the per-rescue
 * body that bwa_paired_sw_thread (bwasw.c:145-268) calls, with the alignment
 * itself batched on the GPU (ibwa_sw_batch).  Pair p: read codes
 * seq[off[p] .. +len[p]); the reference window already extracted by
 * dbset_extract_sequence (bwasw.c:46): ref[ref_off[p] .. +ref_len[p]), its
 * requested length reglen[p] and start beg[p] (in/out, as *beg), l_pac the
 * packed reference length.  Out: n_cigar[p] (0 = rejected, the reference's
 * NULL), cnt[p] = n_mm << 16 | n_gapo << 8 | n_gape, *cigar = malloc'd
 * concatenation of the bwa_cigar_t arrays (op << 29 | len, soft clips op 3).
 */
int ibwa_sw_core_batch(ibwa_ctx_t *ctx, int64_t n, const uint8_t *seq, const uint64_t *off, const uint32_t *len,
                       const uint8_t *ref, const uint64_t *ref_off, const uint32_t *ref_len, const int32_t *reglen,
                       int64_t *beg, int64_t l_pac, int32_t *n_cigar, uint32_t *cnt, uint32_t **cigar);

/*
 * bwa_paired_sw (bwasw.c:270-304) -- the mate rescue of `sampe` -- for one reference
 * database (db offset 0): `pac` is the packed reference as seq_t.data holds it after
 * dbset_load_pac (bns_pac order, 4 bases per byte, MSB first) and l_pac its length.
 * Same effects on seqs[0][i] / seqs[1][i] as the reference (bwa_paired_sw_thread,
 * bwasw.c:145-268): the candidate selection and window placement run on the host, every
 * bwa_sw_core of the batch (<= 2 per pair) is one batched GPU launch (ibwa_sw_core_batch),
 * then the acceptance test and the mapQ / CIGAR / __set_fixed updates are applied in pair
 * order.  A replaced CIGAR is free()d and the new one malloc()ed, as the reference does.
 * Counters: n_tot / n_mapped as the reference's stderr summary ([1] singletons,
 * [0] discordant pairs).  Returns 0, or a negative IBWA_E* code (nothing is modified then).
 */
int ibwa_paired_sw(ibwa_ctx_t *ctx, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                   const ibwa_ref_isize_info_t *ii, const uint8_t *pac, uint64_t l_pac, uint64_t n_tot[2],
                   uint64_t n_mapped[2]);

/*
 * ibwa_paired_sw over several references concatenated at offset[i] (dbset_extract_sequence,
 * dbset.c:306-325): pac[i] / l_pac[i] as seq_t.data / bntseq_t.l_pac of reference i.
 */
int ibwa_paired_sw_dbs(ibwa_ctx_t *ctx, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                       const ibwa_ref_isize_info_t *ii, int n_db, const uint8_t *const *pac, const uint64_t *offset,
                       const uint64_t *l_pac, uint64_t n_tot[2], uint64_t n_mapped[2]);

/*
 * bwa_paired_sw (bwasw.h:12, bwasw.c:270-304) with the reference's own signature: a reference
 * `sampe` links this in place of bwasw.o.  The references of `dbs` are concatenated at their
 * db->offset as dbset_extract_sequence (dbset.c:306-325) reads them; each one's packed
 * sequence is taken from seq_t.data when loaded, else read from its .pac (bntseq_t.fp_pac)
 * as dbset_load_pac does -- neither is modified.  The SW runs on the engine of device 0 that
 * ibwa_gpu_init made (or a new one).  Prints the reference's two stderr summary lines; a HIP
 * failure is reported and abort()s, like the reference's allocation failures.
 */
#ifndef BWASW_H
void bwa_paired_sw(ibwa_ref_dbset_t *dbs, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                   const ibwa_ref_isize_info_t *ii);
#endif

#ifdef __cplusplus
}
#endif
#endif
