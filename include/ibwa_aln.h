/*
 * ibwa_aln.h -- C ABI of the MI355X `ibwa aln` engine (libibwa_amd.so).
 *
 * Plain pointers and sizes only.  Each entry point names the reference
 * interface it replaces.  The drop-in that keeps the reference's own types
 * (`bwa_cal_sa_reg_gap` itself) is in ibwa_bwa_compat.h.
 *
 * Error convention: functions return 0 on success and a negative IBWA_E*
 * code on failure; ibwa_last_error() gives a message.  There is no CPU
 * fallback: without a usable gfx950 device every compute call fails.
 */
#ifndef IBWA_ALN_H
#define IBWA_ALN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
	IBWA_OK = 0,
	IBWA_EHIP = -1,      /* HIP runtime error (no device, OOM, launch failure) */
	IBWA_EINVAL = -2,    /* bad argument / unsupported option combination */
	IBWA_ENOINDEX = -3,  /* index not loaded */
	IBWA_EIO = -4,       /* file I/O */
	IBWA_EOVERFLOW = -5  /* a read exceeded even the large-capacity retry pass */
};

/* gap_opt_t (bwtaln.h:105-115); also the raw 64-byte .sai header (bwtaln.c:192) */
typedef struct {
	int s_mm, s_gapo, s_gape;
	int mode; /* bits 24-31: barcode length */
	int indel_end_skip, max_del_occ, max_entries;
	float fnr;
	int max_diff, max_gapo, max_gape;
	int max_seed_diff, seed_len;
	int n_threads;
	int max_top2;
	int trim_qual;
} ibwa_gap_opt_t;

/* bwt_aln1_t (bwtaln.h:34-38): one SA interval hit, 16 bytes, the .sai record */
typedef struct {
	uint32_t n_mm:8, n_gapo:8, n_gape:8, a:1;
	uint32_t k, l;
	int score;
} ibwa_aln1_t;

#define IBWA_MODE_GAPE     0x01 /* bwtaln.h:95-103 */
#define IBWA_MODE_COMPREAD 0x02
#define IBWA_MODE_LOGGAP   0x04
#define IBWA_MODE_NONSTOP  0x10
#define IBWA_MODE_BAM      0x20
#define IBWA_MODE_BAM_SE   0x40
#define IBWA_MODE_BAM_READ1 0x80
#define IBWA_MODE_BAM_READ2 0x100
#define IBWA_MODE_IL13     0x200

typedef struct ibwa_ctx ibwa_ctx_t;

const char *ibwa_last_error(void);
void ibwa_free(void *p);

/* gap_init_opt (bwtaln.c:21-37) */
void ibwa_gap_init_opt(ibwa_gap_opt_t *opt);
/* bwa_cal_maxdiff (bwtaln.c:39-51) */
int ibwa_cal_maxdiff(int len, double err, double thres);

/* One engine per GPU (device ordinal).  Owns a HIP stream and device buffers. */
int ibwa_ctx_create(int device, ibwa_ctx_t **out);
/* Visible HIP devices (the CLI's -G maps GPU slice g to device g mod this count). */
int ibwa_device_count(int *n);
/* Device memory the library's buffers hold now, and their high-water mark, in bytes, summed over
 * every context of the process (a context borrowing another's index counts only its own buffers).
 * No reference counterpart: the footprint report of bench.py and the CLI's stats line. */
int ibwa_device_bytes(int64_t *now, int64_t *peak);
/* Device arena: one allocation of `bytes` on `device`, made once, from which every later buffer of
 * the process's contexts on that device is carved (a buffer that does not fit is a plain
 * allocation).  Replaces the per-batch scratch allocation of bwa_cal_sa_reg_gap (bwtaln.c:88-97,
 * 139: gap_init_stack / gap_destroy_stack per thread) with memory taken once per process.  A
 * hipMalloc right after another process released much of the HBM waits for the driver to wipe it;
 * reserving the arena while the index loads pays that once, overlapped.  IBWA_EINVAL if the device
 * already has one (the arena lives until the process exits or ibwa_release). */
int ibwa_reserve(int device, uint64_t bytes);
/* Hand the arena of `device` back to the driver now, e.g. before a long host-only phase.  The
 * driver wipes freed memory on the copy engine (~33 GB/s) and an allocation made meanwhile -- by
 * any process -- waits behind that wipe: handing a large arena back right before exit made the next
 * process wait 3.5-5.2 s where an exit holding it often did not (profiles/r05_b2b_rel*.jsonl).  The
 * contexts that carved buffers from it are destroyed first: IBWA_EINVAL while any buffer is still
 * carved.  Afterwards ibwa_reserve may reserve a new arena. */
int ibwa_release(int device);
/* Free and total device memory of `device` (hipMemGetInfo), for sizing an arena. */
int ibwa_device_memory(int device, uint64_t *free_b, uint64_t *total_b);
/* The arena of `device`: its size, the bytes its buffers use now, and their high-water mark. */
int ibwa_arena_stats(int device, uint64_t *size, uint64_t *used, uint64_t *peak);
/* Frees a context.  A context whose index others still borrow (ibwa_ctx_share_index) is freed with
 * its last borrower, so the destroy order of a source and its borrowers does not matter. */
void ibwa_ctx_destroy(ibwa_ctx_t *ctx);

/*
 * Make an FM-index device-resident (replaces the host residency of
 * bwt_restore_bwt, bwtio.c:51-70, as used by bwa_aln_core bwtaln.c:184-189).
 * strand 0 = prefix.bwt, 1 = prefix.rbwt.  `bwt` is the reference's
 * interleaved array (bwt_t.bwt, bwt_size words); L2 = bwt_t.L2[1..4].
 */
int ibwa_ctx_load_bwt(ibwa_ctx_t *ctx, int strand, uint32_t primary, const uint32_t L2[4],
                      const uint32_t *bwt, uint64_t bwt_size);
int ibwa_ctx_load_bwt_file(ibwa_ctx_t *ctx, int strand, const char *path);
/* Copy the index of another context (same process) device-to-device (xGMI peer copy when possible). */
int ibwa_ctx_clone_index(ibwa_ctx_t *dst, const ibwa_ctx_t *src);
/* Use the index of another context on the same device without a copy: its BWT and the structures
 * ibwa_ctx_prepare built (call after it).  Two contexts then align different batches concurrently on
 * one GPU (the CLI's overlapped groups).  src must outlive dst.  While shared, neither context may
 * rebuild or replace the index (load_bwt, build_index, load_sa, clone_index into it, option kmer_k,
 * K-mer tables or a sampled SA the destination would have to build): those return IBWA_EINVAL. */
int ibwa_ctx_share_index(ibwa_ctx_t *dst, const ibwa_ctx_t *src);

/*
 * Batched aln over flat arrays -- the body of bwa_cal_sa_reg_gap
 * (bwtaln.c:80-140) for one batch of n_seqs reads.
 *   seq/off/len : bwa_seq_t.seq of read i (the read reversed, codes 0..5,
 *                 bwaseqio.c:183-191) at seq[off[i] .. off[i]+len[i])
 *   batch_max_len: 0, or the max read length of the *whole* reference batch
 *                 when this call processes only a slice of it (bwtaln.c:89-93
 *                 derive max_diff / max_gapo / stack size from it)
 *   n_aln       : out, per read hit count
 *   aln         : out, malloc'd concatenation of hits in read order (ibwa_free)
 */
int ibwa_aln_batch(ibwa_ctx_t *ctx, const ibwa_gap_opt_t *opt, int64_t n_seqs, const uint8_t *seq,
                   const uint64_t *off, const uint32_t *len, int batch_max_len, int32_t *n_aln,
                   ibwa_aln1_t **aln, int64_t *n_total);

/*
 * Device-resident form used for measurement: stage a batch into HBM once,
 * run the kernels (inputs already resident), then fetch the results.
 */
int ibwa_batch_stage(ibwa_ctx_t *ctx, int64_t n_seqs, const uint8_t *seq, const uint64_t *off,
                     const uint32_t *len);

/*
 * FASTQ ingest on the device -- bwa_read_seq (bwaseqio.c:145-208) over kseq_read (kseq.h:156-195)
 * for strict 4-line records ("@header", one line of sequence bytes: isgraph, none of '>' '+' '@';
 * a line starting with '+'; one line of quality bytes 33..127 as long as the sequence), with the
 * barcode strip (-B: mode >> 24), -I and bwa_trim_read (-q, :74-87), nst_nt4_table codes and the
 * reversal (:197).  raw[0, nbytes) must begin at a record.  Out: *n_rec strict records from its
 * start (at most cap), the *consumed bytes they span, *not_strict = 1 when the next complete
 * record is not strict (the serial kseq reader takes over there; else the block ended inside a
 * record), per record the kept length (-1: not longer than the barcode, skipped as bwaseqio.c:162)
 * and the sequence line's length (rec_len / rec_L may be null).  The kept reads stay in the
 * context (one block at a time) for ibwa_batch_stage_fq.  raw may be pinned (ibwa_host_alloc).
 */
int ibwa_fq_parse(ibwa_ctx_t *ctx, const void *raw, uint64_t nbytes, int mode, int trim_qual, int64_t *n_rec,
                  uint64_t *consumed, int *not_strict, int32_t *rec_len, uint32_t *rec_L, int64_t cap);
/* byte offset (in the block) of record r of the last ibwa_fq_parse (r <= its n_rec); IBWA_EINVAL once
 * another context sharing the parse scratch has parsed since */
int ibwa_fq_offset(const ibwa_ctx_t *ctx, int64_t r, uint64_t *off);
/* dst's parses use src's parse scratch (the raw block, line table, per-record arrays: ~1.7x the
 * block; same device).  Only the kept reads (~0.75x the block) stay per context.  The contexts'
 * ibwa_fq_parse calls must not overlap (each returns with its device work done). */
int ibwa_fq_share_scratch(ibwa_ctx_t *dst, const ibwa_ctx_t *src);
/* kept reads and device time (H2D copy + kernels, ms) of the last ibwa_fq_parse */
int ibwa_fq_stats(const ibwa_ctx_t *ctx, int64_t *kept, double *ms);
/* ibwa_batch_stage from src's last parsed block (same device): its kept reads [first, first + n),
 * max_len = their longest.  Nothing is copied: the batch is a view of src's block, which must not be
 * parsed over (ibwa_fq_parse on src) or destroyed while this context runs or fetches the batch. */
int ibwa_batch_stage_fq(ibwa_ctx_t *ctx, const ibwa_ctx_t *src, int64_t first, int64_t n, int max_len);
/* pinned host memory for the raw blocks */
int ibwa_host_alloc(uint64_t bytes, void **p);
int ibwa_host_free(void *p);
int ibwa_batch_run(ibwa_ctx_t *ctx, const ibwa_gap_opt_t *opt, int batch_max_len);
int ibwa_batch_fetch(ibwa_ctx_t *ctx, int32_t *n_aln, ibwa_aln1_t **aln, int64_t *n_total);
/* The batch's .sai records (bwtaln.c:227-231: per read its int n_aln, then n_aln bwt_aln1_t), in
 * input order, serialised by host threads straight into the caller's buffer.  *bytes = their size;
 * with dst == NULL or cap < *bytes nothing is written (call again with a buffer that large: the
 * device results are copied back once per batch).  *n_total = the hits (may be NULL). */
int ibwa_batch_fetch_sai(ibwa_ctx_t *ctx, void *dst, uint64_t cap, uint64_t *bytes, int64_t *n_total);

/*
 * ibwa_ctx_prepare: the per-index device structures the first ibwa_batch_run with
 * these options would otherwise build on the way (bit-plane Occ layouts and
 * K-mer tables; for max_diff = 0 the exact path's full SA / ISA / 2-bit text,
 * derived from a loaded BWT).  Optional: a caller (the CLI) runs it right
 * after loading the index, while it parses its first reads.  No reference
 * counterpart (bwt_restore_bwt, bwtaln.c:184-189, is the load it follows).
 */
int ibwa_ctx_prepare(ibwa_ctx_t *ctx, const ibwa_gap_opt_t *opt);

typedef struct {
	double ms_width;       /* width kernel (exact path: its read-packing pre-pass), HIP events */
	double ms_search;      /* search kernel (first pass; exact path: k_exact alone) */
	double ms_retry;       /* large-capacity retry pass (0 if none) */
	double ms_total;       /* ibwa_batch_run wall, device-synchronised */
	int64_t n_retry;       /* reads re-run in the large-capacity pass */
	int64_t n_launch_width, n_launch_search;
	int path;              /* 0: width + general search; 1: exact-match path (max_diff == 0);
	                          2: width + persistent gapped search; 3: exact path with the
	                          unique-interval jump (index built by ibwa_ctx_build_index) */
	int kmer_k;            /* K of the K-mer interval table the exact path used (0: none) */
	int64_t n_stack_overflow;  /* first-pass reads whose stack did not fit (re-run) */
	int64_t n_aln_overflow;    /* first-pass reads whose hits did not fit (re-run) */
	int64_t n_heavy;           /* first-pass reads over the iteration budget (re-run) */
	double ms_sw;              /* last ibwa_sw_batch kernel time */
	int64_t n_coop;            /* heavy reads the wave-cooperative pass resolved */
	double ms_coop;            /* its time (width + search), part of ms_retry */
	double ms_sa2pos;          /* last ibwa_sa2pos kernel time */
	int sa2pos_full;           /* 1: it gathered from a full SA, 0: it walked the sampled SA */
	double ms_coop_width;      /* of ms_coop: the heavy reads' widths (k_width) */
	double ms_coop_roots;      /* of ms_coop: their level 0 (k_coop_roots); the rest is k_coop */
	int64_t n_resumed;         /* heavy reads handed on with their search state (the cooperative
	                              pass resumes them instead of starting over) */
	int64_t resume_records;    /* 16 B records those states took (requested, incl. any that did not fit);
	                              the cooperative pass runs them chunk by chunk (part of ms_coop) */
	int64_t resume_records_peak; /* the most records one first-pass chunk's states requested (the
	                              state buffer holds one chunk's states at a time) */
	int64_t resume_records_cap;  /* the state buffer's capacity in 16 B records */
	int64_t coop_pages_peak;     /* the most bucket pages one cooperative launch took from its pool */
	int64_t coop_pages_cap;      /* the largest launch's pool in pages (COOP_PG 16 B entries each) */
	double ms_alloc;             /* wall time the run spent allocating device buffers (hipMalloc) */
} ibwa_run_stats_t;
int ibwa_batch_stats(const ibwa_ctx_t *ctx, ibwa_run_stats_t *st);

/* Named engine options:
 *   "exact_path" (0/1, default 1)  exact-match kernel when max_diff == 0
 *   "exact_jump" (0/1, default 1)  keep full SA / ISA / text at ibwa_ctx_build_index and let
 *                                  the exact path jump over a unique interval's remaining symbols
 *   "jump_derive" (0/1, default 1) for an index loaded from .bwt files, derive those arrays on
 *                                  the device from the BWT at the first -n 0 batch (HBM permitting)
 *   "width_jump" (0/1/2, default 1) k_width steps one-row intervals from the 2-bit text
 *                                  (1: when those arrays are resident; 2: derive them for a
 *                                  gapped batch too; 0: Occ steps only) -- same widths
 *   "width_tab" (0/1, default 1)   k_width takes a chain's first steps (up to gap_tab_k + 1) from
 *                                  the level tables, one round trip for all -- same widths
 *   "kmer_k" (-1 auto, 0 off, 1..16) K-mer interval table length
 *   "gap_tab_k" (-1 auto, 0 off, 1..14) level tables of the first pass: the SA interval of every
 *                                  string of length <= K + 1 per strand; nodes at depth <= K are
 *                                  stored by their strings and expanded from one 32 B load (auto:
 *                                  floor(log4(n)) up to 13, 14 when both tables fit 15 % of the free
 *                                  HBM; the CLI pins 13) -- same hits
 *   "exact_blocks", "lanes_per_chunk"
 *   "gapped_v2" (0/1, default 1)   persistent gapped-search kernel (else the general kernels)
 *   "gap_cap1", "gap_pages_per_block", "gap_hit_slots", "gap_blocks_per_cu", "gap_reads_per_chunk"
 *                                  its per-lane static slots, 128 KiB pages per workgroup pool,
 *                                  first-pass hit slots, residency and batch slice size
 *   "gap_lw" (0/1, default 1), "gap_lw_min_waves" (8)  first pass with its width records in LDS
 *                                  (and resume states), in the workgroup size that keeps the most
 *                                  waves per CU (100 bp: 12, 150 bp: 9) when that is at least the minimum
 *   "gap_iter_budget" (8000)       first-pass iterations before a read goes to the cooperative pass
 *   "gap_early_iters", "gap_early_entries" (3000, 1000)
 *                                  earlier hand-off of a read whose stack holds that many entries
 *   "gap_resume" (0/1, default 1), "gap_resume_gb" (48)  an early hand-off leaves the read's search
 *                                  state (at the next score-level boundary) for the cooperative pass,
 *                                  which resumes it instead of starting over; state buffer size cap
 *                                  ("gap_resume_records": the buffer in 16 B records, for tests)
 *   "gap_resume_recs" (192)        state buffer records per read of a first-pass chunk, or 1.15 x the
 *                                  most an earlier run of the context needed, if more (states that do
 *                                  not fit start over in the cooperative pass: same hits)
 *   "gap_resume_iters", "gap_resume_entries" (2000, 300)  the early hand-off rule when states are left
 *   "gap_resume_ppb" (48), "gap_resume_cap1" (4096)  first-pass pool pages per 256 lanes and static
 *                                  slots per lane when states are left (at most the values above)
 *   "gap_tail_lanes", "gap_tail_iters" (16, 200)  also leave a state when no read is left to claim and
 *                                  at most that many lanes of the wave are busy (0: off)
 *   "coop_waves_per_cu" (12), "coop_pool_gb" (16)  cooperative pass residency and page pool (reads
 *                                  that run out of its pages run again in up to two more launches with
 *                                  the whole pool, then the wide kernel; "coop_pool_pages": the pool
 *                                  in pages, for tests)
 *   "coop_stg_room" (1)            its per-lane staging ring holds this many chains' children (1..4)
 *   "coop_roots" (0/1, default 1)  level 0 of the heavy reads one root chain per lane (k_coop_roots)
 *   "gap_coop" (0/1, default 1)    the cooperative pass (0: heavy reads go to the wide kernel)
 *   "sa_walk" (0/1, default 0)     SA -> coordinate by walking the sampled SA even when the full SA is
 *                                  resident
 *   Test and diagnostics hooks: "gap_stream_per_read" (4), "gap_stream_min" (1 << 20) the first
 *   pass's hit-stream size; "gap_resume_records", "coop_pool_pages" buffer sizes in records / pages;
 *   "diag" (0) per-read iterations and k_width features; "sw_stop" (0) stop k_sw after a pass. */
int ibwa_ctx_set_option(ibwa_ctx_t *ctx, const char *key, long value);

/* The sources this library was built from: the first 16 hex digits of the SHA-256 of the
 * ibwa_amd/csrc/ sources (cpp, h, hip) followed by the include/ headers, each list in byte order of
 * the file names (no reference counterpart; the Python loader refuses a stale build). */
const char *ibwa_build_id(void);

/*
 * The `aln` command line (bwa_aln's getopt loop, bwtaln.c:249-284; same option string and
 * semantics, plus -G INT = number of GPUs) into *opt, starting from gap_init_opt's defaults.
 * argv[0] is the command name.  Returns the index of the first positional argument, -1 on an
 * unknown option.  n_gpus / fn_out (-f) may be NULL.  Thread-safe (getopt is serialised).
 */
int ibwa_aln_parse_args(int argc, char *const *argv, ibwa_gap_opt_t *opt, int *n_gpus, const char **fn_out);

/*
 * Reads of the last ibwa_batch_run that the first pass handed on, and the pass that resolved
 * each: 1 the wave-cooperative pass (coop.hip), 2 the sequential wide pass (gapped.hip, one
 * read per wave), 3 the general kernels (aln.hip), 4 the wave-cooperative pass resuming the first
 * pass's search state (after the read's chunk).  Writes min(cap, n) entries; *n = their count.
 */
int ibwa_batch_retry_info(const ibwa_ctx_t *ctx, int64_t *ids, uint8_t *pass, int64_t cap, int64_t *n);

/* Diagnostics of the last ibwa_batch_run with option "diag" = 1 (gapped path): what 0 = first-pass
 * iterations per read (uint32[n]); 1 = k_width's search-cost features per read (uint16[n][4]:
 * sum of log2 width over both full-length chains, the same over the seed chains, the smaller
 * restart count of the two full chains, of the two seed chains).  what 2 (no option needed): per
 * read the pops (bwtgap.c:129) the first pass made before leaving its resume state, 0 if it left
 * none (uint32[n]): the point where the read's search moves from k_gapped to k_coop. */
int ibwa_batch_diag(const ibwa_ctx_t *ctx, int what, void *out, uint64_t cap_bytes);

/* Tuning knobs (0 = default): per-lane stack entries, per-read hit slots, block size */
int ibwa_ctx_set_tuning(ibwa_ctx_t *ctx, int stack_cap, int aln_cap, int block);

/*
 * On-device index construction (bwa_index, bwtindex.c:42-186, for the BWT
 * part): `codes` is the packed reference (.pac content, one 2-bit code per
 * byte, N already replaced as bns_fasta2bntseq does -- see ibwa_pack_nt4),
 * n < 2^32 - 1.  Builds .bwt (text) and .rbwt (reversed text, bwtmisc.c:160)
 * straight into HBM; the result is bit-identical to `bwa index`.
 * sa_intv > 0 also keeps the sampled suffix arrays (.sa/.rsa, bwt_cal_sa).
 */
int ibwa_ctx_build_index(ibwa_ctx_t *ctx, const uint8_t *codes, uint64_t n, int sa_intv);
/* Geometry of a resident index: primary, L2[1..4], and bwt_size (reference words). */
int ibwa_ctx_bwt_info(const ibwa_ctx_t *ctx, int strand, uint32_t *primary, uint32_t L2[4], uint64_t *bwt_size);
/* Export a resident index in the reference's interleaved .bwt word layout
 * (bwt_dump_bwt, bwtio.c:7-15, after bwt_bwtupdate_core): words[bwt_size]. */
int ibwa_ctx_export_bwt(const ibwa_ctx_t *ctx, int strand, uint32_t *words, uint64_t cap);
/* Export the sampled SA kept by ibwa_ctx_build_index: out[(n+intv)/intv] with out[0] = (u32)-1
 * (bwt.c:56-66); entries 1.. are what bwt_dump_sa writes. */
int ibwa_ctx_export_sa(const ibwa_ctx_t *ctx, int strand, uint32_t *out, uint64_t cap);

/*
 * Batched Smith-Waterman with path: aln_local_core (stdaln.c:529-760) with
 * aln_param_bwa and _thres = 1, as bwa_sw_core (bwasw.c:51) calls it for each
 * mate rescue, plus aln_path2cigar32 (stdaln.c:1010-1040).  Pair p aligns
 * seq1 = ref[off1[p] .. +len1[p]) (the reference window) against seq2 =
 * qry[off2[p] .. +len2[p]) (the read), codes 0..4.  Per pair: score (-1 if a
 * length is 0), path_len, ends[4p..4p+3] = start i, start j, end i, end j
 * (1-based, path[path_len-1] and path[0]), n_cigar; *cigar = malloc'd
 * concatenation of all CIGARs (len << 4 | op, op 0 M, 1 I, 2 D; ibwa_free).
 * Requires min(len1, len2) * 11 <= 32000 (the reference's score rebasing is
 * then unreachable); IBWA_EINVAL otherwise.
 */
int ibwa_sw_batch(ibwa_ctx_t *ctx, int64_t n, const uint8_t *ref, const uint64_t *off1, const uint32_t *len1,
                  const uint8_t *qry, const uint64_t *off2, const uint32_t *len2, int32_t *score,
                  int32_t *path_len, int32_t *ends, int32_t *n_cigar, uint32_t **cigar, int64_t *n_cigar_total);

/*
 * SA -> coordinate.
 *
 * ibwa_ctx_load_sa: make a sampled suffix array device-resident, as
 * bwt_restore_sa (bwtio.c:29-49) loads it into bwt_t: sa[0..n_sa) with
 * sa[0] = (u32)-1, n_sa = (seq_len + sa_intv) / sa_intv; strand 0 = prefix.sa,
 * 1 = prefix.rsa.  ibwa_ctx_load_sa_file reads the .sa/.rsa file itself and
 * applies bwt_restore_sa's primary / seq_len consistency checks (IBWA_EINVAL).
 * An index built by ibwa_ctx_build_index(sa_intv > 0) already has both.
 *
 * ibwa_ctx_expand_sa: derive the full SA of both strands on the device from
 * the sampled ones (one LF walk per sampled row, seq_len steps in all;
 * 2 x 4 B per base of HBM) so that ibwa_sa2pos is one gather per hit.
 *
 * ibwa_sa2pos: bwtdb_sa2seq (dbset.c:240-246) over n hits, i.e. bwt_sa
 * (bwt.c:69-79) on bwt[0] for strand 1 and seq_len - (bwt_sa(bwt[1], k) + len)
 * (u32 arithmetic) for strand 0, plus `offset` (bwtdb_t.offset; 0 for a single
 * database).  Replaces the per-hit calls of bwa_cal_pac_pos (bwase.c:133,
 * :146, :157), bwa_cal_pac_pos_pe (bwape.c:347, :400) and saiset.c:136, :147.
 * Uses the full SA when resident (option "sa_walk" = 1 forces the walk).
 */
int ibwa_ctx_load_sa(ibwa_ctx_t *ctx, int strand, uint32_t sa_intv, const uint32_t *sa, uint64_t n_sa);
int ibwa_ctx_load_sa_file(ibwa_ctx_t *ctx, int strand, const char *path);
int ibwa_ctx_expand_sa(ibwa_ctx_t *ctx);
/* The sampled SA of both strands (bwt_cal_sa's values at interval sa_intv, what `bwa index`
 * writes to .sa / .rsa, bwt.c:48-67) derived on the device from the resident BWT alone. */
int ibwa_ctx_derive_sa(ibwa_ctx_t *ctx, uint32_t sa_intv);
int ibwa_sa2pos(ibwa_ctx_t *ctx, int64_t n, const uint8_t *strand, const uint32_t *k, const uint32_t *len,
                uint64_t offset, uint64_t *pos);

/*
 * Batched banded global alignment: aln_global_core (stdaln.c:345-525) with aln_param_bwa's
 * scores (gap open 26, extend 9, aln_sm_maq) and the given band_width / gap_end, as
 * refine_gapped_core (bwase.c:167-199) calls it with band 50, gap_end 5 for each gapped read.
 * Pair p aligns seq1 = ref[off1[p] .. +len1[p]) against seq2 = qry[off2[p] .. +len2[p]).
 * Per pair: score (0 and path_len 0 if a length is 0), path_len, n_cigar; *cigar = malloc'd
 * concatenation of the CIGARs in aln_path2cigar32 encoding (len << 4 | op: 0 M, 1 I, 2 D).
 */
int ibwa_global_batch(ibwa_ctx_t *ctx, int64_t n, const uint8_t *ref, const uint64_t *off1, const uint32_t *len1,
                      const uint8_t *qry, const uint64_t *off2, const uint32_t *len2, int band, int gap_end,
                      int32_t *score, int32_t *path_len, int32_t *n_cigar, uint32_t **cigar, int64_t *n_cigar_total);

/* Device Occ KAT: bwt_occ4 (bwt.c:157) for n positions k[] on strand s -> cnt[4*n] */
int ibwa_occ4(ibwa_ctx_t *ctx, int strand, int64_t n, const uint32_t *k, uint32_t *cnt);

#ifdef __cplusplus
}
#endif
#endif
