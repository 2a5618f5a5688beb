// engine.h -- internal device/host interface of the aln engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "occ.h"

namespace ibwa {

constexpr uint32_t NIL = 0xFFFFFFFFu;
constexpr uint32_t ST_STACK_OVERFLOW = 1u;  // per-lane stack capacity exceeded -> retry pass
constexpr uint32_t ST_ALN_OVERFLOW = 2u;    // per-read hit slots exceeded      -> retry pass
constexpr uint32_t ST_BAD_SCORE = 4u;       // score outside [0, n_stacks): invalid options
constexpr uint32_t ST_HEAVY = 8u;           // iteration budget of the first pass exceeded -> retry pass

// Batch-level `local_opt` of bwa_cal_sa_reg_gap (bwtaln.c:86-93) as the kernels see it.
struct AlnOpt {
  int s_mm, s_gapo, s_gape, mode;
  int indel_end_skip, max_del_occ, max_entries;
  int fnr_pos;    // opt->fnr > 0: max_diff is per read length (maxdiff_tab)
  int max_diff;   // opt->max_diff when !fnr_pos
  int max_gapo;   // already clamped to the batch max_diff (bwtaln.c:92)
  int max_gape, max_seed_diff, seed_len, max_top2;
  int n_stacks;   // gap_init_stack size (bwtgap.c:18)
};

struct AlnArgs {
  IndexView ix[2];           // ix[0] = .bwt, ix[1] = .rbwt
  const uint8_t *seq;        // bwa_seq_t.seq arrays (read reversed), concatenated
  const uint64_t *off;
  const uint32_t *len;
  const int64_t *ids;        // lane -> read id (nullptr: identity)
  int64_t n;                 // lanes in this launch
  const int16_t *maxdiff_tab;  // [len] -> bwa_cal_maxdiff(len, 0.02, fnr)
  uint2 *wbuf;               // per-lane width arrays {w, bid}
  uint64_t wstride;          // entries per lane
  uint32_t wlen1;            // batch max_len + 1
  uint32_t *heads;           // per-lane bucket heads [n_stacks]
  uint4 *ent;                // per-lane stack entries [cap]
  uint32_t *prev;            // per-lane links [cap]
  uint32_t cap;
  uint4 *aln;                // per-lane hits [aln_cap] (bwt_aln1_t as uint4)
  int32_t *n_aln;            // per lane
  uint32_t aln_cap;
  uint32_t *status;          // per lane ST_* flags
  uint16_t *nN;              // per lane N count (k_width output, may be null)
  uint16_t *feat;            // per lane 4 search-cost features (k_width output, diagnostics, may be null)
  // compact per-read record for the first gapped pass's LDS (k_width output, may be null), cw_words
  // u32 per lane: [0] len | min(nN, 255) << 16 | max_diff << 24; [1, 1 + cw_rw) the read, 16 bases
  // per word; then bytes: per position p <= len the bids of both strands clamped to max_diff + 1
  // (3 bits) and "width equals the previous position's" (1 bit), nibble per strand; then per seed
  // position the same with the bid clamped to max_seed_diff + 1 (2 bits + 1 bit per strand)
  uint32_t *cw;
  uint32_t cw_words, cw_rw;
  // k_width's one-row steps from the text (full SA and 2-bit text per strand, as the exact
  // path's jump); nullptr: every step reads the Occ blocks
  const uint32_t *jsa[2];
  const uint32_t *jtxt[2];
  // the first pass's level tables (GapArgs::ltab): k_width takes a chain's first min(len, tab_k + 1,
  // 15) steps from them; nullptr: off
  const uint2 *ltab[2];
  uint32_t tab_k;
  AlnOpt o;
};

// Kernel arguments of the persistent gapped search (gapped.hip).
struct GapArgs {
  IndexView ix[2];
  const uint4 *o64[2];       // bit-plane Occ blocks (occ64.hip)
  const uint8_t *seq;
  const uint64_t *off;
  const uint32_t *len;
  const int64_t *ids;        // read r of this launch -> input read (nullptr: identity)
  int64_t n;
  int out_by_id;             // outputs indexed by ids[r] (else by r)
  const int16_t *maxdiff_tab;
  uint2 *wbuf;               // widths of read r at wbuf + r * wstride (k_width)
  uint64_t wstride;
  uint32_t wlen1;
  const uint16_t *nN;        // per read N count (k_width)
  uint4 *ent;                // per-lane static slot regions, cap1 slots each
  uint32_t cap1;
  uint32_t hit_slots;        // the last hit_slots static slots hold the read's hits
  uint4 *pool;               // per-workgroup page pools: pages_per_block pages of 2^page_log2 slots
  uint32_t page_log2;
  int max_pages;             // pages a lane may hold
  int pages_per_block;
  uint4 *aln;                // hit stream (bwt_aln1_t as uint4), aln_total slots
  unsigned long long aln_total;
  unsigned long long *aln_next;  // stream fill counter (zeroed once per batch)
  uint64_t *aln_off;         // per read: first hit in the stream
  int32_t *n_aln;
  uint32_t *status;
  uint32_t *iters;           // optional: loop iterations per read (diagnostics)
  unsigned long long *prof;  // optional: per-phase cycle counters [8] (diagnostics kernel)
  uint32_t max_iters;        // iteration budget per read (0: none); over it -> ST_HEAVY
  uint32_t early_iters;      // early hand-off: past this many iterations (0: off) a read whose
  uint32_t early_entries;    //   stack holds more than early_entries entries -> ST_HEAVY
  int lanes_per_wave;        // reads a wave runs at once (64; 1 for heavy reads)
  int free_depth;            // LDS free-slot stack per read (wide kernel)
  // LDS-resident widths (first pass, when they fit): the k_width records (AlnArgs::cw) copied into
  // LDS at a read's claim; 16 bucket heads in a ring; the page table of a lane in global memory
  const uint32_t *cw;        // nullptr: widths from wbuf, heads per bucket, page table in LDS
  uint32_t cw_words, cw_rw;
  uint16_t *ptab_g;          // [lane][GAP_MAX_PAGES]
  // Resume (LDS-width variant): a read past an early hand-off rule runs on to the next score-level
  // boundary and leaves its search state for the cooperative pass instead of being re-run from the
  // start there.  rdump: the states, RD_HDR header records + the live entries in slot order + the
  // hits; rd_next / rd_cap: fill counter and capacity (16 B records); roff[read]: 1 + the state's
  // first record (0: none).  nullptr: every hand-off re-runs from the start.
  uint4 *rdump;
  unsigned long long *rd_next;
  unsigned long long rd_cap;
  uint64_t *roff;
  uint32_t *hpop;            // optional: per read, the pops (bwtgap.c:129) made before its state was left
  uint32_t tail_lanes;       // resume also when no read is left to claim and <= tail_lanes of the wave
  uint32_t tail_iters;       //   are busy, for a read past tail_iters iterations (0: off)
  // Level tables (LW first pass; kmer.hip build_level_tables): per BWT the SA interval of every string
  // of length <= tab_k + 1.  A node at depth <= tab_k is stored by its string (x = code, y = LTAB_MARK |
  // depth) and expanded from one 32 B load of its children's intervals instead of two Occ blocks.
  const uint2 *ltab[2];
  uint32_t tab_k;            // 0: off (resume states leave with intervals: the cooperative pass has no tables)
  AlnOpt o;
};
constexpr uint32_t LTAB_MARK = 0xFFFFFF00u;  // y >= this: a node stored by its string (no l can be: seq_len < it)
constexpr int RD_HDR = 2;  // resume state header: {entries, hits, lowest score, stack size}, {best_score, best_cnt, max_diff, pops}
constexpr int GAP_RING = 16;      // bucket heads of the LDS-width variant: live scores span <= 16
constexpr int GAP_MAX_PAGES = 8;  // page-table entries per lane (global table)
size_t gapped_lds_bytes(int n_stacks, int block, bool wide, int max_pages, int pages_per_block, int lanes_per_wave,
                        int free_depth, int cw_words = 0);
// wide: 24-bit slot links (reads < 4096 bp), for the large-capacity retry pass
hipError_t launch_gapped(const GapArgs &g, unsigned long long *d_counter, int blocks, int block, bool wide,
                         hipStream_t st);

// Wave-cooperative gapped search for heavy reads (coop.hip): one read per wavefront,
// its match chains run across the lanes and committed in the reference's pop order.
constexpr int COOP_MAXLEN = 256;       // longest read the kernel takes (LDS strands / widths)
constexpr int COOP_SEEDMAX = 64;       // longest seed (-l) of a seeded read it takes (LDS seed widths)
constexpr int COOP_PG_LOG2 = 13;       // bucket pages of 8192 entries (128 KiB): 256 pages hold 2M entries
constexpr uint32_t COOP_PG = 1u << COOP_PG_LOG2;
constexpr int COOP_NSTK = 128, COOP_MAXP = 256;
constexpr int COOP_RREC = 256;          // chain records in flight (ring)
struct CoopArgs {
  IndexView ix[2];
  const uint4 *o64[2];
  const uint8_t *seq;
  const uint64_t *off;
  const uint32_t *len;
  const int64_t *ids;        // read r of this launch -> input read (nullptr: identity)
  int64_t n;
  int out_by_id;
  const int16_t *maxdiff_tab;
  const uint2 *wbuf;         // widths of read r at wbuf + r * wstride (k_width)
  uint64_t wstride;
  uint32_t wlen1;
  const uint16_t *nN;
  uint4 *stg;                // per-lane staging rings, 2^stg_log2 entries each, 64 lanes per wave
  uint32_t stg_log2;
  uint32_t *dir;             // per-wave page directories [COOP_NSTK][COOP_MAXP]
  uint32_t *freel;           // per-wave free page stacks [freecap]
  uint32_t freecap;
  uint4 *pool;               // bucket pages (COOP_PG entries each)
  uint32_t pool_pages;
  uint32_t *pool_next;       // global bump pointer into the pool (zeroed per launch)
  uint4 *hits;               // per-wave hit lists [hcap]
  uint4 *recb;               // per-wave hit records of the chain ring [COOP_RREC] (read only at a hit)
  uint32_t hcap;
  uint32_t max_iters;        // runaway guard (loop iterations per read)
  uint4 *aln;                // hit stream
  unsigned long long aln_total;
  unsigned long long *aln_next;
  uint64_t *aln_off;
  int32_t *n_aln;
  uint32_t *status;
  uint32_t *iters;
  unsigned long long *prof;  // diagnostics: per-phase wave cycles (IBWA_PROF_PHASES), may be null
  unsigned long long *wave_t;  // diagnostics: per wave {start, end} shader clock (with prof)
  uint4 *proot;              // root chain records of k_coop_roots [2 n] (nullptr: k_coop runs level 0)
  uint4 *pstore;             // their children, compact
  unsigned long long *pstore_next;  // bump pointer into pstore (entries)
  uint64_t pstore_cap;       // pstore capacity (entries)
  const uint4 *rdump;        // first-pass search states (GapArgs::rdump), roff[read] 1 + offset, 0: none
  const uint64_t *roff;
  // resume_fixup folded in (non-null): as a read ends, fix_status[id] = 0 where it was resolved, else
  // fix_roff[id] = 0 -- no kernel after the launch that would wait for CUs another grid holds
  uint32_t *fix_status;
  uint64_t *fix_roff;
  // >= 0: the widths and N counts are the first pass's own, of read (id - wb_base) of its chunk (right
  // after it: its gap_shadow updates are in them, so a resumed read does not replay them); -1: per
  // launch read (k_width run for this launch)
  int64_t wb_base;
  AlnOpt o;
};
hipError_t launch_coop(const CoopArgs &g, unsigned long long *d_counter, int blocks, hipStream_t st);
// level 0 of the heavy reads, one root chain per lane (g.proot / g.pstore set), before launch_coop
hipError_t launch_coop_roots(const CoopArgs &g, unsigned long long *d_counter, int blocks, hipStream_t st);
// ids (in input order) and statuses of the reads whose status is non-zero (select.hip); tmp == nullptr
// only sizes the rocPRIM scratch into *tmp_bytes
hipError_t select_handed_on(const uint32_t *status, int64_t n, int64_t *ids, uint32_t *sel_status,
                            unsigned long long *d_count, void *tmp, size_t *tmp_bytes, hipStream_t st);
// ids (base + i, in order) and statuses of the reads in [base, base + n) that left a resume state
// (roff != 0); tmp == nullptr only sizes the scratch
hipError_t select_resumed(const uint64_t *roff, int64_t base, int64_t n, const uint32_t *status, int64_t *ids,
                          uint32_t *sel_status, unsigned long long *d_count, void *tmp, size_t *tmp_bytes,
                          hipStream_t st);
// after a cooperative launch over resumed reads ids[0, n): status[id] = 0 where it resolved the read,
// else roff[id] = 0 (the read starts over in the later passes)
hipError_t resume_fixup(const uint32_t *r_status, const int64_t *ids, int64_t n, uint32_t *status, uint64_t *roff,
                        hipStream_t st);
// the order in which the cooperative pass takes the handed-on reads: largest first-pass stack first
// (status bits 16-31); idx[0, n) gets the permutation of the selection, ids_out the ids in that order
hipError_t order_heavy_first(const uint32_t *sel_status, const int64_t *ids, unsigned long long n, uint32_t *keys,
                             uint32_t *idx, int64_t *ids_out, void *tmp, size_t *tmp_bytes, hipStream_t st);

// Kernel arguments of the exact-match path: only what it reads (fewer SGPRs).
struct ExactArgs {
  IndexView ix[2];
  const uint8_t *seq;
  const uint64_t *off;
  const uint32_t *len;
  int64_t n;
  uint4 *aln;
  int32_t *n_aln;
  uint32_t *status;
  uint32_t aln_cap;
  int mode;
  const uint2 *kt0, *kt1;  // K-mer interval tables of .bwt / .rbwt (kmer.hip), or null
  int K;                   // K-mer length (0: no table)
  const uint4 *o64[2];     // bit-plane Occ layouts (occ64.hip)
  // unique-interval jump (optional): full SA / ISA and the 2-bit text of each strand's index
  const uint32_t *sa[2], *isa[2], *txt[2];
  int jump;
};

// Batched local alignment with path (sw.hip).
struct SwArgs {
  const uint8_t *seq1, *seq2;     // reference windows / reads, codes 0..4
  const uint64_t *off1, *off2;
  const uint32_t *len1, *len2;
  int64_t n;
  int max_len1, max_len2;         // size the per-lane scratch
  uint32_t *scratch;              // sw_words_per_lane(max_len1) u32 per lane, lane-minor per wave
  uint64_t words_per_lane;
  uint8_t *tb;                    // sw_tb_per_lane bytes per lane, lane-minor per wave
  uint64_t tb_per_lane;
  int32_t *score, *path_len, *n_cigar;
  int4 *ends;                     // start_i, start_j, end_i, end_j (1-based, stdaln path_t)
  uint32_t *cigar;                // cigar_cap per pair, aln_path2cigar32 encoding (len << 4 | op)
  int cigar_cap;
  int stop_after;                 // diagnostics: 1 after the forward pass, 2 after the reverse pass
  int global_band;                // > 0: aln_global_core alone with this band (and gap_end), no local passes
  int gap_end;
};
hipError_t launch_sw(const SwArgs &a, unsigned long long *d_counter, int blocks, hipStream_t st);
// row p's n_cigar[p] CIGAR words (at cig + p * cap) to out + first[p]
hipError_t launch_pack_cigar(const uint32_t *cig, int cap, const int32_t *n_cigar, const uint64_t *first, int64_t n,
                             uint32_t *out, hipStream_t st);
uint64_t sw_words_per_lane(int max_len1, int max_len2);
uint64_t sw_tb_per_lane(int max_len1, int max_len2);

// SA row -> coordinate (sa2pos.hip): bwt_sa (bwt.c:69-79) inside bwtdb_sa2seq (dbset.c:240-246).
struct SaArgs {
  IndexView ix[2];           // ix[0] = .bwt (strand-1 hits), ix[1] = .rbwt (strand-0 hits)
  const uint32_t *sa[2];     // sampled SA (walk) or full SA (gather) of each index
  uint32_t intv[2];          // sampling interval of each sampled SA
  const uint8_t *strand;     // bwt_aln1_t.a of each hit
  const uint32_t *k, *len;   // SA row and read length of each hit
  int64_t n;
  uint64_t offset;           // bwtdb_t.offset
  uint64_t *pos;             // out
  uint32_t *steps;           // optional out: LF steps of each walk
};
hipError_t launch_sa2pos(const SaArgs &a, bool full, hipStream_t st);
hipError_t expand_sa(const IndexView &ix, const uint32_t *sa_s, uint32_t intv, uint32_t *full, hipStream_t st);
// sampled SA (bwt_cal_sa's values, interval intv) from the BWT alone; tmp: 4 * (n / intv + 1) + 1 words
hipError_t derive_sampled_sa(const IndexView &ix, uint32_t intv, uint32_t *sa_s, uint32_t *tmp, hipStream_t st);
// ISA (seq_len + 1 words) and the 2-bit text from a full SA (full[0] = -1)
hipError_t derive_isa_text(const IndexView &ix, const uint32_t *full, uint32_t *isa, uint32_t *txt2, uint64_t txt_words,
                           hipStream_t st);

hipError_t build_kmer_table(const IndexView &ix, int K, uint2 *table, uint2 *tmp, hipStream_t st);
// first index of level d of a level table: (4^d - 1) / 3 rounded up to a multiple of 4 (level d >= 1 then
// starts 32 B-aligned, so a node's four children are one aligned 32 B load)
__host__ __device__ inline uint64_t ltab_off(uint32_t d) { return d == 0 ? 0ull : ((1ull << (2 * d)) - 1) / 3 + 3; }
hipError_t build_level_tables(const IndexView &ix, int levels, uint2 *t, hipStream_t st);

hipError_t relayout_reference_bwt(const uint32_t *d_ref, uint64_t n_words, uint64_t n_blocks, uint4 *d_out,
                                  hipStream_t st);
hipError_t pack_blocks(const uint32_t *d_sym, uint64_t n_sym_words, const uint4 *d_block_base, uint64_t n_blocks,
                       uint4 *d_out, hipStream_t st);
hipError_t launch_width(const AlnArgs &a, int block, hipStream_t st);
hipError_t launch_search(const AlnArgs &a, int block, hipStream_t st);
hipError_t launch_exact(const AlnArgs &a, const uint4 *o64_0, const uint4 *o64_1, const uint2 *kt0,
                        const uint2 *kt1, int K, uint4 *rec, uint32_t stride, unsigned long long *d_counter,
                        int blocks, hipEvent_t ev_mid, const uint32_t *const jump[6], hipStream_t st);
uint64_t occ64_blocks(uint32_t seq_len);
hipError_t build_occ64(const IndexView &ix, uint4 *out, hipStream_t st);
// bytes of zeros to device memory on stream st by the copy engine (from pinned host zeros): a
// hipMemsetAsync is a kernel, which waits for CUs that another context's persistent grid holds
hipError_t zero_async(void *p, size_t bytes, hipStream_t st);
uint32_t exact_record_stride(int max_len);
hipError_t launch_occ4(const IndexView &ix, int64_t n, const uint32_t *k, uint32_t *cnt, hipStream_t st);
hipError_t build_strand(const uint8_t *T, uint64_t n, uint4 *out_blocks, uint32_t *primary, uint32_t totals[4],
                        uint32_t *sa_sample, uint32_t sa_intv, int *rounds, uint32_t *sa_full, uint32_t *isa_full,
                        hipStream_t st);
hipError_t pack_text2(const uint8_t *T, uint64_t n, uint32_t *out, uint64_t out_words, hipStream_t st);
hipError_t reverse_text(uint8_t *T, uint64_t n, hipStream_t st);

// FASTQ ingest on the device (fastq.hip): strict 4-line records of a raw block -> kept reads
constexpr int FQ_MIN_RDLEN = 35;  // BWA_MIN_RDLEN (bwtaln.h:23): bwa_trim_read keeps at least this
struct FqOpt {
  int l_bc;       // -B barcode length (mode >> 24)
  int trim_qual;  // -q
  int is_64;      // -I: qualities - 31 before trimming
};
struct FqBufs {
  const uint8_t *raw;   // the block, fq_padded_bytes(n) bytes, zero past n
  uint32_t *tile_cnt, *tile_base;
  uint32_t *nl;         // newline positions, cap_lines entries
  uint32_t cap_lines;
  uint32_t *n_lines;    // lines found (at most cap_lines)
  uint32_t *bad;        // first record that is not strict (0xFFFFFFFF: none)
  int32_t *rec_len;     // per record (cap_lines / 4 + 1): kept length, -1 skipped or not strict
  uint32_t *rec_L;      // per record: sequence line length (0: not strict)
  uint64_t *rec_key;    // per record: kept rank << 32 | code offset (exclusive scan; the block is < 4 GiB)
  uint8_t *codes;       // kept reads' reversed nt4 codes, concatenated
  uint64_t *offk;       // per kept read: code offset
  uint32_t *lenk;       // per kept read: length
};
uint64_t fq_padded_bytes(uint64_t n);
constexpr uint32_t FQ_PAD_MAX = 16384;  // fq_padded_bytes(n) - n <= 2 * FQ_PAD_MAX (one tile + the rounding)
// tmp == nullptr: *tmp_bytes = the scans' scratch size
// h_init (pinned host, may be null): {0, 0xFFFFFFFF} for the line and first-bad counters, copied in
// instead of two memsets (a memset is a kernel, which waits for CUs another context's grid holds)
hipError_t fq_parse_launch(const FqBufs &b, uint64_t n, const FqOpt &o, void *tmp, size_t *tmp_bytes, hipStream_t st,
                           const uint32_t *h_init = nullptr);

}  // namespace ibwa
