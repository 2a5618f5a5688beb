// engine.hip -- host side of the C ABI in include/ibwa_aln.h.
//
// Replaces, per batch, the pthread fan-out of bwa_aln_core (bwtaln.c:199-218)
// and the per-thread scratch of bwa_cal_sa_reg_gap (bwtaln.c:88-97, 139) with
// one HIP launch grid over the batch and HBM-resident per-lane scratch.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <chrono>
#include <string>
#include <vector>

#include "engine.h"
#include "ibwa_aln.h"

using namespace ibwa;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                                                    \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) return fail(IBWA_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
  } while (0)

// hipMalloc wall time of this thread (a run reports what it spent: ibwa_run_stats_t.ms_alloc)
thread_local double g_alloc_ms = 0;
// Device bytes the library's buffers hold (all contexts of the process) and their high-water mark.
std::atomic<int64_t> g_dev_bytes{0}, g_dev_peak{0};
void dev_bytes_add(int64_t d) {
  const int64_t now = g_dev_bytes.fetch_add(d) + d;
  int64_t pk = g_dev_peak.load();
  while (now > pk && !g_dev_peak.compare_exchange_weak(pk, now)) {
  }
}

// Device arena (ibwa_reserve): one hipMalloc per device, made once, from which every buffer of the
// process's contexts on that device is carved (first fit, 4 KiB granules, freed ranges coalesce).
// A hipMalloc right after another process released a lot of HBM waits until the driver has wiped
// that memory (measured: 0.5-2.7 s for single allocations of `aln` end 2, profiles/r05_alloc.jsonl);
// a CLI that reserves its arena while it loads the index pays that once, overlapped, instead of in
// the middle of its first groups.  Without a reservation buffers are plain hipMallocs.
struct Arena {
  std::mutex mu;
  char *base = nullptr;
  size_t size = 0, used = 0, peak = 0;
  std::map<size_t, size_t> free_;  // offset -> bytes
  const bool trace = getenv("IBWA_ARENA_TRACE") != nullptr;  // every carve and release, on stderr
  void *alloc(size_t n) {
    n = (n + 4095) & ~(size_t)4095;
    std::lock_guard<std::mutex> lk(mu);
    for (auto it = free_.begin(); it != free_.end(); ++it) {
      if (it->second < n) continue;
      const size_t off = it->first, rest = it->second - n;
      free_.erase(it);
      if (rest) free_[off + n] = rest;
      used += n;
      peak = std::max(peak, used);
      if (trace) fprintf(stderr, "[ibwa_amd arena] +%.3f GB at %.3f GB: used %.3f GB\n", n / 1e9, off / 1e9, used / 1e9);
      return base + off;
    }
    return nullptr;
  }
  bool owns(const void *p) const {
    return base && static_cast<const char *>(p) >= base && static_cast<const char *>(p) < base + size;
  }
  void release(void *p, size_t n) {
    n = (n + 4095) & ~(size_t)4095;
    std::lock_guard<std::mutex> lk(mu);
    size_t off = (size_t)(static_cast<char *>(p) - base);
    used -= n;
    if (trace) fprintf(stderr, "[ibwa_amd arena] -%.3f GB at %.3f GB: used %.3f GB\n", n / 1e9, off / 1e9, used / 1e9);
    auto nx = free_.lower_bound(off);
    if (nx != free_.end() && off + n == nx->first) {  // merge with the next free range
      n += nx->second;
      nx = free_.erase(nx);
    }
    if (nx != free_.begin()) {
      auto pv = std::prev(nx);
      if (pv->first + pv->second == off) {  // and with the previous one
        pv->second += n;
        return;
      }
    }
    free_[off] = n;
  }
};
thread_local hipStream_t g_stream = nullptr;  // the stream of the context this thread's API call works on
constexpr int MAX_DEV = 64;
Arena g_arena[MAX_DEV];

}  // namespace

namespace ibwa {
hipError_t zero_async(void *p, size_t bytes, hipStream_t st) {
  constexpr size_t kZ = 64u << 20;
  static std::once_flag once;
  static void *zeros = nullptr;
  std::call_once(once, []() {
    if (hipHostMalloc(&zeros, kZ, hipHostMallocDefault) != hipSuccess) zeros = nullptr;
    else memset(zeros, 0, kZ);
  });
  if (!zeros) return hipMemsetAsync(p, 0, bytes, st);
  for (size_t o = 0; o < bytes; o += kZ) {
    hipError_t e = hipMemcpyAsync(static_cast<char *>(p) + o, zeros, std::min(kZ, bytes - o), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
}  // namespace ibwa

namespace {

Arena *arena_here() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= MAX_DEV) return nullptr;
  return g_arena[d].base ? &g_arena[d] : nullptr;
}

// A growable device buffer (carved from the device's arena when one is reserved).
struct DBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool borrowed = false;  // another context's buffer (ibwa_ctx_share_index): never freed or grown here
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (borrowed) return fail(IBWA_EINVAL, "a shared index buffer cannot grow (%zu > %zu bytes)", bytes, cap);
    if (p) free_dev(p, cap);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 256);
    static const bool verbose = getenv("IBWA_VERBOSE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    if (Arena *a = arena_here()) p = a->alloc(want);
    if (!p) {
      hipError_t e = hipMalloc(&p, want);
      if (e != hipSuccess) return fail(IBWA_EHIP, "hipMalloc(%zu): %s", want, hipGetErrorString(e));
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g_alloc_ms += ms;
    if (verbose && ms > 20.0) fprintf(stderr, "[ibwa_amd] hipMalloc(%.2f GB) took %.0f ms\n", want / 1e9, ms);
    cap = want;
    dev_bytes_add((int64_t)want);
    return 0;
  }
  static void free_dev(void *q, size_t n) {
    for (Arena &a : g_arena)
      if (a.owns(q)) {
        // the range may still be used by work queued on the owning context's stream (the API call
        // in progress on this thread: g_stream); other contexts never touch it (an index a context
        // lends is never freed while borrowed, and an ingest slot is not parsed over while a lane
        // still reads it)
        if (g_stream) (void)hipStreamSynchronize(g_stream);
        else (void)hipDeviceSynchronize();
        a.release(q, n);
        dev_bytes_add(-(int64_t)n);
        return;
      }
    (void)hipFree(q);
    dev_bytes_add(-(int64_t)n);
  }
  void release() {
    if (p && !borrowed) free_dev(p, cap);
    p = nullptr;
    cap = 0;
    borrowed = false;
  }
  DBuf borrow() const {
    DBuf b;
    b.p = p;
    b.cap = cap;
    b.borrowed = true;
    return b;
  }
  template <class T> T *as() const { return (T *)p; }
};

// A FASTQ parse's device scratch (ibwa_fq_parse): the raw block, its line table, per-record lengths
// and scan keys.  Only the kept reads' codes, offsets and lengths outlive a parse, so the ingest
// contexts of one device that never parse at the same time share one scratch (ibwa_fq_share_scratch).
struct FqScratch {
  int refs = 1;
  const void *last = nullptr;  // the context whose block the line table holds (ibwa_fq_offset)
  DBuf raw, tile, nl, cnt, len, L, key, tmp;
  uint32_t *hinit = nullptr;  // pinned: the parse counters' initial values, then zeros for the padding
  // a block in pageable memory (the CLI's mapped file) goes to the device through two pinned
  // staging chunks, filled by host threads: left to the HIP runtime, a pageable copy locks the
  // file's pages, and unlocking GBs of them cost ~0.3 s at process exit (profiles/r05_e2e_g.json)
  static constexpr size_t kStage = 64u << 20;
  char *stage[2] = {nullptr, nullptr};
  hipEvent_t sev[2] = {nullptr, nullptr};
  void unref() {
    if (--refs > 0) return;
    for (DBuf *b : {&raw, &tile, &nl, &cnt, &len, &L, &key, &tmp}) b->release();
    if (hinit) (void)hipHostFree(hinit);
    for (int i = 0; i < 2; ++i) {
      if (stage[i]) (void)hipHostFree(stage[i]);
      if (sev[i]) (void)hipEventDestroy(sev[i]);
    }
    delete this;
  }
  // src[0, n) to device dst on stream st
  hipError_t h2d(void *dst, const void *src, size_t n, hipStream_t st) {
    hipPointerAttribute_t at;
    const bool pinned = hipPointerGetAttributes(&at, src) == hipSuccess;
    (void)hipGetLastError();  // an unregistered pointer is not an error here
    if (pinned || n < (8u << 20)) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
    for (int i = 0; i < 2; ++i) {
      if (!stage[i]) {
        void *p = nullptr;
        if (hipError_t e = hipHostMalloc(&p, kStage, hipHostMallocDefault)) return e;
        stage[i] = static_cast<char *>(p);
      }
      if (!sev[i])
        if (hipError_t e = hipEventCreateWithFlags(&sev[i], hipEventDisableTiming)) return e;
    }
    const char *s = static_cast<const char *>(src);
    for (size_t o = 0, k = 0; o < n; o += kStage, ++k) {
      const int b = (int)(k & 1);
      const size_t len = std::min(kStage, n - o);
      if (k >= 2)
        if (hipError_t e = hipEventSynchronize(sev[b])) return e;  // its previous chunk has left
      const int T = 8;
      std::thread th[T];
      for (int t = 0; t < T; ++t)
        th[t] = std::thread([&, t]() {
          const size_t a = len * t / T, z = len * (t + 1) / T;
          memcpy(stage[b] + a, s + o + a, z - a);
        });
      for (auto &x : th) x.join();
      if (hipError_t e = hipMemcpyAsync(static_cast<char *>(dst) + o, stage[b], len, hipMemcpyHostToDevice, st)) return e;
      if (hipError_t e = hipEventRecord(sev[b], st)) return e;
    }
    return hipSuccess;
  }
};

}  // namespace

struct ibwa_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[8] = {};
  // index
  DBuf idx[2];
  IndexView ix[2] = {};
  bool loaded[2] = {false, false};
  // staged batch
  DBuf d_seq, d_off, d_len;
  // the staged batch: d_seq / d_off / d_len, or (ibwa_batch_stage_fq) a parsed block's kept reads
  const uint8_t *v_seq = nullptr;
  const uint64_t *v_off = nullptr;
  const uint32_t *v_len = nullptr;
  int64_t n = 0;
  uint64_t seq_bytes = 0;
  int max_len = 0;
  // scratch + outputs
  DBuf d_wbuf, d_heads, d_ent, d_prev, d_aln, d_naln, d_status, d_tab, d_ids;
  DBuf r_aln, r_naln, r_status;  // retry pass outputs
  // results of the last run (host)
  std::vector<int32_t> h_naln;
  std::vector<uint32_t> h_status;
  std::vector<uint4> h_aln;      // n * aln_cap slots
  std::vector<int64_t> retry_ids;                   // every read a later pass resolved (input order)
  std::vector<int64_t> patch_ids;                   // ... of which the wide / general passes' (input order)
  std::vector<std::vector<uint4>> patch_alns;       // their hits (the coop pass writes into d_aln / d_naln)
  DBuf d_selst, d_seltmp;                           // statuses of the handed-on reads, select scratch
  DBuf d_ordk, d_ordi, d_ordids, d_ordtmp;          // the coop pass's order (largest first-pass stack first)
  int coop_roots = 1;                               // option: level 0 of the heavy reads by k_coop_roots
  uint32_t aln_cap_used = 0;
  // sampled suffix arrays kept by ibwa_ctx_build_index
  DBuf sa_s[2];
  // full SA / ISA and 2-bit texts of an index built here: the exact path's unique-interval jump
  DBuf sa_full[2], isa_full[2], txt2[2];
  bool jump_ready = false;
  bool jump_derived = false;  // jump arrays derived from a loaded BWT (ensure_jump), not built here
  int jump_derive = 1;        // option: derive them for a loaded index when HBM allows
  int exact_jump = 1;
  int width_tab = 1;           // option: k_width's first steps from the level tables (first pass)
  int width_jump = 1;         // option: k_width steps one-row intervals from the text (2: derive SA / text for it)
  uint32_t sa_intv = 0;
  bool sa_loaded[2] = {false, false};  // sa_s[s] holds a sampled SA of the resident index
  bool sa_expanded = false;            // sa_full[0/1] derived from the sampled SA (ibwa_ctx_expand_sa)
  int sa_walk = 0;                     // option: always walk the sampled SA (parity / low-memory)
  DBuf h2p_in, h2p_out;                // staging of ibwa_sa2pos
  int build_rounds[2] = {0, 0};
  // tuning
  uint32_t stack_cap = 4096, aln_cap = 8;
  int block = 256;
  int64_t lanes_per_chunk = 1 << 18;
  int exact_path = 1;       // use k_exact when max_diff == 0
  int exact_blocks = 2048;  // persistent grid of k_exact (set from the CU count)
  DBuf d_counter, d_rec;
  int n_cus = 256;
  // persistent gapped search (gapped.hip)
  int gapped_v2 = 1;
  int gap_blocks_per_cu = 3;         // 134 VGPRs -> 3 waves per SIMD
  uint32_t gap_cap1 = 8192;          // per-lane static slots (stack + hit area)
  int gap_pages_per_block = 384;      // 128 KiB pages per 256-lane workgroup pool
  uint32_t gap_hit_slots = 256;      // hits a read may hold in the first pass
  int64_t gap_reads_per_chunk = 1 << 24;  // at most; a batch is cut into equal chunks (each chunk's last reads run alone)
  // early hand-off to the coop pass: a read past 3000 iterations whose stack holds > 1000 entries
  // (swept at 10M reads: 2.28 -> 2.14 s per step; budget 6000-16000 with it: within noise)
  uint32_t gap_early_iters = 3000, gap_early_entries = 1000;
  uint32_t gap_iter_budget = 8000;   // first-pass iterations per read before handing it to the coop pass (swept 1000-8000 at 50M reads: 8000 best)
  DBuf d_nN, d_pool, d_aoff, r_aoff, d_iters;
  // wave-cooperative heavy-read pass (coop.hip)
  int gap_coop = 1;
  int gap_lw = 1;                    // first pass with its widths in LDS (gapped.hip LW) when they fit
  int gap_lw_min_waves = 8;          // ... in a workgroup size that keeps at least this many waves per CU
  int gap_resume = 1;                // early hand-offs leave their search state for the coop pass (LW)
  int gap_resume_gb = 48;            // state buffer: at most this many GiB ...
  // ... sized per read of a first-pass chunk: this many 16 B records (100 bp reads at 1 % need ~160
  // per read at the busiest chunk), or the most an earlier run's chunk needed (x 1.15) if more --
  // states that do not fit are not lost work only: their reads start over in the cooperative pass
  uint32_t gap_resume_recs = 192;
  double resume_need = 0;            // the most records per chunk read a run of this context requested
  int coop_stg_room = 1;             // k_coop's per-lane staging ring: this many chains' children (2: same time)
  int64_t gap_resume_records = 0;    // tests: state buffer of this many 16 B records (0: by gap_resume_gb)
  // the early hand-off rule when the read leaves a resume state (nothing is re-run, so it pays to hand
  // on earlier: swept at 50M reads, flat optimum, profiles/r03_resume_sweep*.log)
  uint32_t gap_resume_iters = 2000, gap_resume_entries = 300;
  // resume in a launch's tail (GapArgs::tail_lanes): 16 / 200 measured 5868 vs 5884 ms per 50M-read
  // step (profiles/r03_tail_sweep.log; 8, 32, 4 / 500 in between)
  uint32_t gap_tail_lanes = 16, gap_tail_iters = 200;
  // first-pass pages per 256-lane pool when states are left (<= gap_pages_per_block): 96 -> 48 cost
  // nothing measurable at 100 or 150 bp (profiles/r04_sweep_mem*.jsonl)
  int gap_resume_ppb = 48;
  uint32_t gap_resume_cap1 = 4096;   // first-pass static slots per lane when states are left (<= gap_cap1)
  DBuf d_cw, d_ptabg;
  DBuf d_rdump, d_roff;
  DBuf d_hpop;           // per read: first-pass pops before its resume state (0: none; ibwa_batch_diag 2)
  bool hpop_valid = false;
  int coop_waves_per_cu = 12;        // 13.3 KiB of LDS and 168 VGPRs per wave (3 waves per SIMD)
  // bucket page pool, GiB (0: by read length -- 10 up to 128 bp, 16 above: at 100 bp 10 GiB costs
  // nothing, 5 322 vs 5 316 ms per 50 M-read step; at 150 bp / 2 % it cost 7 %, profiles/r05_sweep_mem*.jsonl)
  int coop_pool_gb = 0;
  uint64_t pool_bytes(int max_len) const { return (uint64_t)(coop_pool_gb ? coop_pool_gb : max_len <= 128 ? 10 : 16) << 30; }
  uint32_t coop_pool_pages = 0;      // tests: the pool in pages (0: by coop_pool_gb)
  DBuf c_stg, c_dir, c_free, c_pool, c_hits, c_next, c_recb, c_proot, c_pstore;
  bool stream_out = false;           // d_aln is a hit stream indexed by d_aoff
  bool verbose = getenv("IBWA_VERBOSE") != nullptr;
  bool prof_phases = getenv("IBWA_PROF_PHASES") != nullptr;  // diagnostics kernel variant
  int sw_stop_after = getenv("IBWA_SW_STOP") ? atoi(getenv("IBWA_SW_STOP")) : 0;  // diagnostics
  DBuf d_prof;
  int diag = 0;                      // option: keep per-read first-pass iterations and k_width features
  DBuf d_feat;
  unsigned long long stream_len = 0;  // hit-stream records written by the first pass (<= stream_total)
  unsigned long long stream_total = 0;  // hit-stream slots of the last first-pass launch
  uint32_t gap_stream_per_read = 4;     // first-pass hit-stream slots per read
  uint64_t gap_stream_min = 1u << 20;   // ... and at least this many in total
  std::vector<uint64_t> h_aoff;
  std::vector<uint8_t> retry_pass;  // per retry_ids entry: 1 coop, 2 wide, 3 general kernels
  std::vector<int64_t> resumed_ids; // reads the cooperative pass resolved from a resume state (retry_info pass 4)
  bool naln_on_host = true;  // h_naln mirrors d_naln
  bool fetched = false;       // the batch's results are on the host (fetch_to_host; a run resets it)
  std::vector<int32_t> h_cnt;  // per read its hits, patches included (fetch_to_host)
  // K-mer interval tables for the exact-match path (kmer.hip)
  DBuf kt[2], o64[2];
  // level tables of the LW first pass (GapArgs::ltab): strings of length <= gap_tab_k + 1 (0: off;
  // -1: auto, floor(log4(n)) up to 13 -- 2 x 2.9 GB at GRCh37 size -- or 14 with room, ensure_kmer),
  // built with the K-mer tables
  // (ensure_kmer).  Measured at 50 M reads (profiles/r06_sweep_tab.jsonl, hits identical): k_gapped
  // 2 476 ms per step without, 2 149 / 2 027 / 1 947 ms with K = 10 / 12 / 13.
  DBuf ltab[2];
  int gap_tab_k = -1;
  int ltab_K = 0;   // tab_k of the built level tables
  int kmer_k = -1;  // requested K (-1: auto from the genome size, 0: off)
  int kmer_K = 0;   // K of the built tables
  bool kmer_valid = false;
  ibwa_run_stats_t stats = {};
  DBuf sw[15];  // sw_batch's buffers (kept between calls)
  // ibwa_ctx_share_index: the context whose index structures this one borrows, and how many
  // contexts borrow this one's; neither side may rebuild or replace them while shared
  ibwa_ctx *share_src = nullptr;
  int n_borrowers = 0;
  bool destroy_pending = false;  // destroyed while borrowed: freed with its last borrower
  // FASTQ ingest (fastq.hip, ibwa_fq_parse): the last parsed block and its kept reads
  DBuf fq_codes, fq_offk, fq_lenk;  // the last parsed block's kept reads (ibwa_batch_stage_fq's views)
  FqScratch *fqs = nullptr;          // parse scratch, own or shared (ibwa_fq_share_scratch)
  int64_t fq_kept = 0;
  double fq_ms = 0;  // device time of the last parse (H2D copy + kernels), HIP events
};

namespace {

// An API call's entry: the context's device, and its stream for the arena (DBuf::free_dev).
hipError_t enter(const ibwa_ctx *c) {
  g_stream = c->stream;
  return hipSetDevice(c->device);
}

// the pages a cooperative launch took from its pool (a bump counter: freed pages go to per-wave lists)
void note_coop_pages(ibwa_ctx *c, uint32_t pool_pages) {
  uint32_t used = 0;
  if (hipMemcpy(&used, c->c_next.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return;
  c->stats.coop_pages_peak = std::max<int64_t>(c->stats.coop_pages_peak, std::min<uint32_t>(used, pool_pages));
  c->stats.coop_pages_cap = std::max<int64_t>(c->stats.coop_pages_cap, pool_pages);  // the largest launch's pool
}
// An operation that would rebuild or replace index structures shared by ibwa_ctx_share_index
// (borrowed buffers are written in place or cannot grow, and the other context may be aligning).
int refuse_shared(const ibwa_ctx *c, const char *what) {
  if (c->share_src) return fail(IBWA_EINVAL, "%s: this context shares another context's index", what);
  if (c->n_borrowers) return fail(IBWA_EINVAL, "%s: %d other context(s) share this context's index", what, c->n_borrowers);
  return 0;
}
// (Re)build the K-mer tables for the resident index if needed.
int ensure_kmer(ibwa_ctx *c) {
  if (c->kmer_valid) return 0;
  if (int rc = refuse_shared(c, "K-mer tables")) return rc;
  int K = c->kmer_k;
  if (K < 0) {
    // auto: K ~ log4(2n) (past that most K-mers are absent), up to 15 (2 x 8.6 GB for a
    // human genome; K = 16 measured slower: 2 x 34 GB of randomly probed tables),
    // and both tables within 40 % of the free HBM
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    K = 1;
    // at most 14: K = 15 tables (2 x 8.6 GB at GRCh37 size) bought nothing over 14 (2 x 2.1 GB):
    // 5 311 vs 5 316 ms per 50 M-read step, profiles/r05_sweep_mem.jsonl
    while (K < 14 && (1ull << (2 * (K + 1))) <= 2ull * c->ix[0].seq_len &&
           2ull * 8ull * (1ull << (2 * (K + 1))) <= (uint64_t)(0.4 * (double)free_b))
      ++K;
  }
  if (K > 16) K = 16;
  c->kmer_K = 0;
  // bit-plane Occ layouts (occ64.hip), 1 byte per BWT row and strand
  for (int s = 0; s < 2; ++s) {
    if (int rc = c->o64[s].ensure(occ64_blocks(c->ix[s].seq_len) * 64)) return rc;
    HIPCHK(build_occ64(c->ix[s], c->o64[s].as<uint4>(), c->stream));
  }
  if (K > 0) {
    DBuf tmp;
    if (int rc = tmp.ensure((1ull << (2 * (K - 1))) * 8)) return rc;
    for (int s = 0; s < 2; ++s) {
      if (int rc = c->kt[s].ensure((1ull << (2 * K)) * 8)) { tmp.release(); return rc; }
      hipError_t e = build_kmer_table(c->ix[s], K, c->kt[s].as<uint2>(), tmp.as<uint2>(), c->stream);
      if (e != hipSuccess) { tmp.release(); return fail(IBWA_EHIP, "K-mer table: %s", hipGetErrorString(e)); }
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    tmp.release();
    c->kmer_K = K;
  }
  c->ltab_K = 0;
  int TK = c->gap_tab_k;
  if (TK < 0) {
    // auto: as deep as strings of that length still mostly occur, at most 13 (2 x 2.9 GB at GRCh37
    // size); 14 (2 x 11.5 GB) when both tables take at most 15 % of the free HBM: k_gapped 1 935 ->
    // 1 844 ms per 50 M-read step (profiles/r06_sweep_tab2.jsonl).  The CLI pins its K (aln_main.cpp).
    TK = 0;
    while (TK < 13 && (1ull << (2 * (TK + 1))) <= (uint64_t)c->ix[0].seq_len) ++TK;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    if (TK == 13 && (1ull << 30) <= (uint64_t)c->ix[0].seq_len &&
        2.0 * 8.0 * (double)ltab_off(16) <= 0.15 * (double)free_b)
      TK = 14;
  }
  if (TK > 0 && c->ix[0].seq_len < LTAB_MARK) {
    for (int s = 0; s < 2; ++s) {
      if (int rc = c->ltab[s].ensure(ltab_off((uint32_t)TK + 2) * 8)) return rc;
      hipError_t e = build_level_tables(c->ix[s], TK + 1, c->ltab[s].as<uint2>(), c->stream);
      if (e != hipSuccess) return fail(IBWA_EHIP, "level tables: %s", hipGetErrorString(e));
    }
    c->ltab_K = TK;
  }
  c->kmer_valid = true;
  return 0;
}
// The exact path's unique-interval jump needs the full SA, the ISA and the 2-bit text of both
// strands.  An index built here keeps them (ibwa_ctx_build_index); for an index loaded from .bwt
// files (the drop-in, the CLI) they are derived on the device from the BWT alone: the sampled SA
// by an LF walk between marked rows plus list ranking, then the full SA (k_expand_sa), the ISA
// (a scatter) and the text (a gather through the ISA).  Skipped when HBM is short: the exact path
// then runs without the jump (same results).
int derive_sa_locked(ibwa_ctx *c, uint32_t intv) {
  if (c->share_src) return fail(IBWA_EINVAL, "sampled SA: this context shares another context's index");
  HIPCHK(enter(c));
  for (int s = 0; s < 2; ++s) {
    const uint64_t n_nodes = ((uint64_t)c->ix[s].seq_len + intv) / intv;
    DBuf tmp;
    if (int rc = tmp.ensure((4 * n_nodes + 1) * 4)) return rc;
    if (int rc = c->sa_s[s].ensure(n_nodes * 4)) { tmp.release(); return rc; }
    hipError_t e = derive_sampled_sa(c->ix[s], intv, c->sa_s[s].as<uint32_t>(), tmp.as<uint32_t>(), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    tmp.release();
    if (e != hipSuccess) return fail(IBWA_EHIP, "sampled SA from the BWT (strand %d): %s", s, hipGetErrorString(e));
    c->sa_loaded[s] = true;
  }
  c->sa_intv = intv;
  c->sa_expanded = false;
  return 0;
}

int ensure_jump(ibwa_ctx *c) {
  if (c->jump_ready || !c->exact_jump || !c->jump_derive) return 0;
  // a context sharing another's index runs without the jump unless the source had it when shared
  // (the same results; the jump only saves rank queries)
  if (c->share_src) return 0;
  const uint64_t n = c->ix[0].seq_len;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 0;
  // full SA + ISA + text of both strands (~16.6 B per base) and the derivation's temporaries
  if ((double)free_b < (double)n * 18.0 + 4e9 || (double)n * 16.6 > 0.3 * (double)total_b) return 0;
  if (!c->sa_loaded[0] || !c->sa_loaded[1])
    if (int rc = derive_sa_locked(c, 32)) return rc;
  if (int rc = ibwa_ctx_expand_sa(c)) return rc;
  for (int s = 0; s < 2; ++s) {
    const uint64_t words = n / 16 + 4;
    if (int rc = c->isa_full[s].ensure((n + 1) * 4)) return rc;
    if (int rc = c->txt2[s].ensure(words * 4)) return rc;
    HIPCHK(hipMemsetAsync(c->txt2[s].p, 0, words * 4, c->stream));
    HIPCHK(derive_isa_text(c->ix[s], c->sa_full[s].as<uint32_t>(), c->isa_full[s].as<uint32_t>(),
                           c->txt2[s].as<uint32_t>(), words, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  c->jump_ready = true;
  c->jump_derived = true;
  return 0;
}

// Kernel arguments of the persistent gapped search shared by the first and retry passes;
// the caller fills the per-pass scratch and output pointers.
GapArgs gap_args(const ibwa_ctx *c, const AlnArgs &A, const AlnOpt &o, int64_t b0, int64_t cnt) {
  GapArgs G = {};
  G.ix[0] = c->ix[0];
  G.ix[1] = c->ix[1];
  G.o64[0] = c->o64[0].as<uint4>();
  G.o64[1] = c->o64[1].as<uint4>();
  G.seq = A.seq;
  G.off = A.off + b0;
  G.len = A.len + b0;
  G.ids = nullptr;
  G.n = cnt;
  G.maxdiff_tab = A.maxdiff_tab;
  G.wbuf = c->d_wbuf.as<uint2>();
  G.wstride = A.wstride;
  G.wlen1 = A.wlen1;
  G.nN = c->d_nN.as<uint16_t>();
  G.aln_next = c->d_counter.as<unsigned long long>() + 1;
  G.lanes_per_wave = 64;
  G.o = o;
  return G;
}
}  // namespace

extern "C" {

const char *ibwa_last_error(void) { return g_err.c_str(); }
void ibwa_free(void *p) { free(p); }

void ibwa_gap_init_opt(ibwa_gap_opt_t *o) {  // bwtaln.c:21-37
  memset(o, 0, sizeof(*o));
  o->s_mm = 3; o->s_gapo = 11; o->s_gape = 4;
  o->max_diff = -1; o->max_gapo = 1; o->max_gape = 6;
  o->indel_end_skip = 5; o->max_del_occ = 10; o->max_entries = 2000000;
  o->mode = IBWA_MODE_GAPE | IBWA_MODE_COMPREAD;
  o->seed_len = 32; o->max_seed_diff = 2;
  o->fnr = 0.04f;
  o->n_threads = 1;
  o->max_top2 = 30;
  o->trim_qual = 0;
}

int ibwa_cal_maxdiff(int l, double err, double thres) {  // bwtaln.c:39-51
  double elambda = exp(-l * err);
  double sum, y = 1.0;
  int k, x = 1;
  for (k = 1, sum = elambda; k < 1000; ++k) {
    y *= l * err;
    x *= k;
    sum += elambda * y / x;
    if (1.0 - sum < thres) return k;
  }
  return 2;
}

int ibwa_device_count(int *n) {
  int d = 0;
  hipError_t e = hipGetDeviceCount(&d);
  if (e != hipSuccess) return fail(IBWA_EHIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
  if (n) *n = d;
  return 0;
}

int ibwa_device_memory(int device, uint64_t *free_b, uint64_t *total_b) {
  HIPCHK(hipSetDevice(device));
  size_t f = 0, t = 0;
  HIPCHK(hipMemGetInfo(&f, &t));
  if (free_b) *free_b = f;
  if (total_b) *total_b = t;
  return 0;
}

int ibwa_reserve(int device, uint64_t bytes) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return fail(IBWA_EHIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= n || device >= MAX_DEV) return fail(IBWA_EINVAL, "device %d out of range (%d devices)", device, n);
  Arena &a = g_arena[device];
  std::lock_guard<std::mutex> lk(a.mu);
  if (a.base) return fail(IBWA_EINVAL, "device %d already has an arena of %zu bytes", device, a.size);
  if (bytes == 0) return 0;
  HIPCHK(hipSetDevice(device));
  const size_t want = ((size_t)bytes + 4095) & ~(size_t)4095;
  void *p = nullptr;
  e = hipMalloc(&p, want);
  if (e != hipSuccess) return fail(IBWA_EHIP, "hipMalloc(%zu) for the arena: %s", want, hipGetErrorString(e));
  a.base = static_cast<char *>(p);
  a.size = want;
  a.free_[0] = want;
  return 0;
}

int ibwa_release(int device) {
  if (device < 0 || device >= MAX_DEV) return fail(IBWA_EINVAL, "device %d out of range", device);
  Arena &a = g_arena[device];
  std::lock_guard<std::mutex> lk(a.mu);
  if (!a.base) return 0;
  // a buffer still carved from it belongs to a context that may use it again: the contexts go first
  if (a.used > 0)
    return fail(IBWA_EINVAL, "device %d's arena still holds %zu bytes of context buffers (destroy the contexts first)",
                device, a.used);
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipFree(a.base));
  a.base = nullptr;
  a.size = a.used = 0;
  a.free_.clear();
  return 0;
}

int ibwa_arena_stats(int device, uint64_t *size, uint64_t *used, uint64_t *peak) {
  if (device < 0 || device >= MAX_DEV) return fail(IBWA_EINVAL, "device %d out of range", device);
  Arena &a = g_arena[device];
  std::lock_guard<std::mutex> lk(a.mu);
  if (size) *size = a.size;
  if (used) *used = a.used;
  if (peak) *peak = a.peak;
  return 0;
}

int ibwa_device_bytes(int64_t *now, int64_t *peak) {
  if (now) *now = g_dev_bytes.load();
  if (peak) *peak = g_dev_peak.load();
  return 0;
}

int ibwa_ctx_create(int device, ibwa_ctx_t **out) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return fail(IBWA_EHIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= n) return fail(IBWA_EINVAL, "device %d out of range (%d devices)", device, n);
  HIPCHK(hipSetDevice(device));
  ibwa_ctx *c = new ibwa_ctx();
  c->device = device;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
  {
    c->exact_blocks = cus * 8;  // 8 x 256-thread blocks per CU: 32 waves/CU when registers allow
    c->n_cus = cus;
  }
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (auto &x : c->ev) HIPCHK(hipEventCreate(&x));
  *out = c;
  return 0;
}

void ibwa_ctx_destroy(ibwa_ctx_t *c) {
  if (!c) return;
  (void)enter(c);
  (void)hipStreamSynchronize(c->stream);
  // a context whose index other contexts still borrow (ibwa_ctx_share_index) stays alive until the
  // last of them is destroyed: its index buffers are theirs too
  if (c->n_borrowers > 0) {
    c->destroy_pending = true;
    g_stream = nullptr;
    return;
  }
  // the context whose index this one borrowed is destroyed after this one's own buffers are released
  // (their arena release synchronises this context's stream, g_stream)
  ibwa_ctx *src = c->share_src;
  c->share_src = nullptr;
  for (DBuf *b : {&c->h2p_in, &c->h2p_out, &c->idx[0], &c->idx[1], &c->d_seq, &c->d_off, &c->d_len, &c->d_wbuf, &c->d_heads, &c->d_ent,
                  &c->d_prev, &c->d_aln, &c->d_naln, &c->d_status, &c->d_tab, &c->d_ids, &c->r_aln, &c->r_naln,
                  &c->r_status, &c->sa_s[0], &c->sa_s[1], &c->d_counter, &c->kt[0], &c->kt[1], &c->ltab[0], &c->ltab[1], &c->d_rec, &c->o64[0], &c->o64[1], &c->d_nN, &c->d_pool, &c->d_aoff, &c->r_aoff, &c->d_iters, &c->d_prof, &c->sa_full[0], &c->sa_full[1],
                  &c->isa_full[0], &c->isa_full[1], &c->txt2[0], &c->txt2[1], &c->c_dir, &c->c_free, &c->c_hits,
                  &c->c_next, &c->c_pool, &c->c_proot, &c->c_pstore, &c->c_recb, &c->c_stg, &c->d_cw, &c->d_feat,
                  &c->d_hpop, &c->d_ordi, &c->d_ordids, &c->d_ordk, &c->d_ordtmp, &c->d_ptabg, &c->d_rdump, &c->d_roff,
                  &c->d_selst, &c->d_seltmp, &c->fq_codes, &c->fq_lenk, &c->fq_offk})
    b->release();
  if (c->fqs) c->fqs->unref();
  for (auto &b : c->sw) b.release();
  for (auto &x : c->ev) (void)hipEventDestroy(x);
  (void)hipStreamDestroy(c->stream);
  delete c;
  g_stream = nullptr;  // not left naming a destroyed stream
  if (src && --src->n_borrowers == 0 && src->destroy_pending) ibwa_ctx_destroy(src);
}

int ibwa_ctx_set_option(ibwa_ctx_t *c, const char *key, long value) {
  std::string k = key ? key : "";
  if (k == "exact_path") c->exact_path = value != 0;
  else if (k == "kmer_k" && value >= -1 && value <= 16) {
    if (value != c->kmer_k)
      if (int rc = refuse_shared(c, "option kmer_k")) return rc;
    c->kmer_k = (int)value;
    c->kmer_valid = false;
  }
  else if (k == "gap_tab_k" && value >= -1 && value <= 14) {
    if (value != c->gap_tab_k) {
      if (int rc = refuse_shared(c, "option gap_tab_k")) return rc;
      c->kmer_valid = false;  // built with the K-mer tables
    }
    c->gap_tab_k = (int)value;
  }
  else if (k == "exact_blocks" && value > 0) c->exact_blocks = (int)value;
  else if (k == "lanes_per_chunk" && value > 0) c->lanes_per_chunk = value;
  else if (k == "gapped_v2") c->gapped_v2 = value != 0;
  else if (k == "gap_blocks_per_cu" && value > 0 && value <= 8) c->gap_blocks_per_cu = (int)value;
  else if (k == "gap_cap1" && value >= 16 && value <= 65536) c->gap_cap1 = (uint32_t)value;
  else if (k == "gap_pages_per_block" && value >= 1 && value <= 65536) c->gap_pages_per_block = (int)value;
  else if (k == "gap_hit_slots" && value >= 1 && value <= 4096) c->gap_hit_slots = (uint32_t)value;
  else if (k == "gap_reads_per_chunk" && value > 0) c->gap_reads_per_chunk = value;
  else if (k == "gap_iter_budget" && value >= 0) c->gap_iter_budget = (uint32_t)value;
  else if (k == "gap_early_iters" && value >= 0) c->gap_early_iters = (uint32_t)value;
  else if (k == "gap_early_entries" && value >= 0) c->gap_early_entries = (uint32_t)value;
  else if (k == "gap_lw" && (value == 0 || value == 1)) c->gap_lw = (int)value;
  else if (k == "gap_lw_min_waves" && value >= 1 && value <= 32) c->gap_lw_min_waves = (int)value;
  else if (k == "gap_resume" && (value == 0 || value == 1)) c->gap_resume = (int)value;
  else if (k == "gap_resume_gb" && value >= 1 && value <= 256) c->gap_resume_gb = (int)value;
  else if (k == "gap_resume_records" && value >= 0) c->gap_resume_records = (int64_t)value;
  else if (k == "gap_resume_iters" && value >= 0) c->gap_resume_iters = (uint32_t)value;
  else if (k == "gap_resume_entries" && value >= 0) c->gap_resume_entries = (uint32_t)value;
  else if (k == "gap_tail_lanes" && value >= 0 && value <= 64) c->gap_tail_lanes = (uint32_t)value;
  else if (k == "gap_tail_iters" && value >= 0) c->gap_tail_iters = (uint32_t)value;
  else if (k == "gap_resume_ppb" && value >= 1 && value <= 65536) c->gap_resume_ppb = (int)value;
  else if (k == "gap_resume_cap1" && value >= 16 && value <= 65536) c->gap_resume_cap1 = (uint32_t)value;
  else if (k == "coop_roots" && (value == 0 || value == 1)) c->coop_roots = (int)value;
  else if (k == "gap_stream_per_read" && value >= 0 && value <= 4096) c->gap_stream_per_read = (uint32_t)value;
  else if (k == "gap_stream_min" && value >= 1) c->gap_stream_min = (uint64_t)value;
  else if (k == "exact_jump") c->exact_jump = value != 0;
  else if (k == "jump_derive") c->jump_derive = value != 0;
  else if (k == "width_jump" && value >= 0 && value <= 2) c->width_jump = (int)value;
  else if (k == "width_tab" && (value == 0 || value == 1)) c->width_tab = (int)value;
  else if (k == "diag") c->diag = value != 0;
  else if (k == "sa_walk") c->sa_walk = value != 0;
  else if (k == "gap_coop") c->gap_coop = value != 0;
  else if (k == "coop_waves_per_cu" && value > 0 && value <= 16) c->coop_waves_per_cu = (int)value;
  else if (k == "coop_pool_gb" && value >= 0 && value <= 256) c->coop_pool_gb = (int)value;
  else if (k == "coop_stg_room" && value >= 1 && value <= 4) c->coop_stg_room = (int)value;
  else if (k == "coop_pool_pages" && value >= 0 && value <= (1l << 24)) c->coop_pool_pages = (uint32_t)value;
  else if (k == "gap_resume_recs" && value >= 1 && value <= 65536) c->gap_resume_recs = (uint32_t)value;
  else if (k == "sw_stop" && value >= 0 && value <= 2) c->sw_stop_after = (int)value;  // SW phase timing
  else return fail(IBWA_EINVAL, "unknown option %s", k.c_str());
  return 0;
}

int ibwa_ctx_set_tuning(ibwa_ctx_t *c, int stack_cap, int aln_cap, int block) {
  if (stack_cap > 0) c->stack_cap = stack_cap;
  if (aln_cap > 0) c->aln_cap = aln_cap;
  if (block > 0) {
    if (block % 64 || block > 256) return fail(IBWA_EINVAL, "block must be a multiple of 64 and <= 256");
    c->block = block;
  }
  return 0;
}

int ibwa_ctx_load_bwt(ibwa_ctx_t *c, int strand, uint32_t primary, const uint32_t L2[4], const uint32_t *bwt,
                      uint64_t bwt_size) {
  if (strand < 0 || strand > 1) return fail(IBWA_EINVAL, "strand must be 0 (.bwt) or 1 (.rbwt)");
  if (int rc = refuse_shared(c, "load_bwt")) return rc;
  HIPCHK(enter(c));
  const uint32_t seq_len = L2[3];
  const uint64_t n_blocks = ((uint64_t)seq_len + 127) / 128 + 1;
  // expected reference size: 4 words per 128 symbols (+1 final count block) + ceil(n/16) words
  const uint64_t expect = ((uint64_t)seq_len + 127) / 128 * 4 + 4 + ((uint64_t)seq_len + 15) / 16;
  if (bwt_size != expect)
    return fail(IBWA_EINVAL, "bwt_size %llu does not match seq_len %u (expected %llu)", (unsigned long long)bwt_size,
                seq_len, (unsigned long long)expect);
  DBuf tmp;
  if (int rc = tmp.ensure(bwt_size * 4)) return rc;
  if (int rc = c->idx[strand].ensure(n_blocks * 64)) { tmp.release(); return rc; }
  HIPCHK(hipMemcpyAsync(tmp.p, bwt, bwt_size * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(relayout_reference_bwt(tmp.as<uint32_t>(), bwt_size, n_blocks, c->idx[strand].as<uint4>(), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  tmp.release();
  IndexView &ix = c->ix[strand];
  ix.blk = c->idx[strand].as<uint4>();
  ix.primary = primary;
  ix.seq_len = seq_len;
  ix.L2[0] = 0;
  for (int j = 0; j < 4; ++j) ix.L2[j + 1] = L2[j];
  c->loaded[strand] = true;
  c->kmer_valid = false;
  c->jump_ready = false;  // SA / ISA / text belong to an index built here (or are derived again)
  c->jump_derived = false;
  c->sa_loaded[strand] = false;
  c->sa_expanded = false;
  return 0;
}

int ibwa_ctx_load_bwt_file(ibwa_ctx_t *c, int strand, const char *path) {  // bwtio.c:51-70
  FILE *fp = fopen(path, "rb");
  if (!fp) return fail(IBWA_EIO, "cannot open %s", path);
  fseek(fp, 0, SEEK_END);
  long sz = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  if (sz < 20) { fclose(fp); return fail(IBWA_EIO, "%s: too short", path); }
  uint64_t n_words = (uint64_t)(sz - 20) >> 2;
  uint32_t primary, L2[4];
  std::vector<uint32_t> buf(n_words);
  bool ok = fread(&primary, 4, 1, fp) == 1 && fread(L2, 4, 4, fp) == 4 && fread(buf.data(), 4, n_words, fp) == n_words;
  fclose(fp);
  if (!ok) return fail(IBWA_EIO, "%s: short read", path);
  return ibwa_ctx_load_bwt(c, strand, primary, L2, buf.data(), n_words);
}

int ibwa_ctx_clone_index(ibwa_ctx_t *dst, const ibwa_ctx_t *src) {
  if (int rc = refuse_shared(dst, "clone_index")) return rc;
  for (int s = 0; s < 2; ++s) {
    if (!src->loaded[s]) return fail(IBWA_ENOINDEX, "source index not loaded");
    HIPCHK(enter(dst));
    uint64_t bytes = ((uint64_t)src->ix[s].seq_len + 127) / 128 * 64 + 64;
    if (int rc = dst->idx[s].ensure(bytes)) return rc;
    if (src->device == dst->device) {
      HIPCHK(hipMemcpyAsync(dst->idx[s].p, src->idx[s].p, bytes, hipMemcpyDeviceToDevice, dst->stream));
    } else {
      HIPCHK(hipMemcpyPeerAsync(dst->idx[s].p, dst->device, src->idx[s].p, src->device, bytes, dst->stream));
    }
    HIPCHK(hipStreamSynchronize(dst->stream));
    dst->ix[s] = src->ix[s];
    dst->ix[s].blk = dst->idx[s].as<uint4>();
    dst->loaded[s] = true;
    dst->kmer_valid = false;
    dst->sa_loaded[s] = false;
  }
  dst->jump_ready = false;
  dst->sa_expanded = false;
  return 0;
}

int ibwa_ctx_share_index(ibwa_ctx_t *dst, const ibwa_ctx_t *src) {
  if (!dst || !src || dst == src) return fail(IBWA_EINVAL, "share_index: two distinct contexts");
  if (dst->device != src->device) return fail(IBWA_EINVAL, "share_index: contexts on devices %d and %d", dst->device, src->device);
  for (int s = 0; s < 2; ++s)
    if (!src->loaded[s]) return fail(IBWA_ENOINDEX, "source index not loaded");
  if (int rc = refuse_shared(dst, "share_index (destination)")) return rc;
  if (src->share_src) return fail(IBWA_EINVAL, "share_index: the source shares another context's index; share that one");
  HIPCHK(enter(dst));
  HIPCHK(hipStreamSynchronize(src->stream));  // src's structures are complete
  for (int s = 0; s < 2; ++s) {
    for (DBuf *b : {&dst->idx[s], &dst->o64[s], &dst->kt[s], &dst->ltab[s], &dst->sa_s[s], &dst->sa_full[s], &dst->isa_full[s],
                    &dst->txt2[s]})
      b->release();
    dst->idx[s] = src->idx[s].borrow();
    dst->o64[s] = src->o64[s].borrow();
    dst->kt[s] = src->kt[s].borrow();
    dst->ltab[s] = src->ltab[s].borrow();
    dst->sa_s[s] = src->sa_s[s].borrow();
    dst->sa_full[s] = src->sa_full[s].borrow();
    dst->isa_full[s] = src->isa_full[s].borrow();
    dst->txt2[s] = src->txt2[s].borrow();
    dst->ix[s] = src->ix[s];
    dst->loaded[s] = true;
    dst->sa_loaded[s] = src->sa_loaded[s];
    dst->build_rounds[s] = src->build_rounds[s];
  }
  dst->kmer_k = src->kmer_k;
  dst->kmer_K = src->kmer_K;
  dst->gap_tab_k = src->gap_tab_k;
  dst->ltab_K = src->ltab_K;
  dst->kmer_valid = src->kmer_valid;
  dst->sa_intv = src->sa_intv;
  dst->sa_expanded = src->sa_expanded;
  dst->jump_ready = src->jump_ready;
  dst->jump_derived = src->jump_derived;
  dst->jump_derive = src->jump_derive;
  dst->exact_jump = src->exact_jump;
  dst->width_jump = src->width_jump;
  dst->width_tab = src->width_tab;
  dst->share_src = const_cast<ibwa_ctx *>(src);
  ++dst->share_src->n_borrowers;
  return 0;
}

int ibwa_ctx_build_index(ibwa_ctx_t *c, const uint8_t *codes, uint64_t n, int sa_intv) {
  if (n == 0 || n >= 0xFFFFFFFEull) return fail(IBWA_EINVAL, "text length %llu outside [1, 2^32-2)", (unsigned long long)n);
  if (sa_intv < 0) return fail(IBWA_EINVAL, "sa_intv < 0");
  if (int rc = refuse_shared(c, "build_index")) return rc;
  HIPCHK(enter(c));
  DBuf T;
  if (int rc = T.ensure(n)) return rc;
  HIPCHK(hipMemcpyAsync(T.p, codes, n, hipMemcpyHostToDevice, c->stream));
  // keep SA / ISA / text for the exact path's jump when HBM allows (2 x 8.25 B per base)
  c->jump_ready = false;
  bool keep_full = c->exact_jump != 0;
  if (keep_full) {
    size_t free_b = 0, total_b = 0;
    // the kept arrays (16.5 B per base) plus the builder's sort temporaries (~45 B per base)
    // and headroom must fit in what is free now
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || (double)free_b < (double)n * 61.5 + 4e9) keep_full = false;
    if ((double)n * 16.5 > 0.3 * (double)total_b) keep_full = false;
  }
  if (!keep_full)
    for (int s = 0; s < 2; ++s) { c->sa_full[s].release(); c->isa_full[s].release(); c->txt2[s].release(); }
  for (int s = 0; s < 2; ++s) {
    c->loaded[s] = false;
    if (s == 1) HIPCHK(reverse_text(T.as<uint8_t>(), n, c->stream));  // .rpac (bwtmisc.c:160-185)
    const uint64_t n_blocks = (n + 127) / 128 + 1;
    if (int rc = c->idx[s].ensure(n_blocks * 64)) { T.release(); return rc; }
    uint32_t *sa_full = nullptr, *isa_full = nullptr;
    if (keep_full) {
      if (int rc = c->sa_full[s].ensure((n + 1) * 4)) { T.release(); return rc; }
      if (int rc = c->isa_full[s].ensure((n + 1) * 4)) { T.release(); return rc; }
      if (int rc = c->txt2[s].ensure((n / 16 + 4) * 4)) { T.release(); return rc; }
      HIPCHK(pack_text2(T.as<uint8_t>(), n, c->txt2[s].as<uint32_t>(), n / 16 + 4, c->stream));
      sa_full = c->sa_full[s].as<uint32_t>();
      isa_full = c->isa_full[s].as<uint32_t>();
    }
    uint32_t *sa_out = nullptr;
    if (sa_intv > 0) {
      if (int rc = c->sa_s[s].ensure(((n + sa_intv) / sa_intv) * 4)) { T.release(); return rc; }
      sa_out = c->sa_s[s].as<uint32_t>();
    }
    uint32_t primary = 0, tot[4] = {0, 0, 0, 0};
    hipError_t e = build_strand(T.as<uint8_t>(), n, c->idx[s].as<uint4>(), &primary, tot, sa_out, (uint32_t)sa_intv,
                                &c->build_rounds[s], sa_full, isa_full, c->stream);
    if (e != hipSuccess) {
      T.release();
      return fail(IBWA_EHIP, "suffix sort (strand %d): %s", s, hipGetErrorString(e));
    }
    IndexView &ix = c->ix[s];
    ix.blk = c->idx[s].as<uint4>();
    ix.primary = primary;
    ix.seq_len = (uint32_t)n;
    ix.L2[0] = 0;
    ix.L2[1] = tot[0];
    ix.L2[2] = tot[0] + tot[1];
    ix.L2[3] = tot[0] + tot[1] + tot[2];
    ix.L2[4] = tot[0] + tot[1] + tot[2] + tot[3];
    if (ix.L2[4] != n) { T.release(); return fail(IBWA_EHIP, "index build: symbol total %u != n", ix.L2[4]); }
    c->loaded[s] = true;
  }
  c->kmer_valid = false;
  c->sa_intv = (uint32_t)sa_intv;
  c->sa_loaded[0] = c->sa_loaded[1] = sa_intv > 0;
  c->sa_expanded = false;
  c->jump_ready = keep_full;
  T.release();
  return 0;
}

int ibwa_ctx_bwt_info(const ibwa_ctx_t *c, int strand, uint32_t *primary, uint32_t L2[4], uint64_t *bwt_size) {
  if (strand < 0 || strand > 1 || !c->loaded[strand]) return fail(IBWA_ENOINDEX, "index not loaded");
  const IndexView &ix = c->ix[strand];
  if (primary) *primary = ix.primary;
  if (L2) for (int j = 0; j < 4; ++j) L2[j] = ix.L2[j + 1];
  const uint64_t n = ix.seq_len;
  if (bwt_size) *bwt_size = (n + 127) / 128 * 4 + 4 + (n + 15) / 16;
  return 0;
}

int ibwa_ctx_export_bwt(const ibwa_ctx_t *c, int strand, uint32_t *words, uint64_t cap) {
  uint64_t need = 0;
  if (int rc = ibwa_ctx_bwt_info(c, strand, nullptr, nullptr, &need)) return rc;
  if (cap < need) return fail(IBWA_EINVAL, "export buffer too small (%llu < %llu)", (unsigned long long)cap,
                              (unsigned long long)need);
  HIPCHK(enter(c));
  const uint64_t n = c->ix[strand].seq_len, nb = (n + 127) / 128;
  std::vector<uint4> blk((nb + 1) * 4);
  HIPCHK(hipMemcpy(blk.data(), c->idx[strand].p, blk.size() * 16, hipMemcpyDeviceToHost));
  // bwt_bwtupdate_core (bwtmisc.c:122-144): [4 counts][<=8 words] per 128 symbols, then final counts
  uint64_t k = 0;
  for (uint64_t b = 0; b < nb; ++b) {
    const uint4 *p = &blk[b * 4];
    words[k++] = p[0].x; words[k++] = p[0].y; words[k++] = p[0].z; words[k++] = p[0].w;
    const uint32_t w8[8] = {p[1].x, p[1].y, p[1].z, p[1].w, p[2].x, p[2].y, p[2].z, p[2].w};
    const uint64_t nw = std::min<uint64_t>(8, (n - b * 128 + 15) / 16);
    for (uint64_t q = 0; q < nw; ++q) words[k++] = w8[q];
  }
  const IndexView &ix = c->ix[strand];
  for (int j = 0; j < 4; ++j) words[k++] = ix.L2[j + 1] - ix.L2[j];
  return k == need ? 0 : fail(IBWA_EINVAL, "internal: exported %llu words, expected %llu", (unsigned long long)k,
                              (unsigned long long)need);
}

int ibwa_ctx_export_sa(const ibwa_ctx_t *c, int strand, uint32_t *out, uint64_t cap) {
  if (strand < 0 || strand > 1 || !c->loaded[strand] || !c->sa_intv) return fail(IBWA_ENOINDEX, "no sampled SA");
  const uint64_t n = c->ix[strand].seq_len, n_sa = (n + c->sa_intv) / c->sa_intv;
  if (cap < n_sa) return fail(IBWA_EINVAL, "export buffer too small");
  HIPCHK(enter(c));
  HIPCHK(hipMemcpy(out, c->sa_s[strand].p, n_sa * 4, hipMemcpyDeviceToHost));
  out[0] = 0xFFFFFFFFu;  // bwt.c:66
  return 0;
}

int ibwa_ctx_load_sa(ibwa_ctx_t *c, int strand, uint32_t sa_intv, const uint32_t *sa, uint64_t n_sa) {
  if (strand < 0 || strand > 1 || !c->loaded[strand]) return fail(IBWA_ENOINDEX, "index not loaded");
  if (sa_intv == 0) return fail(IBWA_EINVAL, "sa_intv == 0");
  if (int rc = refuse_shared(c, "load_sa")) return rc;
  const uint64_t n = c->ix[strand].seq_len;
  if (n_sa != (n + sa_intv) / sa_intv)
    return fail(IBWA_EINVAL, "n_sa %llu != (seq_len + intv) / intv", (unsigned long long)n_sa);
  if (c->sa_loaded[1 - strand] && c->sa_intv != sa_intv)
    return fail(IBWA_EINVAL, "sa_intv %u differs from the other strand's %u", sa_intv, c->sa_intv);
  HIPCHK(enter(c));
  if (int rc = c->sa_s[strand].ensure(n_sa * 4)) return rc;
  HIPCHK(hipMemcpy(c->sa_s[strand].p, sa, n_sa * 4, hipMemcpyHostToDevice));
  c->sa_intv = sa_intv;
  c->sa_loaded[strand] = true;
  c->sa_expanded = false;
  if (c->jump_ready) c->sa_full[strand].release(), c->isa_full[strand].release(), c->jump_ready = false;
  return 0;
}

int ibwa_ctx_load_sa_file(ibwa_ctx_t *c, int strand, const char *path) {  // bwt_restore_sa, bwtio.c:29-49
  if (strand < 0 || strand > 1 || !c->loaded[strand]) return fail(IBWA_ENOINDEX, "index not loaded");
  FILE *fp = fopen(path, "rb");
  if (!fp) return fail(IBWA_EIO, "cannot open %s", path);
  uint32_t hdr[7];
  if (fread(hdr, 4, 7, fp) != 7) { fclose(fp); return fail(IBWA_EIO, "%s: short header", path); }
  const IndexView &ix = c->ix[strand];
  if (hdr[0] != ix.primary) { fclose(fp); return fail(IBWA_EINVAL, "SA-BWT inconsistency: primary is not the same."); }
  if (hdr[6] != ix.seq_len) { fclose(fp); return fail(IBWA_EINVAL, "SA-BWT inconsistency: seq_len is not the same."); }
  if (hdr[5] == 0) { fclose(fp); return fail(IBWA_EINVAL, "%s: sa_intv 0", path); }
  const uint64_t n_sa = ((uint64_t)ix.seq_len + hdr[5]) / hdr[5];
  std::vector<uint32_t> sa(n_sa);
  sa[0] = 0xFFFFFFFFu;  // bwtio.c:45
  const bool ok = fread(sa.data() + 1, 4, n_sa - 1, fp) == n_sa - 1;
  fclose(fp);
  if (!ok) return fail(IBWA_EIO, "%s: short read", path);
  return ibwa_ctx_load_sa(c, strand, hdr[5], sa.data(), n_sa);
}

int ibwa_ctx_derive_sa(ibwa_ctx_t *c, uint32_t sa_intv) {
  if (!c->loaded[0] || !c->loaded[1]) return fail(IBWA_ENOINDEX, "load both .bwt and .rbwt first");
  if (sa_intv == 0) return fail(IBWA_EINVAL, "sa_intv == 0");
  return derive_sa_locked(c, sa_intv);
}

int ibwa_ctx_expand_sa(ibwa_ctx_t *c) {
  if (!c->sa_loaded[0] || !c->sa_loaded[1]) return fail(IBWA_ENOINDEX, "sampled SA of both strands needed");
  if (c->jump_ready || c->sa_expanded) return 0;  // full SA already resident
  if (c->share_src) return fail(IBWA_EINVAL, "expand_sa: this context shares another context's index");
  HIPCHK(enter(c));
  for (int s = 0; s < 2; ++s) {
    if (int rc = c->sa_full[s].ensure(((uint64_t)c->ix[s].seq_len + 1) * 4)) return rc;
    HIPCHK(expand_sa(c->ix[s], c->sa_s[s].as<uint32_t>(), c->sa_intv, c->sa_full[s].as<uint32_t>(), c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  c->sa_expanded = true;
  return 0;
}

int ibwa_sa2pos(ibwa_ctx_t *c, int64_t n, const uint8_t *strand, const uint32_t *k, const uint32_t *len,
                uint64_t offset, uint64_t *pos) {
  if (n < 0) return fail(IBWA_EINVAL, "n < 0");
  if (!c->loaded[0] || !c->loaded[1]) return fail(IBWA_ENOINDEX, "index not loaded");
  const bool full = (c->jump_ready || c->sa_expanded) && !c->sa_walk;
  if (!full && (!c->sa_loaded[0] || !c->sa_loaded[1])) return fail(IBWA_ENOINDEX, "no suffix array loaded");
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t sl = c->ix[strand[i] ? 0 : 1].seq_len;
    if (k[i] > sl) return fail(IBWA_EINVAL, "hit %lld: row %u > seq_len %u", (long long)i, k[i], sl);
  }
  c->stats.ms_sa2pos = 0;
  if (n == 0) return 0;
  HIPCHK(enter(c));
  // one staging buffer: strand bytes, rows, lengths in; positions + walk lengths out
  const uint64_t o_k = (n + 15) / 16 * 16, o_len = o_k + n * 4, in_bytes = o_len + n * 4;
  if (int rc = c->h2p_in.ensure(in_bytes)) return rc;
  if (int rc = c->h2p_out.ensure(n * 12)) return rc;
  uint8_t *din = c->h2p_in.as<uint8_t>();
  HIPCHK(hipMemcpyAsync(din, strand, n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(din + o_k, k, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(din + o_len, len, n * 4, hipMemcpyHostToDevice, c->stream));
  SaArgs a = {};
  for (int s = 0; s < 2; ++s) {
    a.ix[s] = c->ix[s];
    a.sa[s] = full ? c->sa_full[s].as<uint32_t>() : c->sa_s[s].as<uint32_t>();
    a.intv[s] = full ? 1 : c->sa_intv;
  }
  a.strand = din;
  a.k = reinterpret_cast<const uint32_t *>(din + o_k);
  a.len = reinterpret_cast<const uint32_t *>(din + o_len);
  a.n = n;
  a.offset = offset;
  a.pos = c->h2p_out.as<uint64_t>();
  a.steps = reinterpret_cast<uint32_t *>(c->h2p_out.as<uint8_t>() + n * 8);
  HIPCHK(hipEventRecord(c->ev[0], c->stream));
  HIPCHK(launch_sa2pos(a, full, c->stream));
  HIPCHK(hipEventRecord(c->ev[1], c->stream));
  HIPCHK(hipMemcpyAsync(pos, a.pos, n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->stats.ms_sa2pos = ms;
  c->stats.sa2pos_full = full;
  return 0;
}

int ibwa_host_alloc(uint64_t bytes, void **p) {
  if (!p) return fail(IBWA_EINVAL, "null pointer");
  hipError_t e = hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault);
  if (e != hipSuccess) return fail(IBWA_EHIP, "hipHostMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
  return 0;
}

int ibwa_host_free(void *p) {
  if (p) HIPCHK(hipHostFree(p));
  return 0;
}

int ibwa_fq_parse(ibwa_ctx_t *c, const void *raw, uint64_t nbytes, int mode, int trim_qual, int64_t *n_rec,
                  uint64_t *consumed, int *not_strict, int32_t *rec_len, uint32_t *rec_L, int64_t cap) {
  if (!c || !raw || !n_rec || !consumed || !not_strict || cap < 0) return fail(IBWA_EINVAL, "fq_parse: bad arguments");
  if (nbytes >= 0xFFFF0000ull) return fail(IBWA_EINVAL, "fq_parse: a block of %llu bytes (< 4 GiB)", (unsigned long long)nbytes);
  if (((unsigned)mode >> 24) > 15) return fail(IBWA_EINVAL, "the maximum barcode length is 15");
  *n_rec = 0;
  *consumed = 0;
  *not_strict = 0;
  c->fq_kept = 0;
  c->fq_ms = 0;
  if (nbytes == 0) return 0;
  HIPCHK(enter(c));
  const uint64_t padded = fq_padded_bytes(nbytes);
  // a strict line holds >= 2 bytes, and records of real reads far more: past cap_lines the block
  // simply ends earlier (the caller parses on from *consumed)
  const uint64_t cap_lines = std::min<uint64_t>(nbytes / 12 + 64, 0xFFFFFF00ull);
  const uint64_t max_rec = cap_lines / 4 + 1, n_tiles = padded / 16384;
  if (!c->fqs) c->fqs = new FqScratch();
  FqScratch &S = *c->fqs;
  S.last = nullptr;
  if (int rc = S.raw.ensure(padded)) return rc;
  if (int rc = S.tile.ensure(n_tiles * 8 + 8)) return rc;
  if (int rc = S.nl.ensure(cap_lines * 4)) return rc;
  if (int rc = S.cnt.ensure(16)) return rc;
  if (int rc = S.len.ensure(max_rec * 4)) return rc;
  if (int rc = S.L.ensure(max_rec * 4)) return rc;
  if (int rc = S.key.ensure(max_rec * 8)) return rc;
  // the kept reads' codes: at most half the block (a strict record of L bases takes 2 L + 4 bytes)
  if (int rc = c->fq_codes.ensure(nbytes / 2 + 16)) return rc;
  if (int rc = c->fq_offk.ensure(max_rec * 8)) return rc;
  if (int rc = c->fq_lenk.ensure(max_rec * 4)) return rc;
  FqBufs B;
  B.raw = S.raw.as<uint8_t>();
  B.tile_cnt = S.tile.as<uint32_t>();
  B.tile_base = B.tile_cnt + n_tiles;
  B.nl = S.nl.as<uint32_t>();
  B.cap_lines = (uint32_t)cap_lines;
  B.n_lines = S.cnt.as<uint32_t>();
  B.bad = B.n_lines + 1;
  B.rec_len = S.len.as<int32_t>();
  B.rec_L = S.L.as<uint32_t>();
  B.rec_key = S.key.as<uint64_t>();
  B.codes = c->fq_codes.as<uint8_t>();
  B.offk = c->fq_offk.as<uint64_t>();
  B.lenk = c->fq_lenk.as<uint32_t>();
  const FqOpt o{(int)((unsigned)mode >> 24), trim_qual, (mode & IBWA_MODE_IL13) ? 1 : 0};
  size_t tb = 0;
  HIPCHK(fq_parse_launch(B, nbytes, o, nullptr, &tb, c->stream));
  if (int rc = S.tmp.ensure(tb + 256)) return rc;
  HIPCHK(hipEventRecord(c->ev[6], c->stream));
  // the padding and the counters' initial values come from pinned host memory (copy engine), not
  // from memsets (kernels)
  if (!S.hinit) {
    void *h = nullptr;
    HIPCHK(hipHostMalloc(&h, 8 + 2 * FQ_PAD_MAX, 0));
    memset(h, 0, 8 + 2 * FQ_PAD_MAX);
    static_cast<uint32_t *>(h)[1] = 0xFFFFFFFFu;
    S.hinit = static_cast<uint32_t *>(h);
  }
  HIPCHK(S.h2d(S.raw.p, raw, nbytes, c->stream));
  if (padded - nbytes <= 2 * FQ_PAD_MAX)
    HIPCHK(hipMemcpyAsync(S.raw.as<uint8_t>() + nbytes, S.hinit + 2, padded - nbytes, hipMemcpyHostToDevice, c->stream));
  else
    HIPCHK(hipMemsetAsync(S.raw.as<uint8_t>() + nbytes, 0, padded - nbytes, c->stream));
  HIPCHK(fq_parse_launch(B, nbytes, o, S.tmp.p, &tb, c->stream, S.hinit));
  HIPCHK(hipEventRecord(c->ev[7], c->stream));
  uint32_t cnt[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(cnt, S.cnt.p, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, c->ev[6], c->ev[7]));
  c->fq_ms = ms;
  const uint64_t complete = cnt[0] / 4;
  uint64_t n = std::min<uint64_t>(complete, cnt[1]);
  *not_strict = cnt[1] < complete && n == cnt[1];
  if (n > (uint64_t)cap) {  // the caller takes at most cap records: the block ends at the last of them
    n = (uint64_t)cap;
    *not_strict = 0;
  }
  if (n == 0) return 0;
  uint32_t last_nl = 0;
  HIPCHK(hipMemcpy(&last_nl, S.nl.as<uint32_t>() + 4 * n - 1, 4, hipMemcpyDeviceToHost));
  if (rec_len) HIPCHK(hipMemcpy(rec_len, S.len.p, n * 4, hipMemcpyDeviceToHost));
  if (rec_L) HIPCHK(hipMemcpy(rec_L, S.L.p, n * 4, hipMemcpyDeviceToHost));
  uint64_t key = 0;
  int32_t ll = 0;
  HIPCHK(hipMemcpy(&key, S.key.as<uint64_t>() + n - 1, 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(&ll, S.len.as<int32_t>() + n - 1, 4, hipMemcpyDeviceToHost));
  c->fq_kept = (int64_t)(key >> 32) + (ll >= 0 ? 1 : 0);
  S.last = c;
  *n_rec = (int64_t)n;
  *consumed = (uint64_t)last_nl + 1;
  return 0;
}

int ibwa_fq_share_scratch(ibwa_ctx_t *dst, const ibwa_ctx_t *src) {
  if (!dst || !src || dst == src) return fail(IBWA_EINVAL, "fq_share_scratch: bad arguments");
  if (dst->device != src->device)
    return fail(IBWA_EINVAL, "fq_share_scratch: contexts on devices %d and %d", dst->device, src->device);
  ibwa_ctx *s = const_cast<ibwa_ctx *>(src);
  HIPCHK(enter(s));
  if (!s->fqs) s->fqs = new FqScratch();
  if (dst->fqs == s->fqs) return 0;
  if (dst->fqs) {
    HIPCHK(enter(dst));
    dst->fqs->unref();
  }
  dst->fqs = s->fqs;
  ++dst->fqs->refs;
  return 0;
}

int ibwa_fq_offset(const ibwa_ctx_t *c, int64_t r, uint64_t *off) {
  if (!c || !off || r < 0) return fail(IBWA_EINVAL, "fq_offset: bad arguments");
  *off = 0;
  if (r == 0) return 0;
  HIPCHK(enter(c));
  if (!c->fqs || !c->fqs->nl.p || c->fqs->last != c)
    return fail(IBWA_EINVAL, "fq_offset: this context's block is not the last one parsed in its scratch");
  uint32_t x = 0;
  HIPCHK(hipMemcpy(&x, c->fqs->nl.as<uint32_t>() + 4 * r - 1, 4, hipMemcpyDeviceToHost));
  *off = (uint64_t)x + 1;
  return 0;
}

int ibwa_fq_stats(const ibwa_ctx_t *c, int64_t *kept, double *ms) {
  if (kept) *kept = c->fq_kept;
  if (ms) *ms = c->fq_ms;
  return 0;
}

int ibwa_batch_stage_fq(ibwa_ctx_t *c, const ibwa_ctx_t *src, int64_t first, int64_t n, int max_len) {
  if (!c || !src || first < 0 || n < 0 || first + n > src->fq_kept)
    return fail(IBWA_EINVAL, "stage_fq: reads [%lld, %lld) outside the %lld kept reads of the parsed block",
                (long long)first, (long long)(first + n), (long long)(src ? src->fq_kept : 0));
  if (c->device != src->device) return fail(IBWA_EINVAL, "stage_fq: contexts on devices %d and %d", c->device, src->device);
  if (max_len > 65535) return fail(IBWA_EINVAL, "read length %d > 65535 is not supported", max_len);
  HIPCHK(enter(c));
  HIPCHK(hipStreamSynchronize(src->stream));  // the block is parsed
  // no copy: the batch is a view of the parsed block's kept reads (their codes, offsets into them
  // and lengths), which must stay as they are until this context's runs over it are over -- a
  // copy would be a kernel waiting for CUs that the other contexts' persistent searches hold
  c->v_seq = src->fq_codes.as<uint8_t>();
  c->v_off = src->fq_offk.as<uint64_t>() + first;
  c->v_len = src->fq_lenk.as<uint32_t>() + first;
  c->n = n;
  c->seq_bytes = 0;
  c->max_len = max_len;
  return 0;
}

int ibwa_batch_stage(ibwa_ctx_t *c, int64_t n, const uint8_t *seq, const uint64_t *off, const uint32_t *len) {
  if (n < 0) return fail(IBWA_EINVAL, "n < 0");
  HIPCHK(enter(c));
  uint64_t bytes = 0;
  int max_len = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (len[i] > 65535) return fail(IBWA_EINVAL, "read %lld: length %u > 65535 is not supported", (long long)i, len[i]);
    bytes = std::max<uint64_t>(bytes, off[i] + len[i]);
    max_len = std::max<int>(max_len, (int)len[i]);
  }
  if (int rc = c->d_seq.ensure(bytes + 16)) return rc;
  if (int rc = c->d_off.ensure(n * 8 + 8)) return rc;
  if (int rc = c->d_len.ensure(n * 4 + 4)) return rc;
  if (bytes) HIPCHK(hipMemcpyAsync(c->d_seq.p, seq, bytes, hipMemcpyHostToDevice, c->stream));
  if (n) {
    HIPCHK(hipMemcpyAsync(c->d_off.p, off, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_len.p, len, n * 4, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  c->n = n;
  c->seq_bytes = bytes;
  c->max_len = max_len;
  c->v_seq = c->d_seq.as<uint8_t>();
  c->v_off = c->d_off.as<uint64_t>();
  c->v_len = c->d_len.as<uint32_t>();
  return 0;
}

static int check_opt(const ibwa_gap_opt_t *o) {
  if (o->s_mm <= 0 || o->s_gapo <= 0 || o->s_gape <= 0)
    return fail(IBWA_EINVAL,
                "zero/negative penalties (-M %d -O %d -E %d) are unsupported: the reference reads uninitialised "
                "stack slots (bwtgap.c:60) or crashes on them",
                o->s_mm, o->s_gapo, o->s_gape);
  if (o->seed_len < 0 || o->max_gape < 0 || o->max_gapo < 0) return fail(IBWA_EINVAL, "negative option");
  return 0;
}

// Runs one pass of (width, search) over `lanes` reads.  ids == nullptr: reads base..base+lanes-1.
static int run_pass(ibwa_ctx *c, AlnArgs A, int64_t base, int64_t lanes, const int64_t *d_ids, float *ms_w,
                    float *ms_s) {
  (void)base;
  A.n = lanes;
  A.ids = d_ids;
  HIPCHK(hipEventRecord(c->ev[0], c->stream));
  HIPCHK(launch_width(A, c->block, c->stream));
  HIPCHK(hipEventRecord(c->ev[1], c->stream));
  HIPCHK(launch_search(A, c->block, c->stream));
  HIPCHK(hipEventRecord(c->ev[2], c->stream));
  HIPCHK(hipEventSynchronize(c->ev[2]));
  float a = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
  HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
  *ms_w += a;
  *ms_s += b;
  return 0;
}

int ibwa_batch_run(ibwa_ctx_t *c, const ibwa_gap_opt_t *opt, int batch_max_len) {
  auto t0 = std::chrono::steady_clock::now();
  // host-phase timestamps (IBWA_VERBOSE)
  auto since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  if (!c->loaded[0] || !c->loaded[1]) return fail(IBWA_ENOINDEX, "load both .bwt and .rbwt first");
  if (c->ix[0].seq_len != c->ix[1].seq_len) return fail(IBWA_EINVAL, ".bwt and .rbwt lengths differ");
  if (int rc = check_opt(opt)) return rc;
  c->fetched = false;
  HIPCHK(enter(c));
  memset(&c->stats, 0, sizeof(c->stats));
  g_alloc_ms = 0;
  c->hpop_valid = false;  // set again by a gapped run that leaves resume states
  const int64_t n = c->n;
  const int max_len = std::max(batch_max_len, c->max_len);

  // batch-level local_opt (bwtaln.c:86-93)
  AlnOpt o = {};
  o.s_mm = opt->s_mm; o.s_gapo = opt->s_gapo; o.s_gape = opt->s_gape; o.mode = opt->mode;
  o.indel_end_skip = opt->indel_end_skip; o.max_del_occ = opt->max_del_occ; o.max_entries = opt->max_entries;
  o.fnr_pos = opt->fnr > 0.0f;
  int batch_md = o.fnr_pos ? ibwa_cal_maxdiff(max_len, 0.02, opt->fnr) : opt->max_diff;
  o.max_diff = opt->max_diff;
  o.max_gapo = batch_md < opt->max_gapo ? batch_md : opt->max_gapo;
  o.max_gape = opt->max_gape; o.max_seed_diff = opt->max_seed_diff; o.seed_len = opt->seed_len;
  o.max_top2 = opt->max_top2;
  o.n_stacks = (batch_md + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape;
  if (o.n_stacks <= 0 || o.n_stacks > (1 << 20)) return fail(IBWA_EINVAL, "invalid stack size %d", o.n_stacks);

  // per-length max_diff table
  std::vector<int16_t> tab(max_len + 1);
  for (int l = 0; l <= max_len; ++l) tab[l] = (int16_t)(o.fnr_pos ? ibwa_cal_maxdiff(l, 0.02, opt->fnr) : opt->max_diff);
  if (int rc = c->d_tab.ensure(tab.size() * 2)) return rc;
  HIPCHK(hipMemcpyAsync(c->d_tab.p, tab.data(), tab.size() * 2, hipMemcpyHostToDevice, c->stream));

  AlnArgs A = {};
  A.ix[0] = c->ix[0];
  A.ix[1] = c->ix[1];
  A.seq = c->v_seq;
  A.off = c->v_off;
  A.len = c->v_len;
  A.maxdiff_tab = c->d_tab.as<int16_t>();
  A.wlen1 = (uint32_t)max_len + 1;
  A.wstride = 2ull * A.wlen1 + 2ull * ((uint64_t)std::max(opt->seed_len, 0) + 1);
  A.o = o;
  // k_width's one-row steps from the text (1: when SA / text are resident, 2: derive them)
  if (c->width_jump == 2 && !(c->exact_path && !o.fnr_pos && opt->max_diff == 0))
    if (int rc = ensure_jump(c)) return rc;
  if (c->width_jump && c->jump_ready) {
    for (int s = 0; s < 2; ++s) {
      A.jsa[s] = c->sa_full[s].as<uint32_t>();
      A.jtxt[s] = c->txt2[s].as<uint32_t>();
    }
  }

  const bool exact_path = c->exact_path && !o.fnr_pos && opt->max_diff == 0 && opt->max_entries >= 2;
  c->stats.path = exact_path ? 1 : 0;
  if (exact_path) {
    c->stream_out = false;
    A.aln_cap = c->aln_cap;
    A.n = n;
    if (int rc = c->d_aln.ensure(std::max<int64_t>(n, 1) * (uint64_t)A.aln_cap * 16)) return rc;
    if (int rc = c->d_naln.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
    if (int rc = c->d_status.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
    if (int rc = c->d_counter.ensure(64)) return rc;
    A.aln = c->d_aln.as<uint4>();
    A.n_aln = c->d_naln.as<int32_t>();
    A.status = c->d_status.as<uint32_t>();
    if (int rc = ensure_kmer(c)) return rc;
    if (int rc = ensure_jump(c)) return rc;
    c->stats.kmer_k = c->kmer_K;
    HIPCHK(hipEventRecord(c->ev[0], c->stream));
    const uint32_t stride = exact_record_stride(max_len);
    if (int rc = c->d_rec.ensure(std::max<int64_t>(n, 1) * (uint64_t)stride * 16)) return rc;
    const uint32_t *jump[6] = {c->sa_full[0].as<uint32_t>(), c->sa_full[1].as<uint32_t>(),
                               c->isa_full[0].as<uint32_t>(), c->isa_full[1].as<uint32_t>(),
                               c->txt2[0].as<uint32_t>(), c->txt2[1].as<uint32_t>()};
    const bool use_jump = c->jump_ready && c->exact_jump;
    c->stats.path = use_jump ? 3 : 1;
    HIPCHK(launch_exact(A, c->o64[0].as<uint4>(), c->o64[1].as<uint4>(), c->kt[0].as<uint2>(),
                        c->kt[1].as<uint2>(), c->kmer_K, c->d_rec.as<uint4>(), stride,
                        c->d_counter.as<unsigned long long>(), c->exact_blocks, c->ev[2], use_jump ? jump : nullptr,
                        c->stream));
    HIPCHK(hipEventRecord(c->ev[1], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[1]));
    float ms_pack = 0, ms = 0;
    HIPCHK(hipEventElapsedTime(&ms_pack, c->ev[0], c->ev[2]));
    HIPCHK(hipEventElapsedTime(&ms, c->ev[2], c->ev[1]));
    c->stats.ms_width = ms_pack;  // the exact path's pre-pass: read packing
    c->stats.ms_search = ms;
    c->stats.n_launch_search = 1;
    c->aln_cap_used = A.aln_cap;
    c->h_naln.resize(n);
    c->h_status.clear();
    c->naln_on_host = false;  // results stay in HBM; ibwa_batch_fetch copies them
    c->retry_ids.clear();
    c->patch_ids.clear();
    c->patch_alns.clear();
    c->retry_pass.clear();
    c->resumed_ids.clear();
    c->stats.ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->stats.ms_alloc = g_alloc_ms;
    return 0;
  }

  // persistent gapped search (gapped.hip) when the options fit its entry bit fields
  const bool v2 = c->gapped_v2 && batch_md + 1 <= 31 && o.max_gapo <= 7 && o.max_gape <= 15 &&
                  gapped_lds_bytes(o.n_stacks, 64, true, 0, 0, 1, 4096) <= 65536 && max_len <= 65535;
  float ms_w = 0, ms_s = 0;
  c->stream_out = v2;
  bool resume_states = false;  // the first pass left resume states (GapArgs::rdump)
  c->hpop_valid = false;
  c->resumed_ids.clear();
  float res_ms = 0, res_w = 0;  // the cooperative launches over resumed reads (after each chunk)
  int64_t res_ok = 0;           // reads they resolved
  c->stats.n_resumed = 0;
  c->stats.resume_records = 0;
  c->stats.resume_records_peak = c->stats.resume_records_cap = 0;
  c->stats.coop_pages_peak = c->stats.coop_pages_cap = 0;
  if (v2) {
    if (int rc = ensure_kmer(c)) return rc;
    c->stats.path = 2;
    if (c->width_tab && c->ltab_K > 0 && c->ix[0].seq_len < LTAB_MARK) {  // k_width's leading steps
      A.ltab[0] = c->ltab[0].as<uint2>();
      A.ltab[1] = c->ltab[1].as<uint2>();
      A.tab_k = (uint32_t)c->ltab_K;
    }
    // equal chunks of at most gap_reads_per_chunk reads: every launch ends with a tail in which
    // only its slowest reads still run, so fewer (and balanced) launches waste less -- but no more
    // reads than an earlier run's resume states per read let the state buffer hold (150 bp at 2 %:
    // 3 chunks of 6.7 M instead of 2 of 10 M, whose overflowing states start over: 5160 -> 4972 ms
    // per 20 M reads in the round-4 footprint sweep)
    // LDS: bucket heads + free slots + page table per lane, the page bitmap per workgroup
    const uint32_t LG = 13, P0 = c->gap_cap1;
    const int max_pages = (int)std::min<uint32_t>(7, (65536u - P0) >> LG);
    auto ppb_of = [&](int blk) { return std::max(1, c->gap_pages_per_block * blk / 256); };
    // LDS widths (gapped.hip LW): bids clamped to max_diff + 1 in 3 bits and to max_seed_diff + 1
    // in 2, a ring of 16 bucket heads (the largest penalty <= 15), and 3 workgroups per CU still fit
    const int maxpen = std::max(o.s_mm, std::max(o.s_gapo, o.s_gape));
    const uint32_t cw_rw = (uint32_t)(max_len + 15) / 16;
    const uint32_t cw_sb = max_len > o.seed_len ? (uint32_t)o.seed_len + 1u : 0u;
    const uint32_t cw_words = 1u + cw_rw + ((uint32_t)max_len + 1u + cw_sb + 3u) / 4u;
    // The LDS rows grow with the read (100 bp: 208 B per lane, 3 workgroups of 256 lanes per CU); longer
    // reads take the workgroup size that keeps the most waves per CU (150 bp: 9 of 64 lanes) as long
    // as that is at least gap_lw_min_waves
    int lw_block = 256, lw_waves = 0;
    for (int blk : {256, 128, 64}) {
      const size_t b = gapped_lds_bytes(o.n_stacks, blk, false, max_pages, ppb_of(blk), 64, 0, (int)cw_words);
      if (b > 65536) continue;
      const int waves = std::min<int>(c->gap_blocks_per_cu * 4, (int)(160 * 1024 / b) * (blk / 64));
      if (waves > lw_waves) lw_waves = waves, lw_block = blk;
    }
    const bool lw = c->gap_lw && !c->diag && batch_md <= 6 && o.max_seed_diff >= 0 && o.max_seed_diff <= 2 && maxpen <= 15 &&
                    max_pages <= GAP_MAX_PAGES && lw_waves >= c->gap_lw_min_waves;
    auto lds_of = [&](int blk) {
      return gapped_lds_bytes(o.n_stacks, blk, false, max_pages, ppb_of(blk), 64, 0, lw ? (int)cw_words : 0);
    };
    const int block = lw ? lw_block : lds_of(256) <= 65536 ? 256 : lds_of(128) <= 65536 ? 128 : 64;
    const int ppb = ppb_of(block);
    const size_t lds = lds_of(block);
    const int per_cu = std::max<int>(
        1, std::min<int>(c->gap_blocks_per_cu * 256 / block, (int)(160 * 1024 / std::max<size_t>(lds, 1))));
    const bool resume = lw && c->gap_resume && c->gap_coop && max_len <= COOP_MAXLEN && o.n_stacks <= COOP_NSTK;
    // (Round 5 also overlapped a chunk's cooperative pass with the next chunk's first pass on a
    // second stream; measured 3-10 % slower at 50 M reads in both of its variants, it was removed in
    // round 6: DESIGN §4.4.1.)
    int64_t per_chunk = c->gap_reads_per_chunk;
    if (c->resume_need > 0)  // (the state buffer's bound no lower than 65 536 reads; gap_reads_per_chunk may be)
      per_chunk = std::min<int64_t>(per_chunk, std::max<int64_t>(65536, (int64_t)((double)(((uint64_t)c->gap_resume_gb << 30) / 16) /
                                                                                   (1.15 * c->resume_need))));
    const int64_t n_chunks = (std::max<int64_t>(n, 1) + per_chunk - 1) / per_chunk;
    const int64_t chunk = (std::max<int64_t>(n, 1) + n_chunks - 1) / n_chunks;
    // persistent grid: fills the chip, but a small batch gets only the lanes it can use, so
    // its per-lane scratch and page pools are sized by the batch, not the worst case
    const int blocks = (int)std::min<int64_t>((int64_t)c->n_cus * per_cu, (chunk + block - 1) / block);
    const uint64_t lanes = (uint64_t)blocks * block;
    const uint64_t aln_total = std::max<uint64_t>((uint64_t)n * c->gap_stream_per_read, c->gap_stream_min);
    if (int rc = c->d_wbuf.ensure(chunk * A.wstride * 8)) return rc;
    if (int rc = c->d_nN.ensure(chunk * 2 + 2)) return rc;
    if (lw) {
      if (int rc = c->d_cw.ensure(chunk * (uint64_t)cw_words * 4)) return rc;
      if (int rc = c->d_ptabg.ensure(lanes * GAP_MAX_PAGES * 2)) return rc;
    }
    // resume states of the early hand-offs: per read 1 + the state's offset (0: none), then per state
    // buffer its fill counter and the count of states stored
    uint64_t rd_cap = 0;
    if (resume) {
      // the buffer holds one first-pass chunk's states at a time (cleared after each chunk)
      const double per_read = std::max<double>(c->gap_resume_recs, 1.15 * c->resume_need);
      rd_cap = std::min<uint64_t>(((uint64_t)c->gap_resume_gb << 30) / 16, (uint64_t)((double)chunk * per_read) + (1u << 16));
      if (c->gap_resume_records > 0) rd_cap = (uint64_t)c->gap_resume_records;
      if (int rc = c->d_rdump.ensure(rd_cap * 16)) return rc;
      c->stats.resume_records_cap = (int64_t)rd_cap;
      if (int rc = c->d_roff.ensure(((uint64_t)n + 4) * 8)) return rc;
      HIPCHK(zero_async(c->d_roff.p, ((uint64_t)n + 4) * 8, c->stream));
      if (int rc = c->d_hpop.ensure(((uint64_t)n + 1) * 4)) return rc;
      HIPCHK(zero_async(c->d_hpop.p, ((uint64_t)n + 1) * 4, c->stream));
      resume_states = true;
      c->hpop_valid = true;
    }
    // and smaller static slot regions (4096: 5859 -> 5840 ms per 50M-read step, hits identical,
    // profiles/r03_pool_cap_sweep.log; the page table and max_pages are the same for both sizes)
    const uint32_t P0r = resume ? std::min<uint32_t>(P0, c->gap_resume_cap1) : P0;
    if (int rc = c->d_ent.ensure(lanes * P0r * 16)) return rc;
    // with resume states a read leaves the first pass by 2 000 iterations, so few stacks outgrow the
    // static slots: a smaller page pool (same time at 50M reads, profiles/r03_pool_chunk_sweep.log)
    const int ppb_run = resume ? std::min(ppb, std::max(1, c->gap_resume_ppb * block / 256)) : ppb;
    if (int rc = c->d_pool.ensure((uint64_t)blocks * ppb_run * (16ull << LG))) return rc;
    if (int rc = c->d_aln.ensure(aln_total * 16)) return rc;
    if (int rc = c->d_aoff.ensure(std::max<int64_t>(n, 1) * 8)) return rc;
    if (int rc = c->d_naln.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
    if (int rc = c->d_status.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
    if (int rc = c->d_counter.ensure(64)) return rc;
    HIPCHK(zero_async(c->d_counter.as<unsigned long long>() + 1, 8, c->stream));
    // The reads of chunk [b0, b0 + cnt) that left a resume state go through the cooperative pass right
    // after their chunk's first pass, so the state buffer holds one chunk's states at a time: a read
    // it resolves is done (status 0), one it hands on starts over in the passes below.
    // Launch part: select the resumed reads of chunk [b0, b0 + cnt), order them largest stack first,
    // then k_coop on stream st.  The widths and N counts are the chunk's own first-pass rows, still in
    // place (their gap_shadow updates included).
    struct CoopRun {
      int64_t lanes = 0, b0 = 0, cnt = 0;
      uint32_t pool_pages = 0;
      const int64_t *ids = nullptr;
    };
    auto coop_launch = [&](int64_t b0, int64_t cnt, hipStream_t st, hipEvent_t *evs, CoopRun &R) -> int {
      R = CoopRun();
      R.b0 = b0;
      R.cnt = cnt;
      size_t tb = 0;
      HIPCHK(select_resumed(c->d_roff.as<uint64_t>(), b0, cnt, c->d_status.as<uint32_t>(), nullptr, nullptr, nullptr,
                            nullptr, &tb, st));
      if (int rc = c->d_seltmp.ensure(tb + 16)) return rc;
      if (int rc = c->d_ids.ensure(cnt * 8)) return rc;
      if (int rc = c->d_selst.ensure(cnt * 4)) return rc;
      unsigned long long *d_cnt = c->d_counter.as<unsigned long long>() + 5;
      HIPCHK(select_resumed(c->d_roff.as<uint64_t>(), b0, cnt, c->d_status.as<uint32_t>(), c->d_ids.as<int64_t>(),
                            c->d_selst.as<uint32_t>(), d_cnt, c->d_seltmp.p, &tb, st));
      unsigned long long lanes_u = 0;
      HIPCHK(hipMemcpyAsync(&lanes_u, d_cnt, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const int64_t lanes = (int64_t)lanes_u;
      R.lanes = lanes;
      if (lanes <= 0) return 0;
      uint32_t stg_log2 = 10;
      while ((1u << stg_log2) < (uint32_t)c->coop_stg_room * (9u * (uint32_t)(max_len + 1) + 16u)) ++stg_log2;
      const int full_blocks = c->n_cus * c->coop_waves_per_cu;
      const int blocks = (int)std::min<int64_t>(full_blocks, lanes);
      const uint32_t freecap = 4096, hcap = 4096;
      const uint64_t pool_bytes = std::min<uint64_t>(
          c->pool_bytes(max_len), std::max<uint64_t>(1ull << 30, c->pool_bytes(max_len) / full_blocks * blocks));
      const uint32_t pool_pages = c->coop_pool_pages ? c->coop_pool_pages : (uint32_t)(pool_bytes / (COOP_PG * 16ull));
      R.pool_pages = pool_pages;
      if (int rc = c->c_stg.ensure((uint64_t)blocks * 64 * 16 << stg_log2)) return rc;
      if (int rc = c->c_dir.ensure((uint64_t)blocks * COOP_NSTK * COOP_MAXP * 4)) return rc;
      if (int rc = c->c_free.ensure((uint64_t)blocks * freecap * 4)) return rc;
      if (int rc = c->c_hits.ensure((uint64_t)blocks * hcap * 16)) return rc;
      if (int rc = c->c_recb.ensure((uint64_t)blocks * COOP_RREC * 16)) return rc;
      if (int rc = c->c_pool.ensure((uint64_t)pool_pages * COOP_PG * 16)) return rc;
      if (int rc = c->c_next.ensure(64)) return rc;
      if (int rc = c->r_status.ensure(lanes * 4)) return rc;
      // largest first-pass stack first, as in the main cooperative pass below
      const int64_t *ids = c->d_ids.as<int64_t>();
      if (lanes > 1) {
        size_t ob = 0;
        HIPCHK(order_heavy_first(nullptr, nullptr, lanes, nullptr, nullptr, nullptr, nullptr, &ob, st));
        if (int rc = c->d_ordk.ensure(lanes * 8)) return rc;
        if (int rc = c->d_ordi.ensure(lanes * 8)) return rc;
        if (int rc = c->d_ordids.ensure(lanes * 8)) return rc;
        if (int rc = c->d_ordtmp.ensure(ob + 16)) return rc;
        HIPCHK(order_heavy_first(c->d_selst.as<uint32_t>(), c->d_ids.as<int64_t>(), lanes, c->d_ordk.as<uint32_t>(),
                                 c->d_ordi.as<uint32_t>(), c->d_ordids.as<int64_t>(), c->d_ordtmp.p, &ob, st));
        ids = c->d_ordids.as<int64_t>();
      }
      R.ids = ids;
      CoopArgs K = {};
      K.ix[0] = c->ix[0];
      K.ix[1] = c->ix[1];
      K.o64[0] = c->o64[0].as<uint4>();
      K.o64[1] = c->o64[1].as<uint4>();
      K.seq = A.seq;
      K.off = A.off;
      K.len = A.len;
      K.ids = ids;
      K.n = lanes;
      K.out_by_id = 1;
      K.maxdiff_tab = A.maxdiff_tab;
      K.wstride = A.wstride;
      K.wlen1 = A.wlen1;
      K.wbuf = c->d_wbuf.as<uint2>();
      K.wb_base = b0;
      K.nN = c->d_nN.as<uint16_t>();
      K.stg = c->c_stg.as<uint4>();
      K.stg_log2 = stg_log2;
      K.dir = c->c_dir.as<uint32_t>();
      K.freel = c->c_free.as<uint32_t>();
      K.freecap = freecap;
      K.pool = c->c_pool.as<uint4>();
      K.pool_pages = pool_pages;
      K.pool_next = c->c_next.as<uint32_t>();
      K.hits = c->c_hits.as<uint4>();
      K.recb = c->c_recb.as<uint4>();
      K.rdump = c->d_rdump.as<uint4>();
      K.roff = c->d_roff.as<uint64_t>();
      K.hcap = hcap;
      K.max_iters = 1u << 24;
      K.aln = c->d_aln.as<uint4>();
      K.aln_total = c->stream_total;
      K.aln_next = c->d_counter.as<unsigned long long>() + 1;
      K.aln_off = c->d_aoff.as<uint64_t>();
      K.n_aln = c->d_naln.as<int32_t>();
      K.status = c->r_status.as<uint32_t>();
      K.o = o;
      HIPCHK(hipEventRecord(evs[0], st));
      HIPCHK(hipEventRecord(evs[2], st));
      K.fix_status = c->d_status.as<uint32_t>();  // resume_fixup, as each read ends
      K.fix_roff = c->d_roff.as<uint64_t>();
      HIPCHK(launch_coop(K, c->d_counter.as<unsigned long long>(), blocks, st));
      HIPCHK(hipEventRecord(evs[1], st));
      return 0;
    };
    // Finish part (after the launch's kernels): the reads it resolved, the state buffer's use, and the
    // buffer's fill counter back to 0 for the chunk after next.
    auto coop_finish = [&](CoopRun &R, hipStream_t st, hipEvent_t *evs) -> int {
      unsigned long long *rdn = c->d_roff.as<unsigned long long>() + n;
      if (R.lanes > 0) {
        HIPCHK(hipEventSynchronize(evs[1]));
        note_coop_pages(c, R.pool_pages);
        float t_all = 0, t_w = 0;
        HIPCHK(hipEventElapsedTime(&t_all, evs[0], evs[1]));
        HIPCHK(hipEventElapsedTime(&t_w, evs[0], evs[2]));
        std::vector<uint32_t> rs(R.lanes);
        std::vector<int64_t> rid(R.lanes);
        HIPCHK(hipMemcpyAsync(rs.data(), c->r_status.p, R.lanes * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(rid.data(), R.ids, R.lanes * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        int64_t ok = 0;
        for (int64_t j = 0; j < R.lanes; ++j)
          if (rs[j] == 0) {
            ++ok;
            c->resumed_ids.push_back(rid[j]);
          }
        res_ms += t_all;
        res_w += t_w;
        res_ok += ok;
        if (c->verbose)
          fprintf(stderr, "[ibwa_amd] chunk at %lld: %lld resumed reads through the cooperative pass, %.1f ms\n",
                  (long long)R.b0, (long long)R.lanes, t_all);
      }
      unsigned long long used = 0;
      HIPCHK(hipMemcpyAsync(&used, rdn, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      c->stats.resume_records += (int64_t)used;
      c->stats.resume_records_peak = std::max<int64_t>(c->stats.resume_records_peak, (int64_t)used);
      if (R.cnt >= 65536) c->resume_need = std::max(c->resume_need, (double)used / (double)R.cnt);
      HIPCHK(zero_async(rdn, 8, st));
      HIPCHK(hipEventRecord(evs[3], st));  // the state buffer may be written again
      return 0;
    };
    auto coop_resumed = [&](int64_t b0, int64_t cnt) -> int {
      CoopRun R;
      hipEvent_t evs[4] = {c->ev[3], c->ev[4], c->ev[5], c->ev[6]};
      if (int rc = coop_launch(b0, cnt, c->stream, evs, R)) return rc;
      return coop_finish(R, c->stream, evs);
    };
    for (int64_t b0 = 0; b0 < n; b0 += chunk) {
      const int64_t cnt = std::min(chunk, n - b0);
      AlnArgs B = A;
      B.n = cnt;
      B.off = A.off + b0;
      B.len = A.len + b0;
      B.wbuf = c->d_wbuf.as<uint2>();
      B.nN = c->d_nN.as<uint16_t>();
      GapArgs G = gap_args(c, A, o, b0, cnt);
      G.wbuf = B.wbuf;
      G.nN = B.nN;
      if (lw) {
        B.cw = c->d_cw.as<uint32_t>();
        B.cw_words = cw_words;
        B.cw_rw = cw_rw;
        G.cw = B.cw;
        G.cw_words = cw_words;
        G.cw_rw = cw_rw;
        G.ptab_g = c->d_ptabg.as<uint16_t>();
      }
      G.ent = c->d_ent.as<uint4>();
      if (lw && c->ltab_K > 0 && c->ix[0].seq_len < LTAB_MARK) {
        G.ltab[0] = c->ltab[0].as<uint2>();
        G.ltab[1] = c->ltab[1].as<uint2>();
        G.tab_k = (uint32_t)c->ltab_K;
      }
      G.cap1 = P0r;
      G.hit_slots = std::min<uint32_t>(c->gap_hit_slots, P0r / 2);
      G.pool = c->d_pool.as<uint4>();
      G.page_log2 = LG;
      G.max_pages = max_pages;
      G.pages_per_block = ppb_run;
      G.aln = c->d_aln.as<uint4>();
      G.aln_total = aln_total;
      c->stream_total = aln_total;
      G.aln_off = c->d_aoff.as<uint64_t>() + b0;
      G.n_aln = c->d_naln.as<int32_t>() + b0;
      G.status = c->d_status.as<uint32_t>() + b0;
      G.max_iters = c->gap_iter_budget;
      G.early_iters = resume ? c->gap_resume_iters : c->gap_early_iters;
      G.early_entries = resume ? c->gap_resume_entries : c->gap_early_entries;
      if (resume) {
        G.rdump = c->d_rdump.as<uint4>();
        G.rd_next = c->d_roff.as<unsigned long long>() + n;
        G.rd_cap = rd_cap;
        G.roff = c->d_roff.as<uint64_t>() + b0;
        G.hpop = c->d_hpop.as<uint32_t>() + b0;
        G.tail_lanes = c->gap_tail_lanes;
        G.tail_iters = c->gap_tail_iters;
      }
      if (c->verbose || c->diag) {
        if (int rc = c->d_iters.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
        G.iters = c->d_iters.as<uint32_t>() + b0;
      }
      if (c->diag) {
        if (int rc = c->d_feat.ensure(std::max<int64_t>(n, 1) * 8)) return rc;
        B.feat = c->d_feat.as<uint16_t>() + b0 * 4;
      }
      if (c->prof_phases) {
        if (int rc = c->d_prof.ensure(256)) return rc;
        HIPCHK(hipMemsetAsync(c->d_prof.p, 0, 256, c->stream));
        G.prof = c->d_prof.as<unsigned long long>();
      }
      HIPCHK(hipEventRecord(c->ev[0], c->stream));
      HIPCHK(launch_width(B, c->block, c->stream));
      HIPCHK(hipEventRecord(c->ev[1], c->stream));
      HIPCHK(launch_gapped(G, c->d_counter.as<unsigned long long>(), blocks, block, false, c->stream));
      HIPCHK(hipEventRecord(c->ev[2], c->stream));
      HIPCHK(hipEventSynchronize(c->ev[2]));
      float a = 0, b = 0;
      HIPCHK(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
      HIPCHK(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
      ms_w += a;
      ms_s += b;
      c->stats.n_launch_width++;
      c->stats.n_launch_search++;
      if (c->verbose) {
        std::vector<uint32_t> it(cnt);
        HIPCHK(hipMemcpy(it.data(), G.iters, cnt * 4, hipMemcpyDeviceToHost));
        uint64_t sum = 0;
        uint32_t mx = 0;
        for (uint32_t v : it) { sum += v; mx = std::max(mx, v); }
        std::sort(it.begin(), it.end());
        fprintf(stderr, "[ibwa_amd] k_gapped: %lld reads, %.3g lane-iterations (%.0f per read, p99 %u, p99.99 %u, "
                "max %u), %.1f ms -> %.3g lane-iterations/s\n", (long long)cnt, (double)sum, (double)sum / cnt,
                it[(size_t)(cnt * 0.99)], it[(size_t)(cnt * 0.9999)], mx, b, sum / (b * 1e-3));
      }
      if (c->prof_phases) {
        unsigned long long pf[19];
        HIPCHK(hipMemcpy(pf, c->d_prof.p, sizeof pf, hipMemcpyDeviceToHost));
        const char *nm[4] = {"claim", "pop", "wait", "rest"};
        double tot = (double)(pf[0] + pf[1] + pf[2] + pf[3]);
        fprintf(stderr, "[ibwa_amd] k_gapped phases (wave cycles, %d waves):", blocks * block / 64);
        for (int q = 0; q < 4; ++q) fprintf(stderr, " %s %.1f%%", nm[q], tot > 0 ? 100.0 * pf[q] / tot : 0.0);
        const double wi = pf[9] ? (double)pf[9] : 1.0;
        fprintf(stderr, "; per wave-iteration: exact %.3f push trips %.3f hits %.3f ends %.3f expansions %.3f "
                "claims %.3f (%llu wave-iterations)\n", pf[4] / wi, pf[5] / wi, pf[6] / wi, pf[7] / wi, pf[8] / wi,
                pf[10] / wi, pf[9]);
        const double li = pf[16] ? (double)pf[16] : 1.0;
        fprintf(stderr, "[ibwa_amd] k_gapped loads per live lane-iteration: block %.3f second block %.3f widths %.3f "
                "seed widths %.3f candidate %.3f; exact steps %.3f (unique interval %.3f) (%.3g live lane-iterations)\n",
                pf[11] / li, pf[12] / li, pf[13] / li, pf[14] / li, pf[15] / li, pf[17] / li, pf[18] / li, (double)pf[16]);
      }
      if (resume_states)
        if (int rc = coop_resumed(b0, cnt)) return rc;
    }
  }
  // first pass, in chunks of lanes_per_chunk reads
  const int64_t chunk = std::min<int64_t>(std::max<int64_t>(n, 1), c->lanes_per_chunk);
  A.cap = c->stack_cap;
  if (!v2) A.aln_cap = c->aln_cap;
  if (!v2) {
  if (int rc = c->d_wbuf.ensure(chunk * A.wstride * 8)) return rc;
  if (int rc = c->d_heads.ensure(chunk * (uint64_t)o.n_stacks * 4)) return rc;
  if (int rc = c->d_ent.ensure(chunk * (uint64_t)A.cap * 16)) return rc;
  if (int rc = c->d_prev.ensure(chunk * (uint64_t)A.cap * 4)) return rc;
  if (int rc = c->d_aln.ensure(std::max<int64_t>(n, 1) * (uint64_t)A.aln_cap * 16)) return rc;
  if (int rc = c->d_naln.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
  if (int rc = c->d_status.ensure(std::max<int64_t>(n, 1) * 4)) return rc;
  A.wbuf = c->d_wbuf.as<uint2>();
  A.heads = c->d_heads.as<uint32_t>();
  A.ent = c->d_ent.as<uint4>();
  A.prev = c->d_prev.as<uint32_t>();
  for (int64_t b0 = 0; b0 < n; b0 += chunk) {
    int64_t lanes = std::min(chunk, n - b0);
    // lane-indexed inputs and outputs: shift the base pointers to this chunk
    AlnArgs B = A;
    B.off = A.off + b0;
    B.len = A.len + b0;
    B.aln = c->d_aln.as<uint4>() + b0 * A.aln_cap;
    B.n_aln = c->d_naln.as<int32_t>() + b0;
    B.status = c->d_status.as<uint32_t>() + b0;
    if (int rc = run_pass(c, B, b0, lanes, nullptr, &ms_w, &ms_s)) return rc;
    c->stats.n_launch_width++;
    c->stats.n_launch_search++;
  }
  }  // !v2
  c->stats.ms_width = ms_w;
  c->stats.ms_search = ms_s;
  c->aln_cap_used = A.aln_cap;

  if (c->verbose) fprintf(stderr, "[ibwa_amd] t %.1f ms: first pass done\n", since());
  // results stay in HBM; the reads handed on (non-zero status) are selected on the device
  c->naln_on_host = false;
  c->h_status.clear();
  c->stream_len = 0;
  c->retry_ids.clear();
  c->patch_ids.clear();
  c->patch_alns.clear();
  c->retry_pass.clear();
  std::vector<uint32_t> rstat;
  if (n) {
    size_t tb = 0;
    HIPCHK(select_handed_on(c->d_status.as<uint32_t>(), n, nullptr, nullptr, nullptr, nullptr, &tb, c->stream));
    if (int rc = c->d_seltmp.ensure(tb + 16)) return rc;
    if (int rc = c->d_ids.ensure(n * 8)) return rc;
    if (int rc = c->d_selst.ensure(n * 4)) return rc;
    if (int rc = c->d_counter.ensure(64)) return rc;
    unsigned long long *d_cnt = c->d_counter.as<unsigned long long>() + 3;
    HIPCHK(select_handed_on(c->d_status.as<uint32_t>(), n, c->d_ids.as<int64_t>(), c->d_selst.as<uint32_t>(), d_cnt,
                            c->d_seltmp.p, &tb, c->stream));
    unsigned long long cnt = 0;
    HIPCHK(hipMemcpyAsync(&cnt, d_cnt, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->retry_ids.resize(cnt);
    rstat.resize(cnt);
    if (cnt) {
      HIPCHK(hipMemcpyAsync(c->retry_ids.data(), c->d_ids.p, cnt * 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(rstat.data(), c->d_selst.p, cnt * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  for (size_t j = 0; j < rstat.size(); ++j) {
    const uint32_t s_ = rstat[j];
    if (s_ & ST_BAD_SCORE) return fail(IBWA_EINVAL, "read %lld: score outside the stack range", (long long)c->retry_ids[j]);
    c->stats.n_stack_overflow += (s_ & ST_STACK_OVERFLOW) != 0;
    c->stats.n_aln_overflow += (s_ & ST_ALN_OVERFLOW) != 0;
    c->stats.n_heavy += (s_ & ST_HEAVY) != 0;
  }
  if (resume_states) {
    unsigned long long rs[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpy(rs, c->d_roff.as<unsigned long long>() + n, 32, hipMemcpyDeviceToHost));
    c->stats.n_resumed = (int64_t)(rs[1] + rs[3]);  // states stored in either buffer
    c->stats.n_heavy += res_ok;  // handed on and resolved by the per-chunk cooperative launches
    c->stats.n_coop += res_ok;
    c->stats.ms_coop += res_ms;
    c->stats.ms_coop_width += res_w;
  }
  if (c->verbose) fprintf(stderr, "[ibwa_amd] t %.1f ms: handed-on reads selected, %zu to retry\n", since(), c->retry_ids.size());
  // retry pass: larger stacks / hit arrays for the few reads that overflowed
  std::vector<int64_t> todo = c->retry_ids;
  uint64_t cap = std::max<uint64_t>((uint64_t)c->stack_cap * 16, 65536);
  uint32_t acap = std::max<uint32_t>(c->aln_cap * 64, 4096);
  std::vector<std::pair<int64_t, std::vector<uint4>>> patch;  // (read, hits) of the wide / general passes
  std::vector<uint8_t> found_by(todo.size(), 0);
  std::vector<int64_t> where(todo.size());
  for (size_t j = 0; j < todo.size(); ++j) where[j] = (int64_t)j;
  float ms_r = 0;
  // heavy and overflowing reads: the wave-cooperative kernel first (exact; whatever it cannot
  // hold is flagged and continues below)
  if (v2 && c->gap_coop && !todo.empty() && max_len <= COOP_MAXLEN && o.n_stacks <= COOP_NSTK) {
    std::vector<int64_t> wide_todo, wide_where;
    const int coop_rounds = 4;
    for (int round = 0; round < coop_rounds && !todo.empty(); ++round) {
      const int64_t lanes = (int64_t)todo.size();
      const size_t wide0 = wide_todo.size();
      uint32_t stg_log2 = 10;
      while ((1u << stg_log2) < (uint32_t)c->coop_stg_room * (9u * (uint32_t)(max_len + 1) + 16u)) ++stg_log2;
      // one heavy read per wave at a time: no more waves than heavy reads, and the page pool in
      // proportion (at least 1 GiB).  The reads that run out of pages run again with all of it,
      // shared by 8x fewer concurrent waves each round (the pool is taken page by page, so each of
      // them can grow into the room the others leave): a read whose stack outgrew its share of a
      // busy pool is still resolved cooperatively, instead of by the sequential wide kernel (at
      // coop_pool_gb=10, 150 bp reads at 2 %: minutes; now 1.07x the 16 GiB time, r05_sweep_mem150.jsonl)
      const int full_blocks = c->n_cus * c->coop_waves_per_cu;
      const int blocks = (int)std::min<int64_t>(std::max(1, full_blocks >> (3 * round)), lanes);
      const uint32_t freecap = 4096, hcap = 4096;
      const uint64_t pool_bytes =
          round ? c->pool_bytes(max_len)
                : std::min<uint64_t>(c->pool_bytes(max_len),
                                     std::max<uint64_t>(1ull << 30, c->pool_bytes(max_len) / full_blocks * blocks));
      const uint32_t pool_pages = c->coop_pool_pages ? c->coop_pool_pages : (uint32_t)(pool_bytes / (COOP_PG * 16ull));
      if (int rc = c->d_ids.ensure(lanes * 8)) return rc;
      if (int rc = c->d_wbuf.ensure(lanes * A.wstride * 8)) return rc;
      if (int rc = c->d_nN.ensure(lanes * 2 + 2)) return rc;
      if (int rc = c->c_stg.ensure((uint64_t)blocks * 64 * 16 << stg_log2)) return rc;
      // k_coop_roots: two chain records per read, their children in a compact store (a chain that
      // finds it full leaves level 0 to k_coop).  A root chain stages ~190 children on a GRCh37-sized
      // genome, so the store takes the first pass's page pool when there is one: nothing in it is
      // live between the first pass and the retry passes, which set it up anew.
      uint4 *pstore = nullptr;
      uint64_t pcap = 0;
      if (c->coop_roots) {
        if (int rc = c->c_proot.ensure((uint64_t)lanes * 2 * 16)) return rc;
        if (c->d_pool.cap >= (1ull << 30)) {
          pstore = c->d_pool.as<uint4>();
          pcap = std::min<uint64_t>(c->d_pool.cap / 16, 0xFFFFFFFFull);
        } else {
          pcap = std::min<uint64_t>(1ull << 31, std::max<uint64_t>(1ull << 24, (uint64_t)lanes * 2 * 256));
          if (int rc = c->c_pstore.ensure(pcap * 16)) return rc;
          pstore = c->c_pstore.as<uint4>();
        }
      }
      if (int rc = c->c_dir.ensure((uint64_t)blocks * COOP_NSTK * COOP_MAXP * 4)) return rc;
      if (int rc = c->c_free.ensure((uint64_t)blocks * freecap * 4)) return rc;
      if (int rc = c->c_hits.ensure((uint64_t)blocks * hcap * 16)) return rc;
      if (int rc = c->c_recb.ensure((uint64_t)blocks * COOP_RREC * 16)) return rc;
      if (int rc = c->c_pool.ensure((uint64_t)pool_pages * COOP_PG * 16)) return rc;
      if (int rc = c->c_next.ensure(64)) return rc;
      if (int rc = c->r_status.ensure(lanes * 4)) return rc;
      if (int rc = c->d_counter.ensure(64)) return rc;
      // d_ids holds todo (select_handed_on, input order); the pass takes the reads with the largest
      // first-pass stacks first (its longest reads then do not start near its end) -- which pass or
      // which order resolves a read changes nothing in its results
      if (round) HIPCHK(hipMemcpy(c->d_ids.p, todo.data(), lanes * 8, hipMemcpyHostToDevice));
      const int64_t *coop_ids = c->d_ids.as<int64_t>();
      if (!round && lanes > 1) {
        size_t tb = 0;
        HIPCHK(order_heavy_first(nullptr, nullptr, lanes, nullptr, nullptr, nullptr, nullptr, &tb, c->stream));
        if (int rc = c->d_ordk.ensure(lanes * 8)) return rc;
        if (int rc = c->d_ordi.ensure(lanes * 8)) return rc;
        if (int rc = c->d_ordids.ensure(lanes * 8)) return rc;
        if (int rc = c->d_ordtmp.ensure(tb + 16)) return rc;
        HIPCHK(order_heavy_first(c->d_selst.as<uint32_t>(), c->d_ids.as<int64_t>(), lanes, c->d_ordk.as<uint32_t>(),
                                 c->d_ordi.as<uint32_t>(), c->d_ordids.as<int64_t>(), c->d_ordtmp.p, &tb, c->stream));
        std::vector<uint32_t> perm(lanes);
        HIPCHK(hipMemcpyAsync(perm.data(), c->d_ordi.p, lanes * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int64_t j = 0; j < lanes; ++j) {
          todo[j] = c->retry_ids[perm[j]];
          where[j] = perm[j];
        }
        coop_ids = c->d_ordids.as<int64_t>();
      }
      AlnArgs B = A;
      B.ids = coop_ids;
      B.n = lanes;
      B.wbuf = c->d_wbuf.as<uint2>();
      B.nN = c->d_nN.as<uint16_t>();
      CoopArgs K = {};
      K.wb_base = -1;  // widths from this launch's k_width
      K.ix[0] = c->ix[0];
      K.ix[1] = c->ix[1];
      K.o64[0] = c->o64[0].as<uint4>();
      K.o64[1] = c->o64[1].as<uint4>();
      K.seq = A.seq;
      K.off = A.off;
      K.len = A.len;
      K.ids = B.ids;
      K.n = lanes;
      K.out_by_id = 1;  // n_aln / aln_off of the input read; status per launch read
      K.maxdiff_tab = A.maxdiff_tab;
      K.wbuf = B.wbuf;
      K.wstride = A.wstride;
      K.wlen1 = A.wlen1;
      K.nN = B.nN;
      K.stg = c->c_stg.as<uint4>();
      K.stg_log2 = stg_log2;
      K.dir = c->c_dir.as<uint32_t>();
      K.freel = c->c_free.as<uint32_t>();
      K.freecap = freecap;
      K.pool = c->c_pool.as<uint4>();
      K.pool_pages = pool_pages;
      K.pool_next = c->c_next.as<uint32_t>();
      K.hits = c->c_hits.as<uint4>();
      K.recb = c->c_recb.as<uint4>();
      if (resume_states) {
        K.rdump = c->d_rdump.as<uint4>();
        K.roff = c->d_roff.as<uint64_t>();
      }
      if (c->coop_roots) {
        K.proot = c->c_proot.as<uint4>();
        K.pstore = pstore;
        K.pstore_next = c->c_next.as<unsigned long long>() + 1;
        K.pstore_cap = pcap;
      }
      K.hcap = hcap;
      K.max_iters = 1u << 24;  // runaway guard; a read past it goes to the sequential kernel
      // hits go on the first pass's stream (a read out of room there is flagged and re-run below)
      K.aln = c->d_aln.as<uint4>();
      K.aln_total = c->stream_total;
      K.aln_next = c->d_counter.as<unsigned long long>() + 1;
      K.aln_off = c->d_aoff.as<uint64_t>();
      K.n_aln = c->d_naln.as<int32_t>();
      K.status = c->r_status.as<uint32_t>();
      if (c->verbose) {
        if (int rc = c->d_iters.ensure(lanes * 4)) return rc;
        K.iters = c->d_iters.as<uint32_t>();
      }
      K.o = o;
      if (c->prof_phases) {
        if (int rc = c->d_prof.ensure(512 + (uint64_t)blocks * 16)) return rc;
        HIPCHK(hipMemsetAsync(c->d_prof.p, 0, 512 + (uint64_t)blocks * 16, c->stream));
        K.prof = c->d_prof.as<unsigned long long>();
        K.wave_t = K.prof + 64;
      }
      HIPCHK(hipEventRecord(c->ev[3], c->stream));
      HIPCHK(launch_width(B, c->block, c->stream));
      HIPCHK(hipEventRecord(c->ev[5], c->stream));
      if (K.proot) HIPCHK(launch_coop_roots(K, c->d_counter.as<unsigned long long>(), blocks, c->stream));
      HIPCHK(hipEventRecord(c->ev[6], c->stream));
      HIPCHK(launch_coop(K, c->d_counter.as<unsigned long long>(), blocks, c->stream));
      HIPCHK(hipEventRecord(c->ev[4], c->stream));
      HIPCHK(hipEventSynchronize(c->ev[4]));
      note_coop_pages(c, pool_pages);
      if (c->verbose) fprintf(stderr, "[ibwa_amd] t %.1f ms: coop kernel done\n", since());
      if (c->prof_phases) {
        unsigned long long pf[40];
        HIPCHK(hipMemcpy(pf, c->d_prof.p, sizeof pf, hipMemcpyDeviceToHost));
        const char *nm[6] = {"barriers", "commits", "claims", "loads+consume", "levels", "read set-up"};
        double tot = 0;
        for (int q = 0; q < 6; ++q) tot += (double)pf[q];
        fprintf(stderr, "[ibwa_amd] k_coop phases (wave cycles):");
        for (int q = 0; q < 6; ++q) fprintf(stderr, " %s %.1f%%", nm[q], tot > 0 ? 100.0 * pf[q] / tot : 0.0);
        fprintf(stderr, "; %llu iterations (%.0f cycles each), %llu commits, %llu levels; lanes per iteration: "
                "%.1f running (%.1f fetching an entry, %.1f in an exact tail)\n", pf[6], pf[6] ? tot / pf[6] : 0.0, pf[7],
                pf[8], pf[6] ? (double)pf[9] / pf[6] : 0.0, pf[6] ? (double)pf[10] / pf[6] : 0.0,
                pf[6] ? (double)pf[11] / pf[6] : 0.0);
        const double it = pf[6] ? (double)pf[6] : 1.0;
        fprintf(stderr, "[ibwa_amd] k_coop idle lanes per iteration: barrier %.1f, level drained %.1f, ring %.1f, staging %.1f; "
                "chains %llu (%.0f per level), %llu discarded at %llu barriers, %llu children committed\n",
                pf[12] / it, pf[13] / it, pf[14] / it, pf[15] / it, pf[16], pf[8] ? (double)pf[16] / pf[8] : 0.0, pf[17],
                pf[18], pf[19]);
        fprintf(stderr, "[ibwa_amd] k_coop iterations (running lanes) by chains per level:");
        const char *nb[5] = {"<=2", "<=16", "<=64", "<=256", ">256"};
        for (int q = 0; q < 5; ++q)
          fprintf(stderr, " %s: %.1f%% (%.1f)", nb[q], 100.0 * pf[20 + q] / it, pf[20 + q] ? (double)pf[25 + q] / pf[20 + q] : 0.0);
        fprintf(stderr, "\n");
        fprintf(stderr, "[ibwa_amd] k_coop one-row lane-steps: expanding %.1f%%, exact tail %.1f%% of running; chains by steps:",
                100.0 * pf[30] / (pf[9] ? pf[9] : 1), 100.0 * pf[31] / (pf[9] ? pf[9] : 1));
        const char *cb[4] = {"<4", "<16", "<64", ">=64"};
        for (int q = 0; q < 4; ++q)
          fprintf(stderr, " %s: %llu (%.1f%% of steps)", cb[q], pf[32 + q], 100.0 * pf[36 + q] / (pf[9] ? pf[9] : 1));
        fprintf(stderr, "\n");
        // wave end times (shader clock) relative to the first wave start: the pass's tail
        std::vector<unsigned long long> wt((size_t)blocks * 2);
        HIPCHK(hipMemcpy(wt.data(), K.wave_t, wt.size() * 8, hipMemcpyDeviceToHost));
        // each wave's own duration (the clock is per XCD; the persistent grid starts together)
        std::vector<double> ends;
        for (int w = 0; w < blocks; ++w) ends.push_back((double)(wt[2 * w + 1] - wt[2 * w]));
        std::sort(ends.begin(), ends.end());
        const double last = ends.back() > 0 ? ends.back() : 1.0;
        fprintf(stderr, "[ibwa_amd] k_coop wave durations (fraction of the longest): p10 %.3f p50 %.3f p90 %.3f p99 %.3f\n",
                ends[ends.size() / 10] / last, ends[ends.size() / 2] / last, ends[ends.size() * 9 / 10] / last,
                ends[ends.size() * 99 / 100] / last);
      }
      float a = 0;
      HIPCHK(hipEventElapsedTime(&a, c->ev[3], c->ev[4]));
      ms_r += a;
      std::vector<uint32_t> rs(lanes);
      HIPCHK(hipMemcpyAsync(rs.data(), c->r_status.p, lanes * 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      // reads out of pool pages (reason 3: the pool is shared by the launch's waves) run again in a
      // launch of their own with the whole pool; the others go on to the wide kernel
      std::vector<int64_t> next, next_where;
      for (int64_t j = 0; j < lanes; ++j) {
        if (rs[j] & ST_BAD_SCORE) return fail(IBWA_EINVAL, "score outside the stack range");
        if (rs[j]) {
          const bool again = ((rs[j] >> 8) & 7u) == 3u && round < coop_rounds - 1;
          (again ? next : wide_todo).push_back(todo[j]);
          (again ? next_where : wide_where).push_back(where[j]);
          continue;
        }
        found_by[where[j]] = 1;
      }
      if (c->verbose) {
        uint32_t mx = 0;
        if (K.iters) {
          std::vector<uint32_t> it(lanes);
          HIPCHK(hipMemcpy(it.data(), K.iters, lanes * 4, hipMemcpyDeviceToHost));
          mx = *std::max_element(it.begin(), it.end());
          double sum = 0;
          for (uint32_t v : it) sum += v;
          std::sort(it.begin(), it.end());
          fprintf(stderr, "[ibwa_amd] coop wave-iterations: sum %.3g (%.0f per wave of %d), p50 %u p99 %u p99.9 %u max %u\n",
                  sum, sum / blocks, blocks, it[it.size() / 2], it[(size_t)(it.size() * 0.99)],
                  it[(size_t)(it.size() * 0.999)], mx);
        }
        uint32_t pages = 0;
        HIPCHK(hipMemcpy(&pages, K.pool_next, 4, hipMemcpyDeviceToHost));
        int why[8] = {0};
        for (int64_t j = 0; j < lanes; ++j)
          if (rs[j]) ++why[(rs[j] >> 8) & 7];
        fprintf(stderr, "[ibwa_amd] coop hand-on reasons: len %d, max_entries %d, pool %d, bucket pages %d, guard %d\n",
                why[1], why[2], why[3], why[4], why[5]);
        fprintf(stderr, "[ibwa_amd] coop pass: %lld reads, %zu handed on, max %u wave iterations, %u pages, %.1f ms\n",
                (long long)lanes, next.size(), mx, pages, a);
        if (K.proot) {
          unsigned long long used = 0;
          HIPCHK(hipMemcpy(&used, K.pstore_next, 8, hipMemcpyDeviceToHost));
          std::vector<uint4> pr((size_t)lanes * 2);
          HIPCHK(hipMemcpy(pr.data(), K.proot, pr.size() * 16, hipMemcpyDeviceToHost));
          int64_t fl[3] = {0, 0, 0};
          for (const uint4 &q : pr) ++fl[(q.w & 0xFFu) < 3 ? (q.w & 0xFFu) : 2];
          fprintf(stderr, "[ibwa_amd] coop roots: %.1f children per chain stored (%llu of %llu entries), chains: %lld done, "
                  "%lld hit, %lld skipped\n", (double)used / (double)pr.size(), used, (unsigned long long)K.pstore_cap,
                  (long long)fl[0], (long long)fl[1], (long long)fl[2]);
        }
      }
      if (c->verbose) fprintf(stderr, "[ibwa_amd] t %.1f ms: coop results on host\n", since());
      c->stats.n_coop += lanes - (int64_t)next.size() - (int64_t)(wide_todo.size() - wide0);
      c->stats.ms_coop += a;
      {
        float w = 0, rt = 0;
        HIPCHK(hipEventElapsedTime(&w, c->ev[3], c->ev[5]));
        HIPCHK(hipEventElapsedTime(&rt, c->ev[5], c->ev[6]));
        c->stats.ms_coop_width += w;
        c->stats.ms_coop_roots = rt;
      }
      todo.swap(next);
      where.swap(next_where);
    }
    todo.insert(todo.end(), wide_todo.begin(), wide_todo.end());
    where.insert(where.end(), wide_where.begin(), wide_where.end());
  }
  // first two retry rounds: the persistent gapped kernel with 24-bit slot links and one
  // large static region per read (4 MiB, then 64 MiB; reads < 4096 bp); then the general kernels
  int wide_rounds = v2 && max_len < 4096 ? 2 : 0;
  while (!todo.empty()) {
    const bool wide_round = wide_rounds > 0;
    const uint32_t wide_hits = 4096;
    // live entries never exceed max_entries + 9 (one expansion after the last check)
    const uint64_t need_cap =
        wide_round ? std::min<uint64_t>((uint64_t)opt->max_entries + 64 + wide_hits, wide_rounds == 2 ? 1u << 18 : 1u << 22)
                   : std::min<uint64_t>(cap, (uint64_t)opt->max_entries + 16);
    // keep each retry chunk within ~16 GiB (general kernels) / 48 GiB (gapped wide) of stack scratch
    const uint64_t budget = (wide_round ? 48ull : 16ull) << 30;
    int64_t per = std::max<int64_t>(1, (int64_t)(budget / (need_cap * 20 + acap * 16 + A.wstride * 8 + 64)));
    std::vector<int64_t> next;
    std::vector<int64_t> next_where;
    for (size_t b0 = 0; b0 < todo.size(); b0 += per) {
      int64_t lanes = std::min<int64_t>(per, (int64_t)todo.size() - (int64_t)b0);
      AlnArgs B = A;
      B.cap = (uint32_t)need_cap;
      B.aln_cap = acap;
      if (int rc = c->d_ids.ensure(lanes * 8)) return rc;
      if (int rc = c->d_wbuf.ensure(lanes * A.wstride * 8)) return rc;
      if (int rc = c->d_ent.ensure(lanes * need_cap * 16)) return rc;
      if (!wide_round) {
        if (int rc = c->d_heads.ensure(lanes * (uint64_t)o.n_stacks * 4)) return rc;
        if (int rc = c->d_prev.ensure(lanes * need_cap * 4)) return rc;
      }
      const uint64_t r_total = wide_round ? (uint64_t)lanes * 64 + 65536 : (uint64_t)lanes * acap;
      if (int rc = c->r_aln.ensure(r_total * 16)) return rc;
      if (int rc = c->r_aoff.ensure(lanes * 8)) return rc;
      if (int rc = c->r_naln.ensure(lanes * 4)) return rc;
      if (int rc = c->r_status.ensure(lanes * 4)) return rc;
      HIPCHK(hipMemcpyAsync(c->d_ids.p, todo.data() + b0, lanes * 8, hipMemcpyHostToDevice, c->stream));
      B.wbuf = c->d_wbuf.as<uint2>();
      B.heads = c->d_heads.as<uint32_t>();
      B.ent = c->d_ent.as<uint4>();
      B.prev = c->d_prev.as<uint32_t>();
      B.aln = c->r_aln.as<uint4>();
      B.n_aln = c->r_naln.as<int32_t>();
      B.status = c->r_status.as<uint32_t>();
      float a = 0, b = 0;
      if (wide_round) {
        if (int rc = c->d_nN.ensure(lanes * 2 + 2)) return rc;
        if (int rc = c->d_counter.ensure(64)) return rc;
        B.ids = c->d_ids.as<int64_t>();
        B.n = lanes;
        B.nN = c->d_nN.as<uint16_t>();
        GapArgs G = gap_args(c, A, o, 0, lanes);
        G.ids = B.ids;
        G.out_by_id = 0;
        G.ent = B.ent;
        G.cap1 = (uint32_t)need_cap;
        G.hit_slots = wide_hits;
        G.pool = nullptr;
        G.max_pages = 0;
        G.pages_per_block = 0;
        G.page_log2 = 13;
        G.aln = B.aln;
        G.aln_total = r_total;
        G.aln_next = c->d_counter.as<unsigned long long>() + 2;
        G.aln_off = c->r_aoff.as<uint64_t>();
        G.n_aln = B.n_aln;
        G.status = B.status;
        if (c->verbose) {
          if (int rc = c->d_iters.ensure(lanes * 4)) return rc;
          G.iters = c->d_iters.as<uint32_t>();
        }
        HIPCHK(zero_async(G.aln_next, 8, c->stream));
        // one heavy read per wave: an iteration then costs only that read's path
        const int blk = 64;
        G.lanes_per_wave = 1;
        G.free_depth = 4096;  // 16 KiB of LDS per heavy read: freed slots are reused, not leaked
        HIPCHK(hipEventRecord(c->ev[3], c->stream));
        HIPCHK(launch_width(B, c->block, c->stream));
        HIPCHK(launch_gapped(G, c->d_counter.as<unsigned long long>(), (int)lanes, blk, true, c->stream));
        HIPCHK(hipEventRecord(c->ev[4], c->stream));
        HIPCHK(hipEventSynchronize(c->ev[4]));
        HIPCHK(hipEventElapsedTime(&a, c->ev[3], c->ev[4]));
        if (c->verbose) {
          std::vector<uint32_t> it(lanes);
          HIPCHK(hipMemcpy(it.data(), c->d_iters.p, lanes * 4, hipMemcpyDeviceToHost));
          const uint32_t mx = *std::max_element(it.begin(), it.end());
          fprintf(stderr, "[ibwa_amd]   wide launch: %lld reads, max %u iterations, %.1f ms (%.2f us/iteration)\n",
                  (long long)lanes, mx, a, mx ? a * 1e3 / mx : 0.0);
        }
      } else {
        if (int rc = run_pass(c, B, 0, lanes, c->d_ids.as<int64_t>(), &a, &b)) return rc;
      }
      ms_r += a + b;
      std::vector<int32_t> rn(lanes);
      std::vector<uint32_t> rs(lanes);
      std::vector<uint64_t> ro(lanes);
      std::vector<uint4> ra(r_total);
      HIPCHK(hipMemcpyAsync(rn.data(), c->r_naln.p, lanes * 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(rs.data(), c->r_status.p, lanes * 4, hipMemcpyDeviceToHost, c->stream));
      if (wide_round) HIPCHK(hipMemcpyAsync(ro.data(), c->r_aoff.p, lanes * 8, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(ra.data(), c->r_aln.p, r_total * 16, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      for (int64_t j = 0; j < lanes; ++j) {
        int64_t slot = where[b0 + j];
        if (rs[j] & ST_BAD_SCORE) return fail(IBWA_EINVAL, "score outside the stack range");
        if (rs[j]) {
          next.push_back(todo[b0 + j]);
          next_where.push_back(slot);
          continue;
        }
        const uint64_t first = wide_round ? (rn[j] ? ro[j] : 0) : (uint64_t)j * acap;
        patch.emplace_back(todo[b0 + j], std::vector<uint4>(ra.begin() + first, ra.begin() + first + rn[j]));
        found_by[slot] = wide_round ? 2 : 3;
      }
    }
    if (c->verbose)
      fprintf(stderr, "[ibwa_amd] retry round (%s, cap %llu): %zu reads, %zu still overflow, %.1f ms so far\n",
              wide_round ? "gapped wide" : "general", (unsigned long long)need_cap, todo.size(), next.size(), ms_r);
    if (wide_round) {
      --wide_rounds;  // what still overflows goes to a larger round, then to the general kernels
      todo.swap(next);
      where.swap(next_where);
      continue;
    }
    if (!next.empty()) {
      if (cap >= (uint64_t)opt->max_entries + 16 && acap >= (1u << 20))
        return fail(IBWA_EOVERFLOW, "read %lld overflowed the large-capacity pass", (long long)next[0]);
      cap *= 16;
      acap = std::min<uint32_t>(acap * 16, 1u << 20);
    }
    todo.swap(next);
    where.swap(next_where);
  }
  // the reads the wide / general passes resolved, in input order, for ibwa_batch_fetch to patch in
  std::sort(patch.begin(), patch.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
  c->patch_ids.resize(patch.size());
  c->patch_alns.resize(patch.size());
  for (size_t j = 0; j < patch.size(); ++j) {
    c->patch_ids[j] = patch[j].first;
    c->patch_alns[j].swap(patch[j].second);
  }
  c->retry_pass.swap(found_by);
  // hit-stream records of the first and cooperative passes; a read whose hits did not fit advanced
  // the fill counter but wrote nothing (ST_ALN_OVERFLOW, re-run above): the records end at stream_total
  if (v2 && n) {
    HIPCHK(hipMemcpyAsync(&c->stream_len, c->d_counter.as<unsigned long long>() + 1, 8, hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->stream_len = std::min<unsigned long long>(c->stream_len, c->stream_total);
  }
  c->stats.ms_retry = ms_r + res_ms;
  c->stats.n_retry = (int64_t)c->retry_ids.size() + res_ok;
  c->stats.ms_total =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  c->stats.ms_alloc = g_alloc_ms;
  return 0;
}

int ibwa_batch_retry_info(const ibwa_ctx_t *c, int64_t *ids, uint8_t *pass, int64_t cap, int64_t *n) {
  const int64_t m0 = (int64_t)c->retry_ids.size(), m = m0 + (int64_t)c->resumed_ids.size();
  for (int64_t j = 0; j < std::min(m, cap); ++j) {
    if (ids) ids[j] = j < m0 ? c->retry_ids[j] : c->resumed_ids[j - m0];
    if (pass) pass[j] = j >= m0 ? 4 : j < (int64_t)c->retry_pass.size() ? c->retry_pass[j] : 0;
  }
  if (n) *n = m;
  return 0;
}

int ibwa_batch_diag(const ibwa_ctx_t *c, int what, void *out, uint64_t cap_bytes) {
  if (what == 2) {
    const uint64_t need2 = (uint64_t)c->n * 4;
    if (cap_bytes < need2) return fail(IBWA_EINVAL, "diag buffer too small");
    if (!c->hpop_valid || c->d_hpop.cap < need2) {  // no resume states in the last run
      memset(out, 0, need2);
      return 0;
    }
    if (c->n == 0) return 0;
    HIPCHK(enter(c));
    HIPCHK(hipMemcpy(out, c->d_hpop.p, need2, hipMemcpyDeviceToHost));
    return 0;
  }
  const uint64_t need = what == 0 ? (uint64_t)c->n * 4 : (uint64_t)c->n * 8;
  if (!c->diag || (what != 0 && what != 1)) return fail(IBWA_EINVAL, "set option diag=1 before the run; what = 0 or 1");
  if (cap_bytes < need) return fail(IBWA_EINVAL, "diag buffer too small");
  if (c->n == 0) return 0;
  HIPCHK(enter(c));
  HIPCHK(hipMemcpy(out, (what == 0 ? c->d_iters : c->d_feat).p, need, hipMemcpyDeviceToHost));
  return 0;
}

// the batch's results to the host once (h_naln / h_aoff / h_aln), and per read its hit count with
// the wide / general passes' patches in (c->h_cnt)
// huge pages for a large host array (fewer faults, and fewer page tables to tear down at exit)
static void advise_huge(const void *p, size_t bytes) {
  const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
  const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(uintptr_t)((2u << 20) - 1);
  if (e > a) (void)madvise(reinterpret_cast<void *>(a), e - a, MADV_HUGEPAGE);
}

static int fetch_to_host(ibwa_ctx_t *c) {
  if (c->fetched) return 0;
  const int64_t n = c->n;
  const uint32_t cap = c->aln_cap_used;
  const uint64_t n_slots = c->stream_out ? c->stream_len : (uint64_t)n * cap;
  if (c->h_aln.capacity() < n_slots) {
    std::vector<uint4>().swap(c->h_aln);
    c->h_aln.reserve(n_slots + n_slots / 8);  // not touched yet: huge pages advised first
    advise_huge(c->h_aln.data(), c->h_aln.capacity() * sizeof(uint4));
  }
  c->h_aln.resize(std::max<uint64_t>(n_slots, 1));
  if (n) {
    HIPCHK(enter(c));
    if (!c->naln_on_host) {
      c->h_naln.resize(n);
      HIPCHK(hipMemcpyAsync(c->h_naln.data(), c->d_naln.p, n * 4, hipMemcpyDeviceToHost, c->stream));
      c->naln_on_host = true;
    }
    if (c->stream_out) {
      c->h_aoff.resize(n);
      HIPCHK(hipMemcpyAsync(c->h_aoff.data(), c->d_aoff.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    }
    if (n_slots) HIPCHK(hipMemcpyAsync(c->h_aln.data(), c->d_aln.p, n_slots * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  c->h_cnt.assign(c->h_naln.begin(), c->h_naln.begin() + n);
  for (size_t j = 0; j < c->patch_ids.size(); ++j) c->h_cnt[c->patch_ids[j]] = (int32_t)c->patch_alns[j].size();
  c->fetched = true;
  return 0;
}

int ibwa_batch_fetch_sai(ibwa_ctx_t *c, void *dst, uint64_t cap_bytes, uint64_t *bytes, int64_t *n_total) {
  if (!c || !bytes) return fail(IBWA_EINVAL, "fetch_sai: bad arguments");
  if (int rc = fetch_to_host(c)) return rc;
  const int64_t n = c->n;
  const uint32_t cap = c->aln_cap_used;
  const int32_t *cnt = c->h_cnt.data();
  // per range of reads (one per host thread): its bytes and hits, then the ranges' offsets
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(16, n >> 16));
  std::vector<uint64_t> bo(T + 1, 0), ho(T + 1, 0);
  auto ranges = [&](auto &&fn) {
    if (T == 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(fn, t);
    for (auto &x : th) x.join();
  };
  ranges([&](int t) {
    uint64_t h = 0;
    for (int64_t i = n * t / T; i < n * (t + 1) / T; ++i) h += (uint64_t)cnt[i];
    ho[t + 1] = h;
    bo[t + 1] = h * 16 + (uint64_t)(n * (t + 1) / T - n * t / T) * 4;
  });
  for (int t = 0; t < T; ++t) {
    bo[t + 1] += bo[t];
    ho[t + 1] += ho[t];
  }
  *bytes = bo[T];
  if (n_total) *n_total = (int64_t)ho[T];
  if (!dst || cap_bytes < bo[T]) return 0;
  ranges([&](int t) {
    char *w = static_cast<char *>(dst) + bo[t];
    const int64_t lo = n * t / T;
    size_t rj = std::lower_bound(c->patch_ids.begin(), c->patch_ids.end(), lo) - c->patch_ids.begin();
    for (int64_t i = lo; i < n * (t + 1) / T; ++i) {
      const int32_t k = cnt[i];
      const uint4 *src;
      if (rj < c->patch_ids.size() && c->patch_ids[rj] == i) {
        src = c->patch_alns[rj].data();
        ++rj;
      } else {
        src = c->h_aln.data() + (c->stream_out ? (k ? c->h_aoff[i] : 0) : (uint64_t)i * cap);
      }
      memcpy(w, &k, 4);
      if (k) memcpy(w + 4, src, (size_t)k * 16);
      w += 4 + (size_t)k * 16;
    }
  });
  return 0;
}

int ibwa_batch_fetch(ibwa_ctx_t *c, int32_t *n_aln, ibwa_aln1_t **aln, int64_t *n_total) {
  const int64_t n = c->n;
  const uint32_t cap = c->aln_cap_used;
  // first-pass hits (per-read slots n x cap, or the hit stream + per-read offsets) to the host, with
  // the reads the wide / general passes resolved patched in (the first and cooperative passes wrote
  // theirs into d_naln / d_aln)
  if (int rc = fetch_to_host(c)) return rc;
  const std::vector<int32_t> &cnt = c->h_cnt;
  std::vector<int64_t> at(n + 1, 0);  // output offset of read i
  for (int64_t i = 0; i < n; ++i) at[i + 1] = at[i] + cnt[i];
  const int64_t tot = at[n];
  ibwa_aln1_t *o = (ibwa_aln1_t *)malloc(std::max<int64_t>(tot, 1) * sizeof(ibwa_aln1_t));
  if (!o) return fail(IBWA_EINVAL, "out of host memory");
  // the records in input order, gathered by several host threads (patch_ids ascending)
  auto gather = [&](int64_t lo, int64_t hi) {
    size_t rj = std::lower_bound(c->patch_ids.begin(), c->patch_ids.end(), lo) - c->patch_ids.begin();
    for (int64_t i = lo; i < hi; ++i) {
      const uint4 *src;
      if (rj < c->patch_ids.size() && c->patch_ids[rj] == i) {
        src = c->patch_alns[rj].data();
        ++rj;
      } else {
        src = c->h_aln.data() + (c->stream_out ? (cnt[i] ? c->h_aoff[i] : 0) : i * cap);
      }
      memcpy(o + at[i], src, (size_t)cnt[i] * 16);
      if (n_aln) n_aln[i] = cnt[i];
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, n / 65536));
  if (nt == 1) {
    gather(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(gather, n * t / nt, n * (t + 1) / nt);
    for (auto &x : th) x.join();
  }
  *aln = o;
  if (n_total) *n_total = tot;
  return 0;
}

int ibwa_ctx_prepare(ibwa_ctx_t *c, const ibwa_gap_opt_t *opt) {
  if (!c) return fail(IBWA_EINVAL, "null context");
  HIPCHK(enter(c));
  if (int rc = ensure_kmer(c)) return rc;
  // the condition of ibwa_batch_run's exact path
  if (opt && c->exact_path && !(opt->fnr > 0.0f) && opt->max_diff == 0 && opt->max_entries >= 2)
    if (int rc = ensure_jump(c)) return rc;
  return 0;
}

int ibwa_batch_stats(const ibwa_ctx_t *c, ibwa_run_stats_t *st) {
  *st = c->stats;
  return 0;
}

int ibwa_aln_batch(ibwa_ctx_t *c, const ibwa_gap_opt_t *opt, int64_t n, const uint8_t *seq, const uint64_t *off,
                   const uint32_t *len, int batch_max_len, int32_t *n_aln, ibwa_aln1_t **aln, int64_t *n_total) {
  if (int rc = ibwa_batch_stage(c, n, seq, off, len)) return rc;
  if (int rc = ibwa_batch_run(c, opt, batch_max_len)) return rc;
  return ibwa_batch_fetch(c, n_aln, aln, n_total);
}

}  // extern "C"

namespace {
// k_sw launch over host arrays: the local core (global_band == 0) or aln_global_core alone
int sw_batch(ibwa_ctx_t *c, int64_t n, const uint8_t *ref, const uint64_t *off1, const uint32_t *len1,
             const uint8_t *qry, const uint64_t *off2, const uint32_t *len2, int global_band, int gap_end,
             int32_t *score, int32_t *path_len, int32_t *ends, int32_t *n_cigar, uint32_t **cigar,
             int64_t *n_cigar_total) {
  if (n < 0) return fail(IBWA_EINVAL, "negative pair count");
  *cigar = nullptr;
  if (n_cigar_total) *n_cigar_total = 0;
  if (n == 0) {
    *cigar = (uint32_t *)malloc(4);
    return 0;
  }
  HIPCHK(enter(c));
  int max1 = 0, max2 = 0;
  uint64_t end1 = 0, end2 = 0;
  for (int64_t p = 0; p < n; ++p) {
    if (!global_band && std::min(len1[p], len2[p]) * 11ull > 32000)
      return fail(IBWA_EINVAL, "pair %lld: min(len1, len2) * 11 > 32000", (long long)p);
    if (global_band && (uint64_t)len1[p] * len2[p] > (64ull << 20))
      return fail(IBWA_EINVAL, "pair %lld: %u x %u cells is past the traceback bound", (long long)p, len1[p], len2[p]);
    max1 = std::max<int>(max1, (int)len1[p]);
    max2 = std::max<int>(max2, (int)len2[p]);
    end1 = std::max<uint64_t>(end1, off1[p] + len1[p]);
    end2 = std::max<uint64_t>(end2, off2[p] + len2[p]);
  }
  const int cap = std::max(1, max1 + max2);
  // the context's SW buffers, grown as needed and kept (a per-call hipMalloc / hipFree of the DP
  // scratch cost more than the kernel on a sampe batch)
  DBuf &s1 = c->sw[0], &s2 = c->sw[1], &o1 = c->sw[2], &o2 = c->sw[3], &l1 = c->sw[4], &l2 = c->sw[5], &sc = c->sw[6],
       &pl = c->sw[7], &nc = c->sw[8], &en = c->sw[9], &cg = c->sw[10], &scr = c->sw[11], &tbb = c->sw[12],
       &cf = c->sw[13], &cc = c->sw[14];
  auto release = [&]() {};
  const uint64_t wpl = sw_words_per_lane(max1, max2), tpl = sw_tb_per_lane(max1, max2);
  const uint64_t per_wave = (wpl * 4 + tpl) * 64;
  // a persistent grid within ~32 GiB of DP scratch (5 waves per SIMD at most: 94 VGPRs)
  const int64_t waves = std::max<int64_t>(
      1, std::min<int64_t>({(n + 63) / 64, (int64_t)((32ull << 30) / per_wave), (int64_t)c->n_cus * 20}));
  const int blocks = (int)((waves + 3) / 4);
  int rc = 0;
  if ((rc = s1.ensure(end1 + 16)) || (rc = s2.ensure(end2 + 16)) || (rc = o1.ensure(n * 8)) || (rc = o2.ensure(n * 8)) ||
      (rc = l1.ensure(n * 4)) || (rc = l2.ensure(n * 4)) || (rc = sc.ensure(n * 4)) || (rc = pl.ensure(n * 4)) ||
      (rc = nc.ensure(n * 4)) || (rc = en.ensure(n * 16)) || (rc = cg.ensure((uint64_t)n * cap * 4)) ||
      (rc = scr.ensure((uint64_t)blocks * 4 * wpl * 4 * 64)) || (rc = tbb.ensure((uint64_t)blocks * 4 * tpl * 64)) ||
      (rc = c->d_counter.ensure(64)) || (rc = cf.ensure(n * 8))) {
    release();
    return rc;
  }
  auto chk = [&](hipError_t e, const char *what) {
    if (e != hipSuccess && !rc) rc = fail(IBWA_EHIP, "%s: %s", what, hipGetErrorString(e));
  };
  chk(hipMemcpyAsync(s1.p, ref, end1, hipMemcpyHostToDevice, c->stream), "H2D ref");
  chk(hipMemcpyAsync(s2.p, qry, end2, hipMemcpyHostToDevice, c->stream), "H2D qry");
  chk(hipMemcpyAsync(o1.p, off1, n * 8, hipMemcpyHostToDevice, c->stream), "H2D off1");
  chk(hipMemcpyAsync(o2.p, off2, n * 8, hipMemcpyHostToDevice, c->stream), "H2D off2");
  chk(hipMemcpyAsync(l1.p, len1, n * 4, hipMemcpyHostToDevice, c->stream), "H2D len1");
  chk(hipMemcpyAsync(l2.p, len2, n * 4, hipMemcpyHostToDevice, c->stream), "H2D len2");
  SwArgs A = {};
  A.seq1 = s1.as<uint8_t>(); A.seq2 = s2.as<uint8_t>();
  A.off1 = o1.as<uint64_t>(); A.off2 = o2.as<uint64_t>();
  A.len1 = l1.as<uint32_t>(); A.len2 = l2.as<uint32_t>();
  A.n = n;
  A.max_len1 = max1;
  A.max_len2 = max2;
  A.scratch = scr.as<uint32_t>(); A.words_per_lane = wpl;
  A.tb = tbb.as<uint8_t>(); A.tb_per_lane = tpl;
  A.score = sc.as<int32_t>(); A.path_len = pl.as<int32_t>(); A.n_cigar = nc.as<int32_t>();
  A.ends = en.as<int4>();
  A.cigar = cg.as<uint32_t>(); A.cigar_cap = cap;
  A.stop_after = c->sw_stop_after;
  A.global_band = global_band;
  A.gap_end = gap_end;
  if (!rc) {
    chk(hipEventRecord(c->ev[0], c->stream), "event");
    chk(launch_sw(A, c->d_counter.as<unsigned long long>(), blocks, c->stream), "k_sw");
    chk(hipEventRecord(c->ev[1], c->stream), "event");
  }
  if (!rc) {
    chk(hipMemcpyAsync(score, sc.p, n * 4, hipMemcpyDeviceToHost, c->stream), "D2H score");
    chk(hipMemcpyAsync(path_len, pl.p, n * 4, hipMemcpyDeviceToHost, c->stream), "D2H path_len");
    chk(hipMemcpyAsync(n_cigar, nc.p, n * 4, hipMemcpyDeviceToHost, c->stream), "D2H n_cigar");
    chk(hipMemcpyAsync(ends, en.p, n * 16, hipMemcpyDeviceToHost, c->stream), "D2H ends");
    chk(hipStreamSynchronize(c->stream), "sync");
    float ms = 0;
    if (!rc && hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->stats.ms_sw = ms;
  }
  if (rc) return rc;
  // the CIGARs packed on the device (row p's n_cigar[p] words at its prefix offset), one copy back
  std::vector<uint64_t> first(n);
  int64_t tot = 0;
  for (int64_t p = 0; p < n; ++p) {
    first[p] = (uint64_t)tot;
    tot += n_cigar[p];
  }
  uint32_t *o = (uint32_t *)malloc(std::max<int64_t>(tot, 1) * 4);
  if (!o) return fail(IBWA_EINVAL, "out of host memory");
  if (tot) {
    if ((rc = cc.ensure((uint64_t)tot * 4))) { free(o); return rc; }
    chk(hipMemcpyAsync(cf.p, first.data(), n * 8, hipMemcpyHostToDevice, c->stream), "H2D cigar offsets");
    chk(launch_pack_cigar(cg.as<uint32_t>(), cap, nc.as<int32_t>(), cf.as<uint64_t>(), n, cc.as<uint32_t>(), c->stream),
        "k_pack_cigar");
    chk(hipMemcpyAsync(o, cc.p, (uint64_t)tot * 4, hipMemcpyDeviceToHost, c->stream), "D2H cigar");
    chk(hipStreamSynchronize(c->stream), "sync");
    if (rc) { free(o); return rc; }
  }
  *cigar = o;
  if (n_cigar_total) *n_cigar_total = tot;
  return 0;
}
}  // namespace

extern "C" {

int ibwa_sw_batch(ibwa_ctx_t *c, int64_t n, const uint8_t *ref, const uint64_t *off1, const uint32_t *len1,
                  const uint8_t *qry, const uint64_t *off2, const uint32_t *len2, int32_t *score,
                  int32_t *path_len, int32_t *ends, int32_t *n_cigar, uint32_t **cigar, int64_t *n_cigar_total) {
  return sw_batch(c, n, ref, off1, len1, qry, off2, len2, 0, -1, score, path_len, ends, n_cigar, cigar, n_cigar_total);
}

int ibwa_global_batch(ibwa_ctx_t *c, int64_t n, const uint8_t *ref, const uint64_t *off1, const uint32_t *len1,
                      const uint8_t *qry, const uint64_t *off2, const uint32_t *len2, int band, int gap_end,
                      int32_t *score, int32_t *path_len, int32_t *n_cigar, uint32_t **cigar, int64_t *n_cigar_total) {
  if (band <= 0) return fail(IBWA_EINVAL, "band must be > 0");
  std::vector<int32_t> ends(4 * std::max<int64_t>(n, 1));
  return sw_batch(c, n, ref, off1, len1, qry, off2, len2, band, gap_end, score, path_len, ends.data(), n_cigar, cigar,
                  n_cigar_total);
}

int ibwa_occ4(ibwa_ctx_t *c, int strand, int64_t n, const uint32_t *k, uint32_t *cnt) {
  if (!c->loaded[strand]) return fail(IBWA_ENOINDEX, "index not loaded");
  HIPCHK(enter(c));
  DBuf dk, dc;
  if (int rc = dk.ensure(n * 4 + 4)) return rc;
  if (int rc = dc.ensure(n * 16 + 16)) { dk.release(); return rc; }
  HIPCHK(hipMemcpyAsync(dk.p, k, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(launch_occ4(c->ix[strand], n, dk.as<uint32_t>(), dc.as<uint32_t>(), c->stream));
  HIPCHK(hipMemcpyAsync(cnt, dc.p, n * 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  dk.release();
  dc.release();
  return 0;
}

}  // extern "C"
