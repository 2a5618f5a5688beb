// ingest.h -- `ibwa-amd aln`'s FASTQ input parsed on the GPUs (fastq.hip, ibwa_fq_parse).
//
// bwa_aln_core (bwtaln.c:199-231) reads batches of 0x40000 kept reads with bwa_read_seq
// (bwaseqio.c:145-208).  For an uncompressed FASTQ file the host here only moves bytes: host
// threads pread() the file into pinned buffers, one region at a time (the next region is read
// while the current one is parsed), and each GPU's ingest context parses its piece of the region
// -- strict 4-line records split, checked, barcode / -q trimmed, nt4-encoded and reversed on the
// device (ibwa_fq_parse) -- and keeps the kept reads in HBM.  From the per-record lengths the host
// forms the reference's batches (kSub kept reads each, the records bwa_read_seq skips included) and
// from them groups: consecutive complete batches with the same batch-level max_diff
// (bwtaln.c:86-88), whose slices -- the group's reads in each GPU's piece -- the aligning contexts
// take as views of the parsed block (ibwa_batch_stage_fq, no copy).  A producer thread parses ahead:
// each region goes to the lowest free of `slots` ingest contexts per GPU: a slot is parsed over once
// every group of its previous region has been released (aligned) -- the parse kernels wait for
// CUs that the searches' persistent grids hold, so they must not sit on the launching thread's
// path.  A region's last, incomplete batch is parsed again at
// the start of the next region (its bytes move to the front of the next buffer), except at the
// end of the file.  At the first record that is not strict (FASTA, multi-line, CRLF, a truncated
// tail) -- or a batch whose bytes exceed the carry room -- the rest of the file, from the start
// of the incomplete batch, goes to the host readers (readers.h), whose records are then the
// reference's as before.
#pragma once
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gzsrc.h"
#include "ibwa_aln.h"
#include "readers.h"
#include "sam_common.h"

namespace ibwa_cli {

// A group the GPUs align: per GPU the kept reads [first, first + count) of its parsed piece.
struct DevGroup {
  int64_t n = 0;
  int max_len = 0;
  int slot = 0;  // the ingest contexts (one per GPU) that hold its reads
  std::vector<std::pair<long, long>> trims;  // per batch: bases trimmed, bases read (bwaseqio.c:206)
  std::vector<int64_t> first, count;
};

class FastqGpu {
 public:
  // true when `fn` is a regular file this path can take: uncompressed, or gzip (inflated on the host
  // threads by GzSource, the parse on the GPUs) unless IBWA_GZ_PARALLEL=0
  static bool usable(const char *fn) {
    if (!strcmp(fn, "-")) return false;
    struct stat st;
    if (stat(fn, &st) != 0 || !S_ISREG(st.st_mode)) return false;
    if (!is_gzip(fn)) return true;
    const char *pe = getenv("IBWA_GZ_PARALLEL");
    return !(pe && atoi(pe) == 0);
  }
  static bool is_gzip(const char *fn) {
    FILE *f = fopen(fn, "rb");
    if (!f) return false;
    unsigned char m[2] = {0, 0};
    const size_t got = fread(m, 1, 2, f);
    fclose(f);
    return got == 2 && m[0] == 0x1f && m[1] == 0x8b;
  }

  // ing: n_slots x G ingest contexts, slot-major (ing[slot * G + g] on GPU g); key_of(max_len): the
  // batch-level key that groups share
  FastqGpu(const char *fn, std::vector<ibwa_ctx_t *> ing, int G, int mode, int trim_qual, int sub,
           uint64_t piece_bytes, uint64_t carry_bytes, std::function<int(int)> key_of)
      : all_(std::move(ing)), G_(G), mode_(mode), trim_(trim_qual), sub_(sub), l_bc_((int)((unsigned)mode >> 24)),
        key_of_(std::move(key_of)) {
    n_slots_ = G_ > 0 ? (int)all_.size() / G_ : 0;
    busy_.assign(std::max(n_slots_, 1), 0);
    fd_ = open(fn, O_RDONLY);
    struct stat st;
    fsize_ = fd_ >= 0 && fstat(fd_, &st) == 0 ? (uint64_t)st.st_size : 0;
    // gzip: the reader thread inflates each region (GzSource, on all host threads for BGZF and
    // multi-member files) into pageable buffers; offsets are then offsets of the inflated stream, and
    // the size an estimate until the stream ends
    if (fd_ >= 0 && is_gzip(fn)) {
      src_.reset(new GzSource);
      if (!src_->open(fn)) { ok_ = false; return; }
      fsize_ = src_->size_hint();
    }
    // The file is mapped (IBWA_FQ_MMAP, default 1) and each region handed to the parse where it lies:
    // no pinned buffers (pinning 4.5 GB took ~1 s and unpinning it ~0.5 s at exit -- or, freed while
    // the searches ran, slowed them: profiles/r05_exit.jsonl, r05_e2e_d.json), no carry copies (a
    // region's unfinished batch is simply where the next region starts).  A reader thread faults the
    // next region's pages in while the current one is parsed.
    const char *mv = getenv("IBWA_FQ_MMAP");
    if (fd_ >= 0 && fsize_ > 0 && !src_ && !(mv && !strcmp(mv, "0"))) {
      void *m = mmap(nullptr, fsize_, PROT_READ, MAP_PRIVATE, fd_, 0);
      if (m != MAP_FAILED) map_ = static_cast<const char *>(m);
    }
    // pinned buffers no larger than the file needs (a small input must not pin GBs)
    const uint64_t fs = std::max<uint64_t>((fsize_ + 4095) / 4096 * 4096, 4096);
    piece_ = std::max<uint64_t>(piece_bytes, 4096);
    carry_ = std::min<uint64_t>(std::max<uint64_t>(carry_bytes, 4096), fs);
    // regions of equal size (at most piece_bytes per GPU): the last groups then hold as many reads as
    // the others, so the lanes finish together instead of one short group running alone at the end
    const uint64_t per = piece_ * G_, n_reg = (fs + per - 1) / per;
    chunk_ = std::min<uint64_t>(per, ((fs + n_reg - 1) / n_reg + 4095) / 4096 * 4096);
    for (auto &b : buf_) {
      if (map_) break;
      void *p = nullptr;
      if (src_) {  // pageable, huge pages (ibwa_fq_parse stages pageable blocks through pinned chunks)
        const uint64_t sz = (carry_ + chunk_ + 64 + (2u << 20) - 1) / (2u << 20) * (2u << 20);
        p = aligned_alloc(2u << 20, sz);
        if (!p) { ok_ = false; return; }
        madvise(p, sz, MADV_HUGEPAGE);
        pageable_ = true;
      } else if (ibwa_host_alloc(carry_ + chunk_ + 64, &p)) {
        ok_ = false;
        return;
      }
      b = static_cast<char *>(p);
    }
    ok_ = fd_ >= 0 && n_slots_ >= 1;
    if (!ok_) return;
    start_read(0);
    producer_ = std::thread([this]() { produce(); });
  }
  ~FastqGpu() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (producer_.joinable()) producer_.join();
    if (reader_.joinable()) reader_.join();
    for (char *b : buf_) {
      if (pageable_) free(b);
      else ibwa_host_free(b);
    }
    if (map_ && map_lo_ < fsize_) munmap(const_cast<char *>(map_) + map_lo_, fsize_ - map_lo_);
    if (fd_ >= 0) close(fd_);
  }
  bool ok() const { return ok_; }
  // the host readers take over at this file offset (valid once next() returned false with handoff())
  bool handoff() const { return handoff_; }
  uint64_t handoff_offset() const { return handoff_off_; }
  double parse_s() const { return parse_s_; }
  double inflate_s() const { return inflate_s_; }  // reader-thread time inflating gzip input
  bool gzip() const { return src_ != nullptr; }
  bool bgzf() const { return src_ && src_->bgzf(); }
  uint64_t input_bytes() const { return src_ ? src_->offset() : fsize_; }
  double dev_ms() const { return dev_ms_; }
  int64_t records() const { return n_records_; }
  // GPU g's ingest context of a group
  ibwa_ctx_t *ctx_of(const DevGroup &d, int g) const { return all_[(size_t)d.slot * G_ + g]; }

  // The next group in input order, false when the GPU path is over (the input ended, or handoff()).
  bool next(DevGroup &g) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&]() { return !queue_.empty() || finished_; });
    if (queue_.empty()) return false;
    g = std::move(queue_.front());
    queue_.pop_front();
    return true;
  }
  // a group's reads are no longer used (its alignment has been fetched): its slot may be parsed over
  // once all of its region's groups are released
  void release(const DevGroup &g) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      --busy_[g.slot];
    }
    cv_.notify_all();
  }

 private:
  std::vector<ibwa_ctx_t *> all_;  // slot-major ingest contexts
  std::vector<ibwa_ctx_t *> ing_;  // the slot being parsed
  int G_ = 1, n_slots_ = 0;
  int mode_, trim_, sub_, l_bc_;
  std::function<int(int)> key_of_;
  std::thread producer_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<DevGroup> queue_;
  std::vector<int> busy_;  // per slot: groups of its region not yet released
  bool stop_ = false, finished_ = false;
  int fd_ = -1;
  uint64_t fsize_ = 0, piece_ = 0, carry_ = 0, chunk_ = 0;
  char *buf_[2] = {nullptr, nullptr};  // pinned region buffers (IBWA_FQ_MMAP=0)
  const char *map_ = nullptr;         // the mapped file
  std::unique_ptr<GzSource> src_;     // gzip input: the inflated stream
  bool pageable_ = false;             // buf_ from aligned_alloc (gzip), else pinned
  bool src_end_[2] = {false, false};  // per buffer: the stream ended with it (src_)
  bool src_stop_[2] = {false, false}; // ... or stopped at a problem gzread must see (src_)
  uint64_t map_lo_ = 0;               // ... still mapped from this offset on (consumed regions are unmapped)
  bool ok_ = false, handoff_ = false;
  uint64_t handoff_off_ = 0;
  int cur_ = 0;                 // buffer of the region being parsed
  uint64_t tail_ = 0;           // carried bytes in front of the chunk in buf_[cur_]
  uint64_t tail_file_off_ = 0;  // file offset of the carried bytes' first byte
  uint64_t next_off_ = 0;       // file offset of the next chunk
  uint64_t got_[2] = {0, 0};
  std::thread reader_;
  std::vector<DevGroup> groups_;
  struct Piece {  // one GPU's piece of a region: its records' kept / sequence lengths
    int64_t n_rec = 0;
    uint64_t consumed = 0;
    int not_strict = 0, rc = 0;
    std::vector<int32_t> len;
    std::vector<uint32_t> L;
  };
  std::vector<Piece> pc_;  // per GPU, reused by every region
  double parse_s_ = 0, dev_ms_ = 0, inflate_s_ = 0;
  int64_t n_records_ = 0;

  // regions in turn, each into a slot whose previous region has been released
  void produce() {
    int after = NEXT;
    while (after == NEXT) {
      // the lowest free slot: a slot's buffers are allocated at its first parse, and an allocation
      // can wait long (a process started after one that held most of the HBM), so a short input
      // touches as few slots as it needs
      int slot = -1;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&]() {
          if (stop_) return true;
          for (int q = 0; q < n_slots_; ++q)
            if (busy_[q] == 0) { slot = q; return true; }
          return false;
        });
        if (stop_) break;
      }
      ing_.assign(all_.begin() + (size_t)slot * G_, all_.begin() + (size_t)(slot + 1) * G_);
      after = parse_region();
      {
        std::lock_guard<std::mutex> lk(mu_);
        busy_[slot] = (int)groups_.size();
        for (auto &g : groups_) {
          g.slot = slot;
          queue_.push_back(std::move(g));
        }
        groups_.clear();
        if (after != NEXT) {
          handoff_ = after == HANDOFF;
          finished_ = true;
        }
      }
      cv_.notify_all();
    }
    std::lock_guard<std::mutex> lk(mu_);
    finished_ = true;
    cv_.notify_all();
  }

  // chunk at file offset next_off_ into buf_[b] + carry_ (mapped file: its pages faulted in), by
  // several threads
  void start_read(int b) {
    if (src_) {  // the next chunk of the inflated stream
      char *dst = buf_[b] + carry_;
      reader_ = std::thread([this, b, dst]() {
        const auto t0 = std::chrono::steady_clock::now();
        got_[b] = src_->read(reinterpret_cast<uint8_t *>(dst), chunk_);
        next_off_ += got_[b];
        src_stop_[b] = src_->failed();
        src_end_[b] = src_->eof() || src_->failed();
        inflate_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      });
      return;
    }
    const uint64_t off = next_off_, want = off < fsize_ ? std::min<uint64_t>(chunk_, fsize_ - off) : 0;
    next_off_ = off + want;
    if (map_) {
      got_[b] = want;
      reader_ = std::thread([this, off, want]() {
        const uint64_t pg = 4096, lo = off / pg * pg, hi = std::min<uint64_t>(fsize_, (off + want + pg - 1) / pg * pg);
        const int nt = std::max(1, std::min<int>(ibwa_sam::host_threads(), (int)((hi - lo) >> 26) + 1));
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
          th.emplace_back([&, t]() {
            const uint64_t a = lo + (hi - lo) * t / nt / pg * pg, e = t + 1 == nt ? hi : lo + (hi - lo) * (t + 1) / nt / pg * pg;
            if (e <= a) return;
            if (madvise(const_cast<char *>(map_) + a, e - a, 22 /* MADV_POPULATE_READ */) == 0) return;
            volatile char sink = 0;  // older kernels: touch one byte per page
            for (uint64_t q = a; q < e; q += pg) sink = sink + map_[q];
          });
        for (auto &x : th) x.join();
      });
      return;
    }
    char *dst = buf_[b] + carry_;
    reader_ = std::thread([this, b, off, want, dst]() {
      const int nt = std::max(1, std::min<int>(ibwa_sam::host_threads(), (int)(want >> 24) + 1));
      std::vector<uint64_t> got(nt, 0);
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
          const uint64_t lo = want * t / nt, hi = want * (t + 1) / nt;
          uint64_t p = lo;
          while (p < hi) {
            const ssize_t r = pread(fd_, dst + p, (size_t)std::min<uint64_t>(hi - p, 1u << 30), (off_t)(off + p));
            if (r <= 0) break;
            p += (uint64_t)r;
          }
          got[t] = p - lo;
        });
      for (auto &x : th) x.join();
      uint64_t tot = 0;
      for (int t = 0; t < nt; ++t) {
        if (got[t] != want * (t + 1) / nt - want * t / nt) { tot += got[t]; break; }  // short read: stop there
        tot += got[t];
      }
      got_[b] = tot;
    });
  }

  // Parse the region in buf_[cur_] and form its groups; after them: 1 the next region, 0 the end
  // of the input, -1 the host readers from handoff_off_.
  enum { NEXT = 1, END = 0, HANDOFF = -1 };

  int parse_region() {
    auto key_of = key_of_;
    reader_.join();
    const uint64_t got = got_[cur_];
    // gzip input that stopped at a problem (src_stop): its bytes so far are parsed as not the end of
    // the input, and the host readers take over at the first batch not complete
    const bool src_stop = src_ && src_stop_[cur_];
    const bool eof = src_ ? src_end_[cur_] && !src_stop : next_off_ >= fsize_;
    const char *const base = map_ ? map_ + tail_file_off_ : buf_[cur_] + carry_ - tail_;
    const uint64_t n = tail_ + got;
    // the next chunk is read into the other buffer, behind its carry room, while this region is
    // parsed and aligned (that buffer's previous region went to the GPUs with its parse)
    if (!eof && !src_stop) start_read(cur_ ^ 1);
    groups_.clear();
    if (n == 0) {
      if (!src_stop) return END;
      handoff_off_ = tail_file_off_;
      return HANDOFF;
    }
    // pieces: one per GPU, split at strict record starts (readers.h FastqBulk::rec_at)
    const int G = (int)ing_.size();
    std::vector<uint64_t> cut(G + 1, n);
    cut[0] = 0;
    for (int g = 1; g < G; ++g) {
      uint64_t x = std::max<uint64_t>(cut[g - 1], n * (uint64_t)g / (uint64_t)G);
      cut[g] = n;
      while (x < n) {
        const char *nl = static_cast<const char *>(memchr(base + x, '\n', n - x));
        if (!nl) break;
        x = (uint64_t)(nl + 1 - base);
        FastqBulk::Rec r;
        if (x < n && base[x] == '@' && FastqBulk::rec_at(base + x, base + n, eof, base, r) > 0) { cut[g] = x; break; }
      }
      if (cut[g] < cut[g - 1]) cut[g] = cut[g - 1];
    }
    // each GPU parses its piece (in parallel)
    if ((int)pc_.size() < G) pc_.resize(G);
    std::vector<Piece> &pc = pc_;
    const auto t0 = std::chrono::steady_clock::now();
    {
      std::vector<std::thread> th;
      for (int g = 0; g < G; ++g)
        th.emplace_back([&, g]() {
          Piece &p = pc[g];
          p.n_rec = 0;
          p.consumed = 0;
          p.not_strict = p.rc = 0;
          const uint64_t bytes = cut[g + 1] - cut[g];
          if (!bytes) return;
          // ibwa_fq_parse returns at most cap_lines / 4 + 1 = bytes / 48 + 17 records; the arrays are
          // kept across regions and only ever grow
          const int64_t cap = (int64_t)(bytes / 48 + 17);
          if ((int64_t)p.len.size() < cap) {
            p.len.resize(cap);
            p.L.resize(cap);
          }
          p.rc = ibwa_fq_parse(ing_[g], base + cut[g], bytes, mode_, trim_, &p.n_rec, &p.consumed, &p.not_strict,
                               p.len.data(), p.L.data(), cap);
        });
      for (auto &x : th) x.join();
    }
    parse_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int g = 0; g < G; ++g) {
      if (pc[g].rc) {
        fprintf(stderr, "[ibwa-amd aln] FASTQ parse on GPU %d: %s\n", g, ibwa_last_error());
        handoff_off_ = tail_file_off_;
        return HANDOFF;
      }
      double ms = 0;
      if (cut[g + 1] > cut[g]) ibwa_fq_stats(ing_[g], nullptr, &ms);
      dev_ms_ += ms;
    }
    // the region's records: pieces in order, up to the first one that does not end on its cut
    int g_end = 0;
    bool strict_stop = false;
    uint64_t end_byte = 0;
    for (int g = 0; g < G; ++g) {
      g_end = g + 1;
      end_byte = cut[g] + pc[g].consumed;
      if (end_byte != cut[g + 1] || pc[g].not_strict) {
        strict_stop = pc[g].not_strict != 0;
        break;
      }
    }
    // batches of sub_ kept reads (bwa_read_seq's n_needed; skipped records ride along)
    struct Bt {
      int g0 = 0;
      int64_t r0 = 0, kept = 0;
      int max_len = 0;
      long trimmed = 0, total = 0;
    };
    std::vector<Bt> bts;
    Bt cb;
    bool open_batch = false;
    std::vector<int64_t> kept_before(G + 1, 0);
    int64_t kept_tot = 0, recs = 0;
    for (int g = 0; g < G; ++g) {
      kept_before[g] = kept_tot;
      if (g >= g_end) continue;
      for (int64_t r = 0; r < pc[g].n_rec; ++r) {
        if (!open_batch) {
          cb = Bt();
          cb.g0 = g;
          cb.r0 = r;
          open_batch = true;
        }
        const int32_t len = pc[g].len[r];
        if (len >= 0) {  // bwaseqio.c:176-180, bwa_trim_read
          const long full = (long)pc[g].L[r] - l_bc_;
          cb.total += full;
          cb.trimmed += full - len;
          cb.max_len = std::max<int>(cb.max_len, len);
          ++cb.kept;
          ++kept_tot;
        }
        ++recs;
        if (cb.kept == sub_) {
          bts.push_back(cb);
          open_batch = false;
        }
      }
    }
    kept_before[G] = kept_tot;
    const bool input_end = eof && !strict_stop && end_byte == n;
    uint64_t rewind = end_byte;  // region offset where what follows these groups starts
    if (open_batch) {
      if (input_end) {
        if (cb.kept > 0) bts.push_back(cb);  // the input's last batch
      } else {
        uint64_t off = 0;
        if (cb.r0 > 0 && ibwa_fq_offset(ing_[cb.g0], cb.r0, &off)) {
          fprintf(stderr, "[ibwa-amd aln] FASTQ parse: %s\n", ibwa_last_error());
          handoff_off_ = tail_file_off_;
          return HANDOFF;
        }
        rewind = cut[cb.g0] + off;
        for (int64_t r = cb.r0; r < pc[cb.g0].n_rec; ++r) --recs;  // parsed again
        for (int g = cb.g0 + 1; g < g_end; ++g) recs -= pc[g].n_rec;
      }
    }
    // groups: consecutive batches with the same batch-level key; per GPU the kept reads they hold
    int64_t k0 = 0;
    for (size_t b = 0; b < bts.size();) {
      const int key = key_of(bts[b].max_len);
      DevGroup dg;
      dg.first.assign(G, 0);
      dg.count.assign(G, 0);
      const int64_t ka = k0;
      size_t e = b;
      while (e < bts.size() && key_of(bts[e].max_len) == key) {
        dg.max_len = std::max(dg.max_len, bts[e].max_len);
        dg.trims.emplace_back(bts[e].trimmed, bts[e].total);
        k0 += bts[e].kept;
        ++e;
      }
      dg.n = k0 - ka;
      for (int g = 0; g < G; ++g) {
        const int64_t lo = std::max(ka, kept_before[g]), hi = std::min(k0, kept_before[g + 1]);
        dg.first[g] = hi > lo ? lo - kept_before[g] : 0;
        dg.count[g] = hi > lo ? hi - lo : 0;
      }
      groups_.push_back(std::move(dg));
      b = e;
    }
    n_records_ += recs;
    const uint64_t file_rewind = tail_file_off_ + rewind;
    if (input_end) return END;
    if (strict_stop || eof || src_stop) {  // a record the host readers must see (not strict, truncated, ...)
      handoff_off_ = file_rewind;
      return HANDOFF;
    }
    const uint64_t carry = n - rewind;
    if (carry > carry_) {
      handoff_off_ = file_rewind;
      return HANDOFF;
    }
    // the next region: the carried bytes in front of the next chunk, read meanwhile (mapped file:
    // already there; the page tables of what this region consumed are dropped)
    const int nb = cur_ ^ 1;
    if (map_) {
      const uint64_t pg = 4096, a = tail_file_off_ / pg * pg, e = file_rewind / pg * pg;
      // unmapped, not only dropped: the page tables of 12 GB of mapping cost ~0.1 s at exit
      // (profiles/r05_e2e_i.json, IBWA_ALN_EXIT_PROBE)
      if (e > a && a == map_lo_) {
        munmap(const_cast<char *>(map_) + a, e - a);
        map_lo_ = e;
      } else if (e > a) {
        madvise(const_cast<char *>(map_) + a, e - a, MADV_DONTNEED);
      }
    } else {
      memcpy(buf_[nb] + carry_ - carry, base + rewind, carry);
    }
    tail_ = carry;
    tail_file_off_ = file_rewind;
    cur_ = nb;
    return NEXT;
  }
};

}  // namespace ibwa_cli
