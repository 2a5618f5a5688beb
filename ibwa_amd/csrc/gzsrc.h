// gzsrc.h -- gzip input inflated on all host threads.
//
// The reference reads .fq.gz and BAM through zlib's gzread on the thread that parses the records
// (bwaseqio.c:34-41 via utils.c:61 xzopen; kseq.h:156-195's ks_getc; bamlite.h:8): one inflate
// stream, ~0.3-0.6 GB/s, about 2 M reads/s of 100 bp FASTQ -- a fifth of one GPU's search rate.
// Here a gzip file is mapped and inflated in three ways, by its shape:
//  * BGZF (SAM spec §4.1: bgzip output, every BAM): each member names its own compressed size in a
//    'BC' extra subfield and its uncompressed size in the trailer, so the members of a span are
//    found by walking their headers and every one is inflated straight into its place in the output,
//    the span split over all threads.
//  * other multi-member gzip (concatenated files, block-wise writers): member starts are found
//    speculatively -- every "1f 8b 08" with a plausible header in a window ahead -- and inflated in
//    parallel into buffers of their own, while the calling thread inflates the member the stream is
//    at.  Only the chain that follows each member's true end is kept; a false start is an error or
//    a member nothing chains to, and its work is dropped.
//  * one member: one thread inflates it (deflate's back references make a member one serial stream);
//    callers run that thread ahead of the parse (ByteStream's read-ahead, FastqGpu's reader thread).
// Members are inflated with zlib's gzip wrapper, so their CRC-32 and ISIZE are checked before a byte
// is handed on.  After a member, gzread takes the next bytes as a member only when they start with
// the gzip magic and otherwise ends the stream (trailing bytes ignored); so does this source.  At
// anything gzread reports as an error (a bad CRC, a truncated or corrupt member) the source stops
// with failed() -- at the start of that member for members decoded whole, where zlib found the
// problem for the member being streamed -- and ByteStream continues from offset() with gzread
// itself, which reports the error.  (Which bytes before the error gzread hands on depends on its
// internal 16 KiB output chunks -- one that ends in an error is dropped whole -- so on a corrupt file
// the last records kept can differ from the reference's; on a good file the bytes are gzread's.)
#pragma once
#include <dlfcn.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace ibwa_cli {

inline int gz_threads() {  // the CLI's host thread count (sam_common.h host_threads)
  const char *e = getenv("OMP_NUM_THREADS");
  const int n = e && atoi(e) > 0 ? atoi(e) : (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 32));
}

// libdeflate's whole-buffer gzip decoder, when the system has the library (libdeflate.so.0, loaded
// at run time; IBWA_GZ_LIBDEFLATE=0 turns it off): 1.8x zlib's inflate rate per thread on FASTQ
// members.  It checks CRC-32 and ISIZE like zlib; members whose header carries its own CRC (FHCRC,
// which zlib checks) always go to zlib.  Used for members decoded whole (BGZF, speculative starts).
struct LibDeflate {
  void *(*alloc)() = nullptr;
  int (*gzip_ex)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
  void (*release)(void *) = nullptr;
  static const LibDeflate *get() {
    static const LibDeflate *ld = []() -> const LibDeflate * {
      const char *e = getenv("IBWA_GZ_LIBDEFLATE");
      if (e && atoi(e) == 0) return nullptr;
      void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
      if (!h) return nullptr;
      static LibDeflate L;
      L.alloc = reinterpret_cast<void *(*)()>(dlsym(h, "libdeflate_alloc_decompressor"));
      L.gzip_ex = reinterpret_cast<int (*)(void *, const void *, size_t, void *, size_t, size_t *, size_t *)>(
          dlsym(h, "libdeflate_gzip_decompress_ex"));
      L.release = reinterpret_cast<void (*)(void *)>(dlsym(h, "libdeflate_free_decompressor"));
      return L.alloc && L.gzip_ex && L.release ? &L : nullptr;
    }();
    return ld;
  }
  // one thread's decoder
  struct Dec {
    void *d = nullptr;
    const LibDeflate *L = get();
    Dec() {
      if (L) d = L->alloc();
    }
    ~Dec() {
      if (d) L->release(d);
    }
    // the member at in (at most n bytes) into out[0..cap): 0 success (*used, *got), 3 out too small,
    // other values: bad data
    int member(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *used, uint64_t *got) const {
      size_t ai = 0, ao = 0;
      const int r = L->gzip_ex(d, in, (size_t)n, out, (size_t)cap, &ai, &ao);
      *used = ai;
      *got = ao;
      return r;
    }
  };
};

// One zlib stream that inflates gzip members one after another (windowBits 15 + 16: header, CRC-32
// and ISIZE handled and checked by zlib).
struct GzInflater {
  z_stream zs{};
  bool ok = false;
  GzInflater() { ok = inflateInit2(&zs, 15 + 16) == Z_OK; }
  ~GzInflater() {
    if (ok) inflateEnd(&zs);
  }
  GzInflater(const GzInflater &) = delete;
  GzInflater &operator=(const GzInflater &) = delete;
  const uint8_t *in_end = nullptr;  // end of the mapped input
  // start the member at `in` (the input runs to `end`)
  void start(const uint8_t *in, const uint8_t *end) {
    inflateReset(&zs);
    zs.next_in = const_cast<Bytef *>(in);
    zs.avail_in = 0;
    in_end = end;
  }
  // inflate on into out[0..cap): 1 at the member's end (checked), 0 with out full first, -1 on an
  // error or truncated input.  *got: bytes written.
  int run(uint8_t *out, uint64_t cap, uint64_t *got) {
    *got = 0;
    if (!ok) return -1;
    for (;;) {
      if (zs.avail_in == 0) {
        const uint64_t left = (uint64_t)(in_end - (const uint8_t *)zs.next_in);
        zs.avail_in = (uInt)std::min<uint64_t>(left, 1u << 30);
      }
      if (*got == cap) return 0;
      zs.next_out = out + *got;
      zs.avail_out = (uInt)std::min<uint64_t>(cap - *got, 1u << 30);
      const uInt before = zs.avail_out, in_before = zs.avail_in;
      const int r = inflate(&zs, Z_NO_FLUSH);
      *got += before - zs.avail_out;
      if (r == Z_STREAM_END) return 1;
      if (r == Z_BUF_ERROR && zs.avail_out > 0 && zs.avail_in == 0 && in_before == 0) return -1;  // input ended
      if (r != Z_OK && r != Z_BUF_ERROR) return -1;
      if (zs.avail_out > 0 && zs.avail_in == 0 && (const uint8_t *)zs.next_in >= in_end) {
        // all input given: one more call tells the end of the member from a truncation
        const int r2 = inflate(&zs, Z_NO_FLUSH);
        if (r2 == Z_STREAM_END) return 1;
        return -1;
      }
    }
  }
  const uint8_t *pos() const { return (const uint8_t *)zs.next_in; }
};

class GzSource {
 public:
  // true when fn is a regular file that starts with the gzip magic (mapped; nothing inflated yet)
  bool open(const char *fn) {
    if (!fn || !strcmp(fn, "-")) return false;
    const int fd = ::open(fn, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 18) {
      ::close(fd);
      return false;
    }
    n_ = (uint64_t)st.st_size;
    void *m = mmap(nullptr, n_, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) return false;
    m_ = static_cast<const uint8_t *>(m);
    if (!(m_[0] == 0x1f && m_[1] == 0x8b)) {
      munmap(m, n_);
      m_ = nullptr;
      return false;
    }
    madvise(m, n_, MADV_SEQUENTIAL);
    nt_ = gz_threads();
    const char *e = getenv("IBWA_GZ_THREADS");
    if (e && atoi(e) > 0) nt_ = atoi(e);
    hint_ = estimate_size();
    return true;
  }
  ~GzSource() {
    if (m_) munmap(const_cast<uint8_t *>(m_), n_);
  }
  bool eof() const { return eof_; }
  bool failed() const { return failed_; }
  uint64_t offset() const { return uoff_; }  // uncompressed bytes handed on so far
  uint64_t size_hint() const { return hint_; }
  uint64_t compressed_size() const { return n_; }
  bool bgzf() const { return m_ && bgzf_at(0, nullptr); }
  // Up to cap further bytes of the stream into dst; fewer only at its end or when it stops (failed()).
  uint64_t read(uint8_t *dst, uint64_t cap) {
    uint64_t out = 0;
    while (out < cap && !eof_ && !failed_) {
      if (head_) {  // inside a member: stream it
        uint64_t got = 0;
        const int r = head_->run(dst + out, cap - out, &got);
        out += got;
        if (r < 0) { fail(); break; }
        if (r == 1) {
          cpos_ = (uint64_t)(head_->pos() - m_);
          head_.reset();
          after_member();
        }
        continue;
      }
      uint32_t bs = 0;
      if (bgzf_at(cpos_, &bs)) {
        const uint64_t got = bgzf_span(dst + out, cap - out);
        out += got;
        if (got == 0 && !failed_ && !eof_) {
          if (out > 0) break;                      // the next member does not fit: the next call
          start_head(cpos_);                       // a buffer smaller than one member: stream it
        }
        continue;
      }
      out += speculate(dst + out, cap - out);
      if (out == 0 && !eof_ && !failed_ && !head_) start_head(cpos_);
      else if (!head_ && out < cap && !eof_ && !failed_ && spec_stalled_) break;
    }
    uoff_ += out;
    return out;
  }

 private:
  const uint8_t *m_ = nullptr;
  uint64_t n_ = 0, cpos_ = 0, uoff_ = 0, hint_ = 0;
  int nt_ = 1;
  bool eof_ = false, failed_ = false, spec_stalled_ = false;
  std::unique_ptr<GzInflater> head_;
  double in_seen_ = 0, out_seen_ = 0;  // for the window of speculative starts
  struct Spec {                        // a speculatively inflated member
    int status = 0;                    // 1 whole member, 0 stopped at its buffer limit, -1 error
    uint8_t *p = nullptr;              // its output [off, n) (malloc'd, grown as it inflates)
    uint64_t off = 0, n = 0, cap = 0;
    uint64_t end = 0;                  // compressed offset after it (status 1)
    std::unique_ptr<GzInflater> z;     // status 0: the stream, to go on with
    ~Spec() { free(p); }
    uint64_t size() const { return n - off; }
    const uint8_t *data() const { return p + off; }
    bool grow(uint64_t c) {
      void *q = realloc(p, c);
      if (!q) return false;
      p = static_cast<uint8_t *>(q);
      cap = c;
      return true;
    }
  };
  std::map<uint64_t, std::unique_ptr<Spec>> cache_;

  void fail() { failed_ = true; }
  // after a member ended at cpos_: the end of the file, or bytes gzread would not take as a member,
  // end the stream (gz_look: only the magic starts another member)
  void after_member() {
    if (cpos_ + 2 > n_ || !(m_[cpos_] == 0x1f && m_[cpos_ + 1] == 0x8b)) eof_ = true;
  }
  void start_head(uint64_t pos) {
    head_.reset(new GzInflater);
    head_->start(m_ + pos, m_ + n_);
  }
  // a BGZF member header at p (gzip magic, deflate, FEXTRA with a 'BC' subfield of 2 bytes)
  bool bgzf_at(uint64_t p, uint32_t *bsize) const {
    if (p + 18 > n_) return false;
    const uint8_t *h = m_ + p;
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return false;
    const uint32_t xlen = h[10] | (uint32_t)h[11] << 8;
    if (p + 12 + xlen > n_) return false;
    for (uint32_t q = 0; q + 4 <= xlen;) {
      const uint8_t *s = h + 12 + q;
      const uint32_t sl = s[2] | (uint32_t)s[3] << 8;
      if (s[0] == 'B' && s[1] == 'C' && sl == 2 && q + 6 <= xlen) {
        const uint32_t b = (s[4] | (uint32_t)s[5] << 8) + 1u;
        if (b < 12 + xlen + 8 || p + b > n_) return false;
        if (bsize) *bsize = b;
        return true;
      }
      q += 4 + sl;
    }
    return false;
  }
  // The run of BGZF members from cpos_ whose outputs fit in cap, inflated in parallel into place.
  uint64_t bgzf_span(uint8_t *dst, uint64_t cap) {
    struct Blk {
      uint64_t pos, out;
      uint32_t size, isize;
    };
    std::vector<Blk> b;
    uint64_t p = cpos_, o = 0;
    uint32_t bs = 0;
    while (bgzf_at(p, &bs)) {
      const uint8_t *t = m_ + p + bs - 4;
      const uint32_t isz = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
      if (o + isz > cap) break;
      b.push_back({p, o, bs, isz});
      o += isz;
      p += bs;
    }
    if (b.empty()) return 0;
    // contiguous runs of members per thread, balanced by compressed bytes
    const uint64_t cb = p - cpos_;
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)nt_, b.size() / 4 + 1));
    std::vector<size_t> first(nt + 1, b.size());
    first[0] = 0;
    for (int t = 1; t < nt; ++t) {
      const uint64_t at = cpos_ + cb * t / nt;
      first[t] = std::lower_bound(b.begin(), b.end(), at, [](const Blk &x, uint64_t v) { return x.pos < v; }) - b.begin();
    }
    std::atomic<size_t> bad{b.size()};
    auto work = [&](int t) {
      GzInflater z;
      LibDeflate::Dec ld;
      for (size_t i = first[t]; i < first[t + 1] && i < bad.load(std::memory_order_relaxed); ++i) {
        if (ld.d && !(m_[b[i].pos + 3] & 2)) {
          uint64_t used = 0, got = 0;
          const int r = ld.member(m_ + b[i].pos, b[i].size, dst + b[i].out, b[i].isize, &used, &got);
          if (r == 0 && used == b[i].size && got == b[i].isize) continue;
          // anything else is decided by zlib below (the same checks as gzread's)
        }
        z.start(m_ + b[i].pos, m_ + b[i].pos + b[i].size);
        uint64_t got = 0;
        const int r = z.run(dst + b[i].out, b[i].isize, &got);
        // a member ends exactly at its BSIZE with ISIZE bytes (zlib checked CRC and ISIZE mod 2^32)
        bool good = r == 1 && got == b[i].isize && z.pos() == m_ + b[i].pos + b[i].size;
        if (r == 0 && got == b[i].isize) {  // out full: the member must end right here
          uint8_t x;
          uint64_t g2 = 0;
          good = z.run(&x, 1, &g2) == 1 && g2 == 0 && z.pos() == m_ + b[i].pos + b[i].size;
        }
        if (!good) {
          size_t cur = bad.load();
          while (i < cur && !bad.compare_exchange_weak(cur, i)) {
          }
          return;
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    const size_t ok = bad.load();
    const uint64_t got = ok < b.size() ? b[ok].out : o;
    in_seen_ += (double)((ok < b.size() ? b[ok].pos : p) - cpos_);
    out_seen_ += (double)got;
    if (ok < b.size()) {
      cpos_ = b[ok].pos;
      fail();
      return got;
    }
    cpos_ = p;
    after_member();
    return got;
  }
  // plausible gzip member header at p: magic, deflate, no reserved flag bits
  bool member_at(uint64_t p) const {
    return p + 18 <= n_ && m_[p] == 0x1f && m_[p + 1] == 0x8b && m_[p + 2] == 8 && (m_[p + 3] & 0xe0) == 0;
  }
  // A non-BGZF member at cpos_: the calling thread inflates it into dst while the other threads
  // inflate the plausible member starts of a window ahead into their own buffers; then the chain of
  // whole members that follows it is copied out.
  uint64_t speculate(uint8_t *dst, uint64_t cap) {
    spec_stalled_ = false;
    const double ratio = in_seen_ > 0 ? std::max(1.0, out_seen_ / in_seen_) : 4.0;
    const uint64_t win = std::min<uint64_t>(n_ - cpos_, std::max<uint64_t>((uint64_t)(cap / ratio), 1u << 20));
    const uint64_t lim = std::max<uint64_t>(cap / std::max(nt_, 1), 1u << 20);  // per speculative buffer
    std::vector<uint64_t> cand;
    if (!cache_.count(cpos_)) {
      for (uint64_t p = cpos_ + 1; p + 18 <= cpos_ + win && p + 18 <= n_;) {
        const uint8_t *q = static_cast<const uint8_t *>(memchr(m_ + p, 0x1f, (size_t)(cpos_ + win - p)));
        if (!q) break;
        p = (uint64_t)(q - m_);
        if (member_at(p) && !cache_.count(p)) cand.push_back(p);
        ++p;
      }
    }
    std::atomic<size_t> next{0};
    std::vector<std::unique_ptr<Spec>> res(cand.size());
    auto worker = [&]() {
      LibDeflate::Dec ld;
      for (size_t i; (i = next.fetch_add(1)) < cand.size();) {
        std::unique_ptr<Spec> s(new Spec);
        if (ld.d && !(m_[cand[i] + 3] & 2)) {  // whole member at once (untouched capacity costs nothing)
          uint64_t used = 0, got = 0;
          if (!s->grow(lim)) { s->status = -1; res[i] = std::move(s); continue; }
          const int r = ld.member(m_ + cand[i], n_ - cand[i], s->p, lim, &used, &got);
          if (r == 0) {
            s->status = 1;
            s->n = got;
            s->end = cand[i] + used;
            res[i] = std::move(s);
            continue;
          }
          if (r != 3) { s->status = -1; res[i] = std::move(s); continue; }
          free(s->p);  // larger than lim: zlib keeps the stream to go on with
          s->p = nullptr;
          s->cap = 0;
        }
        s->z.reset(new GzInflater);
        s->z->start(m_ + cand[i], m_ + n_);
        // the buffer doubles from 256 KiB up to lim (a false start usually fails in its first bytes)
        for (uint64_t c = std::min<uint64_t>(lim, 256u << 10);; c = std::min<uint64_t>(lim, 2 * c)) {
          if (!s->grow(c)) { s->status = -1; break; }
          uint64_t got = 0;
          s->status = s->z->run(s->p + s->n, c - s->n, &got);
          s->n += got;
          if (s->status != 0 || c == lim) break;
        }
        if (s->status == 1) {
          s->end = (uint64_t)(s->z->pos() - m_);
          s->z.reset();
        } else if (s->status < 0) {
          s->z.reset();
        }
        res[i] = std::move(s);
      }
    };
    std::vector<std::thread> th;
    const int nw = (int)std::min<size_t>((size_t)std::max(nt_ - 1, 0), cand.size());
    for (int t = 0; t < nw; ++t) th.emplace_back(worker);
    uint64_t out = 0;
    // the member at cpos_: cached from an earlier call, or inflated here
    auto it = cache_.find(cpos_);
    std::unique_ptr<Spec> headspec;
    if (it != cache_.end()) {
      headspec = std::move(it->second);
      cache_.erase(it);
    }
    if (!headspec) {
      GzInflater *z = new GzInflater;
      head_.reset(z);
      z->start(m_ + cpos_, m_ + n_);
      uint64_t got = 0;
      const int r = z->run(dst, cap, &got);
      out = got;
      if (r < 0) fail();
      else if (r == 1) {
        in_seen_ += (double)((uint64_t)(z->pos() - m_) - cpos_);
        out_seen_ += (double)got;
        cpos_ = (uint64_t)(z->pos() - m_);
        head_.reset();
        after_member();
      }
    }
    if (nw == 0) worker();  // (no other thread: the candidates here)
    for (auto &x : th) x.join();
    for (size_t i = 0; i < cand.size(); ++i)
      if (res[i] && res[i]->status >= 0) cache_[cand[i]] = std::move(res[i]);
    if (headspec) cache_[cpos_] = std::move(headspec);
    // the chain of cached members from cpos_
    while (!head_ && !eof_ && !failed_ && out < cap) {
      auto c = cache_.find(cpos_);
      if (c == cache_.end()) break;  // a start outside the window: the next round
      Spec &s = *c->second;
      if (s.size() > cap - out) {  // does not fit: the next call (the part that fits when dst is empty)
        if (out == 0) {
          memcpy(dst, s.data(), cap);
          s.off += cap;
          out += cap;
        }
        spec_stalled_ = true;
        break;
      }
      memcpy(dst + out, s.data(), s.size());
      out += s.size();
      if (s.status == 0) {  // it stopped at its buffer limit: stream the rest from its state
        head_ = std::move(s.z);
        cache_.erase(c);
        break;
      }
      in_seen_ += (double)(s.end - cpos_);
      out_seen_ += (double)s.n;
      cpos_ = s.end;
      cache_.erase(c);
      after_member();
    }
    // speculative results behind the stream's position are false starts
    cache_.erase(cache_.begin(), cache_.lower_bound(cpos_));
    if (!head_ && !eof_ && !failed_ && out < cap && !cache_.count(cpos_)) spec_stalled_ = false;
    return out;
  }
  // uncompressed size, estimated from the first members (BGZF: their ISIZE over BSIZE) or from
  // inflating the first few MB
  uint64_t estimate_size() {
    uint64_t p = 0, o = 0;
    uint32_t bs = 0;
    for (int k = 0; k < 64 && bgzf_at(p, &bs); ++k) {
      const uint8_t *t = m_ + p + bs - 4;
      o += t[0] | (uint64_t)t[1] << 8 | (uint64_t)t[2] << 16 | (uint64_t)t[3] << 24;
      p += bs;
    }
    if (p == 0) {
      GzInflater z;
      z.start(m_, m_ + n_);
      std::vector<uint8_t> tmp(8u << 20);
      uint64_t got = 0;
      z.run(tmp.data(), tmp.size(), &got);
      o = got;
      p = (uint64_t)(z.pos() - m_);
    }
    if (p == 0 || o == 0) return n_ * 4;
    if (p >= n_) return o;
    return (uint64_t)((double)n_ * ((double)o / (double)p) * 1.05) + 4096;
  }
};

// A byte stream over a file with gzread's contract (the reference's reading path): a gzip regular
// file through GzSource, read ahead by a background thread into two buffers; anything else (plain
// files, stdin) through gzread.  A GzSource that stops at a problem hands over to gzread at its
// offset.
class ByteStream {
 public:
  ~ByteStream() { close(); }
  bool open(const char *fn) {
    fn_ = fn;
    std::unique_ptr<GzSource> s(new GzSource);
    const char *pe = getenv("IBWA_GZ_PARALLEL");
    if (!(pe && atoi(pe) == 0) && s->open(fn)) {
      src_ = std::move(s);  // the first read starts the read-ahead (a stream never read costs nothing)
      return true;
    }
    fp_ = strcmp(fn, "-") ? gzopen(fn, "r") : gzdopen(fileno(stdin), "r");
    if (fp_) gzbuffer(fp_, 1 << 20);
    return fp_ != nullptr;
  }
  void close() {
    if (fill_.joinable()) fill_.join();
    src_.reset();
    if (fp_) gzclose(fp_);
    fp_ = nullptr;
  }
  bool parallel() const { return src_ != nullptr; }
  const GzSource *source() const { return src_.get(); }
  // up to n bytes; fewer only at the end of the stream; -1 on an error
  int64_t read(void *dst, uint64_t n) {
    uint8_t *d = static_cast<uint8_t *>(dst);
    uint64_t got = 0;
    while (got < n) {
      if (fp_) {
        const int r = gzread(fp_, d + got, (unsigned)std::min<uint64_t>(n - got, 1u << 30));
        if (r < 0) return got ? (int64_t)got : -1;
        if (r == 0) break;
        got += (uint64_t)r;
        continue;
      }
      if (!src_) break;
      if (pos_ == have_) {
        if (!next_buffer()) break;
        continue;
      }
      const uint64_t k = std::min<uint64_t>(n - got, have_ - pos_);
      memcpy(d + got, buf_[cur_].get() + pos_, k);
      pos_ += k;
      got += k;
    }
    return (int64_t)got;
  }
  // to uncompressed offset off of a stream not read from yet (aln's hand-over from the device parse)
  bool seek(uint64_t off) {
    if (fp_) return gzseek(fp_, (z_off_t)off, SEEK_SET) >= 0;
    std::unique_ptr<uint8_t[]> tmp(new uint8_t[1u << 24]);
    while (off > 0) {
      const int64_t r = read(tmp.get(), std::min<uint64_t>(off, 1u << 24));
      if (r <= 0) return false;
      off -= (uint64_t)r;
    }
    return true;
  }

 private:
  static const uint64_t kBuf = (uint64_t)64 << 20;
  std::string fn_;
  gzFile fp_ = nullptr;
  std::unique_ptr<GzSource> src_;
  std::unique_ptr<uint8_t[]> buf_[2];
  uint64_t filled_[2] = {0, 0};
  int cur_ = 1;
  uint64_t pos_ = 0, have_ = 0;
  bool primed_ = false;
  std::thread fill_;

  void start_fill(int b) {
    fill_ = std::thread([this, b]() { filled_[b] = src_->read(buf_[b].get(), kBuf); });
  }
  // the buffer being filled becomes current, the next fill starts; at the source's end or stop,
  // gzread takes over when the source failed
  bool next_buffer() {
    if (!primed_) {
      for (auto &b : buf_) b.reset(new uint8_t[kBuf]);
      primed_ = true;
      cur_ = 1;
      start_fill(0);
    }
    if (fill_.joinable()) fill_.join();
    const int b = cur_ ^ 1;
    const bool more = !src_->eof() && !src_->failed();
    if (filled_[b] == 0 && !more) {
      if (src_->failed()) {  // gzread from here reports (or skips) exactly what the reference's would
        const uint64_t off = src_->offset();
        src_.reset();
        fp_ = gzopen(fn_.c_str(), "r");
        if (!fp_) return false;
        gzbuffer(fp_, 1 << 20);
        if (gzseek(fp_, (z_off_t)off, SEEK_SET) < 0) return false;
        return true;
      }
      src_.reset();
      return false;
    }
    cur_ = b;
    pos_ = 0;
    have_ = filled_[b];
    filled_[b] = 0;
    if (more) start_fill(b ^ 1);
    else filled_[b ^ 1] = 0;
    return true;
  }
};

}  // namespace ibwa_cli
