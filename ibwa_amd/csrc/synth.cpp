// synth.cpp -- deterministic synthetic genome + read generator.
//
// SURVEY.md §8(d) fixes the synthetic workload: a GRCh37-sized genome (24
// contigs with the chr1..22/X/Y lengths, seeded repeat families, N runs)
// and 100 bp reads with 1 % substitutions and 5 % of reads carrying one
// 1-3 bp indel, qualities 'I'.  Every random draw comes from splitmix64
// keyed by (seed, stream, index) so the output is identical for any thread
// count and on any host -- no libc / numpy RNG anywhere.
//
// N handling mirrors the reference packer: bns_fasta2bntseq (bntseq.c:180-224)
// replaces every ambiguous base, in file order, by lrand48()&3 after
// srand48(11).  ibwa_pack_nt4() restates that with the POSIX 48-bit LCG so
// the repo-owned index builder produces the same .pac as `bwa index`.
#include <cstdint>
#include <cstdio>
#include <unistd.h>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <thread>
#include <algorithm>
#include <zlib.h>

namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// counter-based draw: value #idx of stream `stream` under `seed`
inline uint64_t draw(uint64_t seed, uint64_t stream, uint64_t idx) {
  return splitmix64(splitmix64(seed * 0x100000001B3ull ^ stream) + idx);
}
inline double unif(uint64_t r) { return (r >> 11) * (1.0 / 9007199254740992.0); }

const char kACGT[4] = {'A', 'C', 'G', 'T'};

// GRCh37 primary assembly lengths, chr1..22, X, Y (hg19 .fai)
const uint64_t kGRCh37[24] = {
    249250621, 243199373, 198022430, 191154276, 180915260, 171115067,
    159138663, 146364022, 141213431, 135534747, 135006516, 133851895,
    115169878, 107349540, 102531392, 90354753,  81195210,  78077248,
    59128983,  63025520,  48129895,  51304566,  155270560, 59373566};

inline char comp(char b) {
  return b == 'A' ? 'T' : b == 'C' ? 'G' : b == 'G' ? 'C' : b == 'T' ? 'A' : 'N';
}

struct Family {
  uint64_t off;  // offset of consensus in the family pool
  uint32_t len;
  double div;    // per-copy divergence
};

}  // namespace

extern "C" {

// Fill `lens[24]` with GRCh37 contig lengths scaled by num/den (min 1000).
// Returns the total length.
uint64_t ibwa_synth_grch37_lengths(uint64_t num, uint64_t den, uint64_t *lens) {
  uint64_t tot = 0;
  for (int i = 0; i < 24; ++i) {
    uint64_t l = kGRCh37[i] * num / den;
    if (l < 1000) l = 1000;
    lens[i] = l;
    tot += l;
  }
  return tot;
}

// Generate an ASCII genome into `out` (total = sum(lens) bytes, no newlines).
//   repeat_frac : fraction of bases covered by mutated copies of repeat families
//   n_frac      : approx. fraction of bases in N runs (telomeres + one internal gap per contig)
// Deterministic in (seed, lens, params) regardless of n_threads.
void ibwa_synth_genome(uint64_t seed, int n_contigs, const uint64_t *lens,
                       double repeat_frac, double n_frac, int n_families,
                       char *out, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  uint64_t total = 0;
  for (int c = 0; c < n_contigs; ++c) total += lens[c];
  // 1. unique background, GC ~41 %; parallel over 1 Mb chunks
  const uint64_t CH = 1u << 20;
  uint64_t n_chunks = (total + CH - 1) / CH;
  auto bg = [&](int t) {
    for (uint64_t ch = t; ch < n_chunks; ch += n_threads) {
      uint64_t b = ch * CH, e = std::min(total, b + CH);
      for (uint64_t i = b; i < e; ++i) {
        uint64_t r = draw(seed, 1, i);
        double u = unif(r);
        // P(A)=P(T)=0.295, P(C)=P(G)=0.205
        out[i] = u < 0.295 ? 'A' : u < 0.5 ? 'C' : u < 0.705 ? 'G' : 'T';
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(bg, t);
    for (auto &x : th) x.join();
  }
  // 2. repeat families: consensus lengths 300..6000, divergence 2..20 %
  if (n_families < 1) n_families = 1;
  std::vector<Family> fam(n_families);
  uint64_t pool_len = 0;
  for (int f = 0; f < n_families; ++f) {
    uint64_t r = draw(seed, 2, f);
    // skew toward short elements (Alu-like ~300 bp are the most common)
    double u = unif(r);
    fam[f].len = (uint32_t)(300 + (uint64_t)(u * u * 5700));
    fam[f].div = 0.02 + 0.18 * unif(draw(seed, 3, f));
    fam[f].off = pool_len;
    pool_len += fam[f].len;
  }
  std::vector<char> pool(pool_len);
  for (uint64_t i = 0; i < pool_len; ++i) pool[i] = kACGT[draw(seed, 4, i) & 3];
  // copies placed per contig, deterministically; each contig is one task
  std::vector<uint64_t> coff(n_contigs + 1, 0);
  for (int c = 0; c < n_contigs; ++c) coff[c + 1] = coff[c] + lens[c];
  auto rep = [&](int t) {
    for (int c = t; c < n_contigs; c += n_threads) {
      uint64_t L = lens[c], base = coff[c];
      uint64_t target = (uint64_t)(repeat_frac * L), covered = 0, k = 0;
      uint64_t stream = 100 + (uint64_t)c * 4;
      while (covered < target && k < (1ull << 40)) {
        uint64_t r0 = draw(seed, stream, k * 4 + 0);
        uint64_t r1 = draw(seed, stream, k * 4 + 1);
        ++k;
        const Family &F = fam[r0 % n_families];
        if (F.len >= L) continue;
        uint64_t pos = r1 % (L - F.len);
        bool rc = (r0 >> 40) & 1;
        for (uint32_t j = 0; j < F.len; ++j) {
          uint64_t rr = draw(seed, stream + 1, (k << 13) ^ j ^ (pos << 20));
          char b = rc ? comp(pool[F.off + F.len - 1 - j]) : pool[F.off + j];
          if (unif(rr) < F.div) b = kACGT[(rr >> 3) & 3];
          out[base + pos + j] = b;
        }
        covered += F.len;
      }
      // a few microsatellites (tandem repeats), 0.5 % of the contig
      uint64_t ms_target = L / 200, ms_cov = 0, m = 0;
      while (ms_cov < ms_target && m < (1ull << 32)) {
        uint64_t r = draw(seed, stream + 2, m++);
        uint32_t unit = 1 + (r & 5);             // 1..6
        uint32_t rl = 20 + ((r >> 8) % 180);     // 20..199 bp
        if (rl + 8 >= L) break;
        uint64_t pos = (r >> 20) % (L - rl);
        char motif[8];
        for (uint32_t q = 0; q < unit; ++q) motif[q] = kACGT[(r >> (40 + 2 * q)) & 3];
        for (uint32_t j = 0; j < rl; ++j) out[base + pos + j] = motif[j % unit];
        ms_cov += rl;
      }
      // N runs: 10 kb telomeres (scaled) + one internal gap
      uint64_t tel = std::min<uint64_t>(10000, (uint64_t)(n_frac * L / 4));
      uint64_t gap = (uint64_t)(n_frac * L) > 2 * tel ? (uint64_t)(n_frac * L) - 2 * tel : 0;
      if (n_frac > 0) {
        for (uint64_t j = 0; j < tel && j < L; ++j) out[base + j] = 'N';
        for (uint64_t j = 0; j < tel && j < L; ++j) out[base + L - 1 - j] = 'N';
        if (gap > 0 && L > gap + 2 * tel) {
          uint64_t gpos = tel + draw(seed, stream + 3, 0) % (L - gap - 2 * tel);
          for (uint64_t j = 0; j < gap; ++j) out[base + gpos + j] = 'N';
        }
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(rep, t);
    for (auto &x : th) x.join();
  }
}

// POSIX drand48 family: X' = (a X + c) mod 2^48; srand48(s): X = s<<16 | 0x330E;
// lrand48() = X' >> 17.  Used to restate bntseq.c:181,224 exactly.
static inline uint64_t lcg48(uint64_t x) {
  return (0x5DEECE66Dull * x + 0xBull) & ((1ull << 48) - 1);
}

// Pack ASCII to 2-bit codes (one byte per base, 0..3) the way `bwa index`
// builds .pac: nst_nt4_table (bntseq.c:39-56) then N -> lrand48()&3 in order.
// Returns the number of ambiguous bases replaced.
uint64_t ibwa_pack_nt4(const char *ascii, uint64_t n, uint8_t *codes) {
  uint64_t x = (11ull << 16) | 0x330E, n_amb = 0;
  for (uint64_t i = 0; i < n; ++i) {
    int c;
    switch (ascii[i]) {
      case 'A': case 'a': c = 0; break;
      case 'C': case 'c': c = 1; break;
      case 'G': case 'g': c = 2; break;
      case 'T': case 't': c = 3; break;
      default: c = 4;
    }
    if (c == 4) {
      x = lcg48(x);
      c = (int)((x >> 17) & 3);
      ++n_amb;
    }
    codes[i] = (uint8_t)c;
  }
  return n_amb;
}

// jump the 48-bit LCG ahead by k steps: compose the affine map x -> a x + c
static uint64_t lcg48_skip(uint64_t x, uint64_t k) {
  const uint64_t M = (1ull << 48) - 1;
  uint64_t A = 1, C = 0, a = 0x5DEECE66Dull, c = 0xBull;
  while (k) {
    if (k & 1) { A = (A * a) & M; C = (C * a + c) & M; }
    c = (c * a + c) & M;  // (a,c)∘(a,c) = (a^2, a c + c)
    a = (a * a) & M;
    k >>= 1;
  }
  return (A * x + C) & M;
}

static inline int nt4_of(char ch) {
  switch (ch) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
  }
}

// Multithreaded ibwa_pack_nt4: identical output (each chunk jumps the LCG
// ahead by the number of ambiguous bases before it).
uint64_t ibwa_pack_nt4_mt(const char *ascii, uint64_t n, uint8_t *codes, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  const uint64_t CH = 1ull << 24, nch = (n + CH - 1) / CH;
  std::vector<uint64_t> namb(nch + 1, 0);
  auto count = [&](int t) {
    for (uint64_t ch = t; ch < nch; ch += n_threads) {
      uint64_t b = ch * CH, e = std::min(n, b + CH), k = 0;
      for (uint64_t i = b; i < e; ++i) k += nt4_of(ascii[i]) == 4;
      namb[ch + 1] = k;
    }
  };
  auto fill = [&](int t) {
    for (uint64_t ch = t; ch < nch; ch += n_threads) {
      uint64_t b = ch * CH, e = std::min(n, b + CH);
      uint64_t x = lcg48_skip((11ull << 16) | 0x330E, namb[ch]);
      for (uint64_t i = b; i < e; ++i) {
        int c = nt4_of(ascii[i]);
        if (c == 4) { x = lcg48(x); c = (int)((x >> 17) & 3); }
        codes[i] = (uint8_t)c;
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(count, t);
    for (auto &x : th) x.join();
  }
  for (uint64_t ch = 0; ch < nch; ++ch) namb[ch + 1] += namb[ch];
  {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(fill, t);
    for (auto &x : th) x.join();
  }
  return namb[nch];
}

// Fixed-length ASCII reads -> bwa_seq_t.seq layout (codes, read reversed;
// bwaseqio.c:183-191): seq[i*len .. i*len+len), off[i] = i*len, lens[i] = len.
void ibwa_encode_reads_fixed(const char *ascii, uint64_t n, int len, uint8_t *seq, uint64_t *off, uint32_t *lens,
                             int n_threads) {
  if (n_threads < 1) n_threads = 1;
  auto work = [&](int t) {
    for (uint64_t r = t; r < n; r += n_threads) {
      const char *s = ascii + r * (uint64_t)len;
      uint8_t *o = seq + r * (uint64_t)len;
      for (int j = 0; j < len; ++j) {
        char ch = s[len - 1 - j];
        o[j] = ch == '-' ? 5 : (uint8_t)nt4_of(ch);
      }
      off[r] = r * (uint64_t)len;
      lens[r] = (uint32_t)len;
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
  for (auto &x : th) x.join();
}

// Draw `n_reads` single-end reads of length `len` from `ascii` (length n,
// contigs concatenated; reads never span a contig boundary or an N).
//   sub_rate   : i.i.d. substitution probability (uniform alternative base)
//   indel_frac : fraction of reads carrying one 1-3 bp indel in [10, len-10)
// Output: `seqs` (n_reads*len ASCII bases, fixed stride len), `pos` (0-based
// leftmost genome coordinate), `strand` (0 fwd / 1 rev).  Deterministic in
// (seed, index) for any thread count.
void ibwa_synth_reads(uint64_t seed, const char *ascii, uint64_t n, int n_contigs,
                      const uint64_t *lens, uint64_t n_reads, int len, double sub_rate,
                      double indel_frac, char *seqs, uint64_t *pos, uint8_t *strand,
                      int n_threads) {
  if (n_threads < 1) n_threads = 1;
  std::vector<uint64_t> coff(n_contigs + 1, 0);
  for (int c = 0; c < n_contigs; ++c) coff[c + 1] = coff[c] + lens[c];
  const int span = len + 3;
  auto work = [&](int t) {
    std::vector<char> win(span + 8), rd(len + 8);
    for (uint64_t r = t; r < n_reads; r += n_threads) {
      uint64_t k = 0;
      for (;;) {
        uint64_t x = draw(seed, 10, r * 64 + k++);
        uint64_t p = x % (n > (uint64_t)span ? n - span : 1);
        int ci = (int)(std::upper_bound(coff.begin(), coff.end(), p) - coff.begin()) - 1;
        if (p + span > coff[ci + 1]) continue;
        bool ok = true;
        for (int j = 0; j < span; ++j) {
          char b = ascii[p + j];
          if (b != 'A' && b != 'C' && b != 'G' && b != 'T') { ok = false; break; }
        }
        if (!ok && k < 4096) continue;
        pos[r] = p;
        break;
      }
      uint64_t p = pos[r];
      uint64_t y = draw(seed, 11, r);
      bool rc = y & 1;
      strand[r] = rc;
      // optional indel
      int ilen = 0, ipos = 0, is_ins = 0;
      if (unif(draw(seed, 12, r)) < indel_frac && len > 24) {
        uint64_t z = draw(seed, 13, r);
        ilen = 1 + (int)(z % 3);
        ipos = 10 + (int)((z >> 8) % (uint64_t)(len - 20));
        is_ins = (z >> 20) & 1;
      }
      // build the read from the forward reference window
      int wi = 0;
      for (int j = 0; j < len; ++j) {
        if (ilen && j == ipos) {
          if (is_ins) {
            for (int q = 0; q < ilen && j < len; ++q, ++j)
              rd[j] = kACGT[draw(seed, 14, r * 8 + q) & 3];
            if (j >= len) break;
          } else {
            wi += ilen;  // deletion: skip reference bases
          }
        }
        rd[j] = ascii[p + wi++];
      }
      // substitutions
      for (int j = 0; j < len; ++j) {
        uint64_t s = draw(seed, 15, r * 1024 + j);
        if (unif(s) < sub_rate) {
          int c = (int)(std::find(kACGT, kACGT + 4, rd[j]) - kACGT);
          if (c < 4) rd[j] = kACGT[(c + 1 + (int)((s >> 7) % 3)) & 3];
        }
      }
      char *o = seqs + r * (uint64_t)len;
      if (rc) {
        for (int j = 0; j < len; ++j) o[j] = comp(rd[len - 1 - j]);
      } else {
        memcpy(o, rd.data(), len);
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
  for (auto &x : th) x.join();
}

// Write n fixed-length reads (ASCII, stride len) as FASTQ records "@r%010d", bases, "+", 'I'
// qualities -- the same bytes tools/e2e_aln.py and bench.py's write_fastq produce -- with n_threads
// formatting and writing their share of records at fixed file offsets.  The reads with index
// [first, first + n) are numbered from `first`.  Returns 0, or -1 if the file cannot be written.
int ibwa_synth_write_fastq(const char *path, const char *seqs, uint64_t first, uint64_t n, int len, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  FILE *f = fopen(path, "wb");
  if (!f) return -1;
  const int fd = fileno(f);
  const uint64_t rec = 12 + 1 + (uint64_t)len + 3 + (uint64_t)len + 1;
  std::vector<int> bad(n_threads, 0);
  auto work = [&](int t) {
    const uint64_t lo = n * t / n_threads, hi = n * (t + 1) / n_threads;
    const uint64_t step = 1u << 16;
    std::vector<char> buf(step * rec);
    for (uint64_t a = lo; a < hi; a += step) {
      const uint64_t b = std::min(hi, a + step);
      char *w = buf.data();
      for (uint64_t r = a; r < b; ++r) {
        uint64_t id = first + r;
        w[0] = '@';
        w[1] = 'r';
        for (int d = 11; d >= 2; --d, id /= 10) w[d] = (char)('0' + id % 10);
        w[12] = '\n';
        memcpy(w + 13, seqs + r * (uint64_t)len, len);
        memcpy(w + 13 + len, "\n+\n", 3);
        memset(w + 16 + len, 'I', len);
        w[16 + 2 * len] = '\n';
        w += rec;
      }
      const uint64_t bytes = (b - a) * rec;
      uint64_t done = 0;
      while (done < bytes) {
        const ssize_t x = pwrite(fd, buf.data() + done, bytes - done, (off_t)(a * rec + done));
        if (x <= 0) { bad[t] = 1; return; }
        done += (uint64_t)x;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
  for (auto &x : th) x.join();
  const bool ok = fclose(f) == 0 && std::find(bad.begin(), bad.end(), 1) == bad.end();
  return ok ? 0 : -1;
}

// The same records gzip-compressed, for the compressed-input legs (bench extra.e2e_gz, tests):
// kind 0 BGZF (SAM spec §4.1: members of <= 65 280 input bytes with the 'BC' extra subfield, the
// empty EOF member last), kind 1 plain gzip members of ~4 MiB input each (no BC field: a reader has
// to find them), kind 2 one member.  qual_mode 0: 'I' as ibwa_synth_write_fastq; 1: binned
// qualities in runs (four bins, NovaSeq-like), so the file compresses like real FASTQ (~4x rather
// than ~7x).  Members are deflated on n_threads threads at `level`.
int ibwa_synth_write_fastq_gz(const char *path, const char *seqs, uint64_t first, uint64_t n, int len,
                              int n_threads, int qual_mode, int kind, int level) {
  if (n_threads < 1) n_threads = 1;
  FILE *f = fopen(path, "wb");
  if (!f) return -1;
  const uint64_t rec = 12 + 1 + (uint64_t)len + 3 + (uint64_t)len + 1;
  const uint64_t mem_in = kind == 0 ? 65280 : (4u << 20);
  auto record = [&](char *w, uint64_t r) {
    uint64_t id = first + r;
    w[0] = '@';
    w[1] = 'r';
    for (int d = 11; d >= 2; --d, id /= 10) w[d] = (char)('0' + id % 10);
    w[12] = '\n';
    memcpy(w + 13, seqs + r * (uint64_t)len, len);
    memcpy(w + 13 + len, "\n+\n", 3);
    if (qual_mode == 0) {
      memset(w + 16 + len, 'I', len);
    } else {
      static const char bins[4] = {'F', ':', ',', '#'};
      int b = 0;
      for (int i = 0; i < len; ++i) {
        const uint64_t x = draw(0x51, first + r, (uint64_t)i);
        if ((x & 7) == 0) {  // a bin change every ~8 bases: mostly F, then :, then , and #
          const uint32_t u = (uint32_t)(x >> 8) % 100;
          b = u < 78 ? 0 : u < 92 ? 1 : u < 98 ? 2 : 3;
        }
        w[16 + len + i] = bins[b];
      }
    }
    w[16 + 2 * len] = '\n';
  };
  // one member from in[0..k): gzip header (+ 'BC' for BGZF), raw deflate, CRC-32, ISIZE
  auto member = [&](const char *in, uint64_t k, std::vector<unsigned char> &out) -> bool {
    z_stream zs{};
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    const size_t h0 = out.size(), hl = kind == 0 ? 18 : 10;
    const size_t bound = deflateBound(&zs, (uLong)k);
    out.resize(h0 + hl + bound + 8);
    unsigned char *h = out.data() + h0;
    memset(h, 0, hl);
    h[0] = 0x1f; h[1] = 0x8b; h[2] = 8; h[9] = 0xff;
    if (kind == 0) { h[3] = 4; h[10] = 6; h[12] = 'B'; h[13] = 'C'; h[14] = 2; }
    zs.next_in = (Bytef *)in;
    zs.avail_in = (uInt)k;
    zs.next_out = h + hl;
    zs.avail_out = (uInt)bound;
    const int r = deflate(&zs, Z_FINISH);
    const size_t clen = bound - zs.avail_out;
    deflateEnd(&zs);
    if (r != Z_STREAM_END) return false;
    const uint32_t crc = (uint32_t)crc32(0, (const Bytef *)in, (uInt)k), isz = (uint32_t)k;
    unsigned char *t = h + hl + clen;
    for (int i = 0; i < 4; ++i) { t[i] = (unsigned char)(crc >> (8 * i)); t[4 + i] = (unsigned char)(isz >> (8 * i)); }
    if (kind == 0) {
      const uint32_t bs = (uint32_t)(hl + clen + 8 - 1);
      if (bs > 0xffff) return false;
      h[16] = (unsigned char)bs; h[17] = (unsigned char)(bs >> 8);
    }
    out.resize(h0 + hl + clen + 8);
    return true;
  };
  if (kind == 2) {  // one member, deflated as a stream
    z_stream zs{};
    if (deflateInit2(&zs, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) { fclose(f); return -1; }
    const uint64_t step = 1u << 14;
    std::vector<char> text(step * rec);
    std::vector<unsigned char> out(1u << 22);
    bool ok = true;
    for (uint64_t a = 0; ok && a <= n; a += step) {
      const uint64_t b = std::min(n, a + step);
      for (uint64_t r = a; r < b; ++r) record(text.data() + (r - a) * rec, r);
      zs.next_in = (Bytef *)text.data();
      zs.avail_in = (uInt)((b - a) * rec);
      const int fl = b == n ? Z_FINISH : Z_NO_FLUSH;
      int r = Z_OK;
      do {
        zs.next_out = out.data();
        zs.avail_out = (uInt)out.size();
        r = deflate(&zs, fl);
        const size_t k = out.size() - zs.avail_out;
        if (r == Z_STREAM_ERROR || (k && fwrite(out.data(), 1, k, f) != k)) ok = false;
      } while (ok && (zs.avail_out == 0 || (fl == Z_FINISH && r != Z_STREAM_END)));
      if (b == n) break;
    }
    deflateEnd(&zs);
    return fclose(f) == 0 && ok ? 0 : -1;
  }
  // thread t compresses records [lo, hi) into its own buffer; the buffers are written in order
  std::vector<std::vector<unsigned char>> outb(n_threads);
  std::vector<int> bad(n_threads, 0);
  auto work = [&](int t) {
    const uint64_t lo = n * t / n_threads, hi = n * (t + 1) / n_threads;
    std::vector<char> text;
    text.reserve(mem_in + rec);
    std::vector<char> one(rec);
    std::vector<unsigned char> &out = outb[t];
    out.reserve((size_t)((hi - lo) * rec / 3));
    for (uint64_t r = lo; r < hi; ++r) {
      record(one.data(), r);
      // members split inside records (a member boundary is not a record boundary in general)
      uint64_t o = 0;
      while (o < rec) {
        const uint64_t k = std::min<uint64_t>(rec - o, mem_in - text.size());
        text.insert(text.end(), one.data() + o, one.data() + o + k);
        o += k;
        if (text.size() == mem_in) {
          if (!member(text.data(), text.size(), out)) { bad[t] = 1; return; }
          text.clear();
        }
      }
    }
    if (!text.empty() && !member(text.data(), text.size(), out)) bad[t] = 1;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
  for (auto &x : th) x.join();
  bool ok = std::find(bad.begin(), bad.end(), 1) == bad.end();
  for (auto &b : outb)
    if (ok && !b.empty() && fwrite(b.data(), 1, b.size(), f) != b.size()) ok = false;
  if (ok && kind == 0) {  // the BGZF end-of-file marker
    static const unsigned char eofb[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C',
                                           2, 0, 0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    ok = fwrite(eofb, 1, sizeof eofb, f) == sizeof eofb;
  }
  return fclose(f) == 0 && ok ? 0 : -1;
}

// A .sai file (bwtaln.c:192, :227-231: 64 B header, then per read int32 n_aln and n_aln 16 B
// records) against per-read hit counts and the concatenated 16 B records of n reads.  Returns the
// first read whose records differ, n if the file holds more than those reads, or -1 if they are
// equal (-2: the file cannot be read).
int64_t ibwa_sai_diff(const char *path, uint64_t n, const int32_t *n_aln, const uint8_t *alns) {
  FILE *f = fopen(path, "rb");
  if (!f) return -2;
  std::vector<char> io(1 << 24);
  setvbuf(f, io.data(), _IOFBF, io.size());
  char hdr[64];
  if (fread(hdr, 1, 64, f) != 64) { fclose(f); return 0; }
  std::vector<uint8_t> rec;
  uint64_t p = 0;
  for (uint64_t i = 0; i < n; ++i) {
    int32_t k = 0;
    if (fread(&k, 4, 1, f) != 1 || k != n_aln[i]) { fclose(f); return (int64_t)i; }
    rec.resize((size_t)k * 16);
    if (k && (fread(rec.data(), 16, (size_t)k, f) != (size_t)k || memcmp(rec.data(), alns + p * 16, (size_t)k * 16))) {
      fclose(f);
      return (int64_t)i;
    }
    p += (uint64_t)k;
  }
  const int extra = fgetc(f);
  fclose(f);
  return extra == EOF ? -1 : (int64_t)n;
}

}  // extern "C"
