// aln_main.cpp -- `ibwa-amd aln [options] <prefix> <in.fq>`: the reference's
// aln command (bwtaln.c:243-328, bwa_aln_core :173-241) with the per-batch
// pthread fan-out replaced by the GPU engine (include/ibwa_aln.h).
//
// Kept from the reference: the getopt option set and semantics, gap_opt_t
// written raw as the 64-byte .sai header, 0x40000-read batches, read
// encoding (bwaseqio.c:145-208: barcode strip, -I, -q trimming, reverse /
// reverse-complement), and the per-read `int32 n_aln + n_aln x 16 B` records
// in input order.  Added: -G INT (number of GPUs; a batch is split into
// contiguous slices that keep the batch-level max length, bwtaln.c:89-93).
// Reading the next batch overlaps the GPU work on the current one.
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <cmath>
#include <functional>
#include <algorithm>
#include <string>
#include <thread>
#include <atomic>
#include <type_traits>
#include <vector>

#include "ibwa_aln.h"
#include "ingest.h"
#include "readers.h"
#include "sam_common.h"

namespace {

using ibwa_cli::BamReader;
using ibwa_cli::DevGroup;
using ibwa_cli::FastqBulk;
using ibwa_cli::FastqGpu;
using ibwa_cli::SeqReader;

const auto g_proc_t0 = std::chrono::steady_clock::now();  // process start (static initialisation)
const int kBatch = 0x40000;  // bwtaln.c:193
// A GPU run takes up to kGroup consecutive batches whose batch-level options (bwtaln.c:86-93: the
// max_diff of the batch's longest read, which clamps max_gapo and sizes the stack) are the same,
// so its results are those of running them one by one; a 262 k-read run alone would pay the
// launch tails and host round trips of the passes for every batch.  IBWA_ALN_GROUP /
// IBWA_ALN_SUBBATCH override both (tests: grouped == one batch at a time).
int env_int(const char *k, int dflt) {
  const char *v = getenv(k);
  return v && atoi(v) > 0 ? atoi(v) : dflt;
}
const int kGroup = env_int("IBWA_ALN_GROUP", 16);
const int kSub = env_int("IBWA_ALN_SUBBATCH", kBatch);
const int kMinRdLen = 35;    // BWA_MIN_RDLEN, bwtaln.h:23
const bool kTimes = env_int("IBWA_ALN_TIMES", 0) != 0;
const double kArenaMaxGb = 232.0, kArenaMarginGb = 6.0;  // default device arena (run_aln)

unsigned char nt4[256];

void init_nt4() {  // nst_nt4_table (bntseq.c:39-56)
  memset(nt4, 4, sizeof nt4);
  nt4[(int)'A'] = nt4[(int)'a'] = 0;
  nt4[(int)'C'] = nt4[(int)'c'] = 1;
  nt4[(int)'G'] = nt4[(int)'g'] = 2;
  nt4[(int)'T'] = nt4[(int)'t'] = 3;
  nt4[(int)'-'] = 5;
}

struct Batch {
  std::vector<uint8_t> seq;
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  int max_len = 0;
  std::vector<std::pair<long, long>> trims;  // per 0x40000-read batch: bases trimmed, bases read
  int64_t n() const { return (int64_t)len.size(); }
};

// A GPU run's reads: host-parsed (b) or parsed on the GPUs, staged as views of the parsed block (dg)
struct Group {
  Batch b;
  DevGroup dg;
  bool dev = false;
  int64_t n() const { return dev ? dg.n : b.n(); }
  int max_len() const { return dev ? dg.max_len : b.max_len; }
  const std::vector<std::pair<long, long>> &trims() const { return dev ? dg.trims : b.trims; }
};

// bwa_read_seq (bwaseqio.c:145-208) for FASTQ/FASTA input, bwa_read_bam (:89-143) for BAM: one
// read's barcode strip, -I, -q trimming and reverse into 2-bit codes.  Returns the stored length,
// -1 for a read the reference skips (not longer than the barcode; not on the BAM path).
struct ReadForm {
  bool bam, is_64;
  int l_bc, trim_qual;
  // s / q: the record's sequence and quality (q may be null), l bytes each
  int len_of(const char *s, const char *q, int l, long *n_trimmed, long *n_tot) const {
    (void)s;
    if (!bam && l <= l_bc) return -1;  // bwaseqio.c:162
    const char *qq = q ? q + l_bc : nullptr;
    int len = l - l_bc;
    const int full = len;
    *n_tot += full;
    if (qq && trim_qual >= 1) {  // bwa_trim_read (bwaseqio.c:74-87)
      int sc = 0, mx = 0, max_l = len - 1;
      for (int p = len - 1; p >= kMinRdLen - 1; --p) {
        const unsigned char c = is_64 ? (unsigned char)(char)(qq[p] - 31) : (unsigned char)qq[p];
        sc += trim_qual - (c - 33);
        if (sc < 0) break;
        if (sc > mx) { mx = sc; max_l = p; }
      }
      len = max_l + 1;
      *n_trimmed += full - len;
    }
    return len;
  }
  void put(const char *s, int len, uint8_t *d) const {
    const char *ss = s + l_bc;
    for (int j = 0; j < len; ++j) d[j] = nt4[(unsigned char)ss[len - 1 - j]];  // seq := reverse(read)
  }
};

// A truncated last record (kseq_read's -2, kseq.h:186/:191, which only happens at the end of the
// file; bam_read1's -2/-3 on BAM) ends the input like EOF does: bwa_read_seq's / bwa_read_bam's
// loops (bwaseqio.c:159, :99) stop there and keep every read before it, and bwa_aln_core's next
// read finds nothing.  The record itself is dropped, with a warning (stderr only).
template <class Reader>
int read_serial(Reader &rd, const ReadForm &f, Batch &b, long *n_trimmed, long *n_tot, bool *eof) {
  int l = 0;
  if (*eof) return 0;
  while ((int)b.len.size() < kSub && (l = rd.read()) >= 0) {
    std::string &s = rd.seq, &q = rd.qual;
    const int len = f.len_of(s.data(), q.empty() ? nullptr : q.data(), (int)s.size(), n_trimmed, n_tot);
    if (len < 0) continue;
    const size_t o = b.seq.size();
    b.off.push_back(o);
    b.len.push_back((uint32_t)len);
    if (len > b.max_len) b.max_len = len;
    b.seq.resize(o + len);
    f.put(s.data(), len, b.seq.data() + o);
  }
  if (l < -1) fprintf(stderr, "[ibwa-amd aln] warning: truncated last input record ignored\n");
  if (l < 0) *eof = true;
  return 0;
}

// the records [i0, i1) of the bulk parser into b, in parallel (lengths, then bytes)
void take_bulk(const FastqBulk &fb, size_t i0, size_t i1, const ReadForm &f, Batch &b, long *n_trimmed,
               long *n_tot) {
  const int64_t n = (int64_t)(i1 - i0);
  std::vector<int> ln(n);
  const int nt = std::max(1, std::min<int>(ibwa_sam::host_threads(), (int)(n / 4096) + 1));
  std::vector<long> tr(nt, 0), to(nt, 0);
  const char *base = fb.blk.data();
  ibwa_sam::parallel_chunks(n, [&](int64_t lo, int64_t hi, int t) {
    for (int64_t k = lo; k < hi; ++k) {
      const FastqBulk::Rec &r = fb.recs[i0 + k];
      ln[k] = f.len_of(base + r.s, base + r.q, (int)r.len, &tr[t], &to[t]);
    }
  }, nt);
  for (int t = 0; t < nt; ++t) { *n_trimmed += tr[t]; *n_tot += to[t]; }
  std::vector<uint64_t> off(n);
  uint64_t o = b.seq.size();
  for (int64_t k = 0; k < n; ++k) {
    off[k] = o;
    if (ln[k] >= 0) {
      o += (uint64_t)ln[k];
      b.off.push_back(off[k]);
      b.len.push_back((uint32_t)ln[k]);
      if (ln[k] > b.max_len) b.max_len = ln[k];
    }
  }
  b.seq.resize(o);
  ibwa_sam::parallel_chunks(n, [&](int64_t lo, int64_t hi, int) {
    for (int64_t k = lo; k < hi; ++k)
      if (ln[k] >= 0) f.put(base + fb.recs[i0 + k].s, ln[k], b.seq.data() + off[k]);
  }, nt);
}

// Returns 1 with a batch, 0 at the end of the input, -1 on bad options.
template <class Reader>
int read_batch(Reader &rd, FastqBulk *fb, int mode, int trim_qual, Batch &b, bool *eof) {
  b.seq.clear(); b.off.clear(); b.len.clear(); b.max_len = 0; b.trims.clear();
  long trimmed = 0, total = 0;
  long *n_trimmed = &trimmed, *n_tot = &total;
  const bool bam = std::is_same<Reader, BamReader>::value;
  const ReadForm f{bam, !bam && (mode & IBWA_MODE_IL13) != 0, bam ? 0 : (int)((unsigned)mode >> 24), trim_qual};
  if (((unsigned)mode >> 24) > 15) {
    fprintf(stderr, "[bwa_read_seq] the maximum barcode length is 15.\n");
    return -1;
  }
  auto par = [](int nt, const std::function<void(int)> &g) {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(g, t);
    g(0);
    for (auto &x : th) x.join();
  };
  // the bulk parser's records first (whole strict FASTQ records), then the serial reader
  while (fb && (int)b.len.size() < kSub && fb->more(ibwa_sam::host_threads(), par)) {
    // records the reference skips (barcode) are taken too: the batch is filled up to kSub kept reads
    size_t i1 = fb->qi;
    while ((int)b.len.size() < kSub && fb->qi < fb->recs.size()) {
      i1 = std::min(fb->recs.size(), fb->qi + (size_t)(kSub - (int)b.len.size()));
      take_bulk(*fb, fb->qi, i1, f, b, n_trimmed, n_tot);
      fb->qi = i1;
    }
  }
  if ((int)b.len.size() < kSub) read_serial(rd, f, b, n_trimmed, n_tot, eof);
  b.trims.emplace_back(trimmed, total);
  return b.len.empty() ? 0 : 1;
}

// The batch-level max_diff of a batch whose longest read has max_len (bwtaln.c:86-88).
int batch_key(const ibwa_gap_opt_t &opt, int max_len) {
  return opt.fnr > 0.0f ? ibwa_cal_maxdiff(max_len, 0.02, opt.fnr) : opt.max_diff;
}

// Up to kGroup batches with the same batch-level options into g; a batch whose options differ is
// left in `carry` for the next group.  Returns the batches read (0 at the end), -1 on bad input.
template <class Reader>
int read_group(Reader &rd, FastqBulk *fb, const ibwa_gap_opt_t &opt, Batch &g, Batch &sub, Batch &carry,
               bool &has_carry, bool *eof) {
  g.seq.clear(); g.off.clear(); g.len.clear(); g.max_len = 0; g.trims.clear();
  int nb = 0, key = 0;
  auto append = [&](const Batch &x) {
    const uint64_t base = g.seq.size();
    g.seq.insert(g.seq.end(), x.seq.begin(), x.seq.end());
    for (uint64_t o : x.off) g.off.push_back(base + o);
    g.len.insert(g.len.end(), x.len.begin(), x.len.end());
    g.max_len = std::max(g.max_len, x.max_len);
    g.trims.insert(g.trims.end(), x.trims.begin(), x.trims.end());
  };
  if (has_carry) {
    std::swap(g, carry);
    has_carry = false;
    key = batch_key(opt, g.max_len);
    nb = 1;
  }
  while (nb < kGroup) {
    const int r = read_batch(rd, fb, opt.mode, opt.trim_qual, sub, eof);
    if (r < 0) return -1;
    if (r == 0) break;
    const int k = batch_key(opt, sub.max_len);
    if (nb && k != key) {
      std::swap(carry, sub);
      has_carry = true;
      break;
    }
    key = k;
    if (nb == 0) std::swap(g, sub);
    else append(sub);
    ++nb;
  }
  return nb;
}

void usage(const ibwa_gap_opt_t *o) {
  fprintf(stderr, "\nUsage:   ibwa-amd aln [options] <prefix> <in.fq>\n\n");
  fprintf(stderr, "Options: -n NUM    max #diff (int) or missing prob under 0.02 err rate (float) [%.2f]\n", o->fnr);
  fprintf(stderr, "         -o INT    maximum number or fraction of gap opens [%d]\n", o->max_gapo);
  fprintf(stderr, "         -e INT    maximum number of gap extensions, -1 for disabling long gaps [-1]\n");
  fprintf(stderr, "         -i INT    do not put an indel within INT bp towards the ends [%d]\n", o->indel_end_skip);
  fprintf(stderr, "         -d INT    maximum occurrences for extending a long deletion [%d]\n", o->max_del_occ);
  fprintf(stderr, "         -l INT    seed length [%d]\n", o->seed_len);
  fprintf(stderr, "         -k INT    maximum differences in the seed [%d]\n", o->max_seed_diff);
  fprintf(stderr, "         -m INT    maximum entries in the queue [%d]\n", o->max_entries);
  fprintf(stderr, "         -t INT    number of host threads (recorded in the .sai header) [%d]\n", o->n_threads);
  fprintf(stderr, "         -G INT    number of GPUs [1]\n");
  fprintf(stderr, "         -M INT    mismatch penalty [%d]\n", o->s_mm);
  fprintf(stderr, "         -O INT    gap open penalty [%d]\n", o->s_gapo);
  fprintf(stderr, "         -E INT    gap extension penalty [%d]\n", o->s_gape);
  fprintf(stderr, "         -R INT    stop searching when there are >INT equally best hits [%d]\n", o->max_top2);
  fprintf(stderr, "         -q INT    quality threshold for read trimming down to %dbp [%d]\n", kMinRdLen, o->trim_qual);
  fprintf(stderr, "         -f FILE   file to write output to instead of stdout\n");
  fprintf(stderr, "         -B INT    length of barcode\n");
  fprintf(stderr, "         -c        input sequences are in the color space\n");
  fprintf(stderr, "         -L        log-scaled gap penalty for long deletions\n");
  fprintf(stderr, "         -N        non-iterative mode: search for all n-difference hits (slooow)\n");
  fprintf(stderr, "         -I        the input is in the Illumina 1.3+ FASTQ-like format\n\n");
}

int die(const char *what) {
  fprintf(stderr, "[ibwa-amd aln] %s: %s\n", what, ibwa_last_error());
  return 1;
}

}  // namespace

template <class Reader>
int run_aln(Reader &rd, FastqBulk *fb, const ibwa_gap_opt_t &opt, const std::string &prefix, const char *fn_out,
            int n_gpus, const char *fq_dev, const char *fq_path);

int samse_main(int argc, char *argv[]);  // samse_main.cpp
int sampe_main(int argc, char *argv[]);  // sampe_main.cpp
int index_main(int argc, char *argv[]);  // index_main.cpp
int fa2pac_main(int argc, char *argv[]);
int pac_rev_main(int argc, char *argv[]);

int main(int argc, char *argv[]) {
  // Before the HIP runtime starts: host <-> device copies of every size go through the copy engines.
  // By default the runtime does small ones with shader kernels, which wait until a search grid that
  // holds every CU (the other lane's, or this lane's next one) ends: 1.4 s for an 8-byte copy next
  // to a 1.5 s grid, 0.02 ms with this setting (tools/copy_under_load.hip, profiles/r04_cul_*.txt)
  setenv("GPU_FORCE_BLIT_COPY_SIZE", "0", 0);
  if (argc >= 2 && strcmp(argv[1], "samse") == 0) return samse_main(argc - 1, argv + 1);
  if (argc >= 2 && strcmp(argv[1], "sampe") == 0) return sampe_main(argc - 1, argv + 1);
  if (argc >= 2 && strcmp(argv[1], "index") == 0) return index_main(argc - 1, argv + 1);
  if (argc >= 2 && strcmp(argv[1], "fa2pac") == 0) return fa2pac_main(argc - 1, argv + 1);
  if (argc >= 2 && strcmp(argv[1], "pac_rev") == 0) return pac_rev_main(argc - 1, argv + 1);
  if (argc < 2 || strcmp(argv[1], "aln") != 0) {
    fprintf(stderr, "Usage: ibwa-amd aln [options] <prefix> <in.fq>\n"
                    "       ibwa-amd samse [-n max_occ] [-f out.sam] [-r RG] <prefix> <in.sai> <in.fq>\n"
                    "       ibwa-amd sampe [options] <prefix> <in1.sai> <in2.sai> <in1.fq> <in2.fq>\n"
                    "       ibwa-amd index [-a bwtsw|div|is] [-p prefix] <in.fasta>\n"
                    "       ibwa-amd fa2pac <in.fasta> [<out.prefix>] | pac_rev <in.pac> <out.pac>\n");
    return 1;
  }
  --argc; ++argv;
  init_nt4();
  ibwa_gap_opt_t opt;
  int n_gpus = 1;
  const char *fn_out = nullptr;
  const int first_arg = ibwa_aln_parse_args(argc, argv, &opt, &n_gpus, &fn_out);  // bwtaln.c:249-284 (+ -G)
  if (first_arg < 0) return 1;
  if (first_arg + 2 > argc) {
    usage(&opt);
    return 1;
  }
  if (opt.fnr > 0.0f) {  // bwtaln.c:317-324
    for (int i = 17, k = 0; i <= 250; ++i) {
      int l = ibwa_cal_maxdiff(i, 0.02, opt.fnr);
      if (l != k) fprintf(stderr, "[bwa_aln] %dbp reads: max_diff = %d\n", i, l);
      k = l;
    }
  }
  const std::string prefix = argv[first_arg];
  if (opt.mode & IBWA_MODE_BAM) {  // bwa_open_reads (bwtaln.c:159-171)
    int which = 0;
    if (opt.mode & IBWA_MODE_BAM_SE) which |= 4;
    if (opt.mode & IBWA_MODE_BAM_READ1) which |= 1;
    if (opt.mode & IBWA_MODE_BAM_READ2) which |= 2;
    if (which == 0) which = 7;
    BamReader rd;
    if (!rd.open(argv[first_arg + 1], which)) {
      fprintf(stderr, "[ibwa-amd aln] cannot open %s as BAM\n", argv[first_arg + 1]);
      return 1;
    }
    return run_aln(rd, nullptr, opt, prefix, fn_out, n_gpus, nullptr, argv[first_arg + 1]);
  }
  SeqReader rd;
  if (!rd.open(argv[first_arg + 1])) {
    fprintf(stderr, "[ibwa-amd aln] cannot open %s\n", argv[first_arg + 1]);
    return 1;
  }
  // IBWA_ALN_SERIAL_READ=1: the serial reader only (tests compare the two); an uncompressed FASTQ
  // file is parsed on the GPUs (ingest.h) unless IBWA_ALN_GPU_PARSE=0
  FastqBulk fb(rd);
  const bool serial = env_int("IBWA_ALN_SERIAL_READ", 0) != 0;
  const char *gp = getenv("IBWA_ALN_GPU_PARSE");
  const bool dev_parse = !serial && !(gp && atoi(gp) == 0) && FastqGpu::usable(argv[first_arg + 1]);
  return run_aln(rd, serial ? nullptr : &fb, opt, prefix, fn_out, n_gpus, dev_parse ? argv[first_arg + 1] : nullptr,
                 argv[first_arg + 1]);
}

template <class Reader>
int run_aln(Reader &rd, FastqBulk *fb, const ibwa_gap_opt_t &opt, const std::string &prefix, const char *fn_out,
            int n_gpus, const char *fq_dev, const char *fq_path) {
  FILE *out = fn_out ? fopen(fn_out, "wb") : stdout;
  if (!out) {
    fprintf(stderr, "[ibwa-amd aln] cannot write %s\n", fn_out);
    return 1;
  }
  if (n_gpus < 1) n_gpus = 1;
  ibwa_sam::Phases ph;
  ph.t0 = g_proc_t0;
  ph.mark("startup");  // process start to here: loading, option parsing, opening the input
  // GPU slice g runs on device g mod (visible devices): more slices than devices rehearse the
  // multi-GPU path on fewer GPUs (index replication, the slice split, the ordered writer)
  int n_dev = 0;
  if (ibwa_device_count(&n_dev) || n_dev < 1) return die("no HIP device");
  if (n_gpus > n_dev)
    fprintf(stderr, "[ibwa-amd aln] -G %d on %d visible device(s): slice g runs on device g mod %d\n", n_gpus, n_dev, n_dev);
  // One device arena per GPU, reserved before anything else is allocated (engine.hip Arena): every
  // buffer -- index, ingest slots, the lanes' search scratch -- is carved from it, so no allocation
  // in the middle of the alignment waits for the driver to wipe memory a previous process released.
  // IBWA_ARENA_GB: its size per GPU (0: none); default: the free memory less a margin, at most
  // kArenaMaxGb.
  const int n_used = std::min(n_gpus, n_dev);
  const int n_lanes = std::max(1, std::min(4, env_int("IBWA_ALN_LANES", 2)));
  const char *pm = getenv("IBWA_FQ_PIECE_BYTES"), *cm = getenv("IBWA_FQ_CARRY_BYTES");
  // 1.5 GiB per GPU (~7 M reads of 100 bp): fewer, larger groups than 1 GiB pieces (align phase 6.12-6.2
  // vs 5.71-5.79 s at 50 M reads with 2 GiB, profiles/r05_e2e_i.json; 2.5 and 3 GiB measured no
  // faster); 1.5 GiB aligned as fast as 2 GiB (5.15 vs 5.18-5.36 s) with the arena's peak use 174 ->
  // 160 GB (round 6, profiles/r06_e2e_mem.json: the resume states and width rows scale with the
  // group; first-pass chunks capped at 4 M reads inside a group took 141 GB but +10 %).  An
  // input that the pieces would cut into at most one group per lane (10 M reads of 150 bp: two
  // 1.7 GB groups) is cut into two groups per lane instead: the lanes run their groups side by side
  // either way, and the process stays under ~128 GiB (124 vs 146 GiB for that input, align +6 %,
  // r05_pipe_full_v{2,3}.json) -- so that both ends of a pair can be aligned at once on one GPU.
  // (Back to back, the second process waits for the driver to wipe the first one's memory whatever
  // its size: the wipe runs on the copy engine that also clears the new allocation,
  // profiles/r05_b2b*.jsonl.)
  // FASTQ bytes of the input: the file's size, or for gzip the inflated size GzSource estimates from
  // its first members
  auto fastq_bytes = [](const char *path) -> double {
    struct stat st;
    if (!path || stat(path, &st) != 0) return 0.0;
    if (FastqGpu::is_gzip(path)) {
      ibwa_cli::GzSource g;
      if (g.open(path)) return (double)g.size_hint();
      return 4.0 * (double)st.st_size;
    }
    return (double)st.st_size;
  };
  const double in_bytes = fastq_bytes(fq_path && strcmp(fq_path, "-") ? fq_path : nullptr);
  uint64_t piece = pm && atoll(pm) > 0 ? (uint64_t)atoll(pm) : (uint64_t)3 << 29;
  if (!(pm && atoll(pm) > 0) && fq_dev) {
    const uint64_t fs = (uint64_t)in_bytes;
    const uint64_t per_lane = (uint64_t)n_lanes * (uint64_t)n_gpus;
    if (fs > 0 && fs <= piece * per_lane)
      piece = std::max<uint64_t>((uint64_t)256 << 20, (fs + 2 * per_lane - 1) / (2 * per_lane));
  }
  int cli_tab_k = 0;  // the level tables' K, pinned on the aligning contexts (the arena counts them)
  {
    // The default arena follows the inputs, calibrated on what round 5 measured (GiB; IBWA_ARENA_TRACE=1
    // lists every carve, profiles/r05_arena_trace.log): the index structures (relaid-out BWT, bit
    // planes, K-mer tables of K <= 14: ~7.5x the two .bwt files); per lane a part that does not grow
    // with its group (first-pass slots, page pools, cooperative pool and staging: ~30, ~36 above
    // 128 bp with the larger pool; less for a small group, whose grids are smaller) plus a part per
    // GiB of FASTQ the group holds (resume states, width rows, per-read arrays: ~21.5 at 100 bp; ~16
    // at 150 bp -- fewer reads per GiB -- plus room for the resume states to grow after the first
    // group); the ingest scratch ~1.7x and each ingest slot ~0.8x a region's piece.  Measured peaks:
    // 169 GiB at 100 bp in 1.94 GiB groups (r05_e2e_h.json), 147 GiB at 150 bp in 1.58 GiB groups
    // (r05_pipe_full_v2.json).  An arena larger than the need makes the next process wait for the
    // driver to wipe it (~33 GB/s).  At most kArenaMaxGb.
    auto fbytes = [](const std::string &f) -> double {
      struct stat st;
      return stat(f.c_str(), &st) == 0 ? (double)st.st_size : 0.0;
    };
    const double GiB = (double)(1u << 30);
    // FASTQ bytes of one GPU's group: a region's piece (equal regions of at most `piece` per GPU, as
    // FastqGpu cuts them), or (host readers) up to kGroup batches
    const double fq = in_bytes;
    double grp_b = (double)kGroup * kSub * 300.0;
    if (fq_dev) {
      const double per = (double)piece * n_gpus, n_reg = std::max(1.0, std::ceil(fq / per));
      grp_b = std::min(per, fq / n_reg) / n_gpus;
    }
    const double grp = std::min(fq / n_gpus, grp_b) / GiB;
    // the read length from the first record (plain FASTQ): longer reads take the larger pool
    int first_len = 0;
    if (fq_path && strcmp(fq_path, "-") != 0)
      if (gzFile f = gzopen(fq_path, "rb")) {  // (plain files are read as they are)
        char line[4096];
        if (gzgets(f, line, sizeof line) && line[0] == '@' && gzgets(f, line, sizeof line))
          first_len = (int)strcspn(line, "\r\n");
        gzclose(f);
      }
    const bool long_reads = first_len == 0 || first_len > 128;
    const double fixed = long_reads ? 36.0 : 30.0, per_gib = long_reads ? 20.0 : 21.5;
    // the first pass's level tables (engine gap_tab_k): 2 x 8 B x ((4^(K+2) - 1) / 3) for the K that
    // strings of length K + 1 still mostly occur at, at most 13 (5.7 GB for a GRCh37-sized genome; the
    // engine's auto rule would take 14 -- 23 GB, -5 % k_gapped -- where HBM has room: here the CLI
    // keeps its footprint)
    const double seq_len = 4.0 * fbytes(prefix + ".bwt");
    int tab_k = 0;
    while (tab_k < 13 && std::ldexp(1.0, 2 * (tab_k + 1)) <= seq_len) ++tab_k;
    cli_tab_k = tab_k;
    const double ltab_gb = tab_k ? 2.0 * 8.0 * (std::ldexp(1.0, 2 * (tab_k + 2)) / 3.0) / GiB : 0.0;
    const double need_gb = ltab_gb + 7.5 * (fbytes(prefix + ".bwt") + fbytes(prefix + ".rbwt")) / GiB +
                           n_lanes * (std::min(fixed, 2.0 * fixed * grp) + per_gib * grp) + 1.7 * grp +
                           (n_lanes + 3) * 0.8 * grp + 2.0;
    const char *ag = getenv("IBWA_ARENA_GB");
    std::vector<std::thread> th;
    std::vector<int> rc(n_used, 0);
    std::vector<double> want_gb(n_used, 0.0), ms(n_used, 0.0);
    {  // HIP start-up (device enumeration, the driver's process state) apart from the reservation
      uint64_t fr = 0, tot = 0;
      (void)ibwa_device_memory(0, &fr, &tot);
      ph.mark("gpu runtime start");
    }
    for (int d = 0; d < n_used; ++d)
      th.emplace_back([&, d]() {
        const auto t0 = std::chrono::steady_clock::now();
        uint64_t fr = 0, tot = 0;
        double gb = ag ? atof(ag) : 0.0;
        if (!ag && ibwa_device_memory(d, &fr, &tot) == 0)
          gb = std::min(std::min(kArenaMaxGb, (double)fr / (1u << 30) - kArenaMarginGb), need_gb);
        want_gb[d] = gb;
        if (gb >= 1.0) rc[d] = ibwa_reserve(d, (uint64_t)(gb * (1u << 30)));
        ms[d] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      });
    for (auto &t : th) t.join();
    for (int d = 0; d < n_used; ++d) {
      if (rc[d])
        fprintf(stderr, "[ibwa-amd aln] warning: no arena on GPU %d (%s); buffers are allocated one by one\n", d,
                ibwa_last_error());
      else if (kTimes && want_gb[d] >= 1.0)
        fprintf(stderr, "[ibwa-amd aln] arena on GPU %d: %.1f GiB reserved in %.0f ms\n", d, want_gb[d], ms[d]);
    }
  }
  ph.mark("device arena");  // HIP start-up, and the wait for memory a previous process released
  // FASTQ parsed on the GPUs: n_lanes + 3 ingest contexts per GPU (their own streams and buffers;
  // ingest.h's slots); the first region is read and parsed while the index loads
  std::vector<ibwa_ctx_t *> ing;
  std::unique_ptr<FastqGpu> fg;
  struct Destroy {
    std::vector<ibwa_ctx_t *> &v;
    std::unique_ptr<FastqGpu> &f;
    ~Destroy() {
      f.reset();
      for (auto *x : v) ibwa_ctx_destroy(x);
    }
  } destroy_ing{ing, fg};
  if (fq_dev) {
    // one slot per group a lane can hold and the group being launched, and two more parsed ahead:
    // a parse waits for launch boundaries of the searches (their grids hold every CU), so with one
    // slot ahead the launching thread still waited (6.9 s of waits at 50 M reads, r04_e2e_50m_v2)
    // (the producer parses one region at a time, so a GPU's slots share one parse scratch: only the
    // kept reads stay per slot)
    const int n_slots = n_lanes + 3;
    for (int sl = 0; sl < n_slots; ++sl)
      for (int g = 0; g < n_gpus; ++g) {
        ibwa_ctx_t *x = nullptr;
        if (ibwa_ctx_create(g % n_dev, &x)) return die("ibwa_ctx_create (ingest)");
        if (sl > 0 && ibwa_fq_share_scratch(x, ing[g])) return die("ibwa_fq_share_scratch");
        ing.push_back(x);
      }
    const uint64_t carry = cm && atoll(cm) > 0 ? (uint64_t)atoll(cm) : (uint64_t)256 << 20;
    fg.reset(new FastqGpu(fq_dev, ing, n_gpus, opt.mode, opt.trim_qual, kSub, piece, carry,
                          [opt](int max_len) { return batch_key(opt, max_len); }));
    if (!fg->ok()) {
      fprintf(stderr, "[ibwa-amd aln] cannot read %s for the device parse\n", fq_dev);
      return 1;
    }
  }
  // IBWA_CTX_OPTS="key=value,...": engine options (ibwa_ctx_set_option) for every aligning context --
  // measurement and tuning (e.g. kmer_k=14,coop_pool_gb=10)
  auto ctx_opts = [](ibwa_ctx_t *x) -> int {
    const char *e = getenv("IBWA_CTX_OPTS");
    if (!e) return 0;
    std::string all(e);
    size_t p = 0;
    while (p < all.size()) {
      const size_t q = std::min(all.find(',', p), all.size());
      const std::string kv = all.substr(p, q - p);
      const size_t eq = kv.find('=');
      if (eq != std::string::npos && ibwa_ctx_set_option(x, kv.substr(0, eq).c_str(), atol(kv.c_str() + eq + 1))) {
        fprintf(stderr, "[ibwa-amd aln] IBWA_CTX_OPTS: %s: %s\n", kv.c_str(), ibwa_last_error());
        return 1;
      }
      p = q + 1;
    }
    return 0;
  };
  std::vector<ibwa_ctx_t *> ctx(n_gpus, nullptr);
  for (int g = 0; g < n_gpus; ++g) {
    if (ibwa_ctx_create(g % n_dev, &ctx[g]) || ibwa_ctx_set_option(ctx[g], "gap_tab_k", cli_tab_k) ||
        ctx_opts(ctx[g]))
      return die("ibwa_ctx_create");
    if (g == 0) {
      if (ibwa_ctx_load_bwt_file(ctx[0], 0, (prefix + ".bwt").c_str())) return die("load .bwt");
      if (ibwa_ctx_load_bwt_file(ctx[0], 1, (prefix + ".rbwt").c_str())) return die("load .rbwt");
    } else if (ibwa_ctx_clone_index(ctx[g], ctx[0])) {
      return die("replicate index");
    }
  }
  fwrite(&opt, sizeof opt, 1, out);  // bwtaln.c:192
  ph.mark("load index");

  // the index's device structures for these options are built while the first reads are parsed
  std::vector<int> prep_rc(n_gpus, 0);
  std::vector<std::thread> prep;
  for (int g = 0; g < n_gpus; ++g) prep.emplace_back([&, g]() { prep_rc[g] = ibwa_ctx_prepare(ctx[g], &opt); });
  Group cur;
  Batch sub, carry;
  bool has_carry = false;
  bool eof = false;
  double parse_s = 0;  // wall time of the FASTQ parse (all host threads, or waiting for the GPUs')
  bool dev_active = fg != nullptr, dev_done = false;
  auto timed_read = [&](Group &into) {
    const auto t = std::chrono::steady_clock::now();
    int r = 0;
    into.dev = false;
    if (dev_active) {
      if (fg->next(into.dg)) {
        into.dev = true;
        r = 1;
      } else {
        dev_active = false;
        if (fg->handoff()) {  // the host readers from the first batch the device path did not take
          fprintf(stderr, "[ibwa-amd aln] the host readers take over at byte %llu\n",
                  (unsigned long long)fg->handoff_offset());
          if (!rd.in.seek(fg->handoff_offset())) r = -1;
        } else {
          dev_done = true;  // the input ended on the GPU path
        }
      }
    }
    if (!into.dev && r == 0 && !dev_done) r = read_group(rd, fb, opt, into.b, sub, carry, has_carry, &eof);
    parse_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    return r;
  };
  int64_t tot_seqs = 0;
  std::thread writer;
  std::atomic<bool> write_failed{false};
  struct JoinAtExit {  // an early return still waits for the write in flight
    std::thread &t;
    ~JoinAtExit() {
      if (t.joinable()) t.join();
    }
  } join_writer{writer};
  int have = timed_read(cur);
  for (auto &t : prep) t.join();
  for (int g = 0; g < n_gpus; ++g)
    if (prep_rc[g]) return die("prepare the index");
  ph.mark("read (index prepared meanwhile)");
  // Overlapped groups: lane l's contexts (one per GPU) share lane 0's index and take every
  // n_lanes-th group, so a group's staging, first pass and host work run while the previous group's
  // cooperative pass drains.  Groups finish, and their records are written, in input order.
  std::vector<std::vector<ibwa_ctx_t *>> lctx(n_lanes);
  lctx[0] = ctx;
  for (int l = 1; l < n_lanes; ++l)
    for (int g = 0; g < n_gpus; ++g) {
      ibwa_ctx_t *x = nullptr;
      if (ibwa_ctx_create(g % n_dev, &x) || ctx_opts(x) || ibwa_ctx_share_index(x, ctx[g]))
        return die("a second context on the GPU");
      lctx[l].push_back(x);
    }
  // a slice's .sai records (ibwa_batch_fetch_sai), in buffers that go round: slice thread -> writer
  // -> pool (no allocation or page faults per group once the pool holds a buffer per slice in flight)
  struct SaiBuf {  // 2 MiB-aligned, huge pages advised: fewer faults and page tables (exit costs ~pages)
    char *p = nullptr;
    uint64_t cap = 0, bytes = 0;
    SaiBuf() = default;
    SaiBuf(SaiBuf &&o) noexcept : p(o.p), cap(o.cap), bytes(o.bytes) { o.p = nullptr; o.cap = o.bytes = 0; }
    SaiBuf &operator=(SaiBuf &&o) noexcept {
      std::swap(p, o.p);
      std::swap(cap, o.cap);
      std::swap(bytes, o.bytes);
      return *this;
    }
    ~SaiBuf() { free(p); }
    bool grow(uint64_t n) {
      free(p);
      cap = (n + (2u << 20) - 1) / (2u << 20) * (2u << 20);
      p = static_cast<char *>(aligned_alloc(2u << 20, cap));
      if (!p) return false;
      madvise(p, cap, MADV_HUGEPAGE);
      return true;
    }
  };
  std::mutex pool_mu;
  std::vector<SaiBuf> pool;
  auto take_buf = [&]() {
    std::lock_guard<std::mutex> lk(pool_mu);
    SaiBuf b;
    if (!pool.empty()) {
      b = std::move(pool.back());
      pool.pop_back();
    }
    return b;
  };
  struct Job {
    Group b;
    std::vector<SaiBuf> sai;
    std::vector<int> rc;
    std::vector<std::thread> th;
    std::chrono::steady_clock::time_point t0;
    bool active = false;
  };
  std::vector<Job> jobs(n_lanes);
  struct JoinJobs {  // an early return still waits for the groups in flight
    std::vector<Job> &j;
    ~JoinJobs() {
      for (auto &x : j)
        for (auto &t : x.th)
          if (t.joinable()) t.join();
    }
  } join_jobs{jobs};
  auto launch = [&](Job &J, std::vector<ibwa_ctx_t *> &cx) {
    const int64_t n = J.b.n();
    J.sai.clear();
    J.sai.resize(n_gpus);
    J.rc.assign(n_gpus, 0);
    J.th.clear();
    J.t0 = std::chrono::steady_clock::now();
    J.active = true;
    const int64_t per = (n + n_gpus - 1) / n_gpus;
    // a group parsed on the GPUs is staged as a view of its ingest slot (released in finish());
    // its slices are the group's reads in each GPU's piece
    std::vector<double> stage_ms(n_gpus, 0.0);
    if (J.b.dev)
      for (int g = 0; g < n_gpus; ++g) {
        const auto s0 = std::chrono::steady_clock::now();
        J.rc[g] = ibwa_batch_stage_fq(cx[g], fg->ctx_of(J.b.dg, g), J.b.dg.first[g], J.b.dg.count[g], J.b.dg.max_len);
        stage_ms[g] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s0).count();
      }
    for (int g = 0; g < n_gpus; ++g) {
      J.th.emplace_back([&J, &cx, &opt, &take_buf, g, n, per, sms = stage_ms[g]]() {
        const Group &cur = J.b;
        int64_t b = std::min<int64_t>(n, g * per), e = std::min<int64_t>(n, b + per);
        if (cur.dev) b = 0, e = cur.dg.count[g];
        int64_t tot = 0;
        auto c0 = std::chrono::steady_clock::now();
        int rc = J.rc[g];
        if (!cur.dev) {
          // each slice is staged from its own bytes only: offsets rebased to the slice's first read
          // (reads are contiguous in input order); the batch-level max length still applies
          const Batch &hb = cur.b;
          const uint64_t base = b < e ? hb.off[b] : 0;
          std::vector<uint64_t> off(hb.off.begin() + b, hb.off.begin() + e);
          for (auto &x : off) x -= base;
          // ibwa_aln_batch, in its three steps (IBWA_ALN_TIMES=1: their wall times per slice)
          rc = ibwa_batch_stage(cx[g], e - b, hb.seq.data() + base, off.data(), hb.len.data() + b);
        }
        auto c1 = std::chrono::steady_clock::now();
        if (!rc) rc = ibwa_batch_run(cx[g], &opt, cur.max_len());
        auto c2 = std::chrono::steady_clock::now();
        if (!rc) {  // the records serialised straight into a pooled buffer (grown when too small)
          SaiBuf sb = take_buf();
          uint64_t need = 0;
          rc = ibwa_batch_fetch_sai(cx[g], sb.p, sb.cap, &need, &tot);
          if (!rc && need > sb.cap) {
            if (!sb.grow(need + need / 8)) {
              fprintf(stderr, "[ibwa-amd aln] out of host memory for %llu bytes of records\n", (unsigned long long)need);
              rc = 1;
            } else {
              rc = ibwa_batch_fetch_sai(cx[g], sb.p, sb.cap, &need, &tot);
            }
          }
          sb.bytes = need;
          J.sai[g] = std::move(sb);
        }
        auto c3 = std::chrono::steady_clock::now();
        J.rc[g] = rc;
        if (kTimes) {
          auto ms = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
            return std::chrono::duration<double, std::milli>(y - x).count();
          };
          ibwa_run_stats_t st;
          ibwa_batch_stats(cx[g], &st);
          fprintf(stderr, "[ibwa-amd aln] slice %d: %lld reads, stage %.1f run %.1f (of which allocating %.1f) fetch %.1f ms\n",
                  g, (long long)(e - b), ms(c0, c1) + sms, ms(c1, c2), st.ms_alloc, ms(c2, c3));
        }
      });
    }
  };
  // wait for a group, then hand its records to the writer (bwtaln.c:227-231, input order, one write
  // per slice); the previous group's write has finished first
  auto finish = [&](Job &J) -> int {
    for (auto &t : J.th) t.join();
    J.th.clear();
    J.active = false;
    if (J.b.dev) fg->release(J.b.dg);  // its ingest slot may be parsed over
    for (int g = 0; g < n_gpus; ++g)
      if (J.rc[g]) return die("aln");
    tot_seqs += J.b.n();
    fprintf(stderr, "[bwa_aln_core] calculate SA coordinate... %.2f sec\n",
            std::chrono::duration<double>(std::chrono::steady_clock::now() - J.t0).count());
    fprintf(stderr, "[bwa_aln_core] write to the disk... ");
    if (writer.joinable()) writer.join();
    if (write_failed) {
      fprintf(stderr, "[ibwa-amd aln] write failed\n");
      return 1;
    }
    writer = std::thread([out, &write_failed, &pool_mu, &pool, sai = std::move(J.sai)]() mutable {
      for (auto &b : sai) {
        if (b.bytes && fwrite(b.p, 1, b.bytes, out) != b.bytes) write_failed = true;
        std::lock_guard<std::mutex> lk(pool_mu);
        pool.push_back(std::move(b));
      }
    });
    fprintf(stderr, "0.00 sec\n");
    fprintf(stderr, "[bwa_aln_core] %lld sequences have been processed.\n", (long long)tot_seqs);
    return 0;
  };
  int64_t k = 0;  // groups launched
  // IBWA_ALN_PARSE_ONLY=1 (measurement): the input is read and parsed into groups, nothing is aligned
  const bool parse_only = env_int("IBWA_ALN_PARSE_ONLY", 0) != 0;
  const auto t_parse_only = std::chrono::steady_clock::now();
  while (have > 0 && parse_only) {
    tot_seqs += cur.n();
    if (cur.dev) fg->release(cur.dg);
    have = timed_read(cur);
  }
  if (parse_only) {
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_parse_only).count();
    fprintf(stderr, "[ibwa-amd aln] parse only: %lld reads, %.3f s parsing (%.3f s after the first group) = %.2f M reads/s (%s)\n",
            (long long)tot_seqs, parse_s, s, tot_seqs / std::max(parse_s, 1e-9) / 1e6, fg ? "GPU parse" : "host parse");
  }
  while (have > 0) {
    Job &J = jobs[k % n_lanes];
    if (J.active)  // the oldest group in flight
      if (int rc = finish(J)) return rc;
    if (opt.trim_qual >= 1)  // once per 0x40000-read batch, as bwa_read_seq (bwaseqio.c:206)
      for (const auto &t : cur.trims())
        if (t.second) fprintf(stderr, "[bwa_read_seq] %.1f%% bases are trimmed.\n", 100.0f * t.first / t.second);
    std::swap(J.b, cur);
    launch(J, lctx[k % n_lanes]);
    ++k;
    have = timed_read(cur);  // the next group is parsed while the GPUs work
  }
  for (int64_t q = std::max<int64_t>(0, k - n_lanes); q < k; ++q)
    if (jobs[q % n_lanes].active)
      if (int rc = finish(jobs[q % n_lanes])) return rc;
  ph.mark("align (groups overlapped, next group parsed meanwhile)");
  if (writer.joinable()) writer.join();
  if (write_failed) {
    fprintf(stderr, "[ibwa-amd aln] write failed\n");
    return 1;
  }
  if (out != stdout) fclose(out);
  ph.mark("last records written");
  int64_t dev_now = 0, dev_peak = 0;
  ibwa_device_bytes(&dev_now, &dev_peak);
  ph.print("ibwa-amd aln");
  fprintf(stderr, "[ibwa-amd aln] device memory: peak %.1f GB of engine buffers on %d GPU(s) (%d context(s) per GPU, "
                  "index shared)\n", dev_peak / 1e9, n_gpus, n_lanes);
  for (int d = 0; d < n_used; ++d) {
    uint64_t asz = 0, aused = 0, apeak = 0;
    if (ibwa_arena_stats(d, &asz, &aused, &apeak) == 0 && asz)
      fprintf(stderr, "[ibwa-amd aln] arena on GPU %d: %.1f GB, peak use %.1f GB\n", d, asz / 1e9, apeak / 1e9);
  }
  if (fg) {
    fprintf(stderr, "[ibwa-amd aln] input parsed on the GPUs: %lld records, %.2f s parsing ahead of the alignment (%.0f ms "
                    "of device time: H2D copies + kernels)%s\n",
            (long long)fg->records(), fg->parse_s(), fg->dev_ms(), fg->handoff() ? "; the host readers took the rest" : "");
    if (fg->gzip())
      fprintf(stderr, "[ibwa-amd aln] %s input inflated on %d host threads: %.3f GB in %.2f s of the reader thread "
                      "(ahead of the parse)\n",
              fg->bgzf() ? "BGZF" : "gzip", ibwa_cli::gz_threads(), fg->input_bytes() / 1e9, fg->inflate_s());
  }
  if (parse_s > 0 && fg && !fg->handoff()) {  // every record parsed on the GPUs: the time is waiting
    fprintf(stderr, "[ibwa-amd aln] input: %lld reads parsed on the GPUs, %.2f s waited for parsed groups\n",
            (long long)tot_seqs, parse_s);
  } else if (parse_s > 0) {
    const int nt = fb ? ibwa_sam::host_threads() : 1;
    fprintf(stderr, "[ibwa-amd aln] input parse: %lld reads in %.2f s on %d host threads = %.2f M reads/s (%.3f M per thread)\n",
            (long long)tot_seqs, parse_s, nt, tot_seqs / parse_s / 1e6, tot_seqs / parse_s / 1e6 / nt);
  }
  // Every record is written and every kernel has finished: the process ends here.  Tearing down the
  // contexts, the ingest slots and the pinned buffers one by one only hands back what the driver and
  // the OS reclaim at exit anyway (IBWA_ALN_CLEAN_EXIT=1 does it, for leak checkers).
  if (env_int("IBWA_ALN_CLEAN_EXIT", 0) == 0) {
    if (kTimes)  // the process's own clock at its end: the rest of a timed wall is start-up and exit
      fprintf(stderr, "[ibwa-amd aln] exiting at %.3f s\n",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - g_proc_t0).count());
    fflush(stdout);
    fflush(stderr);
    _exit(have < 0 ? 1 : 0);
  }
  for (int l = n_lanes - 1; l >= 1; --l)  // lanes sharing the index first
    for (auto *x : lctx[l]) ibwa_ctx_destroy(x);
  for (auto *x : ctx) ibwa_ctx_destroy(x);
  return have < 0 ? 1 : 0;
}
