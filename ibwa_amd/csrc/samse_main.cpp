// samse_main.cpp -- `ibwa-amd samse [-n max_occ] [-f out.sam] [-r RG] <prefix> <in.sai> <in.fq>`:
// the reference's samse (bwa_sai2sam_se, bwase.c:643-740) for one reference database, with
// its two compute steps on the GPU:
//   * SA -> coordinate of every chosen hit and every XA hit (bwa_cal_pac_pos, bwase.c:137-165)
//     is one ibwa_sa2pos launch per batch over the resident (full) suffix array;
//   * the banded global alignments of bwa_refine_gapped (refine_gapped_core, bwase.c:167-241)
//     are one ibwa_global_batch launch per batch.
// Everything else is the reference's host logic in its order: bwa_aln2seq_core (bwase.c:29-104,
// hit choice with the POSIX drand48 stream seeded from .ann, bwase.c:662), the approximate
// mapQ (:111-126), the CIGAR end fix-ups, MD/NM (bwa_cal_md1 :243-295), trimmed-read
// correction (:297-331) and bwa_print_sam1 (:451-581).  Reference quirks are kept: samse
// never sets remapped_pos, so MD/NM are computed at pac position 0 (bwase.c:401) and every
// mapped read carries a ZR tag (bwase.c:556-563).  Color-space input (.sai written with -c)
// needs the .nt index and is rejected.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <memory>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "sam_common.h"

using namespace ibwa_sam;

namespace {

int die(const char *what) {
  fprintf(stderr, "[ibwa-amd samse] %s: %s\n", what, ibwa_last_error());
  return 1;
}

template <class Reader>
int run_samse(Reader &rd, FILE *fp_sa, const ibwa_gap_opt_t &opt, const std::string &prefix, int n_occ, FILE *out,
              const std::string &rg_line, const std::string &rg_id) {
  Phases ph;
  Dbs dbs;  // samse: a set of one reference (dbset_restore, dbset.c:135)
  dbs.db.resize(1);
  Bns &b = dbs.db[0].bns;
  // the host's .ann / .amb / .pac on a thread while the GPU takes the index
  bool b_ok = false;
  std::thread host_side([&]() { b_ok = bns_restore(prefix, b); });
  ibwa_ctx_t *ctx = nullptr;
  int gpu_rc = ibwa_ctx_create(0, &ctx) ? 1 : 0;
  if (!gpu_rc && (ibwa_ctx_load_bwt_file(ctx, 0, (prefix + ".bwt").c_str()) ||
                  ibwa_ctx_load_bwt_file(ctx, 1, (prefix + ".rbwt").c_str())))
    gpu_rc = 2;
  if (!gpu_rc && (ibwa_ctx_load_sa_file(ctx, 0, (prefix + ".sa").c_str()) ||
                  ibwa_ctx_load_sa_file(ctx, 1, (prefix + ".rsa").c_str())))
    gpu_rc = 3;
  if (!gpu_rc && ibwa_ctx_expand_sa(ctx)) gpu_rc = 4;
  host_side.join();
  if (gpu_rc == 1) return die("ibwa_ctx_create");
  if (gpu_rc == 2) return die("load .bwt / .rbwt");
  if (gpu_rc == 3) return die("load .sa / .rsa");
  if (gpu_rc == 4) return die("expand SA");
  if (!b_ok) {
    fprintf(stderr, "[ibwa-amd samse] cannot read %s.ann / .amb / .pac\n", prefix.c_str());
    return 1;
  }
  dbs.l_pac = (uint64_t)b.l_pac;
  Drand48 rnd;
  rnd.seed((long)b.seed);  // srand48(bns->seed), bwase.c:662
  Out o{out, {}};
  for (const Ann &a : b.anns) o.s("@SQ\tSN:").s(a.name).s("\tLN:").i(a.len).c('\n');  // dbset_print_sam_SQ
  if (!rg_line.empty()) o.s(rg_line).c('\n');
  o.s("@PG\tID:bwa\tPN:bwa\tVN:ibwa-amd\n");  // bwa_print_sam_PG (main.cpp:31-34) names this program
  o.flush();
  const char *rgid = rg_id.empty() ? nullptr : rg_id.c_str();
  std::vector<ibwa_aln1_t> aln;
  long tot = 0;
  ph.mark("load index");
  // batches of 0x40000 reads (bwa_read_seq); the next one is parsed while this one is processed --
  // strict FASTQ in bulk on host threads (IBWA_SAMSE_SERIAL_READ=1: the serial reader alone)
  std::unique_ptr<ibwa_cli::FastqBulk> fb;
  if constexpr (std::is_same<Reader, ibwa_cli::SeqReader>::value)
    if (!getenv("IBWA_SAMSE_SERIAL_READ")) fb.reset(new ibwa_cli::FastqBulk(rd));
  auto read_batch = [&](std::vector<Read> &v) {
    v.reserve(0x40000);
    take_reads(fb.get(), opt.mode, opt.trim_qual, v, 0x40000, host_threads(),
               [&](Read &r) { return next_read(rd, opt.mode, opt.trim_qual, r); });
  };
  std::vector<Read> seqs, nxt;
  read_batch(nxt);
  for (;;) {
    seqs.swap(nxt);
    ph.mark("read (wait)");
    if (seqs.empty()) break;
    Background bg;
    bg.start([&] { read_batch(nxt); });
    tot += (long)seqs.size();
    // ---- read alignment (bwase.c:671-682)
    for (Read &p : seqs) {
      int32_t n_aln = 0;
      if (fread(&n_aln, 4, 1, fp_sa) != 1) n_aln = 0;
      aln.resize(std::max(n_aln, 1));
      if (n_aln > 0 && fread(aln.data(), sizeof(ibwa_aln1_t), n_aln, fp_sa) != (size_t)n_aln) {
        fprintf(stderr, "[ibwa-amd samse] truncated .sai\n");
        return 1;
      }
      aln2seq(n_aln, aln.data(), p, n_occ, rnd);
    }
    ph.mark("sai+hit choice");
    // ---- SA -> coordinate (bwa_cal_pac_pos, bwase.c:128-165): one launch for the batch
    std::vector<uint8_t> hs;
    std::vector<uint32_t> hk, hl;
    for (const Read &p : seqs) {
      if (p.type == TYPE_UNIQUE || p.type == TYPE_REPEAT) {
        hs.push_back((uint8_t)p.strand); hk.push_back(p.sa); hl.push_back((uint32_t)p.len);
      }
      for (const Multi &q : p.multi) {
        hs.push_back((uint8_t)q.strand); hk.push_back((uint32_t)q.pos); hl.push_back((uint32_t)p.len);
      }
    }
    std::vector<uint64_t> pos(hk.size());
    if (!hk.empty() && ibwa_sa2pos(ctx, (int64_t)hk.size(), hs.data(), hk.data(), hl.data(), 0, pos.data()))
      return die("sa2pos");
    size_t x = 0;
    for (Read &p : seqs) {
      if (p.type == TYPE_UNIQUE || p.type == TYPE_REPEAT) {
        p.pos = pos[x++];
        const int max_diff = opt.fnr > 0.0 ? ibwa_cal_maxdiff(p.len, 0.02, opt.fnr) : opt.max_diff;
        p.seQ = p.mapQ = approx_mapQ(p, max_diff) & 0xff;
      }
      for (Multi &q : p.multi) q.pos = pos[x++];
    }
    ph.mark("sa2pos");
    // ---- bwa_refine_gapped (bwase.c:333-416): one global-alignment launch, MD/NM, trimmed reads
    std::vector<Read *> rp;
    for (Read &p : seqs) rp.push_back(&p);
    if (int rc = refine_gapped(ctx, dbs, rp)) return rc == 1 ? 1 : die("global alignment");
    ph.mark("refine+md");
    // ---- print
    print_parallel(o, (int64_t)seqs.size(),
                   [&](Out &ob, int64_t i) { print_sam1(ob, dbs, seqs[i], nullptr, opt.mode, opt.max_top2, rgid); });
    ph.mark("print");
    fprintf(stderr, "[bwa_aln_core] %ld sequences have been processed.\n", tot);
  }
  ph.print("ibwa-amd samse");
  ibwa_ctx_destroy(ctx);
  return 0;
}

}  // namespace

int samse_main(int argc, char *argv[]) {
  init_tables();
  int c, n_occ = 3;
  const char *fn_out = nullptr;
  std::string rg_line, rg_id;
  optind = 1;
  while ((c = getopt(argc, argv, "hn:f:r:")) >= 0) {  // bwa_sai2sam_se (bwase.c:710-740)
    switch (c) {
      case 'h': break;
      case 'r':
        if (!set_rg(optarg, rg_line, rg_id)) {
          fprintf(stderr, "[bwa_sai2sam_se] malformated @RG line\n");
          return 1;
        }
        break;
      case 'n': n_occ = atoi(optarg); break;
      case 'f': fn_out = optarg; break;
      default: return 1;
    }
  }
  if (optind + 3 > argc) {
    fprintf(stderr, "Usage: ibwa-amd samse [-n max_occ] [-f out.sam] [-r RG] <prefix> <in.sai> <in.fq>\n");
    return 1;
  }
  const std::string prefix = argv[optind];
  FILE *fp_sa = fopen(argv[optind + 1], "rb");
  if (!fp_sa) {
    fprintf(stderr, "[ibwa-amd samse] cannot open %s\n", argv[optind + 1]);
    return 1;
  }
  ibwa_gap_opt_t opt;
  if (fread(&opt, sizeof opt, 1, fp_sa) != 1) {
    fprintf(stderr, "[ibwa-amd samse] %s: no .sai header\n", argv[optind + 1]);
    return 1;
  }
  if (!(opt.mode & IBWA_MODE_COMPREAD)) {
    fprintf(stderr, "[ibwa-amd samse] color-space alignments (aln -c) need the .nt index: not supported\n");
    return 1;
  }
  FILE *out = fn_out ? fopen(fn_out, "w") : stdout;
  if (!out) {
    fprintf(stderr, "[ibwa-amd samse] cannot write %s\n", fn_out);
    return 1;
  }
  int rc;
  if (opt.mode & IBWA_MODE_BAM) {  // bwa_open_reads (bwtaln.c:159-171)
    int which = 0;
    if (opt.mode & IBWA_MODE_BAM_SE) which |= 4;
    if (opt.mode & IBWA_MODE_BAM_READ1) which |= 1;
    if (opt.mode & IBWA_MODE_BAM_READ2) which |= 2;
    if (which == 0) which = 7;
    ibwa_cli::BamReader rd;
    if (!rd.open(argv[optind + 2], which)) return 1;
    rc = run_samse(rd, fp_sa, opt, prefix, n_occ, out, rg_line, rg_id);
  } else {
    ibwa_cli::SeqReader rd;
    if (!rd.open(argv[optind + 2])) {
      fprintf(stderr, "[ibwa-amd samse] cannot open %s\n", argv[optind + 2]);
      return 1;
    }
    rc = run_samse(rd, fp_sa, opt, prefix, n_occ, out, rg_line, rg_id);
  }
  fclose(fp_sa);
  if (out != stdout) fclose(out);
  return rc;
}
