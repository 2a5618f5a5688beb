// index_main.cpp -- `ibwa-amd index`, `fa2pac`, `pac_rev`: the reference's index construction
// (bwa_index, bwtindex.c:42-186) with the suffix sorting on the GPU.
//   fa2pac   bns_fasta2bntseq (bntseq.c:166-254): .pac (2-bit, MSB first, N and every other
//            non-ACGT replaced by lrand48() & 3 from srand48(11)), .ann, .amb, with kseq_read's
//            header semantics (bntseq.c:192: a record without a comment gets "(null)" until a
//            comment buffer exists, and after that the last comment read -- kept);
//   pac_rev  bwa_pac_rev_core (bwtmisc.c:160-185);
//   index    both, then .bwt/.rbwt (bwt_pac2bwt + bwt_bwtupdate_core, i.e. the interleaved
//            layout) and .sa/.rsa (bwt_cal_sa, interval 32) from one ibwa_ctx_build_index call
//            (on-device prefix-doubling suffix sort, bit-identical to `bwa index -a is`).
//            -a is / bwtsw / div all give the same files; -c (color space) is rejected.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "ibwa_aln.h"
#include "readers.h"
#include "sam_common.h"

namespace {

struct Packed {
  std::vector<uint8_t> codes;  // one 2-bit code per byte (the device builder's input)
  int64_t l_pac = 0;
};

// bns_fasta2bntseq (bntseq.c:166-254) + bns_dump (bntseq.c:58-87)
bool fa2pac(const char *fn_fa, const std::string &prefix, Packed &pk) {
  ibwa_sam::init_tables();
  ibwa_cli::SeqReader rd;
  rd.keep_comment = true;
  if (!rd.open(fn_fa)) {
    fprintf(stderr, "[fa2pac] cannot open %s\n", fn_fa);
    return false;
  }
  struct Ann {
    std::string name, anno;
    int64_t offset;
    int32_t len, n_ambs;
  };
  struct Hole {
    int64_t offset;
    int32_t len;
    char amb;
  };
  std::vector<Ann> anns;
  std::vector<Hole> holes;
  ibwa_sam::Lrand48 rnd;
  const uint32_t seed = 11;  // fixed seed for the random generator
  rnd.seed(seed);
  pk.codes.clear();
  int l;
  while ((l = rd.read()) >= 0) {
    Ann a;
    a.name = rd.name;
    a.anno = rd.comment_alloc ? rd.comment : std::string("(null)");
    a.len = l;
    a.offset = anns.empty() ? 0 : anns.back().offset + anns.back().len;
    a.n_ambs = 0;
    int lasts = 0;
    for (int i = 0; i < l; ++i) {
      const unsigned char ch = (unsigned char)rd.seq[i];
      int c = ibwa_sam::nt4[ch];
      if (c >= 4) {
        if (lasts == (int)(signed char)ch) {  // a run of the same ambiguity character
          ++holes.back().len;
        } else {
          holes.push_back({a.offset + i, 1, (char)ch});
          ++a.n_ambs;
        }
        c = (int)(rnd.next() & 3);
      }
      lasts = (int)(signed char)ch;
      pk.codes.push_back((uint8_t)c);
    }
    anns.push_back(a);
    pk.l_pac += (int64_t)rd.seq.size();
  }
  if (pk.l_pac == 0) {
    fprintf(stderr, "[fa2pac] zero length sequence.\n");
    return false;
  }
  // .pac: 4 codes per byte, MSB first; then a 0 byte when l_pac % 4 == 0; then l_pac % 4
  std::vector<uint8_t> pac((size_t)(pk.l_pac + 3) / 4, 0);
  for (int64_t i = 0; i < pk.l_pac; ++i) pac[i >> 2] |= (uint8_t)(pk.codes[i] << ((3 - (i & 3)) << 1));
  if (pk.l_pac % 4 == 0) pac.push_back(0);
  pac.push_back((uint8_t)(pk.l_pac % 4));
  FILE *fp = fopen((prefix + ".pac").c_str(), "wb");
  if (!fp || fwrite(pac.data(), 1, pac.size(), fp) != pac.size()) return false;
  fclose(fp);
  fp = fopen((prefix + ".ann").c_str(), "w");
  if (!fp) return false;
  fprintf(fp, "%lld %d %u\n", (long long)pk.l_pac, (int)anns.size(), seed);
  for (const Ann &a : anns) {
    fprintf(fp, "0 %s", a.name.c_str());
    if (!a.anno.empty()) fprintf(fp, " %s\n", a.anno.c_str());
    else fprintf(fp, "\n");
    fprintf(fp, "%lld %d %d\n", (long long)a.offset, a.len, a.n_ambs);
  }
  fclose(fp);
  fp = fopen((prefix + ".amb").c_str(), "w");
  if (!fp) return false;
  fprintf(fp, "%lld %d %u\n", (long long)pk.l_pac, (int)anns.size(), (unsigned)holes.size());
  for (const Hole &h : holes) fprintf(fp, "%lld %d %c\n", (long long)h.offset, h.len, h.amb);
  fclose(fp);
  return true;
}

// bwa_pac_rev_core (bwtmisc.c:160-185): the reversed text, (l_pac >> 2) + 1 bytes, then l_pac % 4
bool pac_rev(const std::string &fn, const std::string &fn_rev) {
  FILE *fp = fopen(fn.c_str(), "rb");
  if (!fp) return false;
  std::vector<uint8_t> in;
  uint8_t buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof buf, fp)) > 0) in.insert(in.end(), buf, buf + got);
  fclose(fp);
  if (in.empty()) return false;
  const int64_t seq_len = ((int64_t)in.size() - 2) * 4 + in.back();  // bwa_seq_len (bwtmisc.c:43-54)
  const size_t pac_len = (size_t)(seq_len >> 2) + 1;
  std::vector<uint8_t> out(pac_len, 0);
  in.resize(std::max(in.size(), pac_len), 0);
  for (int64_t i = seq_len - 1; i >= 0; --i) {
    const int c = in[i >> 2] >> ((~i & 3) << 1) & 3;
    const uint64_t j = (uint64_t)(seq_len - 1 - i);
    out[j >> 2] |= (uint8_t)(c << ((~j & 3) << 1));
  }
  out.push_back((uint8_t)(seq_len % 4));
  fp = fopen(fn_rev.c_str(), "wb");
  if (!fp || fwrite(out.data(), 1, out.size(), fp) != out.size()) return false;
  fclose(fp);
  return true;
}

int die(const char *what) {
  fprintf(stderr, "[ibwa-amd index] %s: %s\n", what, ibwa_last_error());
  return 1;
}

bool write_words(const std::string &fn, const std::vector<uint32_t> &head, const uint32_t *w, size_t n) {
  FILE *fp = fopen(fn.c_str(), "wb");
  if (!fp) return false;
  bool ok = fwrite(head.data(), 4, head.size(), fp) == head.size() && fwrite(w, 4, n, fp) == n;
  return fclose(fp) == 0 && ok;
}

}  // namespace

int fa2pac_main(int argc, char *argv[]) {
  if (argc < 2) {
    fprintf(stderr, "Usage: ibwa-amd fa2pac <in.fasta> [<out.prefix>]\n");
    return 1;
  }
  Packed pk;
  return fa2pac(argv[1], argc > 2 ? argv[2] : argv[1], pk) ? 0 : 1;
}

int pac_rev_main(int argc, char *argv[]) {
  if (argc < 3) {
    fprintf(stderr, "Usage: ibwa-amd pac_rev <in.pac> <out.pac>\n");
    return 1;
  }
  return pac_rev(argv[1], argv[2]) ? 0 : 1;
}

int index_main(int argc, char *argv[]) {
  std::string prefix;
  int c;
  optind = 1;
  while ((c = getopt(argc, argv, "ca:p:")) >= 0) {  // bwa_index (bwtindex.c:48-60)
    switch (c) {
      case 'a':
        if (strcmp(optarg, "div") && strcmp(optarg, "bwtsw") && strcmp(optarg, "is")) {
          fprintf(stderr, "[bwa_index] unknown algorithm: '%s'.\n", optarg);
          return 1;
        }
        break;  // every algorithm gives the same files; the GPU suffix sort builds them
      case 'p': prefix = optarg; break;
      case 'c':
        fprintf(stderr, "[ibwa-amd index] color-space indexing (-c) is not supported\n");
        return 1;
      default: return 1;
    }
  }
  if (optind + 1 > argc) {
    fprintf(stderr, "Usage: ibwa-amd index [-a bwtsw|div|is] [-p prefix] <in.fasta>\n");
    return 1;
  }
  if (prefix.empty()) prefix = argv[optind];
  Packed pk;
  if (!fa2pac(argv[optind], prefix, pk)) return 1;
  if (!pac_rev(prefix + ".pac", prefix + ".rpac")) {
    fprintf(stderr, "[ibwa-amd index] cannot write %s.rpac\n", prefix.c_str());
    return 1;
  }
  ibwa_ctx_t *ctx = nullptr;
  if (ibwa_ctx_create(0, &ctx)) return die("ibwa_ctx_create");
  ibwa_ctx_set_option(ctx, "exact_jump", 0);  // the CLI only exports the files
  if (ibwa_ctx_build_index(ctx, pk.codes.data(), (uint64_t)pk.l_pac, 32)) return die("build index");
  const char *ext_bwt[2] = {".bwt", ".rbwt"}, *ext_sa[2] = {".sa", ".rsa"};
  for (int s = 0; s < 2; ++s) {
    uint32_t primary = 0, L2[4];
    uint64_t bwt_size = 0;
    if (ibwa_ctx_bwt_info(ctx, s, &primary, L2, &bwt_size)) return die("bwt info");
    std::vector<uint32_t> w(bwt_size);
    if (ibwa_ctx_export_bwt(ctx, s, w.data(), bwt_size)) return die("export bwt");
    // bwt_dump_bwt (bwtio.c:7-15): primary, L2[1..4], the interleaved words
    if (!write_words(prefix + ext_bwt[s], {primary, L2[0], L2[1], L2[2], L2[3]}, w.data(), w.size())) {
      fprintf(stderr, "[ibwa-amd index] cannot write %s%s\n", prefix.c_str(), ext_bwt[s]);
      return 1;
    }
    const uint64_t seq_len = (uint64_t)pk.l_pac, n_sa = (seq_len + 32) / 32;
    std::vector<uint32_t> sa(n_sa);
    if (ibwa_ctx_export_sa(ctx, s, sa.data(), n_sa)) return die("export sa");
    // bwt_dump_sa (bwtio.c:17-27): primary, L2[1..4], sa_intv, seq_len, sa[1..n_sa)
    if (!write_words(prefix + ext_sa[s], {primary, L2[0], L2[1], L2[2], L2[3], 32u, (uint32_t)seq_len}, sa.data() + 1,
                     n_sa - 1)) {
      fprintf(stderr, "[ibwa-amd index] cannot write %s%s\n", prefix.c_str(), ext_sa[s]);
      return 1;
    }
  }
  ibwa_ctx_destroy(ctx);
  return 0;
}
