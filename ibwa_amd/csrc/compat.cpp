// compat.cpp -- bwa_cal_sa_reg_gap in the reference's own types (include/ibwa_bwa_compat.h).
//
// Replaces the per-thread body of bwtaln.c:80-140 and the pthread fan-out
// around it (bwtaln.c:199-218): the batch is flattened once, split into
// contiguous slices, one per GPU (each keeping the batch-level max length,
// bwtaln.c:89-93), and every slice runs on its own engine from a host thread.  Several
// slices may share a GPU (ibwa_gpu_init_ex): they run concurrently on their own streams.
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "ibwa_aln.h"
#include "ibwa_bwa_compat.h"

namespace {

std::mutex g_mu;
std::vector<ibwa_ctx_t *> g_ctx;  // one engine per slice: slices_per_gpu on each GPU, GPU-major
int g_min_slice = 1024;          // fewest reads per slice (the reference's THREAD_BLOCK_SIZE, bwtaln.c:16)

[[noreturn]] void die(const char *what, int rc) {
  fprintf(stderr, "[ibwa_amd] %s failed (%d): %s\n", what, rc, ibwa_last_error());
  abort();
}

void destroy_locked() {
  for (ibwa_ctx_t *c : g_ctx) ibwa_ctx_destroy(c);
  g_ctx.clear();
}

int init_locked(ibwa_ref_bwt_t *const bwt[2], int n_gpus, int slices_per_gpu, int min_slice) {
  destroy_locked();
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev <= 0) n_dev = 0;
  if (n_gpus <= 0 || n_gpus > n_dev) n_gpus = n_dev;
  if (n_gpus <= 0) return IBWA_EHIP;
  if (slices_per_gpu < 1) slices_per_gpu = 1;
  g_min_slice = min_slice > 0 ? min_slice : 1024;
  for (int g = 0; g < n_gpus * slices_per_gpu; ++g) {
    ibwa_ctx_t *c = nullptr;
    if (int rc = ibwa_ctx_create(g / slices_per_gpu, &c)) {
      destroy_locked();
      return rc;
    }
    g_ctx.push_back(c);
    int rc = 0;
    if (g == 0) {
      for (int s = 0; s < 2 && !rc; ++s)
        rc = ibwa_ctx_load_bwt(c, s, bwt[s]->primary, bwt[s]->L2 + 1, bwt[s]->bwt, bwt[s]->bwt_size);
    } else {
      rc = ibwa_ctx_clone_index(c, g_ctx[0]);
    }
    if (rc) {
      destroy_locked();
      return rc;
    }
  }
  return 0;
}

}  // namespace

extern "C" {

int ibwa_gpu_init(ibwa_ref_bwt_t *const bwt[2], int n_gpus) {
  std::lock_guard<std::mutex> lk(g_mu);
  return init_locked(bwt, n_gpus, 1, 1024);
}

int ibwa_gpu_init_ex(ibwa_ref_bwt_t *const bwt[2], int n_gpus, int slices_per_gpu, int min_reads_per_slice) {
  std::lock_guard<std::mutex> lk(g_mu);
  return init_locked(bwt, n_gpus, slices_per_gpu, min_reads_per_slice);
}

void ibwa_gpu_destroy(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  destroy_locked();
}

void bwa_cal_sa_reg_gap(int tid, ibwa_ref_bwt_t *const bwt[2], int n_seqs, ibwa_ref_seq_t *seqs,
                        const ibwa_gap_opt_t *opt) {
  (void)tid;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_ctx.empty())
    if (int rc = init_locked(bwt, 1, 1, 1024)) die("ibwa_gpu_init", rc);
  // reads already processed by a concurrent caller (seq freed) are skipped, so the
  // reference's n_threads > 1 fan-out degenerates to one GPU pass per batch
  std::vector<int> ids;
  ids.reserve(n_seqs > 0 ? n_seqs : 0);
  int max_len = 0;
  for (int i = 0; i < n_seqs; ++i) {
    if (!seqs[i].seq) continue;
    ids.push_back(i);
    max_len = std::max<int>(max_len, (int)seqs[i].len);
  }
  const int64_t n = (int64_t)ids.size();
  if (n == 0) return;
  const int n_gpu = (int)std::min<int64_t>((int64_t)g_ctx.size(), (n + g_min_slice - 1) / g_min_slice);
  const int64_t per = (n + n_gpu - 1) / n_gpu;
  std::vector<int32_t> n_aln(n);
  std::vector<ibwa_aln1_t *> alns(n_gpu, nullptr);
  std::vector<int> rcs(n_gpu, 0);
  auto run = [&](int g) {
    const int64_t b0 = g * per, b1 = std::min<int64_t>(n, b0 + per);
    std::vector<uint64_t> off(b1 - b0);
    std::vector<uint32_t> len(b1 - b0);
    uint64_t tot = 0;
    for (int64_t j = b0; j < b1; ++j) {
      off[j - b0] = tot;
      len[j - b0] = seqs[ids[j]].len;
      tot += len[j - b0];
    }
    std::vector<uint8_t> seq(tot + 1);
    for (int64_t j = b0; j < b1; ++j) memcpy(seq.data() + off[j - b0], seqs[ids[j]].seq, len[j - b0]);
    int64_t n_tot = 0;
    rcs[g] = ibwa_aln_batch(g_ctx[g], opt, b1 - b0, seq.data(), off.data(), len.data(), max_len,
                            n_aln.data() + b0, &alns[g], &n_tot);
  };
  if (n_gpu == 1) {
    run(0);
  } else {
    std::vector<std::thread> th;
    for (int g = 0; g < n_gpu; ++g) th.emplace_back(run, g);
    for (auto &t : th) t.join();
  }
  for (int g = 0; g < n_gpu; ++g)
    if (rcs[g]) die("bwa_cal_sa_reg_gap", rcs[g]);
  // scatter: bwtaln.c:114 resets, :132 result, :134-135 frees
  for (int g = 0; g < n_gpu; ++g) {
    const int64_t b0 = g * per, b1 = std::min<int64_t>(n, b0 + per);
    const ibwa_aln1_t *src = alns[g];
    for (int64_t j = b0; j < b1; ++j) {
      ibwa_ref_seq_t *p = seqs + ids[j];
      const int na = n_aln[j];
      // the reference's array always has >= 4 zeroed slots (bwtgap.c:113-114); the caller free()s it
      p->aln = (ibwa_aln1_t *)calloc(std::max(na, 4), sizeof(ibwa_aln1_t));
      if (!p->aln) die("calloc", IBWA_EHIP);
      if (na) memcpy(p->aln, src, (size_t)na * sizeof(ibwa_aln1_t));
      src += na;
      p->n_aln = na;
      p->sa = 0;
      p->type = IBWA_TYPE_NO_MATCH;
      p->c1 = p->c2 = 0;
      free(p->name);
      free(p->seq);
      free(p->rseq);
      free(p->qual);
      p->name = nullptr;
      p->seq = p->rseq = nullptr;
      p->qual = nullptr;
    }
    ibwa_free(alns[g]);
  }
}

/*
 * bwa_sw_core (bwasw.c:29-112) for a batch of mate rescues: the host checks and
 * post-processing of the reference around one batched aln_local_core launch.
 */
int ibwa_sw_core_batch(ibwa_ctx_t *ctx, int64_t n, const uint8_t *seq, const uint64_t *off, const uint32_t *len,
                       const uint8_t *ref, const uint64_t *ref_off, const uint32_t *ref_len, const int32_t *reglen,
                       int64_t *beg, int64_t l_pac, int32_t *n_cigar, uint32_t *cnt, uint32_t **cigar) {
  *cigar = nullptr;
  std::vector<int64_t> idx;  // pairs that pass the pre-checks (bwasw.c:40-43)
  for (int64_t p = 0; p < n; ++p) {
    n_cigar[p] = 0;
    cnt[p] = 0;
    const int L = (int)len[p];
    if (reglen[p] < 20 || l_pac - beg[p] < L) continue;
    int x = 0;
    for (int k = 0; k < L; ++k) x += seq[off[p] + k] >= 4;
    if (L == 0 || (float)x / L >= 0.25f || L - x < 20) continue;
    idx.push_back(p);
  }
  const int64_t m = (int64_t)idx.size();
  std::vector<uint64_t> o1(m), o2(m);
  std::vector<uint32_t> l1(m), l2(m);
  for (int64_t q = 0; q < m; ++q) {
    o1[q] = ref_off[idx[q]]; l1[q] = ref_len[idx[q]];
    o2[q] = off[idx[q]]; l2[q] = len[idx[q]];
  }
  std::vector<int32_t> score(m), plen(m), ends(4 * m), ncig(m);
  uint32_t *c32 = nullptr;
  int64_t tot = 0;
  if (int rc = ibwa_sw_batch(ctx, m, ref, o1.data(), l1.data(), seq, o2.data(), l2.data(), score.data(), plen.data(),
                             ends.data(), ncig.data(), &c32, &tot))
    return rc;
  std::vector<uint32_t> out;
  std::vector<std::vector<uint32_t>> per(n);
  int64_t q32 = 0;
  for (int64_t q = 0; q < m; ++q) {
    const int64_t p = idx[q];
    const uint32_t *cg = c32 + q32;
    q32 += ncig[q];
    if (score[q] < 0 || ncig[q] == 0) continue;  // ret < 0 (bwasw.c:52-55), or no path
    // aln_path2cigar32 -> bwa_cigar_t op << 29 | len (bwtaln.c:332-342)
    std::vector<uint32_t> c;
    uint32_t x = 0, y = 0;
    for (int k = 0; k < ncig[q]; ++k) {
      const uint32_t op = cg[k] & 0xf, ln = cg[k] >> 4;
      c.push_back(op << 29 | ln);
      if (op == 0) { x += ln; y += ln; } else if (op == 2) x += ln; else y += ln;
    }
    if (x < 20 || y < 20) continue;  // bwasw.c:59-69
    const int si = ends[4 * q], sj = ends[4 * q + 1], ej = ends[4 * q + 3];
    const int L = (int)len[p];
    beg[p] += (si ? si : 1) - 1;
    const int start = (sj ? sj : 1) - 1;
    if (start) c.insert(c.begin(), 3u << 29 | (uint32_t)start);  // soft clips (bwasw.c:71-87)
    if (ej < L) c.push_back(3u << 29 | (uint32_t)(L - ej));
    // mismatches and gaps (bwasw.c:89-108)
    int n_mm = 0, n_gapo = 0, n_gape = 0;
    uint32_t rx = si ? si - 1 : 0, ry = sj ? sj - 1 : 0;
    const uint8_t *rs = ref + ref_off[p], *ss = seq + off[p];
    for (uint32_t v : c) {
      const uint32_t op = v >> 29, ln = v & 0x1fffffffu;
      if (op == 0) {
        for (uint32_t l = 0; l < ln; ++l)
          if (rs[rx + l] < 4 && ss[ry + l] < 4 && rs[rx + l] != ss[ry + l]) ++n_mm;
        rx += ln; ry += ln;
      } else if (op == 2) {
        rx += ln; ++n_gapo; n_gape += (int)ln - 1;
      } else if (op == 1) {
        ry += ln; ++n_gapo; n_gape += (int)ln - 1;
      }
    }
    cnt[p] = (uint32_t)n_mm << 16 | (uint32_t)n_gapo << 8 | (uint32_t)n_gape;
    n_cigar[p] = (int32_t)c.size();
    per[p].swap(c);
  }
  ibwa_free(c32);
  for (int64_t p = 0; p < n; ++p) out.insert(out.end(), per[p].begin(), per[p].end());
  *cigar = (uint32_t *)malloc(std::max<size_t>(out.size(), 1) * 4);
  if (!*cigar) return IBWA_EINVAL;
  if (!out.empty()) memcpy(*cigar, out.data(), out.size() * 4);
  return 0;
}

namespace {
// seq_reverse (bwaseqio.c:55-72) into a copy
void rev_copy(const uint8_t *src, int len, bool comp, uint8_t *dst) {
  for (int i = 0; i < len; ++i) {
    const uint8_t c = src[len - 1 - i];
    dst[i] = comp && c < 4 ? 3 - c : c;
  }
}
}  // namespace

namespace {
// the packed references of a dbset, concatenated at their offsets (dbset_extract_sequence,
// dbset.c:306-325): base x is in the last segment starting at or before x
struct PacSeg {
  const uint8_t *pac;
  uint64_t offset, l_pac;
};
int host_threads_c() {  // as ibwa_sam::host_threads
  const char *e = getenv("OMP_NUM_THREADS");
  int n = e ? atoi(e) : (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 32));
}

struct PacSet {
  std::vector<PacSeg> seg;
  uint64_t l_pac = 0;
  // bases [x, x + n) as 2-bit codes: unpacked from one reference's .pac when the window lies in it
  void extract(uint64_t x, uint32_t n, uint8_t *out) const {
    size_t j = seg.size() - 1;
    while (j > 0 && seg[j].offset > x) --j;
    const uint64_t p0 = x - seg[j].offset;
    if (p0 + n > seg[j].l_pac) {  // crosses into a hole or the next reference: base by base
      for (uint32_t t = 0; t < n; ++t) out[t] = at(x + t);
      return;
    }
    const uint8_t *pac = seg[j].pac;
    for (uint32_t t = 0; t < n; ++t) {
      const uint64_t p = p0 + t;
      out[t] = (pac[p >> 2] >> ((~p & 3) << 1)) & 3;  // bns_pac (bntseq.h)
    }
  }
  uint8_t at(uint64_t x) const {
    size_t j = seg.size() - 1;
    while (j > 0 && seg[j].offset > x) --j;
    const uint64_t p = x - seg[j].offset;
    if (p >= seg[j].l_pac) return 0;  // a hole between references (the reference stops there)
    return (seg[j].pac[p >> 2] >> ((~p & 3) << 1)) & 3;  // bns_pac (bntseq.h)
  }
};

int paired_sw_core(ibwa_ctx_t *ctx, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                   const ibwa_ref_isize_info_t *ii, const PacSet &ps, uint64_t n_tot[2], uint64_t n_mapped[2]);
}  // namespace

int ibwa_paired_sw(ibwa_ctx_t *ctx, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                   const ibwa_ref_isize_info_t *ii, const uint8_t *pac, uint64_t l_pac, uint64_t n_tot[2],
                   uint64_t n_mapped[2]) {
  PacSet ps;
  ps.seg.push_back({pac, 0, l_pac});
  ps.l_pac = l_pac;
  return paired_sw_core(ctx, n_seqs, seqs, popt, ii, ps, n_tot, n_mapped);
}

int ibwa_paired_sw_dbs(ibwa_ctx_t *ctx, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                       const ibwa_ref_isize_info_t *ii, int n_db, const uint8_t *const *pac, const uint64_t *offset,
                       const uint64_t *l_pac, uint64_t n_tot[2], uint64_t n_mapped[2]) {
  PacSet ps;
  for (int i = 0; i < n_db; ++i) {
    ps.seg.push_back({pac[i], offset[i], l_pac[i]});
    ps.l_pac = std::max<uint64_t>(ps.l_pac, offset[i] + l_pac[i]);
  }
  if (ps.seg.empty()) return IBWA_EINVAL;
  return paired_sw_core(ctx, n_seqs, seqs, popt, ii, ps, n_tot, n_mapped);
}

void bwa_paired_sw(ibwa_ref_dbset_t *dbs, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                   const ibwa_ref_isize_info_t *ii) {
  uint64_t n_tot[2] = {0, 0}, n_mapped[2] = {0, 0};
  if (popt->is_sw && ii->avg >= 0.0) {  // bwasw.c:279
    // dbset_load_pac (dbset.c:199-207) without touching the caller's seq_t
    PacSet ps;
    std::vector<std::vector<uint8_t>> own(dbs->count);
    for (int i = 0; i < dbs->count; ++i) {
      const ibwa_ref_seqt_t *sq = dbs->bns[i];
      const uint64_t lp = (uint64_t)sq->bns->l_pac;
      const uint8_t *data = sq->data;
      if (!data) {  // seq_load_pac (dbset.c:103-108)
        own[i].assign(lp / 4 + 1, 0);
        rewind(sq->bns->fp_pac);
        if (fread(own[i].data(), 1, own[i].size(), sq->bns->fp_pac) == 0 && lp) die("reading the .pac", IBWA_EIO);
        data = own[i].data();
      }
      ps.seg.push_back({data, dbs->db[i]->offset, lp});
    }
    ps.l_pac = dbs->l_pac;
    std::lock_guard<std::mutex> lk(g_mu);
    ibwa_ctx_t *ctx = g_ctx.empty() ? nullptr : g_ctx[0];
    ibwa_ctx_t *own_ctx = nullptr;
    if (!ctx) {
      if (int rc = ibwa_ctx_create(0, &own_ctx)) die("ibwa_ctx_create", rc);
      ctx = own_ctx;
    }
    const int rc = paired_sw_core(ctx, n_seqs, seqs, popt, ii, ps, n_tot, n_mapped);
    if (own_ctx) ibwa_ctx_destroy(own_ctx);
    if (rc) die("bwa_paired_sw", rc);
    // bwasw.c:296-299
    fprintf(stderr, "[bwa_paired_sw] %lld out of %lld Q%d singletons are mated.\n", (long long)n_mapped[1],
            (long long)n_tot[1], 17);
    fprintf(stderr, "[bwa_paired_sw] %lld out of %lld Q%d discordant pairs are fixed.\n", (long long)n_mapped[0],
            (long long)n_tot[0], 17);
  }
}

}  // extern "C"

namespace {
int paired_sw_core(ibwa_ctx_t *ctx, int n_seqs, ibwa_ref_seq_t *seqs[2], const ibwa_ref_pe_opt_t *popt,
                   const ibwa_ref_isize_info_t *ii, const PacSet &ps, uint64_t n_tot[2], uint64_t n_mapped[2]) {
  const uint64_t l_pac = ps.l_pac;
  n_tot[0] = n_tot[1] = n_mapped[0] = n_mapped[1] = 0;
  if (!popt->is_sw || ii->avg < 0.0) return 0;  // bwasw.c:279
  const bool std_pe = popt->type == IBWA_PET_STD;
  static const bool stats = getenv("IBWA_SAMPE_STATS") != nullptr;
  const auto c0 = std::chrono::steady_clock::now();
  // ---- pass 1: eligible pairs, candidate windows (bwasw.c:157-219), in contiguous pair ranges on
  // the host threads, then concatenated in pair order
  struct Cand {
    int pair, k;
  };
  struct Part {
    std::vector<Cand> cand;
    std::vector<uint8_t> qbuf, rbuf;
    std::vector<uint64_t> qoff, roff;
    std::vector<uint32_t> qlen, rlen;
    std::vector<int32_t> reglen;
    std::vector<int64_t> beg;
    uint64_t n_tot[2] = {0, 0};
  };
  std::vector<int8_t> single(std::max(n_seqs, 0), -1);
  const int nt = std::max(1, std::min<int>(host_threads_c(), n_seqs / 1024 + 1));
  std::vector<Part> part(nt);
  auto scan = [&](int t) {
    Part &P = part[t];
    const int i0 = (int)((int64_t)n_seqs * t / nt), i1 = (int)((int64_t)n_seqs * (t + 1) / nt);
    for (int i = i0; i < i1; ++i) {
      ibwa_ref_seq_t *p[2] = {seqs[0] + i, seqs[1] + i};
      if (!((p[0]->mapQ >= 17 || p[1]->mapQ >= 17) && (p[0]->extra_flag & IBWA_SAM_FPP) == 0)) continue;
      single[i] = (p[0]->type == IBWA_TYPE_NO_MATCH || p[1]->type == IBWA_TYPE_NO_MATCH) ? 1 : 0;
      ++P.n_tot[single[i]];
      if (popt->type != IBWA_PET_STD && popt->type != IBWA_PET_SOLID) continue;
      for (int k = 0; k < 2; ++k) {
        const ibwa_ref_seq_t *ref = p[1 - k], *mate = p[k];
        if (ref->type == IBWA_TYPE_NO_MATCH) continue;
        const int L = (int)mate->len;
        int64_t b, e;
        // set_right_coordinate / set_left_coordinate (bwasw.c:114-143), in the reference's double arithmetic
        auto right = [&]() {
          b = (int64_t)((int64_t)ref->remapped_pos + ii->avg - 3 * ii->std - mate->len * 1.5);
          e = (int64_t)(b + 6 * ii->std + 2 * mate->len);
          if (b < (int64_t)ref->remapped_pos + (int64_t)ref->len) b = ref->remapped_pos + ref->len;
          if (e > (int64_t)l_pac) e = (int64_t)l_pac;
        };
        auto left = [&]() {
          b = (int64_t)((int64_t)ref->remapped_pos + ref->len - ii->avg - 3 * ii->std - mate->len * 0.5);
          e = (int64_t)(b + 6 * ii->std + 2 * mate->len);
          if (b < 0) b = 0;
          if (e > (int64_t)ref->remapped_pos) e = (int64_t)ref->remapped_pos;
        };
        // the read as bwa_sw_core sees it: a copy (the reference reverses p[k]->seq in place and back)
        const size_t q0 = P.qbuf.size();
        P.qbuf.resize(q0 + L);
        uint8_t *q = P.qbuf.data() + q0;
        if (std_pe) {
          if (ref->strand == 0) { right(); memcpy(q, mate->rseq, L); }
          else { left(); rev_copy(mate->seq, L, false, q); }
        } else {
          if (ref->strand == 0) { if (k == 0) left(); else right(); rev_copy(mate->rseq, L, false, q); }
          else { if (k == 0) right(); else left(); memcpy(q, mate->seq, L); }
        }
        const int rl = (int)(e - b);
        // dbset_extract_sequence (dbset.c:306-325), only for windows bwa_sw_core would extract (bwasw.c:40)
        const size_t r0 = P.rbuf.size();
        uint32_t got = 0;
        if (rl >= 20 && b >= 0 && (uint64_t)b < l_pac) {
          got = (uint32_t)std::min<uint64_t>((uint64_t)rl, l_pac - (uint64_t)b);
          P.rbuf.resize(r0 + got);
          ps.extract((uint64_t)b, got, P.rbuf.data() + r0);
        }
        P.cand.push_back({i, k});
        P.qoff.push_back(q0); P.qlen.push_back((uint32_t)L);
        P.roff.push_back(r0); P.rlen.push_back(got);
        P.reglen.push_back(rl);
        P.beg.push_back(b);
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(scan, t);
    scan(0);
    for (auto &x : th) x.join();
  }
  std::vector<Cand> cand;
  std::vector<uint8_t> qbuf, rbuf;
  std::vector<uint64_t> qoff, roff;
  std::vector<uint32_t> qlen, rlen;
  std::vector<int32_t> reglen;
  std::vector<int64_t> beg;
  {
    size_t nc = 0, nq = 0, nr = 0;
    for (const Part &P : part) { nc += P.cand.size(); nq += P.qbuf.size(); nr += P.rbuf.size(); }
    cand.reserve(nc); qoff.reserve(nc); roff.reserve(nc); qlen.reserve(nc); rlen.reserve(nc);
    reglen.reserve(nc); beg.reserve(nc);
    qbuf.reserve(nq + 1); rbuf.reserve(nr + 1);
    for (Part &P : part) {
      const uint64_t qb = qbuf.size(), rb = rbuf.size();
      cand.insert(cand.end(), P.cand.begin(), P.cand.end());
      for (uint64_t x : P.qoff) qoff.push_back(qb + x);
      for (uint64_t x : P.roff) roff.push_back(rb + x);
      qlen.insert(qlen.end(), P.qlen.begin(), P.qlen.end());
      rlen.insert(rlen.end(), P.rlen.begin(), P.rlen.end());
      reglen.insert(reglen.end(), P.reglen.begin(), P.reglen.end());
      beg.insert(beg.end(), P.beg.begin(), P.beg.end());
      qbuf.insert(qbuf.end(), P.qbuf.begin(), P.qbuf.end());
      rbuf.insert(rbuf.end(), P.rbuf.begin(), P.rbuf.end());
      n_tot[0] += P.n_tot[0];
      n_tot[1] += P.n_tot[1];
      P = Part();
    }
  }
  // ---- pass 2: every bwa_sw_core of the batch in one launch
  const int64_t m = (int64_t)cand.size();
  const auto c1 = std::chrono::steady_clock::now();
  std::vector<int32_t> ncig(m);
  std::vector<uint32_t> cnt(m);
  uint32_t *cig = nullptr;
  qbuf.push_back(0);
  rbuf.push_back(0);
  if (m) {
    if (int rc = ibwa_sw_core_batch(ctx, m, qbuf.data(), qoff.data(), qlen.data(), rbuf.data(), roff.data(), rlen.data(),
                                    reglen.data(), beg.data(), (int64_t)l_pac, ncig.data(), cnt.data(), &cig))
      return rc;
  }
  const auto c2 = std::chrono::steady_clock::now();
  // ---- pass 3: acceptance and fix-up in pair order (bwasw.c:220-265)
  std::vector<uint64_t> cfirst(m);
  for (int64_t j = 0, acc = 0; j < m; ++j) { cfirst[j] = acc; acc += ncig[j]; }
  const double prior_term = -4.343 * log(ii->ap_prior / l_pac);
  const int new_term = (int)(-4.343 * log(.5 * erfc(M_SQRT1_2 * 1.5) + .499));
  // each pair's fix-up reads and writes only its own two reads: contiguous pair ranges on the host
  // threads, the counts summed after
  std::vector<uint64_t> nmap(2 * (size_t)nt, 0);
  std::atomic<int> oom{0};
  auto fix = [&](int t) {
    const int i0 = (int)((int64_t)n_seqs * t / nt), i1 = (int)((int64_t)n_seqs * (t + 1) / nt);
    int64_t j = std::lower_bound(cand.begin(), cand.end(), i0, [](const Cand &c, int v) { return c.pair < v; }) - cand.begin();
    for (int i = i0; i < i1; ++i) {
      if (single[i] < 0) continue;
      ibwa_ref_seq_t *p[2] = {seqs[0] + i, seqs[1] + i};
      const uint32_t *cg[2] = {nullptr, nullptr};
      int nc[2] = {0, 0}, mq_adjust[2] = {255, 255};
      int64_t bg[2] = {0, 0};
      uint32_t ct[2] = {0, 0};
      for (; j < m && cand[j].pair == i; ++j) {
        const int k = cand[j].k;
        bg[k] = beg[j];
        if (!ncig[j]) continue;
        cg[k] = cig + cfirst[j];
        nc[k] = ncig[j];
        ct[k] = cnt[j];
        if (p[k]->type != IBWA_TYPE_NO_MATCH) {  // re-evaluate (bwasw.c:222-236)
          int clip = 0;
          if ((cg[k][0] >> 29) == 3) clip += cg[k][0] & 0x1fffffff;
          if ((cg[k][nc[k] - 1] >> 29) == 3) clip += cg[k][nc[k] - 1] & 0x1fffffff;
          int s_old = (int)((p[k]->n_mm * 9 + p[k]->n_gapo * 13 + p[k]->n_gape * 2) / 3. * 8. + .499);
          int s_new = (int)(((ct[k] >> 16) * 9 + (ct[k] >> 8 & 0xff) * 13 + (ct[k] & 0xff) * 2 + clip * 3) / 3. * 8. + .499);
          s_old += prior_term;
          s_new += new_term;
          if (s_old < s_new) {
            mq_adjust[k] = s_new - s_old;
            cg[k] = nullptr;
            nc[k] = 0;
          } else {
            mq_adjust[k] = s_old - s_new;
          }
        }
      }
      int k = -1, mapQ = 0;
      if (cg[0] && cg[1]) {
        k = p[0]->mapQ < p[1]->mapQ ? 0 : 1;
        mapQ = abs((int)p[1]->mapQ - (int)p[0]->mapQ);
      } else if (cg[0]) {
        k = 0, mapQ = p[1]->mapQ;
      } else if (cg[1]) {
        k = 1, mapQ = p[0]->mapQ;
      }
      if (k < 0 || p[k]->pos == (uint64_t)bg[k]) continue;
      ++nmap[2 * (size_t)t + (size_t)single[i]];
      ibwa_ref_seq_t *fx = p[k], *rf = p[1 - k];
      int tmp = (int)rf->mapQ - fx->mapQ / 2 - 8;
      if (tmp <= 0) tmp = 1;
      if (mapQ > tmp) mapQ = tmp;
      fx->mapQ = rf->mapQ = mapQ;
      fx->seQ = rf->seQ = rf->seQ < (uint64_t)mapQ ? rf->seQ : (uint64_t)mapQ;
      if ((int)fx->mapQ > mq_adjust[k]) fx->mapQ = mq_adjust[k];
      if ((int)fx->seQ > mq_adjust[k]) fx->seQ = mq_adjust[k];
      free(fx->cigar);
      fx->cigar = (uint32_t *)malloc(sizeof(uint32_t) * nc[k]);
      if (!fx->cigar) { oom = 1; return; }
      memcpy(fx->cigar, cg[k], sizeof(uint32_t) * nc[k]);
      fx->n_cigar = nc[k];
      // __set_fixed (bwasw.c:167-178)
      fx->type = IBWA_TYPE_MATESW;
      fx->pos = fx->remapped_pos = (uint64_t)bg[k];
      fx->dbidx = fx->remapped_dbidx = 0;
      fx->seQ = rf->seQ;
      fx->strand = std_pe ? 1 - rf->strand : rf->strand;
      fx->n_mm = ct[k] >> 16;
      fx->n_gapo = ct[k] >> 8 & 0xff;
      fx->n_gape = ct[k] & 0xff;
      fx->extra_flag |= IBWA_SAM_FPP;
      rf->extra_flag |= IBWA_SAM_FPP;
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fix, t);
    fix(0);
    for (auto &x : th) x.join();
  }
  for (int t = 0; t < nt; ++t) {
    n_mapped[0] += nmap[2 * (size_t)t];
    n_mapped[1] += nmap[2 * (size_t)t + 1];
  }
  ibwa_free(cig);
  if (oom) return IBWA_EHIP;
  if (stats) {
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    fprintf(stderr, "[ibwa-amd paired_sw] %d pairs, %lld rescues: windows %.1f, SW %.1f, fix-up %.1f ms\n", n_seqs,
            (long long)m, ms(c0, c1), ms(c1, c2), ms(c2, std::chrono::steady_clock::now()));
  }
  return 0;
}

}  // namespace
