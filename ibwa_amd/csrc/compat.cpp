// compat.cpp -- bwa_cal_sa_reg_gap in the reference's own types (include/ibwa_bwa_compat.h).
//
// Replaces the per-thread body of bwtaln.c:80-140 and the pthread fan-out
// around it (bwtaln.c:199-218): the batch is flattened once, split into
// contiguous slices, one per GPU (each keeping the batch-level max length,
// bwtaln.c:89-93), and every slice runs on its own engine from a host thread.
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "ibwa_aln.h"
#include "ibwa_bwa_compat.h"

namespace {

std::mutex g_mu;
std::vector<ibwa_ctx_t *> g_ctx;

[[noreturn]] void die(const char *what, int rc) {
  fprintf(stderr, "[ibwa_amd] %s failed (%d): %s\n", what, rc, ibwa_last_error());
  abort();
}

void destroy_locked() {
  for (ibwa_ctx_t *c : g_ctx) ibwa_ctx_destroy(c);
  g_ctx.clear();
}

int init_locked(ibwa_ref_bwt_t *const bwt[2], int n_gpus) {
  destroy_locked();
  int n_dev = 0;
  if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev <= 0) n_dev = 0;
  if (n_gpus <= 0 || n_gpus > n_dev) n_gpus = n_dev;
  if (n_gpus <= 0) return IBWA_EHIP;
  for (int g = 0; g < n_gpus; ++g) {
    ibwa_ctx_t *c = nullptr;
    if (int rc = ibwa_ctx_create(g, &c)) {
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
  return init_locked(bwt, n_gpus);
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
    if (int rc = init_locked(bwt, 1)) die("ibwa_gpu_init", rc);
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
  const int n_gpu = (int)std::min<int64_t>((int64_t)g_ctx.size(), (n + 1023) / 1024);
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

}  // extern "C"
