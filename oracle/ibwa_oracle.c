/*
 * ibwa_oracle.c -- TEST INFRASTRUCTURE ONLY (checker + CPU baseline).
 *
 * A plain-C restatement of the reference aln hot path.  Each function names
 * the reference lines it follows.  It is pinned against the golden .sai /
 * Occ fixtures produced by the compiled reference (tests/golden/), and it is
 * the `cpu_baseline` kind "port" in bench.py.  The shipped product never
 * links, loads or calls it.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ibwa_oracle.h"

#define OCC_INTERVAL 128 /* bwt.h:34 */
#define THREAD_BLOCK 1024 /* bwtaln.c:16 */

/* ---------------- index (bwtio.c:51-70, bwt.h:56-63) ---------------- */

or_bwt_t *or_bwt_load(const char *fn)
{
	FILE *fp = fopen(fn, "rb");
	or_bwt_t *b;
	long sz;
	if (!fp) return 0;
	b = (or_bwt_t*)calloc(1, sizeof(*b));
	fseek(fp, 0, SEEK_END);
	sz = ftell(fp);
	b->bwt_size = (uint32_t)((sz - 20) >> 2);
	b->bwt = (uint32_t*)malloc((size_t)b->bwt_size * 4);
	fseek(fp, 0, SEEK_SET);
	if (fread(&b->primary, 4, 1, fp) != 1 || fread(b->L2 + 1, 4, 4, fp) != 4 ||
	    fread(b->bwt, 4, b->bwt_size, fp) != b->bwt_size) {
		fclose(fp); free(b->bwt); free(b); return 0;
	}
	fclose(fp);
	b->L2[0] = 0;
	b->seq_len = b->L2[4];
	b->owns = 1;
	return b;
}

or_bwt_t *or_bwt_wrap(uint32_t primary, const uint32_t L2_1to4[4], uint32_t *words, uint64_t n_words)
{
	or_bwt_t *b = (or_bwt_t*)calloc(1, sizeof(*b));
	b->primary = primary;
	b->L2[0] = 0;
	memcpy(b->L2 + 1, L2_1to4, 16);
	b->seq_len = b->L2[4];
	b->bwt_size = (uint32_t)n_words;
	b->bwt = words;
	b->owns = 0;
	return b;
}

void or_bwt_free(or_bwt_t *b)
{
	if (!b) return;
	if (b->owns) free(b->bwt);
	free(b);
}

void or_free(void *p) { free(p); }

/* ---------------- rank queries (bwt.c:81-214) ---------------- */

/* number of symbol c among the 2-bit bases of y (bwt.c:81-88) */
static inline int cnt2(uint64_t y, int c)
{
	y = ((c & 2) ? y : ~y) >> 1 & ((c & 1) ? y : ~y) & 0x5555555555555555ull;
	return __builtin_popcountll(y);
}

/* 4 bytes of per-symbol counts for one 16-base word (bwt.c:36-45,153-155) */
static inline uint32_t cnt4(uint32_t w)
{
	uint32_t x = 0;
	int i;
	for (i = 0; i < 16; ++i) x += 1u << (((w >> (30 - 2 * i)) & 3) << 3);
	return x;
}

static inline const uint32_t *occ_intv(const or_bwt_t *b, uint32_t k) { return b->bwt + (k / OCC_INTERVAL) * 12; }

/* Occ(c, k): bwt.c:90-113 -- count of c in BWT[0..k] with $ removed */
static uint32_t occ_t(const or_bwt_t *b, uint32_t k, int c, uint32_t *t)
{
	uint32_t n, j, i;
	const uint32_t *p;
	if (k == b->seq_len) return b->L2[c + 1] - b->L2[c];
	if (k == (uint32_t)-1) return 0;
	++*t;
	if (k >= b->primary) --k;
	p = occ_intv(b, k);
	n = p[c];
	p += 4;
	j = k >> 5 << 5;
	for (i = k / OCC_INTERVAL * OCC_INTERVAL; i < j; i += 32, p += 2)
		n += cnt2((uint64_t)p[0] << 32 | p[1], c);
	n += cnt2(((uint64_t)p[0] << 32 | p[1]) & ~((1ull << ((~k & 31) << 1)) - 1), c);
	if (c == 0) n -= ~k & 31; /* masked bases read as A */
	return n;
}

uint32_t or_occ(const or_bwt_t *b, uint32_t k, int c) { uint32_t t = 0; return occ_t(b, k, c, &t); }

/* bwt.c:116-151 */
static void twoocc_t(const or_bwt_t *b, uint32_t k, uint32_t l, int c, uint32_t *ok, uint32_t *ol, uint32_t *t)
{
	uint32_t _k, _l;
	if (k == l) { *ok = *ol = occ_t(b, k, c, t); return; }
	_k = k >= b->primary ? k - 1 : k;
	_l = l >= b->primary ? l - 1 : l;
	if (_l / OCC_INTERVAL != _k / OCC_INTERVAL || k == (uint32_t)-1 || l == (uint32_t)-1) {
		*ok = occ_t(b, k, c, t);
		*ol = occ_t(b, l, c, t);
	} else {
		/* same interval: one block serves both ends */
		uint32_t m, n, i, j;
		const uint32_t *p;
		++*t;
		k = _k; l = _l;
		p = occ_intv(b, k);
		n = p[c];
		p += 4;
		j = k >> 5 << 5;
		for (i = k / OCC_INTERVAL * OCC_INTERVAL; i < j; i += 32, p += 2)
			n += cnt2((uint64_t)p[0] << 32 | p[1], c);
		m = n;
		n += cnt2(((uint64_t)p[0] << 32 | p[1]) & ~((1ull << ((~k & 31) << 1)) - 1), c);
		if (c == 0) n -= ~k & 31;
		*ok = n;
		j = l >> 5 << 5;
		for (; i < j; i += 32, p += 2)
			m += cnt2((uint64_t)p[0] << 32 | p[1], c);
		m += cnt2(((uint64_t)p[0] << 32 | p[1]) & ~((1ull << ((~l & 31) << 1)) - 1), c);
		if (c == 0) m -= ~l & 31;
		*ol = m;
	}
}

/* bwt.c:157-174 */
static void occ4_t(const or_bwt_t *b, uint32_t k, uint32_t cnt[4], uint32_t *t)
{
	uint32_t i, j, x;
	const uint32_t *p;
	if (k == (uint32_t)-1) { memset(cnt, 0, 16); return; }
	++*t;
	if (k >= b->primary) --k;
	p = occ_intv(b, k);
	memcpy(cnt, p, 16);
	p += 4;
	j = k >> 4 << 4;
	for (i = k / OCC_INTERVAL * OCC_INTERVAL, x = 0; i < j; i += 16, ++p) x += cnt4(*p);
	x += cnt4(*p & ~((1U << ((~k & 15) << 1)) - 1)) - (~k & 15);
	cnt[0] += x & 0xff; cnt[1] += x >> 8 & 0xff; cnt[2] += x >> 16 & 0xff; cnt[3] += x >> 24;
}

void or_occ4(const or_bwt_t *b, uint32_t k, uint32_t cnt[4]) { uint32_t t = 0; occ4_t(b, k, cnt, &t); }

/* bwt.c:177-214 */
static void twoocc4_t(const or_bwt_t *b, uint32_t k, uint32_t l, uint32_t ck[4], uint32_t cl[4], uint32_t *t)
{
	uint32_t _k, _l;
	if (k == l) { occ4_t(b, k, ck, t); memcpy(cl, ck, 16); return; }
	_k = k >= b->primary ? k - 1 : k;
	_l = l >= b->primary ? l - 1 : l;
	if (_l / OCC_INTERVAL != _k / OCC_INTERVAL || k == (uint32_t)-1 || l == (uint32_t)-1) {
		occ4_t(b, k, ck, t);
		occ4_t(b, l, cl, t);
	} else {
		uint32_t i, j, x, y;
		const uint32_t *p;
		++*t;
		k = _k; l = _l;
		p = occ_intv(b, k);
		memcpy(ck, p, 16);
		p += 4;
		j = k >> 4 << 4;
		for (i = k / OCC_INTERVAL * OCC_INTERVAL, x = 0; i < j; i += 16, ++p) x += cnt4(*p);
		y = x;
		x += cnt4(*p & ~((1U << ((~k & 15) << 1)) - 1)) - (~k & 15);
		j = l >> 4 << 4;
		for (; i < j; i += 16, ++p) y += cnt4(*p);
		y += cnt4(*p & ~((1U << ((~l & 15) << 1)) - 1)) - (~l & 15);
		memcpy(cl, ck, 16);
		ck[0] += x & 0xff; ck[1] += x >> 8 & 0xff; ck[2] += x >> 16 & 0xff; ck[3] += x >> 24;
		cl[0] += y & 0xff; cl[1] += y >> 8 & 0xff; cl[2] += y >> 16 & 0xff; cl[3] += y >> 24;
	}
}

void or_2occ4(const or_bwt_t *b, uint32_t k, uint32_t l, uint32_t ck[4], uint32_t cl[4])
{
	uint32_t t = 0;
	twoocc4_t(b, k, l, ck, cl, &t);
}

/* bwt.c:235-250: continue an exact backward search over str[0..len-1] */
static int match_exact_alt_n(const or_bwt_t *b, int len, const uint8_t *str, uint32_t *k0, uint32_t *l0, uint32_t *t,
                             uint32_t *steps)
{
	int i;
	uint32_t k = *k0, l = *l0, ok, ol;
	for (i = len - 1; i >= 0; --i) {
		int c = str[i];
		if (c > 3) return 0;
		if (steps) ++*steps;
		twoocc_t(b, k - 1, l, c, &ok, &ol, t);
		k = b->L2[c] + ok + 1;
		l = b->L2[c] + ol;
		if (k > l) return 0;
	}
	*k0 = k; *l0 = l;
	return (int)(l - k + 1);
}

static int match_exact_alt(const or_bwt_t *b, int len, const uint8_t *str, uint32_t *k0, uint32_t *l0, uint32_t *t)
{
	return match_exact_alt_n(b, len, str, k0, l0, t, 0);
}

/* ---------------- options (bwtaln.c:21-51) ---------------- */

void or_gap_init_opt(or_gap_opt_t *o)
{
	memset(o, 0, sizeof(*o));
	o->s_mm = 3; o->s_gapo = 11; o->s_gape = 4;
	o->max_diff = -1; o->max_gapo = 1; o->max_gape = 6;
	o->indel_end_skip = 5; o->max_del_occ = 10; o->max_entries = 2000000;
	o->mode = OR_MODE_GAPE | OR_MODE_COMPREAD;
	o->seed_len = 32; o->max_seed_diff = 2;
	o->fnr = 0.04f;
	o->n_threads = 1;
	o->max_top2 = 30;
	o->trim_qual = 0;
}

/* smallest k with Poisson(l*err) upper tail < thres (bwtaln.c:39-51) */
int or_cal_maxdiff(int l, double err, double thres)
{
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

/* ---------------- widths (bwtaln.c:54-78) ---------------- */

typedef struct { uint32_t w; int bid; } width_t;

static void cal_width(const or_bwt_t *b, int len, const uint8_t *str, width_t *width, uint32_t *t)
{
	uint32_t k = 0, l = b->seq_len, ok, ol;
	int i, bid = 0;
	for (i = 0; i < len; ++i) {
		int c = str[i];
		if (c < 4) {
			twoocc_t(b, k - 1, l, c, &ok, &ol, t);
			k = b->L2[c] + ok + 1;
			l = b->L2[c] + ol;
		}
		if (k > l || c > 3) { k = 0; l = b->seq_len; ++bid; }
		width[i].w = l - k + 1;
		width[i].bid = bid;
	}
	width[len].w = 0;
	width[len].bid = ++bid;
}

/* ---------------- bucketed LIFO priority stack (bwtgap.c:13-79) ---------------- */

typedef struct {
	uint32_t k, l;
	int i, a, state, n_mm, n_gapo, n_gape, last_diff_pos, score;
	int phantom; /* instrumentation: can never be expanded (see gs_push) */
	int mc;      /* instrumentation: a match child (popped right after its parent's expansion) */
	int kind;    /* instrumentation: what pushed it (OR_K_*) */
	int dep;     /* instrumentation: BWT steps from the root (the length of the node's reference string) */
} entry_t;

/* instrumentation: pushes / pops / expansions by kind of entry, summed over all searches since the
 * last or_push_kinds_reset (relaxed atomics; diagnostics for the GPU stack design) */
enum { OR_K_ROOT, OR_K_INS_OPEN, OR_K_DEL_OPEN, OR_K_INS_EXT, OR_K_DEL_EXT, OR_K_MISMATCH, OR_K_MATCH, OR_K_N };
static uint64_t g_kind_push[OR_K_N], g_kind_pop[OR_K_N], g_kind_exp[OR_K_N];
/* instrumentation: by depth (OR_DEP_N - 1 = that or deeper) the expansions (one bwt_2occ4 each), the pops
 * and the exact-tail steps (one bwt_2occ each) -- where the search's rank queries fall (tools/depth_stats.py) */
#define OR_DEP_N 64
static uint64_t g_dep_exp[OR_DEP_N], g_dep_pop[OR_DEP_N], g_dep_tail[OR_DEP_N];
/* pops of match children by depth (popped right after their parent's expansion: a chain of them is what
 * a table of the shallow intervals could fetch ahead), pops at a one-row interval and match-child pops
 * at one (a chain that follows the text) */
static uint64_t g_dep_mcpop[OR_DEP_N], g_uniq_pop, g_uniq_mcpop, g_uniq_tail;
static int g_kinds_on; /* counting is off until the first reset: shared counters would serialise the threads */
void or_push_kinds_reset(void)
{
	g_kinds_on = 1;
	memset(g_kind_push, 0, sizeof g_kind_push);
	memset(g_kind_pop, 0, sizeof g_kind_pop);
	memset(g_kind_exp, 0, sizeof g_kind_exp);
	memset(g_dep_exp, 0, sizeof g_dep_exp);
	memset(g_dep_pop, 0, sizeof g_dep_pop);
	memset(g_dep_tail, 0, sizeof g_dep_tail);
	memset(g_dep_mcpop, 0, sizeof g_dep_mcpop);
	g_uniq_pop = g_uniq_mcpop = g_uniq_tail = 0;
}
void or_depth_hist(uint64_t out[4 * OR_DEP_N + 3])
{
	int i;
	for (i = 0; i < OR_DEP_N; ++i) {
		out[i] = __atomic_load_n(&g_dep_exp[i], __ATOMIC_RELAXED);
		out[OR_DEP_N + i] = __atomic_load_n(&g_dep_pop[i], __ATOMIC_RELAXED);
		out[2 * OR_DEP_N + i] = __atomic_load_n(&g_dep_tail[i], __ATOMIC_RELAXED);
		out[3 * OR_DEP_N + i] = __atomic_load_n(&g_dep_mcpop[i], __ATOMIC_RELAXED);
	}
	out[4 * OR_DEP_N] = __atomic_load_n(&g_uniq_pop, __ATOMIC_RELAXED);
	out[4 * OR_DEP_N + 1] = __atomic_load_n(&g_uniq_mcpop, __ATOMIC_RELAXED);
	out[4 * OR_DEP_N + 2] = __atomic_load_n(&g_uniq_tail, __ATOMIC_RELAXED);
}
static inline int dep_bin(int d) { return d < OR_DEP_N - 1 ? d : OR_DEP_N - 1; }
void or_push_kinds(uint64_t out[3 * OR_K_N])
{
	int i;
	for (i = 0; i < OR_K_N; ++i) {
		out[i] = __atomic_load_n(&g_kind_push[i], __ATOMIC_RELAXED);
		out[OR_K_N + i] = __atomic_load_n(&g_kind_pop[i], __ATOMIC_RELAXED);
		out[2 * OR_K_N + i] = __atomic_load_n(&g_kind_exp[i], __ATOMIC_RELAXED);
	}
}

typedef struct { int n, m; entry_t *e; } bucket_t;
#define OR_CHAIN_W 64
typedef struct {
	int n_stacks, best, n_entries; bucket_t *b; uint32_t pushes, pops, peak, peak_bucket;
	/* instrumentation: entries that can still be expanded when pushed */
	int md_now, score_cap, gape; uint32_t n_real, peak_real;
	/* search-shape counters (tools/dfs_stats.py) */
	uint32_t tails, tail_steps, pruned_m, pruned_w, expansions, hits;
	/* match chains (a popped non-match-child entry and its run of match children + tail):
	 * rounds = sum over windows of W consecutive chains of one level of the longest chain */
	uint32_t chains, rounds, next_mc, ch_len, win_n, win_max, win_level;
	int next_kind; /* instrumentation: kind of the next push (OR_K_*) */
	int next_dep;  /* instrumentation: depth of the next push */
	uint32_t *chl, chl_n, chl_m; /* chain (length << 11 | level) in pop order, when stats are on */
	uint64_t *hset; uint32_t hcap, hn; /* distinct (a,i,k,l) expansions, when stats are on */
	uint32_t split_pop, touch_at_split; /* touches counted before pop number split_pop + 1 (0: off) */
} gstack_t;

/* per-read search statistics (test/bench instrumentation only) */
typedef struct {
	uint32_t pushes, pops, peak_entries, peak_bucket, n_aln, touches, peak_real;
	uint32_t tails, tail_steps, pruned_m, pruned_w, expansions, hits, distinct_exp, chains, rounds;
	uint32_t rounds_g4, rounds_g16, rounds_lvl;
} or_stats_t;
static or_stats_t *g_stats_next; /* consumed by the next or_cal_sa_reg_gap call */
void or_set_stats(or_stats_t *buf) { g_stats_next = buf; }
/* per-read touches of the four bwt_cal_width calls alone (bwtaln.c:123-130; the rest of a read's
 * touches are bwt_match_gap's), consumed by the next or_cal_sa_reg_gap call */
static uint32_t *g_wtouch_next;
void or_set_width_touches(uint32_t *buf) { g_wtouch_next = buf; }
/* per read a pop count p (0: none) and the touches counted before pop p + 1 -- where the GPU's first
 * pass left the read's resume state after p pops (gapped.hip dump_states) -- consumed by the next
 * or_cal_sa_reg_gap call; the bench splits bwt_match_gap's touches of a resumed read there */
static const uint32_t *g_split_pops_next;
static uint32_t *g_split_touch_next;
void or_set_touch_split(const uint32_t *pops, uint32_t *touches) { g_split_pops_next = pops; g_split_touch_next = touches; }

#define SCORE(m, o, e, p) ((m) * (p)->s_mm + (o) * (p)->s_gapo + (e) * (p)->s_gape)
#define ST_M 0
#define ST_I 1
#define ST_D 2

static gstack_t *gs_init(int md, int go, int ge, const or_gap_opt_t *o)
{
	gstack_t *s = (gstack_t*)calloc(1, sizeof(*s));
	int i;
	s->n_stacks = SCORE(md + 1, go + 1, ge + 1, o);
	s->b = (bucket_t*)calloc(s->n_stacks, sizeof(bucket_t));
	for (i = 0; i < s->n_stacks; ++i) { s->b[i].m = 4; s->b[i].e = (entry_t*)calloc(4, sizeof(entry_t)); }
	return s;
}

static void gs_free(gstack_t *s)
{
	int i;
	for (i = 0; i < s->n_stacks; ++i) free(s->b[i].e);
	free(s->hset); free(s->chl); free(s->b); free(s);
}

static void gs_reset(gstack_t *s)
{
	int i;
	for (i = 0; i < s->n_stacks; ++i) s->b[i].n = 0;
	s->best = s->n_stacks;
	s->n_entries = 0;
	s->pushes = s->pops = s->peak = s->peak_bucket = 0;
	s->n_real = s->peak_real = 0;
	s->tails = s->tail_steps = s->pruned_m = s->pruned_w = s->expansions = s->hits = 0;
	s->chains = s->rounds = s->next_mc = s->ch_len = s->win_n = s->win_max = 0;
	s->win_level = ~0u;
	s->chl_n = 0;
	if (s->hset) memset(s->hset, 0, (size_t)s->hcap * 8);
	s->hn = 0;
}

/* distinct-expansion set (instrumentation): open addressing on a 64-bit mix of (a,i,k,l) */
static void gs_note_exp(gstack_t *s, int a, int i, uint32_t k, uint32_t l)
{
	uint64_t h = ((uint64_t)k << 32 | l) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(i << 1 | a) + 1) * 0xC2B2AE3D27D4EB4Full;
	uint32_t j;
	if (!s->hset) return;
	if (!h) h = 1;
	if (2 * (s->hn + 1) > s->hcap) {
		uint64_t *o = s->hset; uint32_t oc = s->hcap, q;
		s->hcap = oc ? oc * 2 : 1024;
		s->hset = (uint64_t*)calloc(s->hcap, 8);
		s->hn = 0;
		for (q = 0; q < oc; ++q) if (o[q]) {
			for (j = (uint32_t)(o[q] >> 20) & (s->hcap - 1); s->hset[j]; j = (j + 1) & (s->hcap - 1));
			s->hset[j] = o[q]; ++s->hn;
		}
		free(o);
	}
	for (j = (uint32_t)(h >> 20) & (s->hcap - 1); s->hset[j]; j = (j + 1) & (s->hcap - 1))
		if (s->hset[j] == h) return;
	s->hset[j] = h; ++s->hn;
}

/* bwtgap.c:45-64.  last_diff_pos: a non-diff push keeps the value already in
 * its slot, which for positive penalties is always the just-popped parent's
 * (SURVEY §7); we pass the parent's value explicitly ("inherit"). */
static void gs_push(gstack_t *s, int a, int i, uint32_t k, uint32_t l, int n_mm, int n_gapo, int n_gape,
                    int state, int ldp, const or_gap_opt_t *o)
{
	int score = SCORE(n_mm, n_gapo, n_gape, o);
	bucket_t *q;
	entry_t *p;
	if (score < 0 || score >= s->n_stacks) { fprintf(stderr, "[oracle] score %d out of range\n", score); abort(); }
	q = s->b + score;
	if (q->n == q->m) { q->m <<= 1; q->e = (entry_t*)realloc(q->e, q->m * sizeof(entry_t)); }
	p = q->e + q->n;
	p->k = k; p->l = l; p->i = i & 0xffff; p->a = a; p->state = state;
	p->n_mm = n_mm & 0xff; p->n_gapo = n_gapo & 0xff; p->n_gape = n_gape & 0xff;
	p->last_diff_pos = ldp;
	p->mc = s->next_mc; s->next_mc = 0;
	p->kind = s->next_kind; s->next_kind = OR_K_MISMATCH;
	p->dep = s->next_dep;
	if (g_kinds_on) __atomic_add_fetch(&g_kind_push[p->kind], 1, __ATOMIC_RELAXED);
	p->score = score & 0x7ff; /* info = score<<21 keeps 11 bits */
	/* phantom: more diffs than the (non-increasing) max_diff allows, or a score the
	 * search stops at once a hit has fixed best_score -- such entries are only counted */
	p->phantom = (n_mm + n_gapo + (s->gape ? n_gape : 0) > s->md_now) || score > s->score_cap;
	if (!p->phantom && ++s->n_real > s->peak_real) s->peak_real = s->n_real;
	++q->n;
	++s->n_entries;
	if (s->best > score) s->best = score;
	++s->pushes;
	if ((uint32_t)s->n_entries > s->peak) s->peak = s->n_entries;
	if ((uint32_t)q->n > s->peak_bucket) s->peak_bucket = q->n;
}

static void gs_pop(gstack_t *s, entry_t *e)
{
	bucket_t *q = s->b + s->best;
	++s->pops;
	*e = q->e[q->n - 1];
	if (g_kinds_on) {
		__atomic_add_fetch(&g_kind_pop[e->kind], 1, __ATOMIC_RELAXED);
		__atomic_add_fetch(&g_dep_pop[dep_bin(e->dep)], 1, __ATOMIC_RELAXED);
		if (e->mc) __atomic_add_fetch(&g_dep_mcpop[dep_bin(e->dep)], 1, __ATOMIC_RELAXED);
		if (e->k == e->l) {
			__atomic_add_fetch(&g_uniq_pop, 1, __ATOMIC_RELAXED);
			if (e->mc) __atomic_add_fetch(&g_uniq_mcpop, 1, __ATOMIC_RELAXED);
		}
	}
	if (!e->phantom) --s->n_real;
	if (!e->mc && s->hset) { /* a chain starts: record the previous one */
		if (s->chains) {
			if (s->chl_n == s->chl_m) { s->chl_m = s->chl_m ? s->chl_m * 2 : 4096; s->chl = (uint32_t*)realloc(s->chl, s->chl_m * 4); }
			s->chl[s->chl_n++] = s->ch_len << 11 | s->win_level;
		}
	}
	if (!e->mc) { /* a chain starts: close the previous one into its window */
		if (s->ch_len > s->win_max) s->win_max = s->ch_len;
		if (s->win_n && (s->win_n == OR_CHAIN_W || (uint32_t)e->score != s->win_level)) {
			s->rounds += s->win_max; s->win_n = 0; s->win_max = 0;
		}
		if (s->ch_len == 0 && s->win_n == 0) s->win_max = 0;
		++s->win_n; s->win_level = e->score; ++s->chains; s->ch_len = 0;
	}
	++s->ch_len;
	--q->n;
	--s->n_entries;
	if (q->n == 0 && s->n_entries) {
		int i;
		for (i = s->best + 1; i < s->n_stacks; ++i) if (s->b[i].n) break;
		s->best = i;
	} else if (s->n_entries == 0) s->best = s->n_stacks;
}

/* bwtgap.c:81-91 */
static void gap_shadow(int x, uint32_t max, int last_diff_pos, width_t *w)
{
	int i, j;
	for (i = j = 0; i < last_diff_pos; ++i) {
		if (w[i].w > (uint32_t)x) w[i].w -= x;
		else if (w[i].w == (uint32_t)x) { w[i].bid = 1; w[i].w = max - (++j); }
	}
}

static int int_log2(uint32_t v) /* bwtgap.c:93-102 */
{
	int c = 0;
	if (v & 0xffff0000u) { v >>= 16; c |= 16; }
	if (v & 0xff00) { v >>= 8; c |= 8; }
	if (v & 0xf0) { v >>= 4; c |= 4; }
	if (v & 0xc) { v >>= 2; c |= 2; }
	if (v & 0x2) c |= 1;
	return c;
}

typedef struct { or_aln1_t *a; int n, m; } alnv_t;

/* bwtgap.c:104-264 */
static void match_gap(const or_bwt_t *const bwts[2], int len, const uint8_t *seq[2], width_t *w[2],
                      width_t *seed_w[2], const or_gap_opt_t *opt, alnv_t *out, gstack_t *stack, uint32_t *t)
{
	int best_score = SCORE(opt->max_diff + 1, opt->max_gapo + 1, opt->max_gape + 1, opt);
	int best_diff = opt->max_diff + 1, max_diff = opt->max_diff;
	int best_cnt = 0, j, nN;
	out->n = 0;
	for (j = nN = 0; j < len; ++j) if (seq[0][j] > 3) ++nN;
	if (nN > max_diff) return;

	gs_reset(stack);
	stack->md_now = max_diff;
	stack->score_cap = 0x7fffffff;
	stack->gape = (opt->mode & OR_MODE_GAPE) != 0;
	stack->next_kind = OR_K_ROOT;
	stack->next_dep = 0;
	gs_push(stack, 0, len, 0, bwts[0]->seq_len, 0, 0, 0, ST_M, 0, opt);
	stack->next_kind = OR_K_ROOT;
	gs_push(stack, 1, len, 0, bwts[0]->seq_len, 0, 0, 0, ST_M, 0, opt);

	while (stack->n_entries) {
		entry_t e;
		int a, i, m, m_seed = 0, hit, allow_diff, allow_M, tmp;
		uint32_t k, l, ck[4], cl[4], occ;
		const or_bwt_t *bwt;
		const uint8_t *str;
		const width_t *sw = 0;
		width_t *width;

		if (stack->n_entries > opt->max_entries) break;
		if (stack->split_pop && stack->pops == stack->split_pop) stack->touch_at_split = *t;
		gs_pop(stack, &e);
		k = e.k; l = e.l;
		a = e.a; i = e.i;
		if (!(opt->mode & OR_MODE_NONSTOP) && (uint32_t)e.score > (uint32_t)(best_score + opt->s_mm)) break;

		m = max_diff - (e.n_mm + e.n_gapo);
		if (opt->mode & OR_MODE_GAPE) m -= e.n_gape;
		if (m < 0) { ++stack->pruned_m; continue; }
		bwt = bwts[1 - a]; str = seq[a]; width = w[a];
		if (seed_w) {
			sw = seed_w[a];
			m_seed = opt->max_seed_diff - (e.n_mm + e.n_gapo);
			if (opt->mode & OR_MODE_GAPE) m_seed -= e.n_gape;
		}
		if (i > 0 && m < width[i - 1].bid) { ++stack->pruned_w; continue; }

		hit = 0;
		if (i == 0) hit = 1;
		else if (m == 0 && (e.state == ST_M || (opt->mode & OR_MODE_GAPE) || e.n_gape == opt->max_gape)) {
			++stack->tails;
			{
				uint32_t ts0 = stack->tail_steps, q;
				hit = match_exact_alt_n(bwt, i, str, &k, &l, t, &stack->tail_steps) != 0;
				stack->ch_len += stack->tail_steps - ts0;
				if (g_kinds_on) {
					for (q = 0; q < stack->tail_steps - ts0; ++q)
						__atomic_add_fetch(&g_dep_tail[dep_bin(e.dep + (int)q)], 1, __ATOMIC_RELAXED);
					if (e.k == e.l) __atomic_add_fetch(&g_uniq_tail, stack->tail_steps - ts0, __ATOMIC_RELAXED);
				}
			}
			if (!hit) continue;
		}
		if (hit) {
			++stack->hits;
			int score = SCORE(e.n_mm, e.n_gapo, e.n_gape, opt), do_add = 1;
			if (out->n == 0) {
				best_score = score;
				best_diff = e.n_mm + e.n_gapo;
				if (opt->mode & OR_MODE_GAPE) best_diff += e.n_gape;
				if (!(opt->mode & OR_MODE_NONSTOP)) {
					max_diff = (best_diff + 1 > opt->max_diff) ? opt->max_diff : best_diff + 1;
					stack->md_now = max_diff;
					stack->score_cap = best_score + opt->s_mm;
				}
			}
			if (score == best_score) best_cnt = (int)((uint32_t)best_cnt + (l - k + 1));
			else if (best_cnt > opt->max_top2) break;
			if (e.n_gapo) {
				for (j = 0; j < out->n; ++j) if (out->a[j].k == k && out->a[j].l == l) break;
				if (j < out->n) do_add = 0;
			}
			if (do_add) {
				or_aln1_t *p;
				gap_shadow(l - k + 1, bwt->seq_len, e.last_diff_pos, width);
				if (out->n == out->m) {
					out->m = out->m ? out->m << 1 : 4;
					out->a = (or_aln1_t*)realloc(out->a, out->m * sizeof(or_aln1_t));
				}
				p = out->a + out->n++;
				memset(p, 0, sizeof(*p));
				p->n_mm = e.n_mm; p->n_gapo = e.n_gapo; p->n_gape = e.n_gape; p->a = a;
				p->k = k; p->l = l; p->score = score;
			}
			continue;
		}

		--i;
		++stack->expansions;
		if (g_kinds_on) {
			__atomic_add_fetch(&g_kind_exp[e.kind], 1, __ATOMIC_RELAXED);
			__atomic_add_fetch(&g_dep_exp[dep_bin(e.dep)], 1, __ATOMIC_RELAXED);
		}
		gs_note_exp(stack, a, i, k, l);
		twoocc4_t(bwt, k - 1, l, ck, cl, t);
		occ = l - k + 1;
		allow_diff = allow_M = 1;
		if (i > 0) {
			int ii = i - (len - opt->seed_len);
			if (width[i - 1].bid > m - 1) allow_diff = 0;
			else if (width[i - 1].bid == m - 1 && width[i].bid == m - 1 && width[i - 1].w == width[i].w) allow_M = 0;
			if (seed_w && ii > 0) {
				if (sw[ii - 1].bid > m_seed - 1) allow_diff = 0;
				else if (sw[ii - 1].bid == m_seed - 1 && sw[ii].bid == m_seed - 1 && sw[ii - 1].w == sw[ii].w) allow_M = 0;
			}
		}
		tmp = (opt->mode & OR_MODE_LOGGAP) ? int_log2(e.n_gape + e.n_gapo) / 2 + 1 : e.n_gapo + e.n_gape;
		if (allow_diff && i >= opt->indel_end_skip + tmp && len - i >= opt->indel_end_skip + tmp) {
			if (e.state == ST_M) {
				if (e.n_gapo < opt->max_gapo) {
					stack->next_kind = OR_K_INS_OPEN;
					stack->next_dep = e.dep;
					gs_push(stack, a, i, k, l, e.n_mm, e.n_gapo + 1, e.n_gape, ST_I, i, opt);
					for (j = 0; j != 4; ++j) {
						uint32_t kk = bwt->L2[j] + ck[j] + 1, ll = bwt->L2[j] + cl[j];
						stack->next_kind = OR_K_DEL_OPEN;
						stack->next_dep = e.dep + 1;
						if (kk <= ll) gs_push(stack, a, i + 1, kk, ll, e.n_mm, e.n_gapo + 1, e.n_gape, ST_D, i + 1, opt);
					}
				}
			} else if (e.state == ST_I) {
				if (e.n_gape < opt->max_gape) {
					stack->next_kind = OR_K_INS_EXT;
					stack->next_dep = e.dep;
					gs_push(stack, a, i, k, l, e.n_mm, e.n_gapo, e.n_gape + 1, ST_I, i, opt);
				}
			} else if (e.state == ST_D) {
				if (e.n_gape < opt->max_gape) {
					if (e.n_gape + e.n_gapo < max_diff || occ < (uint32_t)opt->max_del_occ) {
						for (j = 0; j != 4; ++j) {
							uint32_t kk = bwt->L2[j] + ck[j] + 1, ll = bwt->L2[j] + cl[j];
							stack->next_kind = OR_K_DEL_EXT;
							stack->next_dep = e.dep + 1;
							if (kk <= ll) gs_push(stack, a, i + 1, kk, ll, e.n_mm, e.n_gapo, e.n_gape + 1, ST_D, i + 1, opt);
						}
					}
				}
			}
		}
		if (allow_diff && allow_M) {
			for (j = 1; j <= 4; ++j) {
				int c = (str[i] + j) & 3;
				int is_mm = (j != 4 || str[i] > 3);
				uint32_t kk = bwt->L2[c] + ck[c] + 1, ll = bwt->L2[c] + cl[c];
				stack->next_mc = !is_mm;
				stack->next_kind = is_mm ? OR_K_MISMATCH : OR_K_MATCH;
				stack->next_dep = e.dep + 1;
				if (kk <= ll) gs_push(stack, a, i, kk, ll, e.n_mm + is_mm, e.n_gapo, e.n_gape, ST_M,
				                      is_mm ? i : e.last_diff_pos, opt);
			}
		} else if (str[i] < 4) {
			int c = str[i] & 3;
			uint32_t kk = bwt->L2[c] + ck[c] + 1, ll = bwt->L2[c] + cl[c];
			stack->next_mc = 1;
			stack->next_kind = OR_K_MATCH;
			stack->next_dep = e.dep + 1;
			if (kk <= ll) gs_push(stack, a, i, kk, ll, e.n_mm, e.n_gapo, e.n_gape, ST_M, e.last_diff_pos, opt);
		}
	}
	(void)best_diff;
}

/* Occ-interval touches (SURVEY §8d counting rules) of the exact-match path the
 * GPU takes for max_diff == 0: strand 1 = bwt_match_exact_alt(bwt0, rseq),
 * strand 0 = bwt_match_exact_alt(bwt1, seq), none for reads with an N.  Used
 * to price the GPU path's own algorithmic bytes (it skips bwt_cal_width). */
/* The unique-interval jump: once k == l with m symbols left the
 * GPU reads SA[k], compares the m symbols against the packed text and, if they
 * all match, reads ISA at the final position -- one 64 B touch each (the m <= 256
 * symbols of text span one 64 B line), instead of m Occ steps. */
static void jump_touches(const or_bwt_t *b, int m, const uint8_t *str, uint32_t k, uint32_t l, uint32_t *t)
{
	uint32_t dummy = 0;
	*t += 2 + (uint32_t)((2 * m - 1) / 512);
	if (match_exact_alt(b, m, str, &k, &l, &dummy)) ++*t;
}

/* one exact chain priced with a K-mer table: the first K steps are one lookup;
 * with `jump`, the steps after the interval narrows to one row are priced as a jump */
static void exact_chain_touches(const or_bwt_t *b, int L, const uint8_t *str, int K, int jump, uint32_t *t)
{
	uint32_t k = 0, l = b->seq_len, dummy = 0, ok, ol;
	int i;
	if (K > 0 && L >= K) {
		++*t;
		if (!match_exact_alt(b, K, str + L - K, &k, &l, &dummy)) return;
		L -= K;
	}
	for (i = L - 1; i >= 0; --i) {
		int c = str[i];
		if (jump && k == l) { jump_touches(b, i + 1, str, k, l, t); return; }
		if (c > 3) return;
		twoocc_t(b, k - 1, l, c, &ok, &ol, t);
		k = b->L2[c] + ok + 1;
		l = b->L2[c] + ol;
		if (k > l) return;
	}
}

void or_exact_touches(const or_bwt_t *bwt0, const or_bwt_t *bwt1, int64_t n_seqs, const uint8_t *seq,
                      const uint64_t *off, const uint32_t *len, int mode, int K, int jump, uint32_t *touches)
{
	int64_t r;
	uint8_t *rseq = 0;
	int cap = 0;
	for (r = 0; r < n_seqs; ++r) {
		int L = (int)len[r], j, nN = 0;
		const uint8_t *s = seq + off[r];
		uint32_t t = 0, k, l;
		if (L + 1 > cap) { cap = L + 1; rseq = (uint8_t*)realloc(rseq, cap); }
		for (j = 0; j < L; ++j) {
			nN += s[j] > 3;
			rseq[j] = (mode & OR_MODE_COMPREAD) && s[j] < 4 ? 3 - s[j] : s[j];
		}
		if (nN == 0) {
			exact_chain_touches(bwt0, L, rseq, K, jump, &t);
			exact_chain_touches(bwt1, L, s, K, jump, &t);
		}
		(void)k; (void)l;
		touches[r] = t;
	}
	free(rseq);
}

/* ---------------- batch driver (bwtaln.c:80-140, 151-156, 199-218) ---------------- */

typedef struct {
	const or_bwt_t *bwt[2];
	int64_t n_seqs;
	const uint8_t *seq;
	const uint64_t *off;
	const uint32_t *len;
	const or_gap_opt_t *opt;
	or_gap_opt_t base;  /* batch-level local_opt (bwtaln.c:86-93) */
	int max_len;
	int32_t *n_aln;
	or_aln1_t **per_read;
	uint32_t *touches, *wtouches;
	const uint32_t *split_pops;
	uint32_t *split_touches;
	or_stats_t *stats;
	int64_t next;  /* dynamic claim of THREAD_BLOCK reads (bwtaln.c:100-113) */
	pthread_mutex_t lock;
} batch_t;

static void *worker(void *data)
{
	batch_t *B = (batch_t*)data;
	const or_gap_opt_t *opt = B->opt;
	or_gap_opt_t local = B->base;
	gstack_t *stack = gs_init(local.max_diff, local.max_gapo, local.max_gape, &local);
	if (B->stats) { stack->hcap = 1024; stack->hset = (uint64_t*)calloc(1024, 8); }
	width_t *w[2], *sw[2];
	uint8_t *rseq = (uint8_t*)malloc(B->max_len + 1);
	alnv_t out = {0, 0, 0};
	w[0] = (width_t*)calloc(B->max_len + 1, sizeof(width_t));
	w[1] = (width_t*)calloc(B->max_len + 1, sizeof(width_t));
	sw[0] = (width_t*)calloc(opt->seed_len + 1, sizeof(width_t));
	sw[1] = (width_t*)calloc(opt->seed_len + 1, sizeof(width_t));
	for (;;) {
		int64_t b0, b1, r;
		pthread_mutex_lock(&B->lock);
		b0 = B->next; B->next += THREAD_BLOCK;
		pthread_mutex_unlock(&B->lock);
		if (b0 >= B->n_seqs) break;
		b1 = b0 + THREAD_BLOCK < B->n_seqs ? b0 + THREAD_BLOCK : B->n_seqs;
		for (r = b0; r < b1; ++r) {
			int L = (int)B->len[r], j;
			const uint8_t *seq[2];
			uint32_t t = 0;
			seq[0] = B->seq + B->off[r];
			/* rseq = complement(seq) under COMPREAD, else seq (bwaseqio.c:189-192) */
			for (j = 0; j < L; ++j) {
				int c = seq[0][j];
				rseq[j] = (opt->mode & OR_MODE_COMPREAD) && c < 4 ? 3 - c : c;
			}
			seq[1] = rseq;
			cal_width(B->bwt[0], L, seq[0], w[0], &t);
			cal_width(B->bwt[1], L, seq[1], w[1], &t);
			if (opt->fnr > 0.0) local.max_diff = or_cal_maxdiff(L, 0.02, opt->fnr);
			local.seed_len = opt->seed_len < L ? opt->seed_len : 0x7fffffff;
			if (L > opt->seed_len) {
				cal_width(B->bwt[0], opt->seed_len, seq[0] + (L - opt->seed_len), sw[0], &t);
				cal_width(B->bwt[1], opt->seed_len, seq[1] + (L - opt->seed_len), sw[1], &t);
			}
			if (B->wtouches) B->wtouches[r] = t;
			stack->pushes = stack->pops = stack->peak = stack->peak_bucket = 0;
			stack->split_pop = B->split_pops ? B->split_pops[r] : 0;
			stack->touch_at_split = t;
			match_gap(B->bwt, L, seq, w, L <= opt->seed_len ? 0 : sw, &local, &out, stack, &t);
			B->n_aln[r] = out.n;
			if (B->stats) {
				or_stats_t *st = B->stats + r;
				st->pushes = stack->pushes; st->pops = stack->pops; st->peak_entries = stack->peak;
				st->peak_bucket = stack->peak_bucket; st->n_aln = out.n; st->touches = t;
				st->peak_real = stack->peak_real;
				st->tails = stack->tails; st->tail_steps = stack->tail_steps; st->pruned_m = stack->pruned_m;
				st->pruned_w = stack->pruned_w; st->expansions = stack->expansions; st->hits = stack->hits;
				st->distinct_exp = stack->hn;
				if (stack->ch_len > stack->win_max) stack->win_max = stack->ch_len;
				st->chains = stack->chains; st->rounds = stack->rounds + stack->win_max;
				if (stack->chains) {
					int gi;
					if (stack->chl_n == stack->chl_m) { stack->chl_m = stack->chl_m ? stack->chl_m * 2 : 4096; stack->chl = (uint32_t*)realloc(stack->chl, stack->chl_m * 4); }
					stack->chl[stack->chl_n++] = stack->ch_len << 11 | stack->win_level;
					/* lanes take contiguous groups of g chains, 64 lanes per window, windows within a level */
					for (gi = 0; gi < 3; ++gi) {
						uint32_t g = gi == 0 ? 4 : gi == 1 ? 16 : 0, q = 0, tot = 0;
						while (q < stack->chl_n) {
							uint32_t lev = stack->chl[q] & 2047, e2 = q, mx = 0, lane, gg;
							while (e2 < stack->chl_n && (stack->chl[e2] & 2047) == lev) ++e2; /* level [q, e2) */
							while (q < e2) {
								uint32_t rem = e2 - q;
								gg = g ? g : (rem + 63) / 64; /* g = 0: adaptive, all of the level in one window */
								if (g && rem < 64 * g) gg = (rem + 63) / 64;
								mx = 0;
								for (lane = 0; lane < 64 && q < e2; ++lane) {
									uint32_t sum = 0, j;
									for (j = 0; j < gg && q < e2; ++j, ++q) sum += stack->chl[q] >> 11;
									if (sum > mx) mx = sum;
								}
								tot += mx;
							}
						}
						if (gi == 0) st->rounds_g4 = tot; else if (gi == 1) st->rounds_g16 = tot; else st->rounds_lvl = tot;
					}
				}
			}
			if (out.n) {
				B->per_read[r] = (or_aln1_t*)malloc(out.n * sizeof(or_aln1_t));
				memcpy(B->per_read[r], out.a, out.n * sizeof(or_aln1_t));
			} else B->per_read[r] = 0;
			if (B->touches) B->touches[r] = t;
			if (B->split_touches) B->split_touches[r] = stack->split_pop ? stack->touch_at_split : t;
		}
	}
	free(out.a); free(rseq);
	free(w[0]); free(w[1]); free(sw[0]); free(sw[1]);
	gs_free(stack);
	return 0;
}

int64_t or_cal_sa_reg_gap(const or_bwt_t *bwt0, const or_bwt_t *bwt1, int64_t n_seqs,
                          const uint8_t *seq, const uint64_t *off, const uint32_t *len,
                          const or_gap_opt_t *opt, int n_threads,
                          int32_t *n_aln, or_aln1_t **alns_out, uint32_t *touches_out)
{
	batch_t B;
	int64_t i, tot = 0, p = 0;
	int t;
	pthread_t *tid;
	memset(&B, 0, sizeof(B));
	B.bwt[0] = bwt0; B.bwt[1] = bwt1;
	B.n_seqs = n_seqs; B.seq = seq; B.off = off; B.len = len; B.opt = opt;
	B.n_aln = n_aln; B.touches = touches_out;
	B.stats = g_stats_next;
	g_stats_next = 0;
	B.wtouches = g_wtouch_next;
	g_wtouch_next = 0;
	B.split_pops = g_split_pops_next;
	B.split_touches = g_split_touch_next;
	g_split_pops_next = 0;
	g_split_touch_next = 0;
	B.per_read = (or_aln1_t**)calloc(n_seqs > 0 ? n_seqs : 1, sizeof(or_aln1_t*));
	pthread_mutex_init(&B.lock, 0);
	for (i = 0; i < n_seqs; ++i) if ((int)len[i] > B.max_len) B.max_len = (int)len[i];
	B.base = *opt;
	if (opt->fnr > 0.0) B.base.max_diff = or_cal_maxdiff(B.max_len, 0.02, opt->fnr);
	if (B.base.max_diff < B.base.max_gapo) B.base.max_gapo = B.base.max_diff;
	if (n_threads < 1) n_threads = 1;
	tid = (pthread_t*)calloc(n_threads, sizeof(pthread_t));
	for (t = 0; t < n_threads; ++t) pthread_create(&tid[t], 0, worker, &B);
	for (t = 0; t < n_threads; ++t) pthread_join(tid[t], 0);
	free(tid);
	for (i = 0; i < n_seqs; ++i) tot += n_aln[i];
	*alns_out = (or_aln1_t*)malloc((tot ? tot : 1) * sizeof(or_aln1_t));
	for (i = 0; i < n_seqs; ++i) {
		if (n_aln[i]) memcpy(*alns_out + p, B.per_read[i], n_aln[i] * sizeof(or_aln1_t));
		p += n_aln[i];
		free(B.per_read[i]);
	}
	free(B.per_read);
	pthread_mutex_destroy(&B.lock);
	return tot;
}

/* ======================================================================
 * Smith-Waterman refinement, restating
 * stdaln.c with aln_param_bwa = {gap_open 26, gap_ext 9, gap_end 5,
 * aln_sm_maq, row 5, band 50} (stdaln.c:206-212, :227).  The 32000-score
 * rebasing of the local passes (stdaln.c:581-598, :655-668) is omitted: it is
 * unreachable while min(len1, len2) * 11 <= 32000, which or_aln_local_core
 * requires (returns -2 otherwise).
 * ====================================================================== */
#define SW_Q 26
#define SW_R 9
#define SW_GAP_END 5
#define SW_BAND 50
#define SW_MAXSC 11
#define SW_NEG_INF (-1073741823)
#define SW_M 0
#define SW_I 1
#define SW_D 2
static const int sw_mat[25] = { /* aln_sm_maq (stdaln.c:206-212) */
	 11, -19, -19, -19, -13,
	-19,  11, -19, -19, -13,
	-19, -19,  11, -19, -13,
	-19, -19, -19,  11, -13,
	-13, -13, -13, -13, -13 };

typedef struct { int M, I, D; } sw_cell_t;

/* set_M / set_I / set_D (stdaln.c:271-319): pick the predecessor state, ties as there */
static inline int sw_from_diag(const sw_cell_t *p, int sc, unsigned char *t)
{
	if (p->M >= p->I) {
		if (p->M >= p->D) { *t = SW_M; return p->M + sc; }
		*t = SW_D; return p->D + sc;
	}
	if (p->I > p->D) { *t = SW_I; return p->I + sc; }
	*t = SW_D; return p->D + sc;
}
/* gap state `g` (I or D value of p) opened from p->M or extended; ext = gap_ext or gap_end */
static inline int sw_gap(int pM, int pg, int ext, unsigned char *t)
{
	if (pM - SW_Q > pg) { *t = SW_M; return pM - SW_Q - ext; }
	*t = 1; return pg - ext; /* caller maps 1 to its own state */
}

/* aln_global_core (stdaln.c:345-525): banded global DP, M/I/D, full traceback.
 * seq1 is the i axis (FROM_D steps i), seq2 the j axis (FROM_I steps j). */
int or_aln_global_core(const uint8_t *seq1, int len1, const uint8_t *seq2, int len2,
                       int band_width, int gap_end, or_path_t *path, int *path_len)
{
	int b1, b2, i, j, end, tmp_end, n;
	sw_cell_t *curr, *last, *tswap;
	unsigned char *tM, *tI, *tD; /* traceback per (j, i), full matrix */
	const int W = len1 + 1;
	const int endI = gap_end >= 0 ? gap_end : SW_R; /* set_end_I/D fall back to set_I/D */
	int best, ctype, type;
	if (len1 == 0 || len2 == 0) { *path_len = 0; return 0; }
	if (len1 > len2) { b1 = len1 - len2 + band_width; b2 = band_width; }
	else { b1 = band_width; b2 = len2 - len1 + band_width; }
	if (b1 > len1) b1 = len1;
	if (b2 > len2) b2 = len2;
	tM = (unsigned char*)calloc((size_t)(len2 + 1) * W, 1);
	tI = (unsigned char*)calloc((size_t)(len2 + 1) * W, 1);
	tD = (unsigned char*)calloc((size_t)(len2 + 1) * W, 1);
	curr = (sw_cell_t*)malloc(sizeof(sw_cell_t) * W);
	last = (sw_cell_t*)malloc(sizeof(sw_cell_t) * W);
#define CM(i_, p_, sc_) curr[i_].M = sw_from_diag(p_, sc_, &tM[(size_t)j * W + (i_)])
#define CI(i_, p_, e_) do { unsigned char t_; curr[i_].I = sw_gap((p_)->M, (p_)->I, e_, &t_); tI[(size_t)j * W + (i_)] = t_ == SW_M ? SW_M : SW_I; } while (0)
#define CD(i_, p_, e_) do { unsigned char t_; curr[i_].D = sw_gap((p_)->M, (p_)->D, e_, &t_); tD[(size_t)j * W + (i_)] = t_ == SW_M ? SW_M : SW_D; } while (0)
#define INF(c_) ((c_).M = (c_).I = (c_).D = SW_NEG_INF)
#define SC(i_) sw_mat[seq2[j - 1] * 5 + seq1[(i_) - 1]]
	/* row 0 */
	j = 0;
	INF(curr[0]); curr[0].M = 0;
	for (i = 1; i < b1; ++i) { INF(curr[i]); CD(i, &curr[i - 1], endI); }
	tswap = curr; curr = last; last = tswap;
	/* part 1: rows whose band starts at column 0 */
	tmp_end = b2 < len2 ? b2 : len2 - 1;
	for (j = 1; j <= tmp_end; ++j) {
		INF(curr[0]); CI(0, &last[0], endI);
		end = (j + b1 <= len1 + 1) ? j + b1 - 1 : len1;
		for (i = 1; i != end; ++i) { CM(i, &last[i - 1], SC(i)); CI(i, &last[i], SW_R); CD(i, &curr[i - 1], SW_R); }
		CM(i, &last[i - 1], SC(i)); CD(i, &curr[i - 1], SW_R);
		if (j + b1 - 1 > len1) CI(i, &last[i], endI); else curr[i].I = SW_NEG_INF;
		tswap = curr; curr = last; last = tswap;
	}
	if (j == len2 && b2 != len2 - 1) { /* last row of part 1: end-gap deletions */
		INF(curr[0]); CI(0, &last[0], endI);
		end = (j + b1 <= len1 + 1) ? j + b1 - 1 : len1;
		for (i = 1; i != end; ++i) { CM(i, &last[i - 1], SC(i)); CI(i, &last[i], SW_R); CD(i, &curr[i - 1], endI); }
		CM(i, &last[i - 1], SC(i)); CD(i, &curr[i - 1], endI);
		if (j + b1 - 1 > len1) CI(i, &last[i], endI); else curr[i].I = SW_NEG_INF;
		tswap = curr; curr = last; last = tswap;
		++j;
	}
	/* part 2: bands strictly inside */
	for (; j <= len2 - b2 + 1; ++j) {
		INF(curr[j - b2]);
		end = j + b1 - 1;
		for (i = j - b2 + 1; i != end; ++i) { CM(i, &last[i - 1], SC(i)); CI(i, &last[i], SW_R); CD(i, &curr[i - 1], SW_R); }
		CM(i, &last[i - 1], SC(i)); CD(i, &curr[i - 1], SW_R);
		curr[i].I = SW_NEG_INF;
		tswap = curr; curr = last; last = tswap;
	}
	/* part 3: bands reaching the last column */
	for (; j < len2; ++j) {
		INF(curr[j - b2]);
		for (i = j - b2 + 1; i < len1; ++i) { CM(i, &last[i - 1], SC(i)); CI(i, &last[i], SW_R); CD(i, &curr[i - 1], SW_R); }
		CM(i, &last[len1 - 1], SC(i)); CI(i, &last[i], endI); CD(i, &curr[i - 1], SW_R);
		tswap = curr; curr = last; last = tswap;
	}
	if (j == len2) { /* last row */
		INF(curr[j - b2]);
		for (i = j - b2 + 1; i < len1; ++i) { CM(i, &last[i - 1], SC(i)); CI(i, &last[i], SW_R); CD(i, &curr[i - 1], endI); }
		CM(i, &last[len1 - 1], SC(i)); CI(i, &last[i], endI); CD(i, &curr[i - 1], endI);
		tswap = curr; curr = last; last = tswap;
	}
#undef CM
#undef CI
#undef CD
#undef INF
#undef SC
	/* traceback from (len1, len2) (stdaln.c:487-514) */
	i = len1; j = len2;
	best = last[len1].M; type = tM[(size_t)j * W + i]; ctype = SW_M;
	if (last[len1].I > best) { best = last[len1].I; type = tI[(size_t)j * W + i]; ctype = SW_I; }
	if (last[len1].D > best) { best = last[len1].D; type = tD[(size_t)j * W + i]; ctype = SW_D; }
	n = 0;
	path[n].ctype = (unsigned char)ctype; path[n].i = i; path[n].j = j; ++n;
	do {
		if (ctype == SW_M) { --i; --j; } else if (ctype == SW_I) --j; else --i;
		ctype = type;
		type = ctype == SW_M ? tM[(size_t)j * W + i] : ctype == SW_I ? tI[(size_t)j * W + i] : tD[(size_t)j * W + i];
		path[n].ctype = (unsigned char)ctype; path[n].i = i; path[n].j = j; ++n;
	} while (i || j);
	*path_len = n - 1;
	free(tM); free(tI); free(tD); free(curr); free(last);
	return best;
}

/* aln_local_core (stdaln.c:529-760) with _thres > 0 and no sub-optimal score:
 * forward local pass (packed h<<16|e per seq1 column), banded reverse pass for
 * the start, then the path by aln_global_core with band doubling from 50. */
int or_aln_local_core(const uint8_t *seq1, int len1, const uint8_t *seq2, int len2,
                      or_path_t *path, int *path_len, int thres, int *subo)
{
	const int q = SW_Q, r = SW_R, qr = SW_Q + SW_R, qr_shift = (qr + 1) << 16;
	int32_t *eh;
	int i, j, h, e, f, last_h, score_f = 0, score_r, score_g, end_i = 0, end_j = 0, start_i, start_j, start, end;
	(void)subo;
	if (len1 == 0 || len2 == 0) return -1;
	if ((len1 < len2 ? len1 : len2) * SW_MAXSC > 32000) return -2; /* rebasing not restated */
	if (thres < 0) thres = -thres;
	eh = (int32_t*)calloc(len1 + 2, sizeof(int32_t));
	/* forward pass: row j over seq2, column i over seq1; eh[i-1] = H[j-1][i-1] << 16 | E[j-1][i] */
	for (j = 1; j <= len2; ++j) {
		const int *row = sw_mat + seq2[j - 1] * 5;
		last_h = f = 0;
		for (i = 1; i <= len1; ++i) {
			h = (eh[i - 1] >> 16) + row[seq1[i - 1]];
			if (h < 0) h = 0;
			if (last_h > 0) { /* F: gap along seq1, only after a positive H */
				f = (f > last_h - q) ? f - r : last_h - qr;
				if (h < f) h = f;
			}
			if (eh[i] >= qr_shift) { /* E: gap along seq2, only under an H above q+r */
				const int above = eh[i] >> 16, e_old = eh[i - 1] & 0xffff;
				e = (e_old > above - q) ? e_old - r : above - qr;
				if (h < e) h = e;
				eh[i - 1] = (int32_t)((uint32_t)last_h << 16 | (uint32_t)e);
			} else eh[i - 1] = (int32_t)((uint32_t)last_h << 16);
			last_h = h;
			if (score_f < h) { score_f = h; end_i = i; end_j = j; } /* first maximum in row-major order */
		}
		eh[len1] = (int32_t)((uint32_t)last_h << 16);
	}
	if (score_f < thres) { *path_len = 0; free(eh); return score_f; }
	/* reverse pass from (end_i, end_j) towards the start, in an adaptive band */
	for (i = end_i; i >= 0; --i) eh[i] = 0;
	if (end_i == 0 || end_j == 0) { free(eh); return score_f; }
	score_r = sw_mat[seq1[end_i - 1] * 5 + seq2[end_j - 1]];
	start_i = end_i; start_j = end_j;
	eh[end_i] = (int32_t)((uint32_t)(qr + score_r) << 16);
	start = end_i - 1;
	end = end_i - 3;
	if (end <= 0) end = 0;
	for (j = end_j - 1; j != 0; --j) {
		const int *row = sw_mat + seq2[j - 1] * 5;
		last_h = f = 0;
		for (i = start; i != end; --i) { /* eh[i+1] = H[j+1][i+1] << 16 | E, eh[i] = H above */
			h = (eh[i + 1] >> 16) + row[seq1[i - 1]];
			if (h < 0) h = 0;
			if (last_h > 0) {
				f = (f > last_h - q) ? f - r : last_h - qr;
				if (h < f) h = f;
			}
			{
				const int above = eh[i] >> 16, e_old = eh[i + 1] & 0xffff;
				e = (e_old > above - q) ? e_old - r : above - qr;
				if (e < 0) e = 0;
				if (h < e) h = e;
			}
			eh[i + 1] = (int32_t)((uint32_t)last_h << 16 | (uint32_t)e);
			last_h = h;
			if (score_r < h) {
				score_r = h; start_i = i; start_j = j;
				if (score_r - qr == score_f) { j = 1; break; } /* the start is found */
			}
		}
		eh[i + 1] = (int32_t)((uint32_t)last_h << 16);
		if ((eh[start] >> 16) <= qr) --start;
		if (start <= 0) start = 0;
		end = start_i - (start_j - j) - (score_r + (start_j - j) * SW_MAXSC) / r - 1;
		if (end <= 0) end = 0;
	}
	score_r -= qr;
	/* path: banded global alignment of [start_i, end_i] x [start_j, end_j], band doubling */
	{
		const int span = ((end_i - start_i > end_j - start_j) ? end_i - start_i : end_j - start_j) + 1;
		int bw;
		score_g = 0;
		for (bw = SW_BAND;; bw <<= 1) {
			score_g = or_aln_global_core(seq1 + start_i - 1, end_i - start_i + 1, seq2 + start_j - 1,
			                             end_j - start_j + 1, bw, -1, path, path_len);
			if (score_g == score_r || score_f == score_g) break;
			if (bw > span) break;
		}
		if (score_r > score_g && score_f > score_g) score_f = -1; /* the reference's "potential bug" branch */
		else score_f = score_g;
		for (i = 0; i < *path_len; ++i) { path[i].i += start_i - 1; path[i].j += start_j - 1; }
	}
	free(eh);
	return score_f;
}

/* aln_path2cigar32 (stdaln.c:1010-1040): run-length ops from the start of the path */
int or_path2cigar32(const or_path_t *path, int path_len, uint32_t *cigar)
{
	int i, n;
	if (path_len == 0) return 0;
	cigar[0] = 1u << 4 | path[path_len - 1].ctype;
	for (i = path_len - 2, n = 0; i >= 0; --i) {
		if (path[i].ctype == (cigar[n] & 0xf)) cigar[n] += 1u << 4;
		else cigar[++n] = 1u << 4 | path[i].ctype;
	}
	return n + 1;
}

/* ---------------- SA -> coordinate (bwt.c:69-79, bwtio.c:29-49, dbset.c:240-246) ---------------- */

void or_bwt_info(const or_bwt_t *b, uint32_t *primary, uint32_t *seq_len)
{
	*primary = b->primary;
	*seq_len = b->seq_len;
}

/* bwt_restore_sa (bwtio.c:29-49): header primary, L2[1..4], sa_intv, seq_len, then sa[1..n_sa-1];
 * returns sa[0..n_sa) with sa[0] = (u32)-1, or NULL on a mismatch with the index */
uint32_t *or_sa_load(const char *fn, const or_bwt_t *b, uint32_t *intv, uint64_t *n_sa)
{
	FILE *fp = fopen(fn, "rb");
	uint32_t hdr[7], *sa;
	uint64_t n;
	if (!fp) return 0;
	if (fread(hdr, 4, 7, fp) != 7 || hdr[0] != b->primary || hdr[6] != b->seq_len || hdr[5] == 0) {
		fclose(fp); return 0;
	}
	n = ((uint64_t)b->seq_len + hdr[5]) / hdr[5];
	sa = (uint32_t*)calloc(n, 4);
	sa[0] = (uint32_t)-1;
	if (fread(sa + 1, 4, n - 1, fp) != n - 1) { fclose(fp); free(sa); return 0; }
	fclose(fp);
	*intv = hdr[5];
	*n_sa = n;
	return sa;
}

/* symbol of BWT row r's stored base (bwt_B0, bwt.h:61) */
static inline uint32_t b0(const or_bwt_t *b, uint32_t p)
{
	return b->bwt[p / OCC_INTERVAL * 12 + 4 + p % OCC_INTERVAL / 16] >> ((~p & 0xf) << 1) & 3;
}

/* bwt_invPsi (bwt.h:66-70) */
static inline uint32_t inv_psi(const or_bwt_t *b, uint32_t k)
{
	uint32_t c;
	if (k == b->primary) return 0;
	c = k < b->primary ? b0(b, k) : b0(b, k - 1);
	return b->L2[c] + or_occ(b, k, c);
}

/* bwt_sa (bwt.c:69-79): LF-walk to a sampled row; *steps (optional) += walk length */
uint32_t or_bwt_sa(const or_bwt_t *b, const uint32_t *sa, uint32_t intv, uint32_t k, uint32_t *steps)
{
	uint32_t s = 0;
	while (k % intv != 0) {
		++s;
		k = inv_psi(b, k);
	}
	if (steps) *steps += s;
	return s + sa[k / intv];
}

/* bwtdb_sa2seq (dbset.c:240-246) with db->offset = 0, over a batch:
 * strand 1 -> bwt_sa(bwt[0], k); strand 0 -> bwt[1]->seq_len - (u32)(bwt_sa(bwt[1], k) + len) in u64 (dbset.c:244) */
void or_sa2seq_batch(const or_bwt_t *b0_, const uint32_t *sa0, const or_bwt_t *b1, const uint32_t *sa1,
                     uint32_t intv, int64_t n, const uint8_t *strand, const uint32_t *k, const uint32_t *len,
                     uint64_t *pos, uint32_t *steps)
{
	int64_t i;
	for (i = 0; i < n; ++i) {
		if (strand[i]) pos[i] = or_bwt_sa(b0_, sa0, intv, k[i], steps ? steps + i : 0);
		else pos[i] = (uint64_t)b1->seq_len - (uint32_t)(or_bwt_sa(b1, sa1, intv, k[i], steps ? steps + i : 0) + len[i]);
	}
}
