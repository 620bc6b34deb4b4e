/*
 * lincheck_oracle.c — TEST INFRASTRUCTURE ONLY: the CPU parity oracle and CPU baseline.
 *
 * Plain-C restatement of the reference's analysis path for this suite:
 *   checker/linearizable {:model m :algorithm :linear}    register.clj:109-111, counter.clj:135-137
 *   -> knossos.history preprocessing  [ext, knossos via jepsen 0.3.5, project.clj:11]
 *   -> knossos.linear/analysis        [ext] just-in-time linearization search (Lowe 2017)
 *   -> model step: knossos.model/CASRegister [ext] (register.clj:110), CounterModel
 *      (counter.clj:100-127), LeaderModel (leader.clj:63-75, the :election workload)
 * Knossos is a third-party JVM dependency that is absent from /root/reference and from
 * this image (no JVM, no jar); its published algorithm is restated here. Counter parity is
 * pinned by the reference's KATs (test/jepsen/jgroups/raft_test.clj:6-65); cas-register
 * parity is UNPINNED against Knossos (hand KATs + brute-force permutation checker only).
 *
 * Representation (deliberately different from the product's slot/packed-key layout):
 * pending ops are kept in invocation order in a list; a config is (model value, nil flag,
 * bitmask over list positions). When an op returns, its bit is squeezed out of every
 * config (positions above it shift down by one).
 *
 * explored contract: per RETURN, the number of distinct configs produced by
 * a consistent step during that RETURN's closure (depth >= 1), including the config in
 * which the returning op is linearized (counted before its removal); configs in which the
 * target is linearized are not expanded further.
 */
#include "lincheck_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ model step */

typedef struct {
  int64_t value;
  int32_t nil;
} mstate;

typedef struct {
  int64_t inv_pos, cmp_pos;
  int8_t status; /* 0 none (pending forever), 1 ok, 2 fail, 3 info */
  int8_t f, vflags;
  int64_t v0, v1;
  int32_t pair; /* LeaderModel: the op's (term, leader) pair in the history's ltab */
} oop;

/* LeaderModel: the history's distinct (term, leader) pairs, first appearance first. */
typedef struct {
  int64_t term[64], leader[64];
  int8_t tnil[64];
  int n;
} ltab;

enum { ST_INCONSISTENT = 0, ST_OK = 1, ST_ERROR = -1 };

/* knossos.model/CASRegister.step [ext]; register.clj:16-34 give the value domain.
 * write v -> v; cas [cur new] -> new iff cur = value; read v -> ok iff v nil or v = value. */
static int step_register(mstate s, const oop* o, mstate* out, const char** why) {
  switch (o->f) {
    case OR_F_WRITE:
      if (o->vflags == OR_V_NIL) { out->nil = 1; out->value = 0; }
      else if (o->vflags == OR_V_SCALAR) { out->nil = 0; out->value = o->v0; }
      else { *why = "write with a pair value"; return ST_ERROR; }
      return ST_OK;
    case OR_F_CAS:
      if (o->vflags != OR_V_PAIR) { *why = "cas without [cur new]"; return ST_ERROR; }
      if (s.nil || s.value != o->v0) return ST_INCONSISTENT;
      out->nil = 0; out->value = o->v1;
      return ST_OK;
    case OR_F_READ:
      if (o->vflags == OR_V_NIL) { *out = s; return ST_OK; }
      if (o->vflags != OR_V_SCALAR) { *why = "read with a pair value"; return ST_ERROR; }
      if (s.nil || s.value != o->v0) return ST_INCONSISTENT;
      *out = s;
      return ST_OK;
    default:
      *why = "unknown :f for cas-register";
      return ST_ERROR;
  }
}

/* CounterModel.step, counter.clj:102-127. Clojure +/- throw on long overflow, which makes
 * the checker fail; the oracle reports that as an error (valid? :unknown). */
static int step_counter(mstate s, const oop* o, mstate* out, const char** why) {
  int64_t r;
  out->nil = 0;
  switch (o->f) {
    case OR_F_ADD: /* counter.clj:104 */
      if (o->vflags != OR_V_SCALAR) { *why = ":add needs a scalar delta"; return ST_ERROR; }
      if (__builtin_add_overflow(s.value, o->v0, &r)) { *why = "counter overflow"; return ST_ERROR; }
      out->value = r; return ST_OK;
    case OR_F_DECR: /* counter.clj:106 */
      if (o->vflags != OR_V_SCALAR) { *why = ":decr needs a scalar delta"; return ST_ERROR; }
      if (__builtin_sub_overflow(s.value, o->v0, &r)) { *why = "counter overflow"; return ST_ERROR; }
      out->value = r; return ST_OK;
    case OR_F_READ: /* counter.clj:108-111 */
      if (o->vflags == OR_V_NIL) { out->value = s.value; return ST_OK; }
      if (o->vflags != OR_V_SCALAR) { *why = ":read with a pair value"; return ST_ERROR; }
      if (s.value != o->v0) return ST_INCONSISTENT;
      out->value = s.value; return ST_OK;
    case OR_F_ADD_AND_GET: /* counter.clj:113-119 */
      if (o->vflags == OR_V_PAIR) {
        if (__builtin_add_overflow(s.value, o->v0, &r)) { *why = "counter overflow"; return ST_ERROR; }
        if (r != o->v1) return ST_INCONSISTENT;
        out->value = o->v1; return ST_OK;
      }
      if (o->vflags != OR_V_SCALAR) { *why = ":add-and-get without a delta"; return ST_ERROR; }
      if (__builtin_add_overflow(s.value, o->v0, &r)) { *why = "counter overflow"; return ST_ERROR; }
      out->value = r; return ST_OK;
    case OR_F_DECR_AND_GET: /* counter.clj:121-127 */
      if (o->vflags == OR_V_PAIR) {
        if (__builtin_sub_overflow(s.value, o->v0, &r)) { *why = "counter overflow"; return ST_ERROR; }
        if (r != o->v1) return ST_INCONSISTENT;
        out->value = o->v1; return ST_OK;
      }
      if (o->vflags != OR_V_SCALAR) { *why = ":decr-and-get without a delta"; return ST_ERROR; }
      if (__builtin_sub_overflow(s.value, o->v0, &r)) { *why = "counter overflow"; return ST_ERROR; }
      out->value = r; return ST_OK;
    default:
      *why = "unknown :f for CounterModel"; /* condp throws, counter.clj:102 */
      return ST_ERROR;
  }
}

/* LeaderModel.step, leader.clj:69-75, for (:inspect [leader term]): a map without the term
 * gains (term -> leader); a map holding the term keeps itself when the leaders are equal and is
 * inconsistent otherwise ((empty? state) gives the same map as assoc). The map is kept as the
 * set of its (term, leader) pairs: a bitmask over the history's ltab. Leaders arrive as the
 * caller's ids of serialize-leader's names (nil = "null" = -1, leader.clj:51-54); a nil value
 * destructures to (leader nil, term nil). */
static int step_leader(mstate s, const oop* o, const ltab* L, mstate* out) {
  const int k = o->pair;
  for (uint64_t m = (uint64_t)s.value; m; m &= m - 1) {
    const int q = __builtin_ctzll(m);
    if (L->tnil[q] == L->tnil[k] && L->term[q] == L->term[k] && L->leader[q] != L->leader[k])
      return ST_INCONSISTENT;
  }
  out->nil = 0;
  out->value = (int64_t)((uint64_t)s.value | (1ULL << k));
  return ST_OK;
}

/* ------------------------------------------------------------------ config hash set */

typedef struct {
  uint64_t mask;
  int64_t value;
  int32_t nil;
  int32_t last; /* op linearized last on the way here (-1: none); not part of the key */
} cfg;

typedef struct {
  cfg* keys;
  uint32_t* gen;
  int64_t* pos; /* optional: per slot, the position of the key in a list (the OUT vector) */
  uint32_t cur;
  int64_t cap, count;
} cset;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33; return x;
}
static uint64_t cfg_hash(const cfg* c) {
  return mix64(c->mask * 0x9E3779B97F4A7C15ULL ^ mix64((uint64_t)c->value + (uint64_t)c->nil));
}
static int cset_init2(cset* s, int64_t cap, int with_pos) {
  s->cap = cap; s->count = 0; s->cur = 1;
  s->keys = (cfg*)malloc(sizeof(cfg) * cap);
  s->gen = (uint32_t*)calloc(cap, sizeof(uint32_t));
  s->pos = with_pos ? (int64_t*)malloc(sizeof(int64_t) * cap) : NULL;
  return s->keys && s->gen && (!with_pos || s->pos);
}
static int cset_init(cset* s, int64_t cap) { return cset_init2(s, cap, 0); }
static void cset_free(cset* s) { free(s->keys); free(s->gen); free(s->pos); }
static void cset_clear(cset* s) {
  s->count = 0;
  if (++s->cur == 0) { memset(s->gen, 0, sizeof(uint32_t) * s->cap); s->cur = 1; }
}
static int cset_insert_at(cset* s, const cfg* c, int64_t* at);
static int cset_grow(cset* s) {
  cset n;
  if (!cset_init2(&n, s->cap * 2, s->pos != NULL)) return 0;
  for (int64_t i = 0; i < s->cap; ++i)
    if (s->gen[i] == s->cur) {
      int64_t at;
      cset_insert_at(&n, &s->keys[i], &at);
      if (s->pos) n.pos[at] = s->pos[i];
    }
  cset_free(s);
  *s = n;
  return 1;
}
/* returns 1 if inserted (new), 0 if already present, -1 on OOM; *at = the key's slot */
static int cset_insert_at(cset* s, const cfg* c, int64_t* at) {
  if ((s->count + 1) * 2 > s->cap && !cset_grow(s)) return -1;
  uint64_t m = (uint64_t)s->cap - 1;
  uint64_t h = cfg_hash(c) & m;
  for (;;) {
    if (s->gen[h] != s->cur) {
      s->gen[h] = s->cur; s->keys[h] = *c; s->count++;
      *at = (int64_t)h;
      return 1;
    }
    const cfg* k = &s->keys[h];
    if (k->mask == c->mask && k->value == c->value && k->nil == c->nil) { *at = (int64_t)h; return 0; }
    h = (h + 1) & m;
  }
}
static int cset_insert(cset* s, const cfg* c) {
  int64_t at;
  return cset_insert_at(s, c, &at);
}

typedef struct {
  cfg* v;
  int64_t n, cap;
} cvec;
static int cvec_push(cvec* a, const cfg* c) {
  if (a->n == a->cap) {
    int64_t nc = a->cap ? a->cap * 2 : 64;
    cfg* nv = (cfg*)realloc(a->v, sizeof(cfg) * nc);
    if (!nv) return 0;
    a->v = nv; a->cap = nc;
  }
  a->v[a->n++] = *c;
  return 1;
}

/* squeeze bit p out of a mask: bits above p shift down by one */
static uint64_t squeeze(uint64_t m, int p) {
  uint64_t low = p ? (m & ((1ULL << p) - 1)) : 0;
  uint64_t high = (p >= 63) ? 0 : ((m >> (p + 1)) << p);
  return low | high;
}

/* ------------------------------------------------------------------ process map */

typedef struct {
  int32_t* key;
  int64_t* val;
  uint8_t* used;
  int64_t cap;
} pmap;

static int pmap_init(pmap* m, int64_t n) {
  int64_t cap = 16;
  while (cap < 2 * n + 16) cap <<= 1;
  m->cap = cap;
  m->key = (int32_t*)malloc(sizeof(int32_t) * cap);
  m->val = (int64_t*)malloc(sizeof(int64_t) * cap);
  m->used = (uint8_t*)calloc(cap, 1);
  return m->key && m->val && m->used;
}
static void pmap_free(pmap* m) { free(m->key); free(m->val); free(m->used); }
static int64_t* pmap_slot(pmap* m, int32_t p) {
  uint64_t h = mix64((uint64_t)(uint32_t)p) & (uint64_t)(m->cap - 1);
  while (m->used[h] && m->key[h] != p) h = (h + 1) & (uint64_t)(m->cap - 1);
  if (!m->used[h]) { m->used[h] = 1; m->key[h] = p; m->val[h] = -1; }
  return &m->val[h];
}

/* ------------------------------------------------------------------ search */

static void set_err(oracle_result* r, int code, const char* msg) {
  r->valid = 2;
  r->err_code = code;
  snprintf(r->err, sizeof(r->err), "%s", msg);
}

int32_t oracle_result_size(void) { return (int32_t)sizeof(oracle_result); }

int32_t oracle_check(int32_t model_kind, int64_t init_value, int64_t n, const int64_t* index,
                     const int32_t* process, const int8_t* type, const int8_t* f,
                     const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                     int64_t max_configs, oracle_result* out, int64_t cfg_cap,
                     int64_t* cfg_value, int8_t* cfg_nil, uint64_t* cfg_mask, int64_t* cfg_last) {
  memset(out, 0, sizeof(*out));
  out->valid = 1;
  out->fail_idx = out->fail_inv_idx = out->prev_ok_idx = -1;
  if (model_kind != OR_MODEL_CAS_REGISTER && model_kind != OR_MODEL_COUNTER && model_kind != OR_MODEL_LEADER) {
    set_err(out, -2, "unknown model kind");
    return -2;
  }
#define IDX(pos) (index ? index[(pos)] : (int64_t)(pos))

  /* --- knossos.history preprocessing [ext]: pair each invocation with the next
   * completion of the same process; :ok folds its value into the invocation; :fail drops
   * the pair; :info (or no completion) leaves the invocation pending forever. */
  oop* ops = (oop*)malloc(sizeof(oop) * (n > 0 ? n : 1));
  int64_t* op_of_entry = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
  pmap pm;
  int64_t n_ops = 0;
  int rc = 0;
  if (!ops || !op_of_entry || !pmap_init(&pm, n)) {
    free(ops); free(op_of_entry);
    set_err(out, -3, "out of memory");
    return -3;
  }
  for (int64_t i = 0; i < n && rc == 0; ++i) {
    int64_t* pend = pmap_slot(&pm, process[i]);
    op_of_entry[i] = -1;
    if (type[i] == OR_INVOKE) {
      if (*pend >= 0) { set_err(out, -4, "process invoked while an op was outstanding"); rc = -4; break; }
      oop* o = &ops[n_ops];
      o->inv_pos = i; o->cmp_pos = -1; o->status = 0;
      o->f = f[i]; o->vflags = vflags[i]; o->v0 = v0[i]; o->v1 = v1[i]; o->pair = 0;
      *pend = n_ops; op_of_entry[i] = n_ops; n_ops++;
    } else if (type[i] == OR_OK || type[i] == OR_FAIL || type[i] == OR_INFO) {
      if (*pend < 0) { set_err(out, -4, "completion without an outstanding invocation"); rc = -4; break; }
      oop* o = &ops[*pend];
      o->cmp_pos = i; o->status = type[i];
      if (type[i] == OR_OK) { o->vflags = vflags[i]; o->v0 = v0[i]; o->v1 = v1[i]; }
      op_of_entry[i] = *pend;
      *pend = -1;
    } else {
      set_err(out, -4, "unknown :type");
      rc = -4;
    }
  }
  pmap_free(&pm);
  /* knossos.model.memo [ext] enumerates every op's transition before the search, so an op
   * the model cannot step fails the analysis up front, whether or not the search reaches it.
   * Failed ops never enter the search and are not checked. */
  for (int64_t k = 0; k < n_ops && rc == 0; ++k) {
    const oop* o = &ops[k];
    if (o->status == OR_FAIL) continue;
    const char* why = NULL;
    if (model_kind == OR_MODEL_CAS_REGISTER) {
      if (o->f == OR_F_WRITE && o->vflags == OR_V_PAIR) why = "write with a pair value";
      else if (o->f == OR_F_CAS && o->vflags != OR_V_PAIR) why = "cas without [cur new]";
      else if (o->f == OR_F_READ && o->vflags == OR_V_PAIR) why = "read with a pair value";
      else if (o->f != OR_F_WRITE && o->f != OR_F_CAS && o->f != OR_F_READ) why = "unknown :f for cas-register";
    } else if (model_kind == OR_MODEL_LEADER) {
      if (o->f != OR_F_INSPECT) why = "unknown :f for LeaderModel";
      else if (o->vflags == OR_V_SCALAR) why = ":inspect value is not [leader term]";
    } else {
      if ((o->f == OR_F_ADD || o->f == OR_F_DECR) && o->vflags != OR_V_SCALAR) why = ":add/:decr need a scalar delta";
      else if (o->f == OR_F_READ && o->vflags == OR_V_PAIR) why = ":read with a pair value";
      else if ((o->f == OR_F_ADD_AND_GET || o->f == OR_F_DECR_AND_GET) && o->vflags == OR_V_NIL) why = "*-and-get without a delta";
      else if (o->f < OR_F_READ || o->f > OR_F_DECR_AND_GET || o->f == OR_F_WRITE || o->f == OR_F_CAS) why = "unknown :f for CounterModel";
    }
    if (why) { set_err(out, -6, why); rc = -6; }
  }
  ltab LT;
  LT.n = 0;
  for (int64_t k = 0; k < n_ops && rc == 0 && model_kind == OR_MODEL_LEADER; ++k) {
    oop* o = &ops[k];
    if (o->status == OR_FAIL) continue;
    const int8_t tn = o->vflags == OR_V_NIL;
    const int64_t t = tn ? 0 : o->v1, l = tn ? -1 : o->v0;
    int q = 0;
    while (q < LT.n && !(LT.tnil[q] == tn && LT.term[q] == t && LT.leader[q] == l)) ++q;
    if (q == LT.n) {
      if (LT.n == 64) { set_err(out, -7, "more than 64 distinct (term, leader) pairs (oracle limit)"); rc = -7; break; }
      LT.tnil[q] = tn; LT.term[q] = t; LT.leader[q] = l; LT.n++;
    }
    o->pair = q;
  }
  if (rc) { free(ops); free(op_of_entry); return rc; }

  /* --- knossos.linear/analysis [ext]: reduce over the event stream. */
  int64_t pend_list[64];
  int np = 0;
  cvec F = {0}, L = {0}, NL = {0}, OUT = {0};
  cset S, O;
  /* :last-op per config (only for a failure report, cfg_cap > 0): the op linearized last on the
   * way to it. A RETURN's closure stops where the returning op is linearized, so every config
   * it emits has that op last; a config carried through a RETURN (the op was linearized
   * earlier) keeps its own. Two routes to one config keep the most recent (the closure's). */
  const int track = cfg_cap > 0;
  if (!cset_init(&S, 1024) || !cset_init2(&O, 1024, track)) { set_err(out, -3, "out of memory"); rc = -3; }
  cfg c0 = {0, model_kind == OR_MODEL_LEADER ? 0 : init_value, model_kind == OR_MODEL_CAS_REGISTER ? 1 : 0, -1};
  if (model_kind == OR_MODEL_CAS_REGISTER) c0.value = 0; /* (cas-register) starts at nil */
  if (!rc && !cvec_push(&F, &c0)) rc = -3;
  out->max_frontier = 1;
  int64_t last_ok = -1;

  for (int64_t i = 0; i < n && !rc; ++i) {
    int64_t oi = op_of_entry[i];
    if (oi < 0) continue;
    oop* o = &ops[oi];
    if (type[i] == OR_INVOKE) {
      if (o->status == OR_FAIL) continue; /* failed ops never enter the search */
      if (np == 64) { set_err(out, -5, "more than 64 pending ops"); rc = -5; break; }
      pend_list[np++] = oi;
      continue;
    }
    if (type[i] != OR_OK) continue; /* :info / :fail completions: no-op */

    /* RETURN of op oi: jit-linearizations */
    int p = -1;
    for (int k = 0; k < np; ++k) if (pend_list[k] == oi) { p = k; break; }
    out->n_returns++;
    cset_clear(&S); cset_clear(&O);
    OUT.n = 0; L.n = 0;
    for (int64_t a = 0; a < F.n; ++a) {
      cfg c = F.v[a];
      if (c.mask >> p & 1) {
        c.mask = squeeze(c.mask, p);
        int64_t at;
        int ins = cset_insert_at(&O, &c, &at);
        if (ins < 0) { rc = -3; break; }
        if (ins) {
          if (track) O.pos[at] = OUT.n;
          if (!cvec_push(&OUT, &c)) { rc = -3; break; }
        }
      } else if (!cvec_push(&L, &c)) {
        rc = -3; break;
      }
    }
    while (L.n && !rc) {
      NL.n = 0;
      for (int64_t a = 0; a < L.n && !rc; ++a) {
        const cfg* c = &L.v[a];
        for (int k = 0; k < np; ++k) {
          if (c->mask >> k & 1) continue;
          mstate s = {c->value, c->nil}, s2;
          const char* why = 0;
          int st = model_kind == OR_MODEL_CAS_REGISTER ? step_register(s, &ops[pend_list[k]], &s2, &why)
                   : model_kind == OR_MODEL_LEADER     ? step_leader(s, &ops[pend_list[k]], &LT, &s2)
                                                       : step_counter(s, &ops[pend_list[k]], &s2, &why);
          if (st == ST_ERROR) { set_err(out, -6, why); rc = -6; break; }
          if (st == ST_INCONSISTENT) continue;
          cfg c2 = {c->mask | (1ULL << k), s2.value, s2.nil, (int32_t)pend_list[k]};
          if (model_kind == OR_MODEL_CAS_REGISTER && s2.nil) c2.value = 0;
          int ins = cset_insert(&S, &c2);
          if (ins < 0) { rc = -3; break; }
          if (!ins) continue;
          out->explored++;
          if (k == p) {
            cfg r = c2;
            r.mask = squeeze(r.mask, p);
            int64_t at;
            int ins2 = cset_insert_at(&O, &r, &at);
            if (ins2 < 0) { rc = -3; break; }
            if (ins2) {
              if (track) O.pos[at] = OUT.n;
              if (!cvec_push(&OUT, &r)) { rc = -3; break; }
            } else if (track) {
              OUT.v[O.pos[at]].last = r.last; /* carried through before: the closure's is newer */
            }
          } else if (!cvec_push(&NL, &c2)) {
            rc = -3; break;
          }
          if (max_configs > 0 && (S.count > max_configs || O.count > max_configs)) {
            set_err(out, -7, "max_configs exceeded");
            rc = -7;
            break;
          }
        }
      }
      cvec t = L; L = NL; NL = t;
    }
    if (rc) break;
    if (OUT.n == 0) {
      /* no linearization: report and the pre-failure frontier */
      out->valid = 0;
      out->fail_idx = IDX(i);
      out->fail_inv_idx = IDX(o->inv_pos);
      out->prev_ok_idx = last_ok;
      out->n_fail_cfgs = F.n;
      out->final_frontier = F.n;
      out->n_pending_at_fail = np;
      for (int k = 0; k < np; ++k) out->pending_inv_idx[k] = IDX(ops[pend_list[k]].inv_pos);
      for (int64_t a = 0; a < F.n && a < cfg_cap; ++a) {
        if (cfg_value) cfg_value[a] = F.v[a].value;
        if (cfg_nil) cfg_nil[a] = (int8_t)F.v[a].nil;
        if (cfg_mask) cfg_mask[a] = F.v[a].mask;
        if (cfg_last) cfg_last[a] = F.v[a].last < 0 ? -1 : IDX(ops[F.v[a].last].cmp_pos);
      }
      break;
    }
    cvec t = F; F = OUT; OUT = t;
    for (int k = p; k + 1 < np; ++k) pend_list[k] = pend_list[k + 1];
    np--;
    if (F.n > out->max_frontier) out->max_frontier = F.n;
    last_ok = IDX(i);
  }
  if (out->valid == 1) out->final_frontier = F.n;
  if (rc == -3) set_err(out, -3, "out of memory");
  cset_free(&S); cset_free(&O);
  free(F.v); free(L.v); free(NL.v); free(OUT.v);
  free(ops); free(op_of_entry);
  return rc;
#undef IDX
}

/* ------------------------------------------------------------------ threads over keys */

typedef struct {
  int32_t model_kind, n_hist;
  int64_t init_value, max_configs;
  const int64_t *hist_off, *index, *v0, *v1;
  const int32_t* process;
  const int8_t *type, *f, *vflags;
  oracle_result* out;
  int32_t next; /* shared work counter */
} many_ctx;

static void* many_worker(void* arg) {
  many_ctx* c = (many_ctx*)arg;
  for (;;) {
    int32_t h = __atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (h >= c->n_hist) break;
    int64_t b = c->hist_off[h], e = c->hist_off[h + 1];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oracle_check(c->model_kind, c->init_value, e - b, c->index ? c->index + b : NULL,
                 c->process + b, c->type + b, c->f + b, c->v0 + b, c->v1 + b, c->vflags + b,
                 c->max_configs, &c->out[h], 0, NULL, NULL, NULL, NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    c->out[h].wall_ns = (int64_t)(t1.tv_sec - t0.tv_sec) * 1000000000ll + (t1.tv_nsec - t0.tv_nsec);
  }
  return NULL;
}

int32_t oracle_check_many(int32_t model_kind, int64_t init_value, int32_t n_hist,
                          const int64_t* hist_off, const int64_t* index, const int32_t* process,
                          const int8_t* type, const int8_t* f, const int64_t* v0,
                          const int64_t* v1, const int8_t* vflags, int64_t max_configs,
                          int32_t n_threads, oracle_result* out) {
  many_ctx c = {model_kind, n_hist, init_value, max_configs, hist_off, index, v0, v1,
                process, type, f, vflags, out, 0};
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 512) n_threads = 512;
  pthread_t th[512];
  int started = 0;
  for (int t = 1; t < n_threads; ++t)
    if (pthread_create(&th[started], NULL, many_worker, &c) == 0) started++;
  many_worker(&c);
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* ------------------------------------------------------------------ counter bounds */

/* Sound rejection filter for CounterModel histories.
 * For an observation O (a :read ok of x, or an :add-/:decr-and-get ok [d n], which observes
 * the pre-state n-d / n+d) with invocation at position iO and completion at cO:
 *   A = ops whose :ok completion precedes iO (certainly applied before O),
 *   P = ops invoked before cO, not in A, not O (possibly applied before O).
 *   lo = init + sum_A d + sum_P min(0,d),  hi = init + sum_A d + sum_P max(0,d).
 * Failed ops are dropped; :info ops keep their invocation delta. */
int32_t oracle_counter_bounds(int64_t init_value, int64_t n, const int64_t* index,
                              const int32_t* process, const int8_t* type, const int8_t* f,
                              const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                              int64_t* bad_idx) {
  *bad_idx = -1;
  int64_t* inv_of = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));   /* per completion: its invoke pos */
  int8_t* status = (int8_t*)calloc(n > 0 ? n : 1, 1);                       /* per invoke: completion type */
  int64_t* cmp_of = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));   /* per invoke: completion pos */
  pmap pm;
  pmap_init(&pm, n);
  for (int64_t i = 0; i < n; ++i) {
    int64_t* pend = pmap_slot(&pm, process[i]);
    inv_of[i] = -1; cmp_of[i] = -1;
    if (type[i] == OR_INVOKE) { *pend = i; status[i] = 0; }
    else if (*pend >= 0) { inv_of[i] = *pend; cmp_of[*pend] = i; status[*pend] = type[i]; *pend = -1; }
  }
  pmap_free(&pm);
  /* delta of an op, from its invocation value (+ for add, - for decr) */
#define DELTA(ip) ((f[ip] == OR_F_ADD || f[ip] == OR_F_ADD_AND_GET) ? v0[ip] : \
                   (f[ip] == OR_F_DECR || f[ip] == OR_F_DECR_AND_GET) ? -v0[ip] : 0)
  int64_t CA = 0, CAn = 0, CAp = 0, IN = 0, IP = 0;
  int64_t* pCA = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  int64_t* pCAn = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  int64_t* pCAp = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  int64_t* pIN = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  int64_t* pIP = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  for (int64_t i = 0; i < n; ++i) {
    pCA[i] = CA; pCAn[i] = CAn; pCAp[i] = CAp; pIN[i] = IN; pIP[i] = IP;
    if (type[i] == OR_INVOKE && status[i] != OR_FAIL) {
      int64_t d = DELTA(i);
      IN += d < 0 ? d : 0; IP += d > 0 ? d : 0;
    } else if (type[i] == OR_OK && inv_of[i] >= 0) {
      int64_t d = DELTA(inv_of[i]);
      CA += d; CAn += d < 0 ? d : 0; CAp += d > 0 ? d : 0;
    }
  }
  pCA[n] = CA; pCAn[n] = CAn; pCAp[n] = CAp; pIN[n] = IN; pIP[n] = IP;
  int32_t ok = 1;
  for (int64_t c = 0; c < n; ++c) {
    if (type[c] != OR_OK || inv_of[c] < 0) continue;
    int64_t iv = inv_of[c];
    int64_t x;
    if (f[iv] == OR_F_READ) {
      if (vflags[c] != OR_V_SCALAR) continue;
      x = v0[c];
    } else if ((f[iv] == OR_F_ADD_AND_GET || f[iv] == OR_F_DECR_AND_GET) && vflags[c] == OR_V_PAIR) {
      x = (f[iv] == OR_F_ADD_AND_GET) ? v1[c] - v0[c] : v1[c] + v0[c];
    } else {
      continue;
    }
    int64_t d = DELTA(iv);
    int64_t base = init_value + pCA[iv];
    int64_t lo = base + (pIN[c] - pCAn[iv]) - (d < 0 ? d : 0);
    int64_t hi = base + (pIP[c] - pCAp[iv]) - (d > 0 ? d : 0);
    if (x < lo || x > hi) { ok = 0; *bad_idx = index ? index[c] : c; break; }
  }
#undef DELTA
  free(inv_of); free(status); free(cmp_of);
  free(pCA); free(pCAn); free(pCAp); free(pIN); free(pIP);
  return ok;
}
