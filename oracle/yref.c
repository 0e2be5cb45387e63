/* oracle/yref.c — sequential CPU restatement of Yjs 13.5.16 (+ lib0 0.2.42).
 * TEST INFRASTRUCTURE ONLY — see yref.h for scope and citation conventions.
 *
 * Structure mirrors the Yjs objects the reference manipulates:
 *   lib0 decoding / encoding ........ L0@1937 (readVarUint U, readVarInt T, readVarString E, readAny B)
 *                                      L0@7250 (writeVarUint x, writeVarInt I, writeVarString j, writeAny G)
 *   readClientsStructRefs ........... Y@19286
 *   integrateStructs ................ Y@19963
 *   readAndApplyDeleteSet ........... Y@11619
 *   Item (getMissing/integrate/...).. Y@75928
 *   splitItem ....................... Y@74439 (oi)
 *   struct store helpers ............ Y@29100 (addStruct Un, findIndexSS Ln, getItemCleanStart/End)
 *   transaction cleanup ............. Y@30960 (tryToMergeWithLeft Yn, tryGcDeleteSet zn,
 *                                      tryMergeDeleteSet Bn, cleanupTransactions qn)
 *   DeleteSet ....................... Y@10246 (sortAndMergeDeleteSet le, createDeleteSetFromStructStore ue,
 *                                      writeDeleteSet fe)
 *   encode .......................... Y@18809 (writeStructs Ae, writeClientsStructs ve), Y@22002
 *   contents ........................ Y@68955.. (GC, Binary, Deleted, Doc, Embed, Format, JSON, Any,
 *                                      String, Type)
 */
#define _GNU_SOURCE
#include "yref.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ errors */
static __thread char g_err[256];
static void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char *yo_last_error(void) { return g_err; }
void yo_free(void *p) { free(p); }

static void *xmalloc(size_t n) {
  void *p = malloc(n ? n : 1);
  if (!p) { fprintf(stderr, "yref: out of memory\n"); abort(); }
  return p;
}
static void *xrealloc(void *p, size_t n) {
  p = realloc(p, n ? n : 1);
  if (!p) { fprintf(stderr, "yref: out of memory\n"); abort(); }
  return p;
}
static void *xcalloc(size_t a, size_t b) {
  void *p = calloc(a ? a : 1, b ? b : 1);
  if (!p) { fprintf(stderr, "yref: out of memory\n"); abort(); }
  return p;
}

/* ------------------------------------------------------------------ byte buffer (lib0 encoder) */
typedef struct { uint8_t *p; size_t n, cap; } buf_t;
static void bput(buf_t *b, const void *src, size_t n) {
  if (b->n + n > b->cap) {
    size_t c = b->cap ? b->cap * 2 : 256;
    while (c < b->n + n) c *= 2;
    b->p = xrealloc(b->p, c);
    b->cap = c;
  }
  memcpy(b->p + b->n, src, n);
  b->n += n;
}
static void bu8(buf_t *b, uint8_t v) { bput(b, &v, 1); }
/* writeVarUint L0@7250: 7-bit groups, uint32 semantics */
static void bvu(buf_t *b, uint32_t v) {
  while (v > 127) { bu8(b, (uint8_t)(0x80 | (v & 0x7f))); v >>= 7; }
  bu8(b, (uint8_t)v);
}
static void bvstr(buf_t *b, const uint8_t *s, uint32_t n) { bvu(b, n); bput(b, s, n); }

/* ------------------------------------------------------------------ decoder (lib0 decoding) */
typedef struct { const uint8_t *p; size_t n, pos; int err; } dec_t;
/* readVarUint L0@1937 (U): 32-bit shift-or accumulation; reading past the end or a 6th
 * continuation byte raises "Integer out of range!". */
static uint32_t dvu(dec_t *d) {
  uint32_t v = 0;
  int shift = 0;
  for (;;) {
    if (d->pos >= d->n) { d->err = 1; return 0; }
    uint8_t r = d->p[d->pos++];
    if (shift < 32) v |= (uint32_t)(r & 0x7f) << shift;
    shift += 7;
    if (r < 0x80) return v;
    if (shift > 35) { d->err = 1; return 0; }
  }
}
static uint8_t du8(dec_t *d) {
  if (d->pos >= d->n) { d->err = 1; return 0; }
  return d->p[d->pos++];
}
/* readVarInt (T): returns magnitude & sign separately (we only need to skip / print it). */
static int64_t dvi(dec_t *d) {
  uint8_t r = du8(d);
  uint64_t num = r & 0x3f;
  int shift = 6;
  int neg = (r & 0x40) != 0;
  if (d->err) return 0;
  if (!(r & 0x80)) return neg ? -(int64_t)num : (int64_t)num;
  for (;;) {
    r = du8(d);
    if (d->err) return 0;
    if (shift < 32) num |= (uint64_t)((uint32_t)(r & 0x7f) << shift) & 0xffffffffu;
    shift += 7;
    if (r < 0x80) { num &= 0xffffffffu; return neg ? -(int64_t)num : (int64_t)num; }
    if (shift > 41) { d->err = 1; return 0; }
  }
}
static const uint8_t *dbytes(dec_t *d, uint32_t n) {
  if (d->err || d->n - d->pos < n) { d->err = 1; return NULL; }
  const uint8_t *p = d->p + d->pos;
  d->pos += n;
  return p;
}
/* decodeURIComponent(escape(bytes)) of lib0's readVarString (L0@1937 E): shortest-form UTF-8 of
 * scalar values only; anything else throws URIError (and Y.applyUpdate with it) */
static int utf8_ok(const uint8_t *s, uint32_t n) {
  for (uint32_t i = 0; i < n;) {
    uint32_t c = s[i], need, lo;
    if (c < 0x80) { i++; continue; }
    if ((c & 0xE0) == 0xC0) { need = 1; c &= 0x1F; lo = 0x80; }
    else if ((c & 0xF0) == 0xE0) { need = 2; c &= 0x0F; lo = 0x800; }
    else if ((c & 0xF8) == 0xF0) { need = 3; c &= 0x07; lo = 0x10000; }
    else return 0;
    if (n - i - 1 < need) return 0;
    for (uint32_t j = 1; j <= need; j++) {
      if ((s[i + j] & 0xC0) != 0x80) return 0;
      c = (c << 6) | (s[i + j] & 0x3F);
    }
    if (c < lo || c > 0x10FFFF || (c >= 0xD800 && c <= 0xDFFF)) return 0;
    i += need + 1;
  }
  return 1;
}
/* readVarString: the bytes, checked */
static const uint8_t *dstr(dec_t *d, uint32_t *len) {
  uint32_t k = dvu(d);
  const uint8_t *p = dbytes(d, k);
  if (!d->err && !utf8_ok(p, k)) d->err = 1;
  if (len) *len = k;
  return p;
}
/* skips one lib0 `any` (readAny B) */
static void dskip_any(dec_t *d, int depth) {
  if (depth > 20000) { d->err = 1; return; }  /* lib0 readAny recurses without a limit */
  uint8_t t = du8(d);
  if (d->err) return;
  switch (t) {
    case 127: case 126: case 121: case 120: return;
    case 125: dvi(d); return;
    case 124: dbytes(d, 4); return;
    case 123: case 122: dbytes(d, 8); return;
    case 119: dstr(d, NULL); return;
    case 118: {
      uint32_t n = dvu(d);
      for (uint32_t i = 0; i < n && !d->err; i++) { dstr(d, NULL); dskip_any(d, depth + 1); }
      return;
    }
    case 117: {
      uint32_t n = dvu(d);
      for (uint32_t i = 0; i < n && !d->err; i++) dskip_any(d, depth + 1);
      return;
    }
    case 116: { uint32_t n = dvu(d); dbytes(d, n); return; }
    default: d->err = 1; return;
  }
}

/* ------------------------------------------------------------------ strings & hashing */
typedef struct { uint8_t *p; uint32_t n; } ystr; /* owned bytes */
static ystr ystr_dup(const uint8_t *p, uint32_t n) {
  ystr s;
  s.p = xmalloc(n + 1);
  if (n) memcpy(s.p, p, n);
  s.p[n] = 0;
  s.n = n;
  return s;
}
static uint64_t hbytes(const uint8_t *p, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}
static int ystr_eq(const uint8_t *a, uint32_t an, const uint8_t *b, uint32_t bn) {
  return an == bn && (an == 0 || memcmp(a, b, an) == 0);
}

/* ordered string map (JS Map<string, V> with insertion order) */
typedef struct { ystr key; uint64_t h; void *val; } omap_ent;
typedef struct { omap_ent *e; uint32_t n, cap; int32_t *idx; uint32_t icap; } omap;
static void omap_rehash(omap *m, uint32_t icap) {
  free(m->idx);
  m->idx = xmalloc(sizeof(int32_t) * icap);
  for (uint32_t i = 0; i < icap; i++) m->idx[i] = -1;
  m->icap = icap;
  for (uint32_t i = 0; i < m->n; i++) {
    uint32_t s = (uint32_t)m->e[i].h & (icap - 1);
    while (m->idx[s] >= 0) s = (s + 1) & (icap - 1);
    m->idx[s] = (int32_t)i;
  }
}
static omap_ent *omap_find(omap *m, const uint8_t *k, uint32_t kn) {
  if (!m->icap) return NULL;
  uint64_t h = hbytes(k, kn);
  uint32_t s = (uint32_t)h & (m->icap - 1);
  while (m->idx[s] >= 0) {
    omap_ent *e = &m->e[m->idx[s]];
    if (e->h == h && ystr_eq(e->key.p, e->key.n, k, kn)) return e;
    s = (s + 1) & (m->icap - 1);
  }
  return NULL;
}
static omap_ent *omap_set(omap *m, const uint8_t *k, uint32_t kn, void *val) {
  omap_ent *e = omap_find(m, k, kn);
  if (e) { e->val = val; return e; }
  if (m->n == m->cap) { m->cap = m->cap ? m->cap * 2 : 8; m->e = xrealloc(m->e, sizeof(omap_ent) * m->cap); }
  e = &m->e[m->n++];
  e->key = ystr_dup(k, kn);
  e->h = hbytes(k, kn);
  e->val = val;
  if (m->n * 2 > m->icap) omap_rehash(m, m->icap ? m->icap * 2 : 16);
  else {
    uint32_t s = (uint32_t)e->h & (m->icap - 1);
    while (m->idx[s] >= 0) s = (s + 1) & (m->icap - 1);
    m->idx[s] = (int32_t)(m->n - 1);
  }
  return e;
}
static void omap_free(omap *m) {
  for (uint32_t i = 0; i < m->n; i++) free(m->e[i].key.p);
  free(m->e);
  free(m->idx);
  memset(m, 0, sizeof *m);
}

/* ------------------------------------------------------------------ structs, contents, types */
enum { K_GC = 0, K_ITEM = 1, K_SKIP = 2 };
enum { CT_DELETED = 1, CT_JSON = 2, CT_BINARY = 3, CT_STRING = 4, CT_EMBED = 5, CT_FORMAT = 6, CT_TYPE = 7, CT_ANY = 8, CT_DOC = 9 };
enum { PT_NONE = 0, PT_ROOT = 1, PT_ID = 2, PT_TYPE = 3 };

typedef struct { uint32_t client, clock; } yid;
typedef struct ytype ytype;
typedef struct ys ys;

typedef struct {
  uint8_t ref;
  uint32_t dlen;          /* CT_DELETED */
  ystr *el;               /* CT_ANY / CT_JSON: encoded element bytes */
  uint32_t nel, elcap;
  uint16_t *u16;          /* CT_STRING (UTF-16 code units) */
  uint32_t nu16;
  ystr raw;               /* CT_BINARY/EMBED/FORMAT/DOC: verbatim content bytes */
  ytype *type;            /* CT_TYPE */
} ycontent;

struct ys {
  uint8_t kind;           /* K_GC / K_ITEM / K_SKIP */
  uint8_t deleted, keep, countable;
  yid id;
  uint32_t len;
  ys *left, *right;
  int has_origin, has_rorigin;
  yid origin, rorigin;
  int ptag;               /* parent representation: PT_* */
  ytype *parent;          /* PT_ROOT / PT_TYPE resolved type */
  yid parent_id;          /* PT_ID (unresolved) */
  int has_psub;
  ystr psub;
  ycontent c;
  uint64_t mark_before, mark_conf; /* YATA scan sets (Y@77594 itemsBeforeOrigin / conflictingItems) */
  ys *all_next;           /* ownership list */
};

struct ytype {
  int type_ref;           /* -1 AbstractType (unknown root), 0 Array, 1 Map, 2 Text, 3 XmlElement, 4 XmlFragment, 5 XmlHook, 6 XmlText */
  ystr node_name;         /* XmlElement nodeName / XmlHook hookName (encoded verbatim) */
  ys *start;              /* _start */
  omap map;               /* _map: parentSub -> ys* (insertion ordered) */
  ys *item;               /* _item (NULL for root types) */
  int64_t length;
  ytype *all_next;
};

typedef struct {
  uint32_t client;
  ys **s;
  uint32_t n, cap;
} client_structs;

typedef struct { uint32_t clock, len; } dsitem;
typedef struct { uint32_t client; dsitem *r; uint32_t n, cap; } dsclient;
typedef struct { dsclient *c; uint32_t n, cap; } dset; /* insertion ordered */

struct yo_doc {
  uint32_t client_id;
  int compat;
  omap share;             /* root name -> ytype* */
  client_structs *cl;     /* store.clients (insertion ordered) */
  uint32_t ncl, capcl;
  int32_t *clidx;
  uint32_t clicap;
  ys *all;
  ytype *all_types;
  uint64_t epoch;
  uint64_t rng;
};

static ys *ys_new(yo_doc *d) {
  ys *s = xcalloc(1, sizeof(ys));
  s->all_next = d->all;
  d->all = s;
  return s;
}
static ytype *ytype_new(yo_doc *d, int ref) {
  ytype *t = xcalloc(1, sizeof(ytype));
  t->type_ref = ref;
  t->all_next = d->all_types;
  d->all_types = t;
  return t;
}

/* content helpers -------------------------------------------------------- */
static uint32_t content_len(const ycontent *c) {
  switch (c->ref) {
    case CT_DELETED: return c->dlen;
    case CT_ANY: case CT_JSON: return c->nel;
    case CT_STRING: return c->nu16;
    default: return 1;
  }
}
static int content_countable(const ycontent *c) {
  /* ContentDeleted and ContentFormat are not countable (Y@69588, $r) */
  return !(c->ref == CT_DELETED || c->ref == CT_FORMAT);
}
static void el_push(ycontent *c, ystr s) {
  if (c->nel == c->elcap) { c->elcap = c->elcap ? c->elcap * 2 : 4; c->el = xrealloc(c->el, sizeof(ystr) * c->elcap); }
  c->el[c->nel++] = s;
}
static void content_free(ycontent *c) {
  for (uint32_t i = 0; i < c->nel; i++) free(c->el[i].p);
  free(c->el);
  free(c->u16);
  free(c->raw.p);
  memset(c, 0, sizeof *c);
}
static void content_set_deleted(ycontent *c, uint32_t len) {
  content_free(c);
  c->ref = CT_DELETED;
  c->dlen = len;
}
/* ContentX.splice(offset): keeps [0,off) in c, returns right part (Y@69588.. splice) */
static int content_splice(ycontent *c, uint32_t off, ycontent *right) {
  memset(right, 0, sizeof *right);
  right->ref = c->ref;
  switch (c->ref) {
    case CT_DELETED: right->dlen = c->dlen - off; c->dlen = off; return 0;
    case CT_ANY: case CT_JSON:
      for (uint32_t i = off; i < c->nel; i++) el_push(right, c->el[i]);
      c->nel = off;
      return 0;
    case CT_STRING: {
      right->nu16 = c->nu16 - off;
      right->u16 = xmalloc(sizeof(uint16_t) * (right->nu16 + 1));
      memcpy(right->u16, c->u16 + off, sizeof(uint16_t) * right->nu16);
      c->nu16 = off;
      /* 13.5.16 ContentString.splice: a split surrogate pair becomes U+FFFD on both sides */
      uint16_t hi = off ? c->u16[off - 1] : 0;
      if (hi >= 0xD800 && hi <= 0xDBFF) {
        c->u16[off - 1] = 0xFFFD;
        if (right->nu16) right->u16[0] = 0xFFFD;
      }
      return 0;
    }
    default:
      set_err("Method unimplemented");
      return -1;
  }
}
/* ContentX.mergeWith (mergeable classes: Deleted, JSON, Any, String) */
static int content_merge(ycontent *a, ycontent *b) {
  switch (a->ref) {
    case CT_DELETED: a->dlen += b->dlen; return 1;
    case CT_ANY: case CT_JSON:
      for (uint32_t i = 0; i < b->nel; i++) el_push(a, b->el[i]);
      b->nel = 0;
      return 1;
    case CT_STRING:
      a->u16 = xrealloc(a->u16, sizeof(uint16_t) * (a->nu16 + b->nu16 + 1));
      memcpy(a->u16 + a->nu16, b->u16, sizeof(uint16_t) * b->nu16);
      a->nu16 += b->nu16;
      return 1;
    default: return 0;
  }
}

/* ------------------------------------------------------------------ store */
static client_structs *store_get(yo_doc *d, uint32_t client) {
  if (!d->clicap) return NULL;
  uint32_t h = (client * 2654435761u) & (d->clicap - 1);
  while (d->clidx[h] >= 0) {
    if (d->cl[d->clidx[h]].client == client) return &d->cl[d->clidx[h]];
    h = (h + 1) & (d->clicap - 1);
  }
  return NULL;
}
static void store_rehash(yo_doc *d, uint32_t cap) {
  free(d->clidx);
  d->clidx = xmalloc(sizeof(int32_t) * cap);
  for (uint32_t i = 0; i < cap; i++) d->clidx[i] = -1;
  d->clicap = cap;
  for (uint32_t i = 0; i < d->ncl; i++) {
    uint32_t h = (d->cl[i].client * 2654435761u) & (cap - 1);
    while (d->clidx[h] >= 0) h = (h + 1) & (cap - 1);
    d->clidx[h] = (int32_t)i;
  }
}
static client_structs *store_add_client(yo_doc *d, uint32_t client) {
  if (d->ncl == d->capcl) { d->capcl = d->capcl ? d->capcl * 2 : 8; d->cl = xrealloc(d->cl, sizeof(client_structs) * d->capcl); }
  client_structs *c = &d->cl[d->ncl++];
  memset(c, 0, sizeof *c);
  c->client = client;
  if (d->ncl * 2 > d->clicap) store_rehash(d, d->clicap ? d->clicap * 2 : 16);
  else {
    uint32_t h = (client * 2654435761u) & (d->clicap - 1);
    while (d->clidx[h] >= 0) h = (h + 1) & (d->clicap - 1);
    d->clidx[h] = (int32_t)(d->ncl - 1);
  }
  return c;
}
static void cs_insert(client_structs *c, uint32_t pos, ys *s) {
  if (c->n == c->cap) { c->cap = c->cap ? c->cap * 2 : 8; c->s = xrealloc(c->s, sizeof(ys *) * c->cap); }
  memmove(c->s + pos + 1, c->s + pos, sizeof(ys *) * (c->n - pos));
  c->s[pos] = s;
  c->n++;
}
static void cs_remove(client_structs *c, uint32_t pos) {
  memmove(c->s + pos, c->s + pos + 1, sizeof(ys *) * (c->n - pos - 1));
  c->n--;
}
/* getState (On) */
static uint32_t get_state(yo_doc *d, uint32_t client) {
  client_structs *c = store_get(d, client);
  if (!c || c->n == 0) return 0;
  ys *l = c->s[c->n - 1];
  return l->id.clock + l->len;
}
/* findIndexSS (Ln): index of the struct containing `clock`; -1 ⇒ Yjs throws unexpectedCase */
static int64_t find_index(client_structs *c, uint32_t clock) {
  if (!c || c->n == 0) return -1;
  int64_t lo = 0, hi = (int64_t)c->n - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) / 2;
    ys *s = c->s[mid];
    if (s->id.clock <= clock) {
      if (clock < s->id.clock + s->len) return mid;
      lo = mid + 1;
    } else hi = mid - 1;
  }
  return -1;
}
/* addStruct (Un) */
static int add_struct(yo_doc *d, ys *s) {
  client_structs *c = store_get(d, s->id.client);
  if (!c) c = store_add_client(d, s->id.client);
  else {
    ys *l = c->s[c->n - 1];
    if (l->id.clock + l->len != s->id.clock) { set_err("Unexpected case"); return -1; }
  }
  cs_insert(c, c->n, s);
  return 0;
}
/* getItem (Rn/Tn) */
static ys *get_item(yo_doc *d, yid id) {
  client_structs *c = store_get(d, id.client);
  int64_t i = find_index(c, id.clock);
  return i < 0 ? NULL : c->s[i];
}

/* ------------------------------------------------------------------ transactions & delete sets */
static dsclient *ds_client(dset *ds, uint32_t client, int create) {
  for (uint32_t i = 0; i < ds->n; i++) if (ds->c[i].client == client) return &ds->c[i];
  if (!create) return NULL;
  if (ds->n == ds->cap) { ds->cap = ds->cap ? ds->cap * 2 : 8; ds->c = xrealloc(ds->c, sizeof(dsclient) * ds->cap); }
  dsclient *c = &ds->c[ds->n++];
  memset(c, 0, sizeof *c);
  c->client = client;
  return c;
}
/* addToDeleteSet (ae) */
static void ds_add(dset *ds, uint32_t client, uint32_t clock, uint32_t len) {
  dsclient *c = ds_client(ds, client, 1);
  if (c->n == c->cap) { c->cap = c->cap ? c->cap * 2 : 8; c->r = xrealloc(c->r, sizeof(dsitem) * c->cap); }
  c->r[c->n].clock = clock;
  c->r[c->n].len = len;
  c->n++;
}
static int cmp_dsitem(const void *a, const void *b) {
  const dsitem *x = a, *y = b;
  return x->clock < y->clock ? -1 : x->clock > y->clock;
}
/* sortAndMergeDeleteSet (le, Y@10246). JS Array.sort is stable; ties merge either way. */
static void ds_sort_merge(dset *ds) {
  for (uint32_t k = 0; k < ds->n; k++) {
    dsclient *c = &ds->c[k];
    if (c->n > 1) {
      /* stable insertion-merge sort via qsort on (clock, original index) */
      qsort(c->r, c->n, sizeof(dsitem), cmp_dsitem);
    }
    uint32_t e, n;
    for (e = 1, n = 1; e < c->n; e++) {
      dsitem *s = &c->r[n - 1];
      dsitem r = c->r[e];
      if ((uint64_t)s->clock + s->len >= r.clock) {
        uint64_t ne = (uint64_t)r.clock + r.len - s->clock;
        if (ne > s->len) s->len = (uint32_t)ne;
      } else {
        if (n < e) c->r[n] = r;
        n++;
      }
    }
    if (c->n) c->n = n;
  }
}
static void ds_free(dset *ds) {
  for (uint32_t i = 0; i < ds->n; i++) free(ds->c[i].r);
  free(ds->c);
  memset(ds, 0, sizeof *ds);
}

typedef struct { uint32_t client, clock; } svent;
typedef struct { svent *e; uint32_t n, cap; } svmap; /* insertion ordered Map<client,clock> */
static void sv_set(svmap *m, uint32_t client, uint32_t clock) {
  for (uint32_t i = 0; i < m->n; i++) if (m->e[i].client == client) { m->e[i].clock = clock; return; }
  if (m->n == m->cap) { m->cap = m->cap ? m->cap * 2 : 8; m->e = xrealloc(m->e, sizeof(svent) * m->cap); }
  m->e[m->n].client = client;
  m->e[m->n].clock = clock;
  m->n++;
}
static int sv_get(const svmap *m, uint32_t client, uint32_t *clock) {
  for (uint32_t i = 0; i < m->n; i++) if (m->e[i].client == client) { *clock = m->e[i].clock; return 1; }
  return 0;
}
/* getStateVector (In): store.clients insertion order */
static void get_state_vector(yo_doc *d, svmap *out) {
  out->n = 0;
  for (uint32_t i = 0; i < d->ncl; i++) {
    client_structs *c = &d->cl[i];
    if (!c->n) continue;
    ys *l = c->s[c->n - 1];
    sv_set(out, c->client, l->id.clock + l->len);
  }
}

typedef struct {
  yo_doc *doc;
  dset ds;                /* deleteSet */
  svmap before;           /* beforeState */
  ys **merge;             /* _mergeStructs */
  uint32_t nmerge, capmerge;
  int local;
} txn;

static void txn_push_merge(txn *t, ys *s) {
  if (t->nmerge == t->capmerge) { t->capmerge = t->capmerge ? t->capmerge * 2 : 16; t->merge = xrealloc(t->merge, sizeof(ys *) * t->capmerge); }
  t->merge[t->nmerge++] = s;
}

static void txn_begin(txn *t, yo_doc *d, int local) {
  memset(t, 0, sizeof *t);
  t->doc = d;
  t->local = local;
  get_state_vector(d, &t->before);
}

/* ------------------------------------------------------------------ split / clean start / clean end */
/* splitItem (oi, Y@74439) */
static ys *split_item(txn *t, ys *l, uint32_t diff) {
  ys *r = ys_new(t->doc);
  r->kind = K_ITEM;
  r->id.client = l->id.client;
  r->id.clock = l->id.clock + diff;
  r->left = l;
  r->has_origin = 1;
  r->origin.client = l->id.client;
  r->origin.clock = l->id.clock + diff - 1;
  r->right = l->right;
  r->has_rorigin = l->has_rorigin;
  r->rorigin = l->rorigin;
  r->ptag = l->ptag;
  r->parent = l->parent;
  r->parent_id = l->parent_id;
  r->has_psub = l->has_psub;
  if (l->has_psub) r->psub = ystr_dup(l->psub.p, l->psub.n);
  if (content_splice(&l->c, diff, &r->c) < 0) return NULL;
  r->len = content_len(&r->c);
  r->countable = (uint8_t)content_countable(&r->c);
  if (l->deleted) r->deleted = 1;
  if (l->keep) r->keep = 1;
  l->right = r;
  if (r->right) r->right->left = r;
  txn_push_merge(t, r);
  if (r->has_psub && r->right == NULL && r->parent) omap_set(&r->parent->map, r->psub.p, r->psub.n, r);
  l->len = diff;
  return r;
}
/* findIndexCleanStart (Pn) */
static int64_t find_index_clean_start(txn *t, client_structs *c, uint32_t clock) {
  int64_t i = find_index(c, clock);
  if (i < 0) return -1;
  ys *s = c->s[i];
  if (s->id.clock < clock && s->kind == K_ITEM) {
    ys *r = split_item(t, s, clock - s->id.clock);
    if (!r) return -1;
    cs_insert(c, (uint32_t)i + 1, r);
    return i + 1;
  }
  return i;
}
/* getItemCleanStart (Vn) */
static ys *get_item_clean_start(txn *t, yid id) {
  client_structs *c = store_get(t->doc, id.client);
  int64_t i = find_index_clean_start(t, c, id.clock);
  return i < 0 ? NULL : c->s[i];
}
/* getItemCleanEnd (Fn) */
static ys *get_item_clean_end(txn *t, yid id) {
  client_structs *c = store_get(t->doc, id.client);
  int64_t i = find_index(c, id.clock);
  if (i < 0) return NULL;
  ys *s = c->s[i];
  if (id.clock != s->id.clock + s->len - 1 && s->kind != K_GC) {
    ys *r = split_item(t, s, id.clock - s->id.clock + 1);
    if (!r) return NULL;
    cs_insert(c, (uint32_t)i + 1, r);
  }
  return s;
}
/* replaceStruct ($n) */
static void replace_struct(yo_doc *d, ys *old, ys *nw) {
  client_structs *c = store_get(d, old->id.client);
  int64_t i = find_index(c, old->id.clock);
  c->s[i] = nw;
}

static yid last_id(const ys *s) {
  yid r = s->id;
  r.clock += s->len - 1;
  return r;
}
static int id_eq(int ha, yid a, int hb, yid b) {
  if (!ha || !hb) return ha == hb;
  return a.client == b.client && a.clock == b.clock;
}

/* ------------------------------------------------------------------ delete / gc */
static void item_delete(txn *t, ys *s);
/* ContentType.delete (ni.delete) */
static void type_delete_children(txn *t, ytype *ty) {
  for (ys *e = ty->start; e; e = e->right) {
    if (!e->deleted) item_delete(t, e);
    else txn_push_merge(t, e);
  }
  for (uint32_t i = 0; i < ty->map.n; i++) {
    ys *e = ty->map.e[i].val;
    if (!e->deleted) item_delete(t, e);
    else txn_push_merge(t, e);
  }
}
/* Item.delete */
static void item_delete(txn *t, ys *s) {
  if (s->deleted) return;
  ytype *p = s->parent;
  if (s->countable && !s->has_psub && p) p->length -= s->len;
  s->deleted = 1;
  ds_add(&t->ds, s->id.client, s->id.clock, s->len);
  if (s->c.ref == CT_TYPE && s->c.type) type_delete_children(t, s->c.type);
}
static void item_gc(yo_doc *d, ys *s, int parent_gcd);
/* ContentType.gc */
static void type_gc(yo_doc *d, ytype *ty) {
  ys *e = ty->start;
  while (e) { ys *nx = e->right; item_gc(d, e, 1); e = nx; }
  ty->start = NULL;
  for (uint32_t i = 0; i < ty->map.n; i++) {
    ys *e2 = ty->map.e[i].val;
    while (e2) { ys *lf = e2->left; item_gc(d, e2, 1); e2 = lf; }
  }
  omap_free(&ty->map);
}
/* Item.gc */
static void item_gc(yo_doc *d, ys *s, int parent_gcd) {
  if (s->kind != K_ITEM) return;
  if (s->c.ref == CT_TYPE && s->c.type) type_gc(d, s->c.type);
  if (parent_gcd) {
    ys *g = ys_new(d);
    g->kind = K_GC;
    g->deleted = 1;
    g->id = s->id;
    g->len = s->len;
    replace_struct(d, s, g);
  } else {
    content_set_deleted(&s->c, s->len);
  }
}

/* ------------------------------------------------------------------ Item.getMissing / integrate */
static ytype *root_type(yo_doc *d, const uint8_t *name, uint32_t n) {
  omap_ent *e = omap_find(&d->share, name, n);
  if (e) return e->val;
  ytype *t = ytype_new(d, -1);
  omap_set(&d->share, name, n, t);
  return t;
}

/* returns missing client or -1 (none); -2 on error */
static int64_t get_missing(txn *t, ys *s) {
  yo_doc *d = t->doc;
  if (s->has_origin && s->origin.client != s->id.client && s->origin.clock >= get_state(d, s->origin.client)) return s->origin.client;
  if (s->has_rorigin && s->rorigin.client != s->id.client && s->rorigin.clock >= get_state(d, s->rorigin.client)) return s->rorigin.client;
  if (s->ptag == PT_ID && s->id.client != s->parent_id.client && s->parent_id.clock >= get_state(d, s->parent_id.client)) return s->parent_id.client;
  if (s->has_origin) {
    s->left = get_item_clean_end(t, s->origin);
    if (!s->left) { set_err("Unexpected case"); return -2; }
    s->origin = last_id(s->left);
  }
  if (s->has_rorigin) {
    s->right = get_item_clean_start(t, s->rorigin);
    if (!s->right) { set_err("Unexpected case"); return -2; }
    s->rorigin = s->right->id;
  }
  if ((s->left && s->left->kind == K_GC) || (s->right && s->right->kind == K_GC)) {
    s->ptag = PT_NONE;
    s->parent = NULL;
  }
  if (s->ptag == PT_NONE) {
    if (s->left && s->left->kind == K_ITEM) {
      s->ptag = s->left->parent ? PT_TYPE : PT_NONE;
      s->parent = s->left->parent;
      if (s->has_psub) free(s->psub.p);
      s->has_psub = s->left->has_psub;
      if (s->left->has_psub) s->psub = ystr_dup(s->left->psub.p, s->left->psub.n);
    }
    if (s->right && s->right->kind == K_ITEM) {
      s->ptag = s->right->parent ? PT_TYPE : PT_NONE;
      s->parent = s->right->parent;
      if (s->has_psub) free(s->psub.p);
      s->has_psub = s->right->has_psub;
      if (s->right->has_psub) s->psub = ystr_dup(s->right->psub.p, s->right->psub.n);
    }
  } else if (s->ptag == PT_ID) {
    ys *pi = get_item(d, s->parent_id);
    if (!pi) { set_err("Unexpected case"); return -2; }
    if (pi->kind == K_GC || pi->c.ref != CT_TYPE) {
      /* GC parent, or a ContentDeleted former type item: `content.type` is undefined */
      s->ptag = PT_NONE;
      s->parent = NULL;
    } else {
      s->ptag = PT_TYPE;
      s->parent = pi->c.type;
    }
  }
  return -1;
}

static void gc_integrate(txn *t, ys *g, uint32_t offset) {
  if (offset > 0) { g->id.clock += offset; g->len -= offset; }
  add_struct(t->doc, g);
}

/* Item.integrate (Y@77594) */
static int item_integrate(txn *t, ys *s, uint32_t offset) {
  yo_doc *d = t->doc;
  if (offset > 0) {
    s->id.clock += offset;
    yid lid = { s->id.client, s->id.clock - 1 };
    s->left = get_item_clean_end(t, lid);
    if (!s->left) { set_err("Unexpected case"); return -1; }
    s->has_origin = 1;
    s->origin = last_id(s->left);
    ycontent right;
    if (content_splice(&s->c, offset, &right) < 0) return -1;
    content_free(&s->c);
    s->c = right;
    s->len -= offset;
  }
  if (s->parent) {
    ytype *p = s->parent;
    if ((!s->left && (!s->right || s->right->left != NULL)) || (s->left && s->left->right != s->right)) {
      ys *left = s->left;
      ys *o;
      if (left) o = left->right;
      else if (s->has_psub) {
        omap_ent *e = omap_find(&p->map, s->psub.p, s->psub.n);
        o = e ? e->val : NULL;
        while (o && o->left) o = o->left;
      } else o = p->start;
      uint64_t before = ++d->epoch;
      uint64_t conf = ++d->epoch;
      while (o && o != s->right) {
        o->mark_before = before;
        o->mark_conf = conf;
        if (id_eq(s->has_origin, s->origin, o->has_origin, o->origin)) {
          if (o->id.client < s->id.client) {
            left = o;
            conf = ++d->epoch;
          } else if (id_eq(s->has_rorigin, s->rorigin, o->has_rorigin, o->rorigin)) {
            break;
          }
        } else if (o->has_origin) {
          ys *oo = get_item(d, o->origin);
          if (oo && oo->mark_before == before) {
            if (oo->mark_conf != conf) {
              left = o;
              conf = ++d->epoch;
            }
          } else break;
        } else break;
        o = o->right;
      }
      s->left = left;
    }
    if (s->left) {
      ys *r = s->left->right;
      s->right = r;
      s->left->right = s;
    } else {
      ys *r;
      if (s->has_psub) {
        omap_ent *e = omap_find(&p->map, s->psub.p, s->psub.n);
        r = e ? e->val : NULL;
        while (r && r->left) r = r->left;
      } else {
        r = p->start;
        p->start = s;
      }
      s->right = r;
    }
    if (s->right) s->right->left = s;
    else if (s->has_psub) {
      omap_set(&p->map, s->psub.p, s->psub.n, s);
      if (s->left) item_delete(t, s->left);
    }
    if (!s->has_psub && s->countable && !s->deleted) p->length += s->len;
    if (add_struct(d, s) < 0) return -1;
    /* content.integrate: ContentDeleted marks deleted & records in the txn delete set;
     * ContentType binds the type to this item (Y@73441 _integrate). */
    if (s->c.ref == CT_DELETED) {
      ds_add(&t->ds, s->id.client, s->id.clock, s->c.dlen);
      s->deleted = 1;
    } else if (s->c.ref == CT_TYPE && s->c.type) {
      s->c.type->item = s;
    }
    if ((p->item && p->item->deleted) || (s->has_psub && s->right)) item_delete(t, s);
  } else {
    /* parent unknown: integrate a GC struct in its place */
    ys *g = ys_new(d);
    g->kind = K_GC;
    g->deleted = 1;
    g->id = s->id;
    g->len = s->len;
    gc_integrate(t, g, 0);
  }
  return 0;
}

/* ------------------------------------------------------------------ decode (readClientsStructRefs Y@19286) */
typedef struct { uint32_t client; ys **refs; uint32_t n, i; } refs_t;
typedef struct { refs_t *r; uint32_t n, cap; } clients_refs;

static refs_t *cr_get(clients_refs *cr, uint32_t client) {
  for (uint32_t k = 0; k < cr->n; k++) if (cr->r[k].client == client) return &cr->r[k];
  return NULL;
}

static uint16_t *utf8_to_utf16(const uint8_t *s, uint32_t n, uint32_t *out_n, int *bad) {
  uint16_t *o = xmalloc(sizeof(uint16_t) * (n + 1));
  uint32_t k = 0;
  for (uint32_t i = 0; i < n;) {
    uint32_t c = s[i];
    uint32_t extra = 0;
    if (c < 0x80) extra = 0;
    else if ((c & 0xE0) == 0xC0) { c &= 0x1F; extra = 1; }
    else if ((c & 0xF0) == 0xE0) { c &= 0x0F; extra = 2; }
    else if ((c & 0xF8) == 0xF0) { c &= 0x07; extra = 3; }
    else { *bad = 1; c = 0xFFFD; }
    i++;
    for (uint32_t j = 0; j < extra; j++) {
      if (i >= n || (s[i] & 0xC0) != 0x80) { *bad = 1; break; }
      c = (c << 6) | (s[i] & 0x3F);
      i++;
    }
    if (c >= 0x10000) {
      c -= 0x10000;
      o[k++] = (uint16_t)(0xD800 + (c >> 10));
      o[k++] = (uint16_t)(0xDC00 + (c & 0x3FF));
    } else o[k++] = (uint16_t)c;
  }
  *out_n = k;
  return o;
}
static void utf16_to_utf8(buf_t *b, const uint16_t *u, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    uint32_t c = u[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && u[i + 1] >= 0xDC00 && u[i + 1] <= 0xDFFF) {
      c = 0x10000 + ((c - 0xD800) << 10) + (u[i + 1] - 0xDC00);
      i++;
    } else if (c >= 0xD800 && c <= 0xDFFF) c = 0xFFFD; /* lone surrogate (Yjs would throw) */
    uint8_t t[4];
    if (c < 0x80) { t[0] = (uint8_t)c; bput(b, t, 1); }
    else if (c < 0x800) { t[0] = (uint8_t)(0xC0 | (c >> 6)); t[1] = (uint8_t)(0x80 | (c & 0x3F)); bput(b, t, 2); }
    else if (c < 0x10000) { t[0] = (uint8_t)(0xE0 | (c >> 12)); t[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); t[2] = (uint8_t)(0x80 | (c & 0x3F)); bput(b, t, 3); }
    else { t[0] = (uint8_t)(0xF0 | (c >> 18)); t[1] = (uint8_t)(0x80 | ((c >> 12) & 0x3F)); t[2] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); t[3] = (uint8_t)(0x80 | (c & 0x3F)); bput(b, t, 4); }
  }
}

/* JSON.parse(readString()) of ContentJSON / ContentEmbed / ContentFormat values throws in Yjs on
 * text that cannot start a JSON value (and on the empty string): treat as a decode error. */
static int json_start_ok(const uint8_t *p, uint32_t k) {
  if (k == 0) return 0;
  uint8_t c = p[0];
  return c == '{' || c == '[' || c == '"' || c == 't' || c == 'f' || c == 'n' || c == 'u' || c == '-' ||
         (c >= '0' && c <= '9') || c == ' ' || c == '\t' || c == '\n' || c == '\r';
}

/* readItemContent (hi / ai table) */
static int read_content(yo_doc *doc, dec_t *d, uint8_t info, ycontent *c) {
  memset(c, 0, sizeof *c);
  c->ref = info & 31;
  size_t st;
  switch (c->ref) {
    case CT_DELETED: c->dlen = dvu(d); break;
    case CT_JSON: {
      uint32_t n = dvu(d);
      for (uint32_t i = 0; i < n && !d->err; i++) {
        st = d->pos;
        uint32_t k;
        const uint8_t *js = dstr(d, &k);
        if (!d->err && !json_start_ok(js, k)) d->err = 1;
        if (!d->err) el_push(c, ystr_dup(d->p + st, (uint32_t)(d->pos - st)));
      }
      break;
    }
    case CT_BINARY: case CT_EMBED: {
      st = d->pos;
      uint32_t k;
      const uint8_t *js = c->ref == CT_EMBED ? dstr(d, &k) : (k = dvu(d), dbytes(d, k));
      if (!d->err && c->ref == CT_EMBED && !json_start_ok(js, k)) d->err = 1;
      if (!d->err) c->raw = ystr_dup(d->p + st, (uint32_t)(d->pos - st));
      break;
    }
    case CT_STRING: {
      uint32_t k;
      const uint8_t *s = dstr(d, &k);
      if (!d->err) {
        int bad = 0;
        c->u16 = utf8_to_utf16(s, k, &c->nu16, &bad);
        if (bad) d->err = 1; /* decodeURIComponent(escape(...)) throws on invalid UTF-8 */
      }
      break;
    }
    case CT_FORMAT: {
      st = d->pos;
      uint32_t k;
      dstr(d, NULL);
      const uint8_t *js = dstr(d, &k);
      if (!d->err && !json_start_ok(js, k)) d->err = 1;
      if (!d->err) c->raw = ystr_dup(d->p + st, (uint32_t)(d->pos - st));
      break;
    }
    case CT_TYPE: {
      uint32_t tr = dvu(d);
      ytype *t = ytype_new(doc, (int)tr);
      if (tr == 3 || tr == 5) {
        st = d->pos;
        dstr(d, NULL);
        if (!d->err) t->node_name = ystr_dup(d->p + st, (uint32_t)(d->pos - st));
      } else if (tr > 6) d->err = 1;
      c->type = t;
      break;
    }
    case CT_ANY: {
      uint32_t n = dvu(d);
      for (uint32_t i = 0; i < n && !d->err; i++) {
        st = d->pos;
        dskip_any(d, 0);
        if (!d->err) el_push(c, ystr_dup(d->p + st, (uint32_t)(d->pos - st)));
      }
      break;
    }
    case CT_DOC: {
      st = d->pos;
      dstr(d, NULL);
      dskip_any(d, 0);
      if (!d->err) c->raw = ystr_dup(d->p + st, (uint32_t)(d->pos - st));
      break;
    }
    default: d->err = 1; break;
  }
  return d->err ? -1 : 0;
}

static int read_structs(yo_doc *doc, dec_t *d, clients_refs *cr) {
  uint32_t nclients = dvu(d);
  for (uint32_t ci = 0; ci < nclients && !d->err; ci++) {
    uint32_t nstructs = dvu(d);
    uint32_t client = dvu(d);
    uint32_t clock = dvu(d);
    if (d->err) break;
    if (nstructs > d->n - d->pos) { d->err = 1; break; }
    refs_t *r = cr_get(cr, client);
    if (!r) {
      if (cr->n == cr->cap) { cr->cap = cr->cap ? cr->cap * 2 : 8; cr->r = xrealloc(cr->r, sizeof(refs_t) * cr->cap); }
      r = &cr->r[cr->n++];
      memset(r, 0, sizeof *r);
      r->client = client;
    } else {
      /* Map.set replaces an earlier section of the same client */
      r->n = 0;
      r->i = 0;
    }
    r->refs = xrealloc(r->refs, sizeof(ys *) * (nstructs ? nstructs : 1));
    for (uint32_t i = 0; i < nstructs && !d->err; i++) {
      uint8_t info = du8(d);
      if (d->err) break;
      ys *s = ys_new(doc);
      s->id.client = client;
      s->id.clock = clock;
      switch (info & 31) {
        case 0: s->kind = K_GC; s->deleted = 1; s->len = dvu(d); break;
        case 10: s->kind = K_SKIP; s->deleted = 1; s->len = dvu(d); break;
        default: {
          s->kind = K_ITEM;
          int cant_copy_parent = (info & 0xC0) == 0;
          if (info & 0x80) { s->has_origin = 1; s->origin.client = dvu(d); s->origin.clock = dvu(d); }
          if (info & 0x40) { s->has_rorigin = 1; s->rorigin.client = dvu(d); s->rorigin.clock = dvu(d); }
          if (cant_copy_parent) {
            uint32_t pinfo = dvu(d);
            if (pinfo == 1) {
              uint32_t k;
              const uint8_t *nm = dstr(d, &k);
              if (!d->err) { s->ptag = PT_ROOT; s->parent = root_type(doc, nm, k); }
            } else {
              s->ptag = PT_ID;
              s->parent_id.client = dvu(d);
              s->parent_id.clock = dvu(d);
            }
            if (info & 0x20) {
              uint32_t k;
              const uint8_t *ps = dstr(d, &k);
              if (!d->err) { s->has_psub = 1; s->psub = ystr_dup(ps, k); }
            }
          }
          if (read_content(doc, d, info, &s->c) < 0) break;
          /* own-client references at or past the item's clock: Yjs takes them as present
           * (getMissing) and fails to find them (a TypeError in integrateStructs): refused */
          if ((s->has_origin && s->origin.client == client && s->origin.clock >= clock) ||
              (s->has_rorigin && s->rorigin.client == client && s->rorigin.clock >= clock) ||
              (cant_copy_parent && s->ptag == PT_ID && s->parent_id.client == client && s->parent_id.clock >= clock)) {
            d->err = 1;
            break;
          }
          s->len = content_len(&s->c);
          s->countable = (uint8_t)content_countable(&s->c);
          break;
        }
      }
      if (d->err) break;
      r->refs[r->n++] = s;
      clock += s->len;
    }
  }
  return d->err ? -1 : 0;
}

/* ------------------------------------------------------------------ integrateStructs (Y@19963) */
static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return x < y ? -1 : x > y;
}

static int integrate_structs(txn *t, clients_refs *cr, int *pending) {
  yo_doc *d = t->doc;
  uint32_t nids = cr->n;
  uint32_t *ids = xmalloc(sizeof(uint32_t) * (nids + 1));
  for (uint32_t k = 0; k < cr->n; k++) ids[k] = cr->r[k].client;
  qsort(ids, nids, sizeof(uint32_t), cmp_u32);
  ys **stack = NULL;
  uint32_t nstack = 0, capstack = 0;
  svmap state = { 0 };
  int rc = 0;
  *pending = 0;
#define NEXT_TARGET(out)                                                  \
  do {                                                                    \
    out = NULL;                                                           \
    while (nids > 0) {                                                    \
      refs_t *tt = cr_get(cr, ids[nids - 1]);                             \
      if (tt && tt->n != tt->i) { out = tt; break; }                      \
      nids--;                                                             \
    }                                                                     \
  } while (0)
  refs_t *cur;
  NEXT_TARGET(cur);
  if (!cur) { free(ids); return 0; }
  ys *u = cur->refs[cur->i++];
  for (;;) {
    if (u->kind != K_SKIP) {
      uint32_t local;
      if (!sv_get(&state, u->id.client, &local)) { local = get_state(d, u->id.client); sv_set(&state, u->id.client, local); }
      int64_t offset = (int64_t)local - (int64_t)u->id.clock;
      if (offset < 0) {
        /* gap: the rest of this client's refs would go to pendingStructs */
        *pending = 1;
        break;
      } else {
        int64_t missing = get_missing(t, u);
        if (missing == -2) { rc = -1; break; }
        if (missing >= 0) {
          if (nstack == capstack) { capstack = capstack ? capstack * 2 : 16; stack = xrealloc(stack, sizeof(ys *) * capstack); }
          stack[nstack++] = u;
          refs_t *tt = cr_get(cr, (uint32_t)missing);
          if (!tt || tt->n == tt->i) { *pending = 1; break; }
          u = tt->refs[tt->i++];
          continue;
        } else if (offset == 0 || offset < (int64_t)u->len) {
          if (u->kind == K_GC) gc_integrate(t, u, (uint32_t)offset);
          else if (item_integrate(t, u, (uint32_t)offset) < 0) { rc = -1; break; }
          sv_set(&state, u->id.client, u->id.clock + u->len);
        }
      }
    }
    if (nstack > 0) u = stack[--nstack];
    else if (cur && cur->i < cur->n) u = cur->refs[cur->i++];
    else {
      NEXT_TARGET(cur);
      if (!cur) break;
      u = cur->refs[cur->i++];
    }
  }
#undef NEXT_TARGET
  free(stack);
  free(state.e);
  free(ids);
  return rc;
}

/* ------------------------------------------------------------------ readAndApplyDeleteSet (Y@11619) */
static int read_apply_ds(txn *t, dec_t *d, int *pending) {
  yo_doc *doc = t->doc;
  uint32_t n = dvu(d);
  for (uint32_t i = 0; i < n && !d->err; i++) {
    uint32_t client = dvu(d);
    uint32_t nr = dvu(d);
    if (d->err) break;
    client_structs *c = store_get(doc, client);
    uint32_t state = get_state(doc, client);
    for (uint32_t k = 0; k < nr; k++) {
      uint32_t clock = dvu(d);
      uint32_t len = dvu(d);
      if (d->err) break;
      uint64_t end = (uint64_t)clock + len;
      if (clock < state) {
        if (state < end) *pending = 1;
        int64_t ti = find_index(c, clock);
        if (ti < 0) { set_err("Unexpected case"); return -1; }
        ys *l = c->s[ti];
        if (!l->deleted && l->id.clock < clock) {
          ys *r = split_item(t, l, clock - l->id.clock);
          if (!r) return -1;
          cs_insert(c, (uint32_t)ti + 1, r);
          ti++;
        }
        while ((uint32_t)ti < c->n) {
          l = c->s[ti++];
          if (l->id.clock < end) {
            if (!l->deleted) {
              if (end < (uint64_t)l->id.clock + l->len) {
                ys *r = split_item(t, l, (uint32_t)(end - l->id.clock));
                if (!r) return -1;
                cs_insert(c, (uint32_t)ti, r);
              }
              item_delete(t, l);
            }
          } else break;
        }
      } else if (len > 0) {
        *pending = 1;
      }
    }
  }
  return d->err ? -1 : 0;
}

/* ------------------------------------------------------------------ cleanup (Y@30960..) */
/* Item.mergeWith */
static int item_merge_with(ys *a, ys *b) {
  if (a->kind != b->kind) return 0;
  if (a->kind == K_GC) { a->len += b->len; return 1; }
  yid la = last_id(a);
  if (!(b->has_origin && b->origin.client == la.client && b->origin.clock == la.clock)) return 0;
  if (a->right != b) return 0;
  if (!id_eq(a->has_rorigin, a->rorigin, b->has_rorigin, b->rorigin)) return 0;
  if (a->id.client != b->id.client || a->id.clock + a->len != b->id.clock) return 0;
  if (a->deleted != b->deleted) return 0;
  if (a->c.ref != b->c.ref) return 0;
  if (!content_merge(&a->c, &b->c)) return 0;
  if (b->keep) a->keep = 1;
  a->right = b->right;
  if (a->right) a->right->left = a;
  a->len += b->len;
  return 1;
}
/* tryToMergeWithLeft (Yn) */
static void try_merge_left(client_structs *c, uint32_t pos) {
  ys *l = c->s[pos - 1];
  ys *r = c->s[pos];
  if (l->deleted == r->deleted && l->kind == r->kind) {
    if (item_merge_with(l, r)) {
      cs_remove(c, pos);
      if (r->kind == K_ITEM && r->has_psub && r->parent) {
        omap_ent *e = omap_find(&r->parent->map, r->psub.p, r->psub.n);
        if (e && e->val == r) e->val = l;
      }
    }
  }
}

static void txn_cleanup(txn *t) {
  yo_doc *d = t->doc;
  ds_sort_merge(&t->ds);
  svmap after = { 0 };
  get_state_vector(d, &after);
  /* tryGcDeleteSet (zn) */
  for (uint32_t k = 0; k < t->ds.n; k++) {
    dsclient *dc = &t->ds.c[k];
    client_structs *c = store_get(d, dc->client);
    for (int64_t di = (int64_t)dc->n - 1; di >= 0; di--) {
      dsitem it = dc->r[di];
      uint64_t end = (uint64_t)it.clock + it.len;
      int64_t si = find_index(c, it.clock);
      if (si < 0) continue;
      for (; (uint32_t)si < c->n && c->s[si]->id.clock < end; si++) {
        ys *s = c->s[si];
        if (s->kind == K_ITEM && s->deleted && !s->keep) item_gc(d, s, 0);
      }
    }
  }
  /* tryMergeDeleteSet (Bn) */
  for (uint32_t k = 0; k < t->ds.n; k++) {
    dsclient *dc = &t->ds.c[k];
    client_structs *c = store_get(d, dc->client);
    for (int64_t di = (int64_t)dc->n - 1; di >= 0; di--) {
      dsitem it = dc->r[di];
      int64_t fi = find_index(c, it.clock + it.len - 1);
      int64_t si = (int64_t)c->n - 1;
      if (1 + fi < si) si = 1 + fi;
      for (; si > 0 && c->s[si]->id.clock >= it.clock; si--) try_merge_left(c, (uint32_t)si);
    }
  }
  /* merge changed client ranges (afterState vs beforeState) */
  for (uint32_t k = 0; k < after.n; k++) {
    uint32_t client = after.e[k].client, clock = after.e[k].clock;
    uint32_t bc = 0;
    sv_get(&t->before, client, &bc);
    if (bc != clock) {
      client_structs *c = store_get(d, client);
      int64_t fp = find_index(c, bc);
      if (fp < 1) fp = 1;
      for (int64_t i = (int64_t)c->n - 1; i >= fp; i--) try_merge_left(c, (uint32_t)i);
    }
  }
  /* _mergeStructs */
  for (uint32_t i = 0; i < t->nmerge; i++) {
    yid id = t->merge[i]->id;
    client_structs *c = store_get(d, id.client);
    int64_t p = find_index(c, id.clock);
    if (p < 0) continue;
    if ((uint32_t)(p + 1) < c->n) try_merge_left(c, (uint32_t)p + 1);
    if (p > 0) try_merge_left(c, (uint32_t)p);
  }
  /* remote txn touching our own client id ⇒ Yjs picks a new random client id */
  if (!t->local) {
    uint32_t a = 0, b = 0;
    int ha = sv_get(&after, d->client_id, &a), hb = sv_get(&t->before, d->client_id, &b);
    if (ha != hb || a != b) {
      d->rng = d->rng * 6364136223846793005ull + 1442695040888963407ull;
      d->client_id = (uint32_t)(d->rng >> 32);
    }
  }
  free(after.e);
  ds_free(&t->ds);
  free(t->before.e);
  free(t->merge);
}

/* ------------------------------------------------------------------ public: apply */
yo_doc *yo_doc_new(uint32_t client_id, int compat) {
  yo_doc *d = xcalloc(1, sizeof(yo_doc));
  d->client_id = client_id;
  d->compat = compat == 135 ? 135 : 136;
  d->rng = 0x9E3779B97F4A7C15ull ^ client_id;
  return d;
}
uint32_t yo_client_id(yo_doc *d) { return d->client_id; }

void yo_doc_free(yo_doc *d) {
  if (!d) return;
  for (ys *s = d->all; s;) {
    ys *n = s->all_next;
    content_free(&s->c);
    if (s->has_psub) free(s->psub.p);
    free(s);
    s = n;
  }
  for (ytype *t = d->all_types; t;) {
    ytype *n = t->all_next;
    omap_free(&t->map);
    free(t->node_name.p);
    free(t);
    t = n;
  }
  omap_free(&d->share);
  for (uint32_t i = 0; i < d->ncl; i++) free(d->cl[i].s);
  free(d->cl);
  free(d->clidx);
  free(d);
}

int yo_apply_update(yo_doc *doc, const uint8_t *u, size_t n) {
  dec_t d = { u, n, 0, 0 };
  clients_refs cr = { 0 };
  g_err[0] = 0;
  /* the struct section is decoded completely before anything is integrated (Y@21330) */
  if (read_structs(doc, &d, &cr) < 0) {
    for (uint32_t k = 0; k < cr.n; k++) free(cr.r[k].refs);
    free(cr.r);
    set_err("Integer out of range!");
    return YO_E_DECODE;
  }
  txn t;
  txn_begin(&t, doc, 0);
  int pending = 0, pending_ds = 0;
  int rc = integrate_structs(&t, &cr, &pending);
  if (rc == 0 && !pending) {
    if (read_apply_ds(&t, &d, &pending_ds) < 0) {
      if (!g_err[0]) set_err("Integer out of range!");
      rc = YO_E_DECODE;
    }
  }
  txn_cleanup(&t);
  for (uint32_t k = 0; k < cr.n; k++) free(cr.r[k].refs);
  free(cr.r);
  if (rc < 0) return rc == YO_E_DECODE ? rc : YO_E_INTERNAL;
  if (pending || pending_ds) { set_err("update has missing dependencies (pending)"); return YO_E_PENDING; }
  return YO_OK;
}

/* ------------------------------------------------------------------ encode */
static void write_parent(buf_t *b, yo_doc *d, ys *s) {
  ytype *p = s->parent;
  if (p && p->item == NULL) {
    for (uint32_t i = 0; i < d->share.n; i++) {
      if (d->share.e[i].val == p) {
        bu8(b, 1);
        bvstr(b, d->share.e[i].key.p, d->share.e[i].key.n);
        return;
      }
    }
  } else if (p && p->item) {
    bu8(b, 0);
    bvu(b, p->item->id.client);
    bvu(b, p->item->id.clock);
    return;
  }
  /* unreachable for integrated items */
  bu8(b, 1);
  bvu(b, 0);
}
/* Item.write / GC.write with offset (Y@80416, Y@68955) */
static void write_struct(buf_t *b, yo_doc *d, ys *s, uint32_t off) {
  if (s->kind == K_GC) {
    bu8(b, 0);
    bvu(b, s->len - off);
    return;
  }
  int has_o = off > 0 ? 1 : s->has_origin;
  yid o = s->origin;
  if (off > 0) { o.client = s->id.client; o.clock = s->id.clock + off - 1; }
  uint8_t info = (uint8_t)((s->c.ref & 31) | (has_o ? 0x80 : 0) | (s->has_rorigin ? 0x40 : 0) | (s->has_psub ? 0x20 : 0));
  bu8(b, info);
  if (has_o) { bvu(b, o.client); bvu(b, o.clock); }
  if (s->has_rorigin) { bvu(b, s->rorigin.client); bvu(b, s->rorigin.clock); }
  if (!has_o && !s->has_rorigin) {
    write_parent(b, d, s);
    if (s->has_psub) bvstr(b, s->psub.p, s->psub.n);
  }
  ycontent *c = &s->c;
  switch (c->ref) {
    case CT_DELETED: bvu(b, c->dlen - off); break;
    case CT_ANY: case CT_JSON:
      bvu(b, c->nel - off);
      for (uint32_t i = off; i < c->nel; i++) bput(b, c->el[i].p, c->el[i].n);
      break;
    case CT_STRING: {
      buf_t t = { 0 };
      utf16_to_utf8(&t, c->u16 + off, c->nu16 - off);
      bvstr(b, t.p, (uint32_t)t.n);
      free(t.p);
      break;
    }
    case CT_TYPE:
      bvu(b, (uint32_t)c->type->type_ref);
      if (c->type->node_name.n) bput(b, c->type->node_name.p, c->type->node_name.n);
      break;
    default: bput(b, c->raw.p, c->raw.n); break;
  }
}

typedef struct { uint32_t client, clock; } cc_t;
static int cmp_cc_desc(const void *a, const void *b) {
  const cc_t *x = a, *y = b;
  return x->client > y->client ? -1 : x->client < y->client;
}

static void write_sv_map(buf_t *b, yo_doc *d, svmap *m) {
  cc_t *e = xmalloc(sizeof(cc_t) * (m->n + 1));
  for (uint32_t i = 0; i < m->n; i++) { e[i].client = m->e[i].client; e[i].clock = m->e[i].clock; }
  if (d->compat == 136) qsort(e, m->n, sizeof(cc_t), cmp_cc_desc);
  bvu(b, m->n);
  for (uint32_t i = 0; i < m->n; i++) { bvu(b, e[i].client); bvu(b, e[i].clock); }
  free(e);
}

static int read_sv(const uint8_t *sv, size_t n, svmap *out) {
  dec_t d = { sv, n, 0, 0 };
  uint32_t k = dvu(&d);
  for (uint32_t i = 0; i < k && !d.err; i++) {
    uint32_t c = dvu(&d), cl = dvu(&d);
    if (!d.err) sv_set(out, c, cl);
  }
  return d.err ? -1 : 0;
}

int yo_encode_state_as_update(yo_doc *d, const uint8_t *sv, size_t svlen, uint8_t **out, size_t *outlen) {
  svmap target = { 0 };
  if (sv && svlen && read_sv(sv, svlen, &target) < 0) { free(target.e); set_err("Integer out of range!"); return YO_E_DECODE; }
  buf_t b = { 0 };
  /* writeClientsStructs (ve, Y@19025) */
  svmap sm = { 0 }, cur = { 0 };
  for (uint32_t i = 0; i < target.n; i++)
    if (get_state(d, target.e[i].client) > target.e[i].clock) sv_set(&sm, target.e[i].client, target.e[i].clock);
  get_state_vector(d, &cur);
  for (uint32_t i = 0; i < cur.n; i++) {
    uint32_t x;
    if (!sv_get(&target, cur.e[i].client, &x)) sv_set(&sm, cur.e[i].client, 0);
  }
  bvu(&b, sm.n);
  cc_t *e = xmalloc(sizeof(cc_t) * (sm.n + 1));
  for (uint32_t i = 0; i < sm.n; i++) { e[i].client = sm.e[i].client; e[i].clock = sm.e[i].clock; }
  qsort(e, sm.n, sizeof(cc_t), cmp_cc_desc);
  for (uint32_t i = 0; i < sm.n; i++) {
    client_structs *c = store_get(d, e[i].client);
    uint32_t clock = e[i].clock;
    if (clock < c->s[0]->id.clock) clock = c->s[0]->id.clock;
    int64_t st = find_index(c, clock);
    bvu(&b, c->n - (uint32_t)st);
    bvu(&b, e[i].client);
    bvu(&b, clock);
    write_struct(&b, d, c->s[st], clock - c->s[st]->id.clock);
    for (uint32_t k = (uint32_t)st + 1; k < c->n; k++) write_struct(&b, d, c->s[k], 0);
  }
  free(e);
  /* createDeleteSetFromStructStore (ue) + writeDeleteSet (fe) */
  dset ds = { 0 };
  for (uint32_t i = 0; i < d->ncl; i++) {
    client_structs *c = &d->cl[i];
    for (uint32_t k = 0; k < c->n; k++) {
      ys *s = c->s[k];
      if (s->deleted) {
        uint32_t clock = s->id.clock, len = s->len;
        while (k + 1 < c->n && c->s[k + 1]->deleted) { len += c->s[k + 1]->len; k++; }
        ds_add(&ds, c->client, clock, len);
      }
    }
  }
  uint32_t *order = xmalloc(sizeof(uint32_t) * (ds.n + 1));
  for (uint32_t i = 0; i < ds.n; i++) order[i] = i;
  if (d->compat == 136) {
    for (uint32_t i = 1; i < ds.n; i++) { /* insertion sort by client desc */
      uint32_t x = order[i];
      int64_t j = (int64_t)i - 1;
      while (j >= 0 && ds.c[order[j]].client < ds.c[x].client) { order[j + 1] = order[j]; j--; }
      order[j + 1] = x;
    }
  }
  bvu(&b, ds.n);
  for (uint32_t i = 0; i < ds.n; i++) {
    dsclient *c = &ds.c[order[i]];
    bvu(&b, c->client);
    bvu(&b, c->n);
    for (uint32_t k = 0; k < c->n; k++) { bvu(&b, c->r[k].clock); bvu(&b, c->r[k].len); }
  }
  free(order);
  ds_free(&ds);
  free(sm.e);
  free(cur.e);
  free(target.e);
  *out = b.p;
  *outlen = b.n;
  return YO_OK;
}

int yo_encode_state_vector(yo_doc *d, uint8_t **out, size_t *outlen) {
  buf_t b = { 0 };
  svmap sv = { 0 };
  get_state_vector(d, &sv);
  write_sv_map(&b, d, &sv);
  free(sv.e);
  *out = b.p;
  *outlen = b.n;
  return YO_OK;
}

/* ------------------------------------------------------------------ toJSON (YMap.toJSON Y@51558, YArray.toJSON) */
static void json_str(buf_t *b, const uint8_t *s, uint32_t n) {
  bu8(b, '"');
  for (uint32_t i = 0; i < n; i++) {
    uint8_t c = s[i];
    if (c == '"' || c == '\\') { bu8(b, '\\'); bu8(b, c); }
    else if (c == '\n') bput(b, "\\n", 2);
    else if (c == '\r') bput(b, "\\r", 2);
    else if (c == '\t') bput(b, "\\t", 2);
    else if (c == '\b') bput(b, "\\b", 2);
    else if (c == '\f') bput(b, "\\f", 2);
    else if (c < 0x20) { char t[8]; snprintf(t, sizeof t, "\\u%04x", c); bput(b, t, 6); }
    else bu8(b, c);
  }
  bu8(b, '"');
}
static void json_num(buf_t *b, double v) {
  char t[40];
  if (v != v || v == 1.0 / 0.0 || v == -1.0 / 0.0) { bput(b, "null", 4); return; }
  if (v == (double)(int64_t)v && v > -9e15 && v < 9e15) snprintf(t, sizeof t, "%lld", (long long)(int64_t)v);
  else snprintf(t, sizeof t, "%.17g", v);
  bput(b, t, strlen(t));
}
/* any → JSON text; returns 0 if the value is `undefined` (nothing written) */
static int any_json(buf_t *b, dec_t *d) {
  uint8_t t = du8(d);
  switch (t) {
    case 127: return 0;
    case 126: bput(b, "null", 4); return 1;
    case 125: json_num(b, (double)dvi(d)); return 1;
    case 124: {
      const uint8_t *p = dbytes(d, 4);
      uint32_t x = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
      float f;
      memcpy(&f, &x, 4);
      json_num(b, (double)f);
      return 1;
    }
    case 123: {
      const uint8_t *p = dbytes(d, 8);
      uint64_t x = 0;
      for (int i = 0; i < 8; i++) x = (x << 8) | p[i];
      double f;
      memcpy(&f, &x, 8);
      json_num(b, f);
      return 1;
    }
    case 122: dbytes(d, 8); bput(b, "null", 4); return 1;
    case 121: bput(b, "false", 5); return 1;
    case 120: bput(b, "true", 4); return 1;
    case 119: { uint32_t n = dvu(d); const uint8_t *p = dbytes(d, n); json_str(b, p, n); return 1; }
    case 118: {
      uint32_t n = dvu(d);
      bu8(b, '{');
      int first = 1;
      for (uint32_t i = 0; i < n && !d->err; i++) {
        uint32_t k = dvu(d);
        const uint8_t *kp = dbytes(d, k);
        buf_t v = { 0 };
        if (any_json(&v, d)) {
          if (!first) bu8(b, ',');
          first = 0;
          json_str(b, kp, k);
          bu8(b, ':');
          bput(b, v.p, v.n);
        }
        free(v.p);
      }
      bu8(b, '}');
      return 1;
    }
    case 117: {
      uint32_t n = dvu(d);
      bu8(b, '[');
      for (uint32_t i = 0; i < n && !d->err; i++) {
        if (i) bu8(b, ',');
        if (!any_json(b, d)) bput(b, "null", 4);
      }
      bu8(b, ']');
      return 1;
    }
    case 116: {
      uint32_t n = dvu(d);
      const uint8_t *p = dbytes(d, n);
      bu8(b, '{');
      for (uint32_t i = 0; i < n; i++) { char t2[24]; snprintf(t2, sizeof t2, "%s\"%u\":%u", i ? "," : "", i, p[i]); bput(b, t2, strlen(t2)); }
      bu8(b, '}');
      return 1;
    }
    default: d->err = 1; return 0;
  }
}
static void type_json(buf_t *b, ytype *t, int as_map);
/* JSON of content element `i` of an item; returns 0 for undefined */
static int element_json(buf_t *b, ys *s, uint32_t i) {
  ycontent *c = &s->c;
  switch (c->ref) {
    case CT_ANY: { dec_t d = { c->el[i].p, c->el[i].n, 0, 0 }; return any_json(b, &d); }
    case CT_JSON: {
      dec_t d = { c->el[i].p, c->el[i].n, 0, 0 };
      uint32_t n = dvu(&d);
      const uint8_t *p = dbytes(&d, n);
      if (n == 9 && memcmp(p, "undefined", 9) == 0) return 0;
      bput(b, p, n);
      return 1;
    }
    case CT_BINARY: {
      dec_t d = { c->raw.p, c->raw.n, 0, 0 };
      uint32_t n = dvu(&d);
      const uint8_t *p = dbytes(&d, n);
      bu8(b, '{');
      for (uint32_t k = 0; k < n; k++) { char t2[24]; snprintf(t2, sizeof t2, "%s\"%u\":%u", k ? "," : "", k, p[k]); bput(b, t2, strlen(t2)); }
      bu8(b, '}');
      return 1;
    }
    case CT_TYPE: type_json(b, c->type, c->type->type_ref == 1); return 1;
    case CT_STRING: {
      buf_t t = { 0 };
      utf16_to_utf8(&t, c->u16 + i, 1);
      json_str(b, t.p, (uint32_t)t.n);
      free(t.p);
      return 1;
    }
    default: bput(b, "null", 4); return 1;
  }
}
static void type_json(buf_t *b, ytype *t, int as_map) {
  if (t->type_ref == 2) { /* Y.Text → string */
    buf_t s = { 0 };
    for (ys *e = t->start; e; e = e->right)
      if (!e->deleted && e->c.ref == CT_STRING) utf16_to_utf8(&s, e->c.u16, e->c.nu16);
    json_str(b, s.p, (uint32_t)s.n);
    free(s.p);
    return;
  }
  if (as_map) {
    bu8(b, '{');
    int first = 1;
    for (uint32_t i = 0; i < t->map.n; i++) {
      ys *s = t->map.e[i].val;
      if (s->deleted) continue;
      buf_t v = { 0 };
      if (element_json(&v, s, s->len - 1)) {
        if (!first) bu8(b, ',');
        first = 0;
        json_str(b, t->map.e[i].key.p, t->map.e[i].key.n);
        bu8(b, ':');
        bput(b, v.p, v.n);
      }
      free(v.p);
    }
    bu8(b, '}');
  } else {
    bu8(b, '[');
    int first = 1;
    for (ys *s = t->start; s; s = s->right) {
      if (s->deleted || !s->countable) continue;
      for (uint32_t i = 0; i < s->len; i++) {
        if (!first) bu8(b, ',');
        first = 0;
        if (!element_json(b, s, i)) bput(b, "null", 4);
      }
    }
    bu8(b, ']');
  }
}
int yo_root_json(yo_doc *d, const char *name, int kind, uint8_t **out, size_t *outlen) {
  ytype *t = root_type(d, (const uint8_t *)name, (uint32_t)strlen(name));
  if (t->type_ref < 0) t->type_ref = kind == 0 ? 1 : 0;
  buf_t b = { 0 };
  type_json(&b, t, kind == 0);
  *out = b.p;
  *outlen = b.n;
  return YO_OK;
}

/* ------------------------------------------------------------------ local ops (typeMapSet Y@49334, typeMapDelete, typeListInsertGenerics Y@47498, typeListDelete) */
static int local_finish(txn *t) {
  txn_cleanup(t);
  return YO_OK;
}
static ys *new_local_item(yo_doc *d, ytype *p, ys *left, ys *right) {
  ys *s = ys_new(d);
  s->kind = K_ITEM;
  s->id.client = d->client_id;
  s->id.clock = get_state(d, d->client_id);
  s->left = left;
  if (left) { s->has_origin = 1; s->origin = last_id(left); }
  s->right = right;
  if (right) { s->has_rorigin = 1; s->rorigin = right->id; }
  s->ptag = PT_TYPE;
  s->parent = p;
  return s;
}
int yo_map_set(yo_doc *d, const char *root, const char *key, const uint8_t *any, size_t anylen) {
  ytype *p = root_type(d, (const uint8_t *)root, (uint32_t)strlen(root));
  if (p->type_ref < 0) p->type_ref = 1;
  dec_t chk = { any, anylen, 0, 0 };
  dskip_any(&chk, 0);
  if (chk.err || chk.pos != anylen) { set_err("bad any value"); return YO_E_ARG; }
  txn t;
  txn_begin(&t, d, 1);
  omap_ent *e = omap_find(&p->map, (const uint8_t *)key, (uint32_t)strlen(key));
  ys *left = e ? e->val : NULL;
  ys *s = new_local_item(d, p, left, NULL);
  s->has_psub = 1;
  s->psub = ystr_dup((const uint8_t *)key, (uint32_t)strlen(key));
  s->c.ref = CT_ANY;
  el_push(&s->c, ystr_dup(any, (uint32_t)anylen));
  s->len = 1;
  s->countable = 1;
  int rc = item_integrate(&t, s, 0);
  local_finish(&t);
  return rc < 0 ? YO_E_INTERNAL : YO_OK;
}
int yo_map_delete(yo_doc *d, const char *root, const char *key) {
  ytype *p = root_type(d, (const uint8_t *)root, (uint32_t)strlen(root));
  if (p->type_ref < 0) p->type_ref = 1;
  txn t;
  txn_begin(&t, d, 1);
  omap_ent *e = omap_find(&p->map, (const uint8_t *)key, (uint32_t)strlen(key));
  if (e) item_delete(&t, e->val);
  return local_finish(&t);
}
int yo_array_insert(yo_doc *d, const char *root, uint32_t index, const uint8_t *anys, size_t len, uint32_t count) {
  ytype *p = root_type(d, (const uint8_t *)root, (uint32_t)strlen(root));
  if (p->type_ref < 0) p->type_ref = 0;
  if (index > p->length) { set_err("Length exceeded!"); return YO_E_ARG; }
  txn t;
  txn_begin(&t, d, 1);
  /* typeListInsertGenerics: find the item left of `index`, splitting if needed */
  ys *left = NULL;
  if (index > 0) {
    uint32_t n = index;
    for (ys *o = p->start; o; o = o->right) {
      if (!o->deleted && o->countable) {
        if (n <= o->len) {
          if (n < o->len) { yid id = { o->id.client, o->id.clock + n }; get_item_clean_start(&t, id); }
          left = o;
          break;
        }
        n -= o->len;
      }
    }
  }
  ys *right = left ? left->right : p->start;
  ys *s = new_local_item(d, p, left, right);
  s->c.ref = CT_ANY;
  dec_t dd = { anys, len, 0, 0 };
  for (uint32_t i = 0; i < count; i++) {
    size_t st = dd.pos;
    dskip_any(&dd, 0);
    if (dd.err) { set_err("bad any value"); local_finish(&t); return YO_E_ARG; }
    el_push(&s->c, ystr_dup(anys + st, (uint32_t)(dd.pos - st)));
  }
  s->len = count;
  s->countable = 1;
  int rc = count ? item_integrate(&t, s, 0) : 0;
  local_finish(&t);
  return rc < 0 ? YO_E_INTERNAL : YO_OK;
}
int yo_array_delete(yo_doc *d, const char *root, uint32_t index, uint32_t length) {
  ytype *p = root_type(d, (const uint8_t *)root, (uint32_t)strlen(root));
  if (p->type_ref < 0) p->type_ref = 0;
  if (length == 0) return YO_OK;
  txn t;
  txn_begin(&t, d, 1);
  /* typeListDelete: locate the first item to delete, splitting at `index` */
  ys *o = p->start;
  for (; o && index > 0; o = o->right) {
    if (!o->deleted && o->countable) {
      if (index < o->len) { yid id = { o->id.client, o->id.clock + index }; get_item_clean_start(&t, id); }
      index -= o->len;
    }
  }
  while (length > 0 && o) {
    if (!o->deleted) {
      if (length < o->len) { yid id = { o->id.client, o->id.clock + length }; get_item_clean_start(&t, id); }
      item_delete(&t, o);
      length -= o->len;
    }
    o = o->right;
  }
  local_finish(&t);
  if (length > 0) { set_err("array length exceeded"); return YO_E_ARG; }
  return YO_OK;
}
