/*
 * ie_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline, kind "port").
 *
 * A literal CPU restatement of the reference's `{key}` interpolation hot path. Nothing in the
 * product (interpolation-engine_amd/) links, calls or loads this file; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg do, and only as the checker.
 *
 * Followed line by line (reference @ /root/reference, read as text):
 *   interpolate_inserts     src/interpolation_engine/interpolation_engine.py:497-541
 *                           rust-project/src/interp.rs:31-89           (dialect IE_DIALECT_RS)
 *   get_simple_insertkey    interpolation_engine.py:477-495 / interp.rs:11-29
 *   get_interpdata          interpolation_engine.py:430-467 / interp.rs:91-137
 *   recursive_(un)escape    interpolation_engine.py:1436-1460 / interp.rs:147-177 (string leaves)
 *
 * Python str methods are restated on UTF-8 bytes: every pattern used here ('{', '}', '\\{',
 * '\\}', '.〠', '〠.') is itself valid UTF-8, and UTF-8 is self-synchronising, so byte-level
 * non-overlapping left-to-right replace/count/find/rfind select exactly the code-point-level
 * matches of CPython's str methods.
 *
 * Pinning: checked against tests/golden/*.jsonl, vectors produced by the reference Python module
 * itself (tests/golden/gen_golden.py). The Rust dialect is restated from source only and is
 * "parity unpinned" (no Rust toolchain, and the crate does not build: SURVEY §8c).
 *
 * Deviation, by necessity: the reference loops forever on self-referential inserts (py:516 has no
 * bound); this restatement stops at the IE_ITER_CAP / IE_SIZE_CAP caps of include/ie_amd.h and
 * reports IE_DIVERGED, exactly like the device path.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/ie_amd.h"

/* ------------------------------------------------------------------------------------------ */
/* growable byte string                                                                        */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  char* p;
  size_t n, cap;
} sb;

static void sb_reserve(sb* b, size_t need) {
  if (need <= b->cap) return;
  size_t c = b->cap ? b->cap : 64;
  while (c < need) c *= 2;
  b->p = (char*)realloc(b->p, c);
  b->cap = c;
}
static void sb_put(sb* b, const char* s, size_t n) {
  sb_reserve(b, b->n + n + 1);
  if (n) memcpy(b->p + b->n, s, n);
  b->n += n;
}
static void sb_clear(sb* b) { b->n = 0; }
static void sb_free(sb* b) {
  free(b->p);
  b->p = NULL;
  b->n = b->cap = 0;
}
static void sb_swap(sb* a, sb* b) {
  sb t = *a;
  *a = *b;
  *b = t;
}

/* str.replace(pat, rep): non-overlapping, left to right (CPython semantics) */
static void str_replace(sb* out, const char* s, size_t n, const char* pat, size_t pn,
                        const char* rep, size_t rn) {
  sb_clear(out);
  sb_reserve(out, n + 1);
  size_t i = 0, run = 0;
  while (i + pn <= n) {
    const char* hit = (const char*)memchr(s + i, pat[0], n - pn + 1 - i);
    if (!hit) break;
    i = (size_t)(hit - s);
    if (memcmp(s + i, pat, pn) == 0) {
      sb_put(out, s + run, i - run);
      sb_put(out, rep, rn);
      i += pn;
      run = i;
    } else {
      i++;
    }
  }
  sb_put(out, s + run, n - run);
}

/* str.count(pat), non-overlapping */
static size_t str_count(const char* s, size_t n, const char* pat, size_t pn) {
  size_t c = 0, i = 0;
  while (i + pn <= n) {
    const char* hit = (const char*)memchr(s + i, pat[0], n - pn + 1 - i);
    if (!hit) break;
    i = (size_t)(hit - s);
    if (memcmp(s + i, pat, pn) == 0) {
      c++;
      i += pn;
    } else {
      i++;
    }
  }
  return c;
}

static long str_find(const char* s, size_t n, char c, size_t from) {
  if (from >= n) return -1;
  const char* hit = (const char*)memchr(s + from, c, n - from);
  return hit ? (long)(hit - s) : -1;
}
static long str_rfind(const char* s, size_t n, char c) {
  const char* hit = n ? (const char*)memrchr(s, c, n) : NULL;
  return hit ? (long)(hit - s) : -1;
}

/* constants py:41-43, 500-503 / interp.rs:7-9, 38-41 */
static const char ESC_START[] = "\\{";
static const char ESC_STOP[] = "\\}";
static const char PH_START[] = ".\xE3\x80\xA0"; /* '.〠' */
static const char PH_STOP[] = "\xE3\x80\xA0.";  /* '〠.' */

/* ------------------------------------------------------------------------------------------ */
/* inserts table                                                                              */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  char* key;
  size_t key_len;
  char* text;
  size_t text_len;
  int kind;
  uint32_t vid;
} entry;

typedef struct ieo_ctx {
  int dialect;
  int has_dir;
  entry* e;
  size_t ne;
  uint32_t* slot; /* entry index + 1 */
  size_t cap;
  size_t maxtext;
  char hhmm[8], hhmmss[12];
} ieo_ctx;

static uint64_t fnv(const char* s, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)s[i]) * 1099511628211ull;
  return h;
}

static long ctx_find(const ieo_ctx* c, const char* k, size_t kn) {
  size_t m = c->cap - 1, i = (size_t)fnv(k, kn) & m;
  for (;;) {
    uint32_t s = c->slot[i];
    if (!s) return -1;
    const entry* e = &c->e[s - 1];
    if (e->key_len == kn && memcmp(e->key, k, kn) == 0) return (long)(s - 1);
    i = (i + 1) & m;
  }
}

ieo_ctx* ieo_new(const ie_kv* kv, uint64_t n, int32_t dialect, const ie_clock* now,
                 int32_t has_dir) {
  ieo_ctx* c = (ieo_ctx*)calloc(1, sizeof(ieo_ctx));
  c->dialect = dialect;
  c->has_dir = has_dir;
  c->cap = 16;
  while (c->cap < 2 * n + 2) c->cap *= 2;
  c->slot = (uint32_t*)calloc(c->cap, sizeof(uint32_t));
  c->e = (entry*)calloc(n ? n : 1, sizeof(entry));
  for (uint64_t i = 0; i < n; i++) {
    long at = ctx_find(c, kv[i].key, kv[i].key_len);
    entry* e;
    if (at >= 0) { /* duplicate key: dict semantics, the last one wins */
      e = &c->e[at];
      free(e->key);
      free(e->text);
    } else {
      e = &c->e[c->ne++];
      size_t m = c->cap - 1, j = (size_t)fnv(kv[i].key, kv[i].key_len) & m;
      while (c->slot[j]) j = (j + 1) & m;
      c->slot[j] = (uint32_t)(c->ne);
    }
    e->key = (char*)malloc(kv[i].key_len + 1);
    memcpy(e->key, kv[i].key, kv[i].key_len);
    e->key_len = kv[i].key_len;
    e->text = (char*)malloc(kv[i].text_len + 1);
    memcpy(e->text, kv[i].text, kv[i].text_len);
    e->text_len = kv[i].text_len;
    e->kind = kv[i].kind;
    e->vid = (uint32_t)i;
  }
  c->maxtext = 8; /* the clock strings */
  for (size_t i = 0; i < c->ne; i++)
    if (c->e[i].text_len > c->maxtext) c->maxtext = c->e[i].text_len;
  int h = now ? now->hour : 0, mi = now ? now->minute : 0, s = now ? now->second : 0;
  snprintf(c->hhmm, sizeof c->hhmm, "%02d:%02d", h, mi);
  snprintf(c->hhmmss, sizeof c->hhmmss, "%02d:%02d:%02d", h, mi, s);
  return c;
}

void ieo_free(ieo_ctx* c) {
  if (!c) return;
  for (size_t i = 0; i < c->ne; i++) {
    free(c->e[i].key);
    free(c->e[i].text);
  }
  free(c->e);
  free(c->slot);
  free(c);
}

/* a resolved value: a table entry, or a clock string */
typedef struct {
  int kind;
  const char* text;
  size_t text_len;
  uint32_t vid;
} value;

/* ------------------------------------------------------------------------------------------ */
/* get_interpdata  py:430-467 / interp.rs:91-137                                               */
/* ------------------------------------------------------------------------------------------ */
static int all_ascii_digits(const char* s, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (s[i] < '0' || s[i] > '9') return 0;
  return 1;
}

static int get_interpdata(const ieo_ctx* c, const char* k, size_t kn, value* v) {
  /* 'HH:MM' / 'HH:MM:SS'  py:433-436, interp.rs:97-104 */
  if (kn == 5 && memcmp(k, "HH:MM", 5) == 0) {
    v->kind = IE_KIND_STR;
    v->text = c->hhmm;
    v->text_len = 5;
    v->vid = IE_VID_CLOCK_HHMM;
    return IE_OK_STR;
  }
  if (kn == 8 && memcmp(k, "HH:MM:SS", 8) == 0) {
    v->kind = IE_KIND_STR;
    v->text = c->hhmmss;
    v->text_len = 8;
    v->vid = IE_VID_CLOCK_HHMMSS;
    return IE_OK_STR;
  }
  int is_arg;
  if (c->dialect == IE_DIALECT_PY) {
    /* py:437: a.startswith("ARG") and a[3:].isdigit()  (ASCII digits restated) ; '' py:446 */
    is_arg = kn > 3 && memcmp(k, "ARG", 3) == 0 && all_ascii_digits(k + 3, kn - 3);
    if (!is_arg && kn == 0) return IE_E_INTERP;
  } else {
    /* interp.rs:105 '' first, then interp.rs:109 starts_with("ARG") && all ascii digit */
    if (kn == 0) return IE_E_INTERP;
    is_arg = kn >= 3 && memcmp(k, "ARG", 3) == 0 && all_ascii_digits(k + 3, kn - 3);
  }
  long at = ctx_find(c, k, kn);
  if (at >= 0) {
    const entry* e = &c->e[at];
    v->kind = e->kind;
    v->text = e->text;
    v->text_len = e->text_len;
    v->vid = e->vid;
    return IE_OK_STR;
  }
  if (is_arg) return IE_E_INTERP; /* py:440-442 / interp.rs:113-115: no inserts-dir lookup */
  /* py:452-461 / interp.rs:122-134: with an inserts directory the caller adds every key a file
   * answers to the inserts (after them) before building the context, so a miss is a miss there
   * too; a key that is not a canonical relative file name (absolute, an empty, '.' or '..'
   * component, a NUL: os.path.join may leave the directory) is left to the host */
  if (c->has_dir) {
    int odd = 0;
    size_t c0 = 0;
    for (size_t j = 0; j <= kn && !odd; j++) {
      if (j < kn && k[j] == 0) odd = 1;
      if (j == kn || k[j] == '/') {
        size_t cl = j - c0;
        odd |= cl == 0 || (cl == 1 && k[c0] == '.') || (cl == 2 && k[c0] == '.' && k[c0 + 1] == '.');
        c0 = j + 1;
      }
    }
    return odd ? IE_NEEDS_HOST : IE_E_INTERP;
  }
  return IE_E_INTERP; /* py:465-467 / interp.rs:136 */
}

/* get_interpdata called with a RAW value as the key (py:512 after a typed simple result) */
static int get_interpdata_raw_py(const ieo_ctx* c, const value* key, value* v) {
  if (key->kind == IE_KIND_STR) return get_interpdata(c, key->text, key->text_len, v);
  if (key->kind == IE_KIND_LIST || key->kind == IE_KIND_DICT) return IE_E_UNHASHABLE; /* `in` on dict */
  return c->has_dir ? IE_NEEDS_HOST : IE_E_INTERP; /* int/float/bool/None: never a str key */
}

/* ------------------------------------------------------------------------------------------ */
/* get_simple_insertkey  py:477-495 (code points) / interp.rs:11-29 (chars)                    */
/* returns 1 when the reference returns a truthy key (py) / Some (rs)                           */
/* ------------------------------------------------------------------------------------------ */
static size_t utf8_len(unsigned char b) {
  if (b < 0x80) return 1;
  if ((b & 0xE0) == 0xC0) return 2;
  if ((b & 0xF0) == 0xE0) return 3;
  if ((b & 0xF8) == 0xF0) return 4;
  return 1;
}

static int simple_key(int dialect, const char* s, size_t n, size_t* koff, size_t* klen) {
  /* count code points */
  size_t nch = 0;
  for (size_t i = 0; i < n; i += utf8_len((unsigned char)s[i])) nch++;
  if (dialect == IE_DIALECT_RS) {
    if (nch < 2 || s[0] != '{' || s[n - 1] != '}') return 0; /* interp.rs:14-16 */
  }
  long depth = 0;
  size_t ci = 0;
  for (size_t i = 0; i < n; i += utf8_len((unsigned char)s[i]), ci++) {
    char ch = s[i];
    if (ch == '}') depth -= 1;
    if ((depth == 0) != (ci == 0 || ci == nch - 1)) return 0;
    if (ch == '{') depth += 1;
  }
  /* content[1:-1] (py:495) / chars[1..len-1] (interp.rs:28) */
  if (nch <= 2) {
    *koff = 0;
    *klen = 0;
    return dialect == IE_DIALECT_RS; /* py: '' is falsy; rs: Some("") for "{}" */
  }
  size_t first = utf8_len((unsigned char)s[0]);
  size_t last = n;
  do {
    last--;
  } while (last > 0 && (((unsigned char)s[last]) & 0xC0) == 0x80);
  *koff = first;
  *klen = last - first;
  return 1;
}

int ieo_simple_insertkey(const char* s, uint64_t n, int32_t dialect, uint64_t* koff, uint64_t* klen) {
  size_t o = 0, l = 0;
  int r = simple_key(dialect, s, n, &o, &l);
  *koff = o;
  *klen = l;
  return r;
}

/* ------------------------------------------------------------------------------------------ */
/* interpolate_inserts  py:497-541 / interp.rs:31-89                                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int status;
  sb str;  /* IE_OK_STR */
  value v; /* IE_OK_VALUE */
} result;

static void protect(sb* content, sb* tmp) {
  /* py:505-508 / py:532-535 / interp.rs:42-43, 82-83 */
  str_replace(tmp, content->p, content->n, ESC_START, 2, PH_START, 4);
  str_replace(content, tmp->p, tmp->n, ESC_STOP, 2, PH_STOP, 4);
}
static void restore(sb* content, sb* tmp) {
  /* py:537-540 / py:525-528 / interp.rs:60-62, 86-87 */
  str_replace(tmp, content->p, content->n, PH_START, 4, ESC_START, 2);
  str_replace(content, tmp->p, tmp->n, PH_STOP, 4, ESC_STOP, 2);
}

static int splice_allowed(int dialect, int kind) {
  if (dialect == IE_DIALECT_PY) /* py:530 type(v) in (str, int, list) */
    return kind == IE_KIND_STR || kind == IE_KIND_INT || kind == IE_KIND_LIST;
  /* interp.rs:71-80 String | Number | Array */
  return kind == IE_KIND_STR || kind == IE_KIND_INT || kind == IE_KIND_FLOAT || kind == IE_KIND_LIST;
}

static void interpolate(const ieo_ctx* c, const char* s0, size_t n0, result* r, int depth);

static void interpolate(const ieo_ctx* c, const char* s0, size_t n0, result* r, int depth) {
  sb content = {0}, tmp = {0}, key = {0};
  sb_put(&content, s0, n0);
  protect(&content, &tmp);
  r->status = IE_OK_STR;

  size_t koff, klen;
  if (depth > 900) { /* CPython's recursion limit (1000 frames) ends the simple-path recursion */
    r->status = IE_DIVERGED;
    goto done;
  }
  if (simple_key(c->dialect, content.p, content.n, &koff, &klen)) {
    /* py:510-514 — both branches call interpolate_inserts on a string equal to insertkey;
       rs interp.rs:45-52 — same, then value_to_string before the lookup */
    result inner = {0};
    size_t sko, skl;
    if (simple_key(c->dialect, content.p + koff, klen, &sko, &skl)) {
      sb_clear(&key);
      sb_put(&key, "{", 1);
      sb_put(&key, content.p + koff + sko, skl);
      sb_put(&key, "}", 1);
      interpolate(c, key.p, key.n, &inner, depth + 1);
    } else {
      interpolate(c, content.p + koff, klen, &inner, depth + 1);
    }
    if (inner.status == IE_OK_STR) {
      r->status = get_interpdata(c, inner.str.p ? inner.str.p : "", inner.str.n, &r->v);
    } else if (inner.status == IE_OK_VALUE) {
      if (c->dialect == IE_DIALECT_PY)
        r->status = get_interpdata_raw_py(c, &inner.v, &r->v);
      else /* value_to_string(&inner) */
        r->status = get_interpdata(c, inner.v.text, inner.v.text_len, &r->v);
    } else {
      r->status = inner.status;
    }
    if (r->status == IE_OK_STR) r->status = IE_OK_VALUE;
    sb_free(&inner.str);
    goto done;
  }

  size_t iters = 0;
  while (str_find(content.p, content.n, '{', 0) != -1) { /* py:516 */
    if (++iters > IE_ITER_CAP(n0) || content.n > IE_SIZE_CAP(n0, c->maxtext)) {
      r->status = IE_DIVERGED;
      goto done;
    }
    size_t n_starts = str_count(content.p, content.n, "{", 1) - str_count(content.p, content.n, ESC_START, 2);
    size_t n_stops = str_count(content.p, content.n, "}", 1) - str_count(content.p, content.n, ESC_STOP, 2);
    if (n_starts != n_stops) { /* py:517-519 / interp.rs:55-62 */
      r->status = IE_E_ASSERT_BRACES;
      goto done;
    }
    long outer_from = str_rfind(content.p, content.n, '{');                /* py:520 */
    long inner_to = str_find(content.p, content.n, '}', (size_t)outer_from + 1); /* py:521 */
    if (outer_from == -1 || inner_to == -1) {
      if (c->dialect == IE_DIALECT_RS) { /* interp.rs:63-66: .unwrap() on None */
        r->status = IE_E_RS_PANIC;
        goto done;
      }
      break; /* py:522 */
    }
    /* py:525-528 key with placeholders restored */
    sb_clear(&key);
    sb_put(&key, content.p + outer_from + 1, (size_t)(inner_to - outer_from - 1));
    restore(&key, &tmp);
    value v;
    int st = get_interpdata(c, key.p ? key.p : "", key.n, &v); /* py:529 */
    if (st != IE_OK_STR) {
      r->status = st;
      goto done;
    }
    if (!splice_allowed(c->dialect, v.kind)) { /* py:530 / interp.rs:76-79 */
      r->status = IE_E_ASSERT_TYPE;
      goto done;
    }
    /* py:531 content[:outer_from] + str(v) + content[outer_to:] */
    sb_clear(&tmp);
    sb_put(&tmp, content.p, (size_t)outer_from);
    sb_put(&tmp, v.text, v.text_len);
    sb_put(&tmp, content.p + inner_to + 1, content.n - (size_t)inner_to - 1);
    sb_swap(&tmp, &content);
    protect(&content, &tmp); /* py:532-535 */
  }
  restore(&content, &tmp); /* py:537-540 */
  sb_swap(&r->str, &content);

done:
  sb_free(&content);
  sb_free(&tmp);
  sb_free(&key);
}

/* ------------------------------------------------------------------------------------------ */
/* C API used by tests/ and bench.py                                                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct ieo_out {
  int32_t status;
  uint32_t vid;
  char* bytes; /* malloc'd, for IE_OK_STR */
  uint64_t len;
} ieo_out;

int ieo_interpolate(const ieo_ctx* c, const char* s, uint64_t n, ieo_out* o) {
  result r = {0};
  interpolate(c, s, n, &r, 0);
  o->status = r.status;
  o->vid = r.status == IE_OK_VALUE ? r.v.vid : IE_VID_NONE;
  o->bytes = NULL;
  o->len = 0;
  if (r.status == IE_OK_STR) {
    o->bytes = (char*)malloc(r.str.n + 1);
    if (r.str.n) memcpy(o->bytes, r.str.p, r.str.n);
    o->len = r.str.n;
  }
  sb_free(&r.str);
  return r.status;
}

void ieo_out_free(ieo_out* o) {
  free(o->bytes);
  o->bytes = NULL;
}

/* recursive_escape / recursive_unescape on a string leaf: py:1449-1453 / py:1437-1440 */
uint64_t ieo_escape(const char* s, uint64_t n, int unescape, char** out) {
  sb a = {0}, b = {0};
  if (unescape) {
    str_replace(&a, s, n, ESC_START, 2, "{", 1);
    str_replace(&b, a.p, a.n, ESC_STOP, 2, "}", 1);
  } else {
    str_replace(&a, s, n, "{", 1, ESC_START, 2);
    str_replace(&b, a.p, a.n, "}", 1, ESC_STOP, 2);
  }
  sb_free(&a);
  *out = b.p;
  return b.n;
}

void ieo_free_bytes(char* p) { free(p); }

/* ---- timed batch for bench.py's cpu_baseline (and bulk parity checks) ---- */
typedef struct {
  const ieo_ctx* c;
  const uint8_t* bytes;
  const uint64_t* offsets;
  uint64_t lo, hi;
  uint8_t* status;
  uint64_t* out_len;
  uint64_t* out_hash; /* FNV-1a of each output (0 if not OK_STR) */
  uint32_t* vid;
  int32_t mode; /* 0: interpolate_inserts; 1: then the `unescape` command on the result (py:1660-1667);
                  2: the `unescape` command alone */
  const ieo_ctx* const* ctxs; /* table sets: string i against ctxs[table_id[i]] (else c) */
  const uint32_t* table_id;
} job;

/* recursive_unescape of one string (py:1436-1440): two plain str.replace passes */
static void unescape_str(sb* out, const char* s, size_t n) {
  sb a = {0};
  str_replace(&a, s, n, ESC_START, 2, "{", 1);
  str_replace(out, a.p ? a.p : "", a.n, ESC_STOP, 2, "}", 1);
  sb_free(&a);
}

/* the unescape command's transform of a string item (py:1665-1666): recursive_unescape, then
 * recursive_interpolate. recursive_interpolate re-enters the result of an item that is a
 * whole-string '{key}' as written (py:1463-1464) unless that result is an int/float/bool/None
 * value; such items report IE_RECURSE (the device does the same; callers walk them). */
static void unescape_command(const ieo_ctx* c, const char* s, size_t n, result* r) {
  sb b = {0};
  unescape_str(&b, s, n);
  interpolate(c, b.p ? b.p : "", b.n, r, 0);
  size_t ko, kl;
  if (c->dialect == IE_DIALECT_PY && (r->status == IE_OK_STR || r->status == IE_OK_VALUE) &&
      simple_key(IE_DIALECT_PY, b.p ? b.p : "", b.n, &ko, &kl) &&
      (r->status == IE_OK_STR || r->v.kind == IE_KIND_STR || r->v.kind == IE_KIND_LIST || r->v.kind == IE_KIND_DICT)) {
    if (r->status == IE_OK_STR) r->v.vid = IE_VID_NONE;
    r->status = IE_RECURSE;
    sb_free(&r->str);
  }
  sb_free(&b);
}

static void* run_job(void* p) {
  job* j = (job*)p;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    result r = {0};
    const ieo_ctx* c = j->ctxs ? j->ctxs[j->table_id[i]] : j->c;
    const char* s = (const char*)j->bytes + j->offsets[i];
    const size_t n = j->offsets[i + 1] - j->offsets[i];
    if (j->mode == 2) {
      unescape_command(c, s, n, &r); /* the command alone on the item */
    } else {
      interpolate(c, s, n, &r, 0);
      if (j->mode == 1 && r.status == IE_OK_STR) { /* config 4's step: then the command on the result */
        result r2 = {0};
        unescape_command(c, r.str.p ? r.str.p : "", r.str.n, &r2);
        sb_free(&r.str);
        r = r2;
      }
    }
    if (j->status) j->status[i] = (uint8_t)r.status;
    if (j->out_len) j->out_len[i] = r.status == IE_OK_STR ? r.str.n : 0;
    if (j->out_hash) j->out_hash[i] = r.status == IE_OK_STR ? fnv(r.str.p ? r.str.p : "", r.str.n) : 0;
    if (j->vid) j->vid[i] = (r.status == IE_OK_VALUE || r.status == IE_RECURSE) ? r.v.vid : IE_VID_NONE;
    sb_free(&r.str);
  }
  return NULL;
}

/* returns wall seconds; threads split the batch into contiguous, byte-balanced shards */
static double run_batch(const ieo_ctx* c, const ieo_ctx* const* ctxs, const uint32_t* table_id,
                        const uint8_t* bytes, const uint64_t* offsets, uint64_t n, int32_t nthreads,
                        uint8_t* status, uint64_t* out_len, uint64_t* out_hash, uint32_t* vid, int32_t mode) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  job jobs[256];
  pthread_t th[256];
  uint64_t total = offsets[n] - offsets[0];
  uint64_t lo = 0;
  for (int t = 0; t < nthreads; t++) {
    uint64_t target = offsets[0] + total * (uint64_t)(t + 1) / (uint64_t)nthreads;
    uint64_t hi = lo;
    if (t == nthreads - 1) {
      hi = n;
    } else { /* first string index whose start >= target */
      uint64_t a = lo, b = n;
      while (a < b) {
        uint64_t m = (a + b) / 2;
        if (offsets[m] < target) a = m + 1; else b = m;
      }
      hi = a;
    }
    jobs[t] = (job){c, bytes, offsets, lo, hi, status, out_len, out_hash, vid, mode, ctxs, table_id};
    lo = hi;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

double ieo_run_batch_mode(const ieo_ctx* c, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                          int32_t nthreads, uint8_t* status, uint64_t* out_len, uint64_t* out_hash,
                          uint32_t* vid, int32_t mode) {
  return run_batch(c, NULL, NULL, bytes, offsets, n, nthreads, status, out_len, out_hash, vid, mode);
}

/* a table-set batch (config 5's forked states): string i against ctxs[table_id[i]] */
double ieo_run_batch_sets(const ieo_ctx* const* ctxs, const uint32_t* table_id, const uint8_t* bytes,
                          const uint64_t* offsets, uint64_t n, int32_t nthreads, uint8_t* status,
                          uint64_t* out_len, uint64_t* out_hash, uint32_t* vid) {
  return run_batch(NULL, ctxs, table_id, bytes, offsets, n, nthreads, status, out_len, out_hash, vid, 0);
}

double ieo_run_batch(const ieo_ctx* c, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                     int32_t nthreads, uint8_t* status, uint64_t* out_len, uint64_t* out_hash,
                     uint32_t* vid) {
  return ieo_run_batch_mode(c, bytes, offsets, n, nthreads, status, out_len, out_hash, vid, 0);
}

uint64_t ieo_fnv1a(const uint8_t* p, uint64_t n) { return fnv((const char*)p, n); }

/* ---- bulk checker: FNV-1a of every result of a device batch (packed or views), so a test can
 * compare a whole BASELINE-size batch with ieo_run_batch's hashes. starts[i], lens[i] locate
 * string i in bytes; strings whose status is not IE_OK_STR hash to 0 (as ieo_run_batch). ---- */
typedef struct {
  const uint8_t* bytes;
  const uint64_t* starts;
  const uint64_t* lens;
  const uint8_t* status;
  uint64_t lo, hi;
  uint64_t* out_hash;
} hjob;

static void* run_hash(void* p) {
  hjob* j = (hjob*)p;
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->out_hash[i] = j->status[i] == IE_OK_STR ? fnv((const char*)j->bytes + j->starts[i], j->lens[i]) : 0;
  return NULL;
}

void ieo_hash_spans(const uint8_t* bytes, const uint64_t* starts, const uint64_t* lens, const uint8_t* status,
                    uint64_t n, int32_t nthreads, uint64_t* out_hash) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  hjob jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; t++)
    jobs[t] = (hjob){bytes, starts, lens, status, n * (uint64_t)t / (uint64_t)nthreads,
                     n * (uint64_t)(t + 1) / (uint64_t)nthreads, out_hash};
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_hash, &jobs[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}
