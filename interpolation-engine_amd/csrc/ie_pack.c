// ie_pack.c — the host side's store packing as a CPython module (_ie_pack): InsertsTableSet.update's
// changes [(dict index, key, value)] -> the ie_kv records and table ids ie_table_set_store takes,
// pointing straight into an ASCII str's own bytes (no copy) or into one buffer the other texts are
// transcoded into across host threads (no per-object UTF-8 cache left behind on the caller's
// strings), and the
// stored values written back into the table set's value list by the ids the library handed out.
// Host-only code (gcc), no device calls: the library keeps the C ABI, this only feeds it.
//
// Rendering (the splice text, py:531 / interp.rs:314): a str is its own text, an int (not a bool)
// is str(int) in both dialects; anything else goes through the caller's render(v, dialect).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <emmintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

typedef struct {
  const char* key;
  uint64_t key_len;
  const char* text;
  uint64_t text_len;
  int32_t kind;
  uint32_t reserved;
} kv_rec;  // = ie_kv (include/ie_amd.h)

enum { KIND_STR = 0, KIND_INT = 1 };

#ifndef IE_PACK_ID
#define IE_PACK_ID "unstamped"
#endif
__attribute__((used)) static const char kPackId[] = "IE_BUILD_ID:" IE_PACK_ID;  // (__graft_entry__.built_id)

// A text that is not ASCII: transcoded into the call's buffer (one pass, each thread's jobs back to
// back in a region sized by their bounds), across the threads with the GIL released. The records
// point into str objects the call OWNS a reference to (held in `keep`, which the caller holds until
// the library has read the records): pack() takes a tuple snapshot of the changes (the change tuples
// are immutable), pack_dicts() holds every key and value it points into. Another thread that
// rebinds a list item or a dict value meanwhile then frees nothing the records (or the transcode
// threads, or the library behind a ctypes call that released the GIL) still read.
typedef struct {
  const void* src;
  uint64_t len;  // code units
  int kind;      // 1, 2, 4 bytes per unit; KIND_JOB_INT: str() of ival
  int64_t ival;
  uint64_t rec;  // record index * 2 + (0: key, 1: text)
  uint64_t off, out;
} job_t;
enum { KIND_JOB_INT = 8 };

static inline uint8_t* put_cp(uint8_t* o, uint32_t c) {  // one code point (surrogates: 3 bytes, as 'surrogatepass')
  if (c < 0x80) {
    *o++ = (uint8_t)c;
  } else if (c < 0x800) {
    *o++ = (uint8_t)(0xC0 | (c >> 6));
    *o++ = (uint8_t)(0x80 | (c & 0x3F));
  } else if (c < 0x10000) {
    *o++ = (uint8_t)(0xE0 | (c >> 12));
    *o++ = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
    *o++ = (uint8_t)(0x80 | (c & 0x3F));
  } else {
    *o++ = (uint8_t)(0xF0 | (c >> 18));
    *o++ = (uint8_t)(0x80 | ((c >> 12) & 0x3F));
    *o++ = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
    *o++ = (uint8_t)(0x80 | (c & 0x3F));
  }
  return o;
}

// the most UTF-8 bytes a job can make (the output buffer is sized by these: one pass, no count pass
// over the source first)
static uint64_t utf8_bound(const job_t* j) {
  if (j->kind == KIND_JOB_INT) return 24;
  return j->len * (j->kind == 4 ? 4u : j->kind == 2 ? 3u : 2u);
}

// the job's UTF-8 at o; returns the bytes written (16 units at a time where all are ASCII)
static uint64_t transcode(const job_t* j, uint8_t* o) {
  if (j->kind == KIND_JOB_INT) {
    char tmp[24];
    const int n = snprintf(tmp, sizeof tmp, "%lld", (long long)j->ival);
    memcpy(o, tmp, (size_t)n);
    return (uint64_t)n;
  }
  uint8_t* const o0 = o;
  const uint64_t len = j->len;
  uint64_t i = 0;
  // 16 units at a time: the block's ASCII units packed to bytes and stored whole, `o` advanced past
  // the ASCII prefix only; the first wider unit after it is written on its own, and the next block
  // starts right after it (a slot's bound leaves room for the 16-byte store)
  if (j->kind == 1) {
    const uint8_t* d = (const uint8_t*)j->src;
    while (i + 16 <= len) {
      const __m128i v = _mm_loadu_si128((const __m128i*)(d + i));
      _mm_storeu_si128((__m128i*)o, v);
      const unsigned wide = (unsigned)_mm_movemask_epi8(v);
      if (!wide) {
        o += 16;
        i += 16;
        continue;
      }
      const unsigned p = (unsigned)__builtin_ctz(wide);
      o = put_cp(o + p, d[i + p]);
      i += p + 1;
    }
  } else if (j->kind == 2) {
    const uint16_t* d = (const uint16_t*)j->src;
    const __m128i hi = _mm_set1_epi16((short)0xFF80);
    while (i + 16 <= len) {
      const __m128i v0 = _mm_loadu_si128((const __m128i*)(d + i)), v1 = _mm_loadu_si128((const __m128i*)(d + i + 8));
      _mm_storeu_si128((__m128i*)o, _mm_packus_epi16(v0, v1));
      const __m128i a0 = _mm_cmpeq_epi16(_mm_and_si128(v0, hi), _mm_setzero_si128());
      const __m128i a1 = _mm_cmpeq_epi16(_mm_and_si128(v1, hi), _mm_setzero_si128());
      const unsigned wide = ~(unsigned)_mm_movemask_epi8(_mm_packs_epi16(a0, a1)) & 0xFFFFu;
      if (!wide) {
        o += 16;
        i += 16;
        continue;
      }
      const unsigned p = (unsigned)__builtin_ctz(wide);
      o = put_cp(o + p, d[i + p]);
      i += p + 1;
    }
  } else {
    const uint32_t* d = (const uint32_t*)j->src;
    const __m128i hi = _mm_set1_epi32((int)0xFFFFFF80u);
    while (i + 16 <= len) {
      const __m128i v0 = _mm_loadu_si128((const __m128i*)(d + i)), v1 = _mm_loadu_si128((const __m128i*)(d + i + 4));
      const __m128i v2 = _mm_loadu_si128((const __m128i*)(d + i + 8)), v3 = _mm_loadu_si128((const __m128i*)(d + i + 12));
      // (an ASCII lane packs to itself; a wider one's byte is garbage, past the prefix kept)
      _mm_storeu_si128((__m128i*)o, _mm_packus_epi16(_mm_packs_epi32(v0, v1), _mm_packs_epi32(v2, v3)));
      const __m128i z = _mm_setzero_si128();
      const __m128i a01 = _mm_packs_epi32(_mm_cmpeq_epi32(_mm_and_si128(v0, hi), z), _mm_cmpeq_epi32(_mm_and_si128(v1, hi), z));
      const __m128i a23 = _mm_packs_epi32(_mm_cmpeq_epi32(_mm_and_si128(v2, hi), z), _mm_cmpeq_epi32(_mm_and_si128(v3, hi), z));
      const unsigned wide = ~(unsigned)_mm_movemask_epi8(_mm_packs_epi16(a01, a23)) & 0xFFFFu;
      if (!wide) {
        o += 16;
        i += 16;
        continue;
      }
      const unsigned p = (unsigned)__builtin_ctz(wide);
      o = put_cp(o + p, d[i + p]);
      i += p + 1;
    }
  }
  if (j->kind == 1)
    for (const uint8_t* d = (const uint8_t*)j->src; i < len; i++) o = put_cp(o, d[i]);
  else if (j->kind == 2)
    for (const uint16_t* d = (const uint16_t*)j->src; i < len; i++) o = put_cp(o, d[i]);
  else
    for (const uint32_t* d = (const uint32_t*)j->src; i < len; i++) o = put_cp(o, d[i]);
  return (uint64_t)(o - o0);
}

typedef struct {
  job_t* jobs;
  uint64_t lo, hi;
  uint8_t* buf;
  uint64_t base;  // the span's region: the bounds of the jobs before it
} span_t;

// a span's jobs back to back from its region's start (the region holds their bounds: the used
// part is dense, and a reused buffer is touched in about the same pages call after call)
static void* run_span(void* arg) {
  span_t* sp = (span_t*)arg;
  uint64_t at = sp->base;
  for (uint64_t k = sp->lo; k < sp->hi; k++) {
    sp->jobs[k].off = at;
    sp->jobs[k].out = transcode(&sp->jobs[k], sp->buf + at);
    at += sp->jobs[k].out;
  }
  return NULL;
}

// one pass over the jobs across up to `threads` threads (split by code units, not by count)
static void run_jobs(job_t* jobs, uint64_t n, uint8_t* buf, int threads) {
  uint64_t units = 0;
  for (uint64_t k = 0; k < n; k++) units += jobs[k].len * (uint64_t)jobs[k].kind;
  if (threads > 16) threads = 16;
  if (threads < 1 || units < (1u << 20)) threads = 1;
  span_t sp[16];
  pthread_t th[16];
  uint64_t k = 0, acc = 0, bsum = 0;
  for (int w = 0; w < threads; w++) {
    sp[w].jobs = jobs;
    sp[w].buf = buf;
    sp[w].lo = k;
    sp[w].base = bsum;
    const uint64_t want = units * (uint64_t)(w + 1) / (uint64_t)threads;
    while (k < n && (acc < want || w == threads - 1)) acc += jobs[k].len * (uint64_t)jobs[k].kind, bsum += utf8_bound(&jobs[k]), k++;
    sp[w].hi = k;
  }
  int started[16] = {0};
  for (int w = 1; w < threads; w++) started[w] = pthread_create(&th[w], NULL, run_span, &sp[w]) == 0;
  run_span(&sp[0]);
  for (int w = 1; w < threads; w++) {
    if (started[w]) pthread_join(th[w], NULL);
    else run_span(&sp[w]);
  }
}

typedef struct {
  job_t* p;
  uint64_t n, cap;
} jobs_t;

static job_t* new_job(jobs_t* J) {
  if (J->n == J->cap) {
    const uint64_t cap = J->cap ? 2 * J->cap : 1024;
    job_t* q = (job_t*)PyMem_RawRealloc(J->p, cap * sizeof(job_t));
    if (!q) {
      PyErr_NoMemory();
      return NULL;
    }
    J->p = q;
    J->cap = cap;
  }
  job_t* j = &J->p[J->n++];
  j->ival = 0;
  return j;
}

// the record's UTF-8 ('surrogatepass', as _native.enc): an ASCII str is its own UTF-8 (a pointer
// into it); any other becomes a job
static int utf8_of(PyObject* s, jobs_t* J, uint64_t rec, const char** p, uint64_t* n) {
  if (PyUnicode_READY(s) < 0) return -1;
  if (PyUnicode_IS_ASCII(s)) {
    *p = (const char*)PyUnicode_DATA(s);
    *n = (uint64_t)PyUnicode_GET_LENGTH(s);
    return 0;
  }
  job_t* j = new_job(J);
  if (!j) return -1;
  j->src = PyUnicode_DATA(s);
  j->len = (uint64_t)PyUnicode_GET_LENGTH(s);
  j->kind = PyUnicode_KIND(s);
  j->rec = rec;
  *p = NULL;
  *n = 0;
  return 0;
}

// The transcode buffer outlives the call only until the records are used: when its capsule goes,
// the buffer is kept for the next call instead of freed (a store loop packs tens of MB per
// iteration: a fresh mapping each time costs its page faults, and its unmapping, again). The GIL
// guards the slot.
static uint8_t* spare_buf = NULL;
static size_t spare_cap = 0;

static uint8_t* take_buf(size_t need, size_t* cap) {
  if (spare_buf && spare_cap >= need) {
    uint8_t* b = spare_buf;
    *cap = spare_cap;
    spare_buf = NULL;
    spare_cap = 0;
    return b;
  }
  *cap = need + need / 4;  // (headroom: a loop's texts grow call by call, and a fresh buffer faults again)
  return (uint8_t*)PyMem_RawMalloc(*cap);
}

typedef struct {
  uint8_t* p;
  size_t cap;
} held_t;

static void free_buf(PyObject* capsule) {
  held_t* h = (held_t*)PyCapsule_GetPointer(capsule, "ie_pack.buf");
  if (!h) return;
  if (!spare_buf || spare_cap < h->cap) {  // (keep the larger one)
    PyMem_RawFree(spare_buf);
    spare_buf = h->p;
    spare_cap = h->cap;
  } else {
    PyMem_RawFree(h->p);
  }
  PyMem_RawFree(h);
}

// one record: key k, value v (the delete marker: kind -1); 0, or -1 with the Python error set
static int pack_kv(PyObject* k, PyObject* v, kv_rec* r, uint64_t i, jobs_t* J, PyObject* keep, PyObject* del,
                   PyObject* render, PyObject* dialect) {
  if (!PyUnicode_Check(k)) {
    PyErr_SetString(PyExc_TypeError, "insert keys must be str");
    return -1;
  }
  memset(r, 0, sizeof *r);
  if (utf8_of(k, J, 2 * i, &r->key, &r->key_len) < 0) return -1;
  if (v == del) {
    r->kind = -1;
    return 0;
  }
  PyObject* text = NULL;
  if (PyUnicode_CheckExact(v)) {
    r->kind = KIND_STR;
    text = v;
  } else if (PyLong_CheckExact(v)) {
    r->kind = KIND_INT;
    int overflow = 0;
    const long long x = PyLong_AsLongLongAndOverflow(v, &overflow);
    if (!overflow && !(x == -1 && PyErr_Occurred())) {  // (str(int) formatted with the texts: no str object)
      job_t* j = new_job(J);
      if (!j) return -1;
      j->src = NULL;
      j->len = 0;
      j->ival = x;
      j->kind = KIND_JOB_INT;
      j->rec = 2 * i + 1;
      r->text = NULL;
      r->text_len = 0;
      return 0;
    }
    PyErr_Clear();
    text = PyObject_Str(v);
    if (!text || PyList_Append(keep, text) < 0) {
      Py_XDECREF(text);
      return -1;
    }
    Py_DECREF(text);
  } else {
    PyObject* kt = PyObject_CallFunctionObjArgs(render, v, dialect, NULL);  // (kind, text)
    if (!kt) return -1;
    if (PyList_Append(keep, kt) < 0) {
      Py_DECREF(kt);
      return -1;
    }
    Py_DECREF(kt);
    if (!PyTuple_Check(kt) || PyTuple_GET_SIZE(kt) != 2 || !PyUnicode_Check(PyTuple_GET_ITEM(kt, 1))) {
      PyErr_SetString(PyExc_TypeError, "render must return (kind, str)");
      return -1;
    }
    r->kind = (int32_t)PyLong_AsLong(PyTuple_GET_ITEM(kt, 0));
    if (r->kind == -1 && PyErr_Occurred()) return -1;
    text = PyTuple_GET_ITEM(kt, 1);
  }
  return utf8_of(text, J, 2 * i + 1, &r->text, &r->text_len);
}

// the texts that are not ASCII: transcoded into one buffer sized by their bounds (across the
// threads, the GIL released); then the records point there and `keep` holds the buffer
static int finish(kv_rec* kv, jobs_t* J, PyObject* keep, int threads) {
  if (!J->n) return 0;
  uint64_t total = 0;
  for (uint64_t k = 0; k < J->n; k++) total += utf8_bound(&J->p[k]);
  size_t cap = 0;
  uint8_t* buf = take_buf(total + 16, &cap);
  held_t* held = (held_t*)PyMem_RawMalloc(sizeof(held_t));
  if (!buf || !held) {
    PyMem_RawFree(buf);
    PyMem_RawFree(held);
    PyErr_NoMemory();
    return -1;
  }
  held->p = buf;
  held->cap = cap;
  Py_BEGIN_ALLOW_THREADS
  run_jobs(J->p, J->n, buf, threads);  // (each job's .off / .out: where it wrote, how many bytes)
  Py_END_ALLOW_THREADS
  for (uint64_t k = 0; k < J->n; k++) {
    kv_rec* r = &kv[J->p[k].rec / 2];
    if (J->p[k].rec & 1) r->text = (const char*)buf + J->p[k].off, r->text_len = J->p[k].out;
    else r->key = (const char*)buf + J->p[k].off, r->key_len = J->p[k].out;
  }
  PyObject* capsule = PyCapsule_New(held, "ie_pack.buf", free_buf);
  if (!capsule) {
    PyMem_RawFree(buf);
    PyMem_RawFree(held);
    return -1;
  }
  const int rc = PyList_Append(keep, capsule);
  Py_DECREF(capsule);
  return rc;
}

// pack(changes, n_tables, delete, render, dialect, threads) -> (kv: bytearray, table_ids: bytearray,
// keep) (keep: what the records point into besides the changes' own strs; alive until the call)
static PyObject* pack(PyObject* self, PyObject* args) {
  (void)self;
  PyObject *changes, *del, *render, *dialect;
  long long n_tables;
  int threads = 1;
  if (!PyArg_ParseTuple(args, "OLOOO|i", &changes, &n_tables, &del, &render, &dialect, &threads)) return NULL;
  // a snapshot the call owns (a list the caller mutates later cannot free a change under us)
  PyObject* seq = PySequence_Tuple(changes);
  if (!seq) return NULL;
  const Py_ssize_t n = PyTuple_GET_SIZE(seq);
  PyObject* kvb = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(n * sizeof(kv_rec)));
  PyObject* tidb = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(n * 4));
  PyObject* keep = PyList_New(0);
  jobs_t J = {NULL, 0, 0};
  if (!kvb || !tidb || !keep || PyList_Append(keep, seq) < 0) goto fail;
  kv_rec* kv = (kv_rec*)PyByteArray_AS_STRING(kvb);
  uint32_t* tid = (uint32_t*)PyByteArray_AS_STRING(tidb);
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* c = PyTuple_GET_ITEM(seq, i);
    if (!PyTuple_CheckExact(c) || PyTuple_GET_SIZE(c) != 3) {
      PyErr_SetString(PyExc_TypeError, "a change is a (dict index, key, value) tuple");
      goto fail;
    }
    const long long tb = PyLong_AsLongLong(PyTuple_GET_ITEM(c, 0));
    if (tb == -1 && PyErr_Occurred()) goto fail;
    if (!PyUnicode_Check(PyTuple_GET_ITEM(c, 1))) {
      PyErr_SetString(PyExc_TypeError, "insert keys must be str");
      goto fail;
    }
    if (tb < 0 || tb >= n_tables) {
      PyErr_SetString(PyExc_IndexError, "dict index beyond the table set");
      goto fail;
    }
    tid[i] = (uint32_t)tb;
    if (pack_kv(PyTuple_GET_ITEM(c, 1), PyTuple_GET_ITEM(c, 2), &kv[i], (uint64_t)i, &J, keep, del, render, dialect) < 0)
      goto fail;
  }
  if (finish(kv, &J, keep, threads) < 0) goto fail;
  PyMem_RawFree(J.p);
  Py_DECREF(seq);
  return Py_BuildValue("(NNN)", kvb, tidb, keep);
fail:
  PyMem_RawFree(J.p);
  Py_DECREF(seq);
  Py_XDECREF(kvb);
  Py_XDECREF(tidb);
  Py_XDECREF(keep);
  return NULL;
}

// pack_dicts(dicts, render, dialect, threads) -> (kv: bytearray, kv_start: bytearray (n+1 u64), keep):
// every dict's items in order (a table set's build, ie_table_set_build; kv i gets value id i)
static PyObject* pack_dicts(PyObject* self, PyObject* args) {
  (void)self;
  PyObject *dicts, *render, *dialect;
  int threads = 1;
  if (!PyArg_ParseTuple(args, "OOO|i", &dicts, &render, &dialect, &threads)) return NULL;
  PyObject* seq = PySequence_Fast(dicts, "dicts must be a sequence");
  if (!seq) return NULL;
  const Py_ssize_t nd = PySequence_Fast_GET_SIZE(seq);
  Py_ssize_t n = 0;
  for (Py_ssize_t t = 0; t < nd; t++) {
    PyObject* d = PySequence_Fast_GET_ITEM(seq, t);
    if (!PyDict_Check(d)) {
      Py_DECREF(seq);
      PyErr_SetString(PyExc_TypeError, "a table set is built from dicts");
      return NULL;
    }
    n += PyDict_GET_SIZE(d);
  }
  PyObject* kvb = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)((n ? n : 1) * sizeof(kv_rec)));
  PyObject* stb = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)((nd + 1) * 8));
  PyObject* keep = PyList_New(0);
  jobs_t J = {NULL, 0, 0};
  if (!kvb || !stb || !keep) goto fail;
  // every key and value the records may point into, owned by the call (a dict entry rebound by
  // another thread, or a temporary dict the caller drops, frees nothing the records still read)
  PyObject* hold = PyTuple_New(2 * n);
  if (!hold || PyList_Append(keep, hold) < 0) {
    Py_XDECREF(hold);
    goto fail;
  }
  Py_DECREF(hold);  // (keep owns it)
  kv_rec* kv = (kv_rec*)PyByteArray_AS_STRING(kvb);
  uint64_t* st = (uint64_t*)PyByteArray_AS_STRING(stb);
  Py_ssize_t i = 0;
  st[0] = 0;
  for (Py_ssize_t t = 0; t < nd; t++) {
    PyObject* d = PySequence_Fast_GET_ITEM(seq, t);
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(d, &pos, &k, &v)) {
      if (i >= n) {
        PyErr_SetString(PyExc_RuntimeError, "a dict changed size while packing");
        goto fail;
      }
      Py_INCREF(k);
      Py_INCREF(v);
      PyTuple_SET_ITEM(hold, 2 * i, k);
      PyTuple_SET_ITEM(hold, 2 * i + 1, v);
      if (pack_kv(k, v, &kv[i], (uint64_t)i, &J, keep, NULL, render, dialect) < 0) goto fail;
      i++;
    }
    st[t + 1] = (uint64_t)i;
  }
  if (finish(kv, &J, keep, threads) < 0) goto fail;
  PyMem_RawFree(J.p);
  Py_DECREF(seq);
  return Py_BuildValue("(NNN)", kvb, stb, keep);
fail:
  PyMem_RawFree(J.p);
  Py_DECREF(seq);
  Py_XDECREF(kvb);
  Py_XDECREF(stb);
  Py_XDECREF(keep);
  return NULL;
}

// assign(values, changes, vids, delete[, in_table]) -> None: values[vids[i]] = the stored value (None
// for a delete), the list grown with None as the ids need; ids 0xFFFFFFFF are skipped. With
// in_table, a str or int value is not held: the marker goes in its place and the value is read back
// from the table's mirror when asked for (ie_table_value), so a store does not keep (and later free)
// the caller's KB-long texts
static PyObject* assign(PyObject* self, PyObject* args) {
  (void)self;
  PyObject *values, *changes, *vids, *del, *in_table = NULL;
  if (!PyArg_ParseTuple(args, "O!OOO|O", &PyList_Type, &values, &changes, &vids, &del, &in_table)) return NULL;
  Py_buffer vb;
  if (PyObject_GetBuffer(vids, &vb, PyBUF_SIMPLE) < 0) return NULL;
  PyObject* seq = PySequence_Fast(changes, "changes must be a sequence");
  if (!seq) {
    PyBuffer_Release(&vb);
    return NULL;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  if (vb.len < (Py_ssize_t)(n * 4)) {
    PyErr_SetString(PyExc_ValueError, "fewer ids than changes");
    goto fail;
  }
  const uint32_t* id = (const uint32_t*)vb.buf;
  for (Py_ssize_t i = 0; i < n; i++) {
    if (id[i] == 0xFFFFFFFFu) continue;
    while (PyList_GET_SIZE(values) <= (Py_ssize_t)id[i])
      if (PyList_Append(values, Py_None) < 0) goto fail;
    PyObject* v = PyTuple_GET_ITEM(PySequence_Fast_GET_ITEM(seq, i), 2);
    if (v == del) v = Py_None;
    else if (in_table && (PyUnicode_CheckExact(v) || PyLong_CheckExact(v))) v = in_table;
    Py_INCREF(v);
    if (PyList_SetItem(values, (Py_ssize_t)id[i], v) < 0) goto fail;  // (steals v, drops the old value)
  }
  Py_DECREF(seq);
  PyBuffer_Release(&vb);
  Py_RETURN_NONE;
fail:
  Py_DECREF(seq);
  PyBuffer_Release(&vb);
  return NULL;
}

// A batch of strings -> (one bytes blob of their UTF-8, one bytes object of uint64 offsets[n+1]):
// _native.pack's work without a Python-level encode and join per string (a map step's KB-long
// leaves). ASCII strs are copied from their own buffer; the others encoded as _native.enc does
// (utf-8, surrogatepass); bytes objects taken as they are.
static PyObject* pack_strs(PyObject* self, PyObject* arg) {
  (void)self;
  PyObject* seq = PySequence_Fast(arg, "pack_strs takes a sequence");
  if (!seq) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  PyObject* enc = PyList_New(n);  // (the encoded form of each non-ASCII str, else None)
  PyObject* offs = enc ? PyBytes_FromStringAndSize(NULL, (Py_ssize_t)((n + 1) * sizeof(uint64_t))) : NULL;
  if (!offs) {
    Py_XDECREF(enc);
    Py_DECREF(seq);
    return NULL;
  }
  uint64_t* o = (uint64_t*)PyBytes_AS_STRING(offs);
  uint64_t total = 0;
  o[0] = 0;
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* s = items[i];
    PyObject* e = Py_None;
    Py_ssize_t len;
    if (PyUnicode_Check(s) && PyUnicode_IS_ASCII(s)) {
      len = PyUnicode_GET_LENGTH(s);
    } else if (PyUnicode_Check(s)) {
      e = PyUnicode_AsEncodedString(s, "utf-8", "surrogatepass");
      if (!e) goto fail;
      len = PyBytes_GET_SIZE(e);
    } else if (PyBytes_Check(s)) {
      len = PyBytes_GET_SIZE(s);
    } else {
      PyErr_SetString(PyExc_TypeError, "pack_strs takes str or bytes items");
      goto fail;
    }
    if (e == Py_None) Py_INCREF(e);
    PyList_SET_ITEM(enc, i, e);
    total += (uint64_t)len;
    o[i + 1] = total;
  }
  PyObject* blob = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)total);
  if (!blob) goto fail;
  char* w = PyBytes_AS_STRING(blob);
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* s = items[i];
    PyObject* e = PyList_GET_ITEM(enc, i);
    const uint64_t len = o[i + 1] - o[i];
    const char* src = e != Py_None ? PyBytes_AS_STRING(e) : PyUnicode_Check(s) ? (const char*)PyUnicode_DATA(s) : PyBytes_AS_STRING(s);
    if (len) memcpy(w + o[i], src, len);
  }
  Py_DECREF(enc);
  Py_DECREF(seq);
  PyObject* r = PyTuple_Pack(2, blob, offs);
  Py_DECREF(blob);
  Py_DECREF(offs);
  return r;
fail:
  Py_DECREF(enc);
  Py_DECREF(offs);
  Py_DECREF(seq);
  return NULL;
}

static PyMethodDef methods[] = {
    {"pack_strs", pack_strs, METH_O, "strings -> (UTF-8 blob, uint64 offsets[n+1] as bytes)"},
    {"pack", pack, METH_VARARGS, "changes -> (ie_kv records, table ids, keep-alive list)"},
    {"assign", assign, METH_VARARGS, "store the values under the ids the library handed out"},
    {"pack_dicts", pack_dicts, METH_VARARGS, "dicts -> (ie_kv records, kv_start, keep-alive list)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_ie_pack", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__ie_pack(void) { return PyModule_Create(&module); }
