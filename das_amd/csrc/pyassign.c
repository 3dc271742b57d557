/* Answer materialisation for the drop-in API (CPython extension das_amd._assign).
 *
 * The reference's answer is a Python set of Assignment objects
 * (pattern_matcher.py:370-384; DistributedAtomSpace.query prints str(set),
 * distributed_atom_space.py:298-321).  Building one OrderedAssignment per row
 * through assign()/freeze() costs microseconds of interpreter time per
 * binding; this module builds the same objects from a fetched binding table in
 * C: the instance __dict__ the Python class would hold after freeze()
 * (pattern_matcher.OrderedAssignment / UnorderedAssignment), with the same
 * `hash` value -- hash(frozenset(mapping.items())) for ordered rows,
 * hash((hash(frozenset(symbols.items())), hash(frozenset(values.items()))))
 * for unordered ones -- computed by the interpreter's own hash functions.
 * Handle strings are shared: one str per distinct atom id (`strs`, indexed
 * through `lut`), so a row costs one dict, a few tuples and two frozensets.
 *
 * format_set(s) returns str(s) for a set of assignments, taking repr() of an
 * OrderedAssignment's mapping in C instead of calling its Python __repr__.
 * hex_list / hex_pairs format the handle rows of DBInterface answers.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

static PyObject *s_variables, *s_hash, *s_frozen, *s_mapping, *s_values, *s_symbols;

static int get_u32(PyObject *o, Py_buffer *b, const char *what) {
  if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) return -1;
  if (b->itemsize != 4) {
    PyErr_Format(PyExc_TypeError, "%s: expected a 4-byte integer buffer", what);
    PyBuffer_Release(b);
    return -1;
  }
  return 0;
}

static PyObject *new_instance(PyTypeObject *cls, PyObject *empty, PyObject *dict) {
  PyObject *obj = cls->tp_new(cls, empty, NULL);
  if (!obj) return NULL;
  PyObject **dp = _PyObject_GetDictPtr(obj);
  if (!dp) {
    Py_DECREF(obj);
    PyErr_SetString(PyExc_TypeError, "assignment class has no __dict__");
    return NULL;
  }
  Py_XSETREF(*dp, dict);   /* steals dict */
  return obj;
}

/* hash(frozenset(d.items())) without building the items and the frozenset:
 * the interpreter's tuple hash (xxHash lanes) of each (key, value) pair and
 * its frozenset hash (shuffled XOR over the entries; the empty slots of the
 * table cancel out, and a set of <= 4 entries has no dummy slots).  Checked
 * against the interpreter at import (fast_hash_ok); otherwise, and for more
 * than 4 entries, items_hash below is used. */
#define XXPRIME_1 11400714785074694791ULL
#define XXPRIME_2 14029467366897019727ULL
#define XXPRIME_5 2870177450012600261ULL
#define XXROTATE(x) ((x << 31) | (x >> 33))
static int fast_hash_ok = 0;

static Py_uhash_t pair_hash(Py_uhash_t a, Py_uhash_t b) {
  Py_uhash_t acc = XXPRIME_5;
  acc += a * XXPRIME_2; acc = XXROTATE(acc); acc *= XXPRIME_1;
  acc += b * XXPRIME_2; acc = XXROTATE(acc); acc *= XXPRIME_1;
  acc += 2 ^ (XXPRIME_5 ^ 3527539UL);
  if (acc == (Py_uhash_t)-1) return 1546275796;
  return acc;
}
static Py_uhash_t shuffle_bits(Py_uhash_t h) { return ((h ^ 89869747UL) ^ (h << 16)) * 3644798167UL; }
/* frozenset of n <= 4 distinct elements with these hashes (8-slot table, no dummies) */
static Py_hash_t small_frozenset_hash(const Py_uhash_t *h, Py_ssize_t n) {
  Py_uhash_t hash = 0;
  for (Py_ssize_t i = 0; i < n; ++i) hash ^= shuffle_bits(h[i]);   /* empty slots cancel out */
  hash ^= ((Py_uhash_t)n + 1) * 1927868237UL;
  hash ^= (hash >> 11) ^ (hash >> 25);
  hash = hash * 69069U + 907133923UL;
  if (hash == (Py_uhash_t)-1) hash = 590923713UL;
  return (Py_hash_t)hash;
}

/* hash(frozenset(d.items())) */
static Py_hash_t items_hash(PyObject *d) {
  PyObject *items = PyDict_Items(d);
  if (!items) return -1;
  PyObject *fs = PyFrozenSet_New(items);
  Py_DECREF(items);
  if (!fs) return -1;
  Py_hash_t h = PyObject_Hash(fs);
  Py_DECREF(fs);
  return h;
}

/* row value -> shared handle string */
static PyObject *value_of(const uint32_t *lut, Py_ssize_t nlut, PyObject *strs, uint32_t id) {
  if ((Py_ssize_t)id >= nlut) {
    PyErr_SetString(PyExc_IndexError, "atom id outside the lookup table");
    return NULL;
  }
  const uint32_t k = lut[id];
  if ((Py_ssize_t)k >= PyList_GET_SIZE(strs)) {
    PyErr_SetString(PyExc_IndexError, "atom id without a handle string");
    return NULL;
  }
  return PyList_GET_ITEM(strs, k);   /* borrowed */
}

/* add_rows(out_set, cls, kind, names, cols, lut, strs)
 *   kind 0 ordered / 1 unordered; names: tuple of k variable names; cols: u32
 *   buffer (k, n) row-major by column; lut: u32 buffer id -> index in strs. */
static PyObject *add_rows(PyObject *self, PyObject *args) {
  PyObject *out, *cls, *names, *colso, *luto, *strs;
  int kind;
  if (!PyArg_ParseTuple(args, "O!OiO!OOO!", &PySet_Type, &out, &cls, &kind, &PyTuple_Type, &names, &colso, &luto,
                        &PyList_Type, &strs))
    return NULL;
  if (!PyType_Check(cls)) {
    PyErr_SetString(PyExc_TypeError, "cls must be a type");
    return NULL;
  }
  Py_buffer cb, lb;
  if (get_u32(colso, &cb, "cols") < 0) return NULL;
  if (get_u32(luto, &lb, "lut") < 0) {
    PyBuffer_Release(&cb);
    return NULL;
  }
  const Py_ssize_t k = PyTuple_GET_SIZE(names);
  const Py_ssize_t n = k ? (cb.len / 4) / k : 0;
  const uint32_t *cols = (const uint32_t *)cb.buf, *lut = (const uint32_t *)lb.buf;
  const Py_ssize_t nlut = lb.len / 4;
  PyObject *empty = PyTuple_New(0), *vars = PyFrozenSet_New(names);
  PyObject *result = NULL;
  if (!empty || !vars) goto done;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject *d = PyDict_New();
    if (!d) goto done;
    if (PyDict_SetItem(d, s_variables, vars) < 0 || PyDict_SetItem(d, s_frozen, Py_True) < 0) {
      Py_DECREF(d);
      goto done;
    }
    Py_hash_t h;
    if (kind == 0) {
      PyObject *m = PyDict_New(), *vals = PyTuple_New(k);
      if (!m || !vals) {
        Py_XDECREF(m); Py_XDECREF(vals); Py_DECREF(d);
        goto done;
      }
      int bad = 0;
      for (Py_ssize_t c = 0; c < k && !bad; ++c) {
        PyObject *v = value_of(lut, nlut, strs, cols[c * n + i]);
        if (!v || PyDict_SetItem(m, PyTuple_GET_ITEM(names, c), v) < 0) bad = 1;
        else {
          Py_INCREF(v);
          PyTuple_SET_ITEM(vals, c, v);
        }
      }
      PyObject *fv = bad ? NULL : PyFrozenSet_New(vals);
      Py_DECREF(vals);
      if (fv && fast_hash_ok && k <= 4) {
        Py_uhash_t lanes[4];
        for (Py_ssize_t c = 0; c < k; ++c)
          lanes[c] = pair_hash((Py_uhash_t)PyObject_Hash(PyTuple_GET_ITEM(names, c)),
                               (Py_uhash_t)PyObject_Hash(value_of(lut, nlut, strs, cols[c * n + i])));
        h = small_frozenset_hash(lanes, k);
      } else {
        h = fv ? items_hash(m) : -1;
      }
      if (h == -1 || PyDict_SetItem(d, s_mapping, m) < 0 || PyDict_SetItem(d, s_values, fv) < 0) {
        Py_XDECREF(fv); Py_DECREF(m); Py_DECREF(d);
        goto done;
      }
      Py_DECREF(fv);
      Py_DECREF(m);
    } else {
      /* symbols: var -> count, values: value -> count (assign(), :207-214) */
      PyObject *sym = PyDict_New(), *val = PyDict_New();
      if (!sym || !val) {
        Py_XDECREF(sym); Py_XDECREF(val); Py_DECREF(d);
        goto done;
      }
      int bad = 0;
      for (Py_ssize_t c = 0; c < k && !bad; ++c) {
        PyObject *var = PyTuple_GET_ITEM(names, c);
        PyObject *v = value_of(lut, nlut, strs, cols[c * n + i]);
        if (!v) { bad = 1; break; }
        PyObject *cs = PyDict_GetItemWithError(sym, var), *cv = PyDict_GetItemWithError(val, v);
        if (PyErr_Occurred()) { bad = 1; break; }
        PyObject *ns = PyLong_FromLong(cs ? PyLong_AsLong(cs) + 1 : 1);
        PyObject *nv = PyLong_FromLong(cv ? PyLong_AsLong(cv) + 1 : 1);
        if (!ns || !nv || PyDict_SetItem(sym, var, ns) < 0 || PyDict_SetItem(val, v, nv) < 0) bad = 1;
        Py_XDECREF(ns);
        Py_XDECREF(nv);
      }
      Py_hash_t hs = bad ? -1 : items_hash(sym), hv = hs == -1 ? -1 : items_hash(val);
      PyObject *pair = hv == -1 ? NULL : Py_BuildValue("(nn)", (Py_ssize_t)hs, (Py_ssize_t)hv);
      h = pair ? PyObject_Hash(pair) : -1;
      Py_XDECREF(pair);
      if (h == -1 || PyDict_SetItem(d, s_symbols, sym) < 0 || PyDict_SetItem(d, s_values, val) < 0) {
        Py_DECREF(sym); Py_DECREF(val); Py_DECREF(d);
        goto done;
      }
      Py_DECREF(sym);
      Py_DECREF(val);
    }
    PyObject *hh = PyLong_FromSsize_t((Py_ssize_t)h);
    if (!hh || PyDict_SetItem(d, s_hash, hh) < 0) {
      Py_XDECREF(hh); Py_DECREF(d);
      goto done;
    }
    Py_DECREF(hh);
    PyObject *obj = new_instance((PyTypeObject *)cls, empty, d);
    if (!obj) goto done;
    int rc = PySet_Add(out, obj);
    Py_DECREF(obj);
    if (rc < 0) goto done;
  }
  result = Py_None;
  Py_INCREF(result);
done:
  Py_XDECREF(empty);
  Py_XDECREF(vars);
  PyBuffer_Release(&cb);
  PyBuffer_Release(&lb);
  return result;
}

/* format_set(s, ordered_cls) == str(s) */
static PyObject *format_set(PyObject *self, PyObject *args) {
  PyObject *s, *ocls;
  if (!PyArg_ParseTuple(args, "OO", &s, &ocls)) return NULL;
  if (!PyAnySet_Check(s)) return PyObject_Str(s);
  if (PySet_GET_SIZE(s) == 0) return PyObject_Repr(s);
  PyObject *parts = PyList_New(0), *it = PyObject_GetIter(s), *x, *res = NULL;
  if (!parts || !it) goto done;
  while ((x = PyIter_Next(it))) {
    PyObject *r;
    if ((PyObject *)Py_TYPE(x) == ocls) {
      PyObject **dp = _PyObject_GetDictPtr(x);
      PyObject *m = dp && *dp ? PyDict_GetItemWithError(*dp, s_mapping) : NULL;
      r = m ? PyObject_Repr(m) : PyObject_Repr(x);
    } else {
      r = PyObject_Repr(x);
    }
    Py_DECREF(x);
    if (!r || PyList_Append(parts, r) < 0) {
      Py_XDECREF(r);
      goto done;
    }
    Py_DECREF(r);
  }
  if (PyErr_Occurred()) goto done;
  {
    PyObject *sep = PyUnicode_FromString(", ");
    PyObject *body = sep ? PyUnicode_Join(sep, parts) : NULL;
    Py_XDECREF(sep);
    if (body) res = PyUnicode_FromFormat("{%U}", body);
    Py_XDECREF(body);
  }
done:
  Py_XDECREF(parts);
  Py_XDECREF(it);
  return res;
}

/* Handle strings of answer rows (HipDB.get_matched_links & co., the
 * reference's [(handle, targets)] lists, redis_mongo_db.py:235-279): a
 * 32-char lowercase hex str per digest, written straight into the str's
 * buffer (the Python path formats ~3x slower through bytes.hex() + slicing),
 * with a small direct-mapped cache so a target repeated across rows (a
 * schema node) is one shared str. */
static const char HEXD[] = "0123456789abcdef";

static PyObject *hex_str(const uint32_t *w) {
  PyObject *s = PyUnicode_New(32, 127);
  if (!s) return NULL;
  Py_UCS1 *p = PyUnicode_1BYTE_DATA(s);
  const uint8_t *b = (const uint8_t *)w;          /* digest bytes in memory order (little-endian words) */
  for (int i = 0; i < 16; ++i) {
    p[2 * i] = (Py_UCS1)HEXD[b[i] >> 4];
    p[2 * i + 1] = (Py_UCS1)HEXD[b[i] & 15];
  }
  return s;
}

#define HEX_CACHE 4096
typedef struct {
  uint32_t id[HEX_CACHE];
  PyObject *s[HEX_CACHE];
} HexCache;

static void hc_init(HexCache *c) {
  for (int i = 0; i < HEX_CACHE; ++i) {
    c->id[i] = 0xFFFFFFFFu;
    c->s[i] = NULL;
  }
}
static void hc_free(HexCache *c) {
  for (int i = 0; i < HEX_CACHE; ++i) Py_XDECREF(c->s[i]);
}
/* new reference to the str of atom `id` (digest words at w) */
static PyObject *hc_get(HexCache *c, uint32_t id, const uint32_t *w) {
  const uint32_t slot = (id * 2654435761u) >> 20;   /* 12 bits */
  if (c->id[slot] == id && c->s[slot]) {
    Py_INCREF(c->s[slot]);
    return c->s[slot];
  }
  PyObject *s = hex_str(w);
  if (!s) return NULL;
  Py_XDECREF(c->s[slot]);
  Py_INCREF(s);
  c->s[slot] = s;
  c->id[slot] = id;
  return s;
}

/* digest words of row r of column col: dig indexed by ids (the host mirror,
 * ids = (k, n) u32), or dig = (k, n, 4) gathered per column (ids None) */
typedef struct {
  const uint32_t *dig, *ids;
  Py_ssize_t n_dig, n;
} HexSrc;

static const uint32_t *src_row(const HexSrc *h, int col, Py_ssize_t r, uint32_t *id) {
  if (!h->ids) {
    *id = 0xFFFFFFFFu;                              /* no id: uncached */
    return h->dig + ((Py_ssize_t)col * h->n + r) * 4;
  }
  *id = h->ids[(Py_ssize_t)col * h->n + r];
  if ((Py_ssize_t)*id >= h->n_dig) {
    PyErr_SetString(PyExc_IndexError, "hex: atom id outside the digest table");
    return NULL;
  }
  return h->dig + (Py_ssize_t)*id * 4;
}

static PyObject *src_str(HexCache *c, const HexSrc *h, int col, Py_ssize_t r) {
  uint32_t id;
  const uint32_t *w = src_row(h, col, r, &id);
  if (!w) return NULL;
  return id == 0xFFFFFFFFu ? hex_str(w) : hc_get(c, id, w);
}

static int open_src(PyObject *dig, PyObject *ids, int k, Py_ssize_t n, Py_buffer *db, Py_buffer *ib, HexSrc *h) {
  if (get_u32(dig, db, "digests") < 0) return -1;
  h->dig = (const uint32_t *)db->buf;
  h->n_dig = db->len / 16;
  h->n = n;
  h->ids = NULL;
  if (ids != Py_None) {
    if (get_u32(ids, ib, "ids") < 0) {
      PyBuffer_Release(db);
      return -1;
    }
    if (ib->len / 4 < (Py_ssize_t)k * n) {
      PyErr_SetString(PyExc_ValueError, "hex: ids shorter than k * n");
      PyBuffer_Release(ib);
      PyBuffer_Release(db);
      return -1;
    }
    h->ids = (const uint32_t *)ib->buf;
  } else if (h->n_dig < (Py_ssize_t)k * n) {
    PyErr_SetString(PyExc_ValueError, "hex: digests shorter than k * n rows");
    PyBuffer_Release(db);
    return -1;
  }
  return 0;
}

/* hex_list(digests, ids | None, n[, store]) -> [str] of column 0.  store:
 * a list indexed by atom id holding each handle str made so far (None until
 * then): repeated answers share their str objects instead of formatting
 * them again (HipDB keeps one per prefetched KB) */
static PyObject *hex_list(PyObject *self, PyObject *args) {
  PyObject *dig, *ids, *store = Py_None;
  Py_ssize_t n;
  if (!PyArg_ParseTuple(args, "OOn|O", &dig, &ids, &n, &store)) return NULL;
  if (store != Py_None && (!PyList_Check(store) || ids == Py_None)) {
    PyErr_SetString(PyExc_TypeError, "hex_list: store must be a list (with ids)");
    return NULL;
  }
  Py_buffer db, ib;
  HexSrc h;
  if (open_src(dig, ids, 1, n, &db, &ib, &h) < 0) return NULL;
  HexCache *c = PyMem_Malloc(sizeof(HexCache));
  PyObject *out = c ? PyList_New(n) : NULL;
  if (c) hc_init(c);
  else PyErr_NoMemory();
  const Py_ssize_t ns = store != Py_None ? PyList_GET_SIZE(store) : 0;
  for (Py_ssize_t r = 0; out && r < n; ++r) {
    PyObject *s = NULL;
    if (ns) {
      const Py_ssize_t id = (Py_ssize_t)h.ids[r];
      if (id < ns) {
        PyObject *have = PyList_GET_ITEM(store, id);
        if (have != Py_None) {
          Py_INCREF(have);
          PyList_SET_ITEM(out, r, have);
          continue;
        }
        uint32_t aid;
        const uint32_t *w = src_row(&h, 0, r, &aid);
        s = w ? hex_str(w) : NULL;
        if (s) {
          Py_INCREF(s);
          PyList_SetItem(store, id, s);                /* steals the extra reference; drops the None */
        }
      }
    }
    if (!s) s = PyErr_Occurred() ? NULL : src_str(c, &h, 0, r);
    if (!s) {
      Py_CLEAR(out);
      break;
    }
    PyList_SET_ITEM(out, r, s);
  }
  if (c) {
    hc_free(c);
    PyMem_Free(c);
  }
  if (ids != Py_None) PyBuffer_Release(&ib);
  PyBuffer_Release(&db);
  return out;
}

/* hex_pairs(digests, ids | None, k, n, tuple_targets) ->
 * [(link, [t0 .. t_{k-2}]) | (link, (t0 ..))] over k columns of n rows */
static PyObject *hex_pairs(PyObject *self, PyObject *args) {
  PyObject *dig, *ids;
  int k, tup;
  Py_ssize_t n;
  if (!PyArg_ParseTuple(args, "OOinp", &dig, &ids, &k, &n, &tup)) return NULL;
  if (k < 1) {
    PyErr_SetString(PyExc_ValueError, "hex_pairs: k >= 1 columns");
    return NULL;
  }
  Py_buffer db, ib;
  HexSrc h;
  if (open_src(dig, ids, k, n, &db, &ib, &h) < 0) return NULL;
  HexCache *c = PyMem_Malloc(sizeof(HexCache));
  PyObject *out = c ? PyList_New(n) : NULL;
  if (c) hc_init(c);
  else PyErr_NoMemory();
  for (Py_ssize_t r = 0; out && r < n; ++r) {
    PyObject *link = src_str(c, &h, 0, r);
    PyObject *tg = link ? (tup ? PyTuple_New(k - 1) : PyList_New(k - 1)) : NULL;
    PyObject *pair = tg ? PyTuple_New(2) : NULL;
    if (!pair) {
      Py_XDECREF(link);
      Py_XDECREF(tg);
      Py_CLEAR(out);
      break;
    }
    PyTuple_SET_ITEM(pair, 0, link);
    PyTuple_SET_ITEM(pair, 1, tg);
    PyList_SET_ITEM(out, r, pair);
    for (int col = 1; col < k; ++col) {
      PyObject *s = src_str(c, &h, col, r);
      if (!s) {
        Py_CLEAR(out);
        break;
      }
      if (tup) PyTuple_SET_ITEM(tg, col - 1, s);
      else PyList_SET_ITEM(tg, col - 1, s);
    }
  }
  if (c) {
    hc_free(c);
    PyMem_Free(c);
  }
  if (ids != Py_None) PyBuffer_Release(&ib);
  PyBuffer_Release(&db);
  return out;
}

/* seed(cache, strs, ids, arity) -> None: cache[strs[i]] = (ids[i], 2, arity)
 * (strs[i] a handle str, or a (handle, targets) pair)
 * for every handle not yet in the dict (HipDB's handle cache: the links of a
 * pattern answer become host lookups for get_link_targets / get_link_type;
 * the reference's Redis answers carry the same pairs, redis_mongo_db.py:235-252) */
static PyObject *seed(PyObject *self, PyObject *args) {
  PyObject *cache, *strs, *ids;
  long arity;
  if (!PyArg_ParseTuple(args, "O!O!Ol", &PyDict_Type, &cache, &PyList_Type, &strs, &ids, &arity)) return NULL;
  Py_buffer ib;
  if (get_u32(ids, &ib, "ids") < 0) return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(strs);
  if (ib.len / 4 < n) {
    PyBuffer_Release(&ib);
    PyErr_SetString(PyExc_ValueError, "seed: fewer ids than handles");
    return NULL;
  }
  const uint32_t *id = (const uint32_t *)ib.buf;
  PyObject *two = PyLong_FromLong(2), *ar = PyLong_FromLong(arity);
  int bad = !two || !ar;
  for (Py_ssize_t i = 0; !bad && i < n; ++i) {
    PyObject *h = PyList_GET_ITEM(strs, i);
    if (PyTuple_Check(h) && PyTuple_GET_SIZE(h) > 0) h = PyTuple_GET_ITEM(h, 0);   /* a (link, targets) pair */
    const int has = PyDict_Contains(cache, h);
    if (has < 0) { bad = 1; break; }
    if (has) continue;
    PyObject *v = PyTuple_New(3), *x = v ? PyLong_FromUnsignedLong(id[i]) : NULL;
    if (!x) { Py_XDECREF(v); bad = 1; break; }
    PyTuple_SET_ITEM(v, 0, x);
    Py_INCREF(two);
    PyTuple_SET_ITEM(v, 1, two);
    Py_INCREF(ar);
    PyTuple_SET_ITEM(v, 2, ar);
    if (PyDict_SetItem(cache, h, v) < 0) bad = 1;
    Py_DECREF(v);
  }
  Py_XDECREF(two);
  Py_XDECREF(ar);
  PyBuffer_Release(&ib);
  if (bad) return NULL;
  Py_RETURN_NONE;
}

/* ---- query-shape cache hits (pattern_matcher._lower) ---------------------
 * shape(expr): the structure key pattern_matcher._shape builds, nodes
 * appended to `nodes` in walk order; NULL with no exception set = no shape
 * (_NoShape: an unordered link type, a link whose targets are all nodes, an
 * unknown expression kind). */
static PyObject *s_k, *s_atom_type, *s_name, *s_type, *s_ordered, *s_targets, *s_link_type, *s_term, *s_terms,
    *s_handle, *s_copy, *s_tags;

static PyObject *shape_of(PyObject *e, PyObject *nodes, PyObject *unordered, int depth) {
  if (depth > 64) return NULL;
  PyObject *k = PyObject_GetAttr(e, s_k);
  if (!k) { PyErr_Clear(); return NULL; }
  const char *ks = PyUnicode_Check(k) ? PyUnicode_AsUTF8(k) : NULL;
  PyObject *out = NULL;
  if (!ks) { PyErr_Clear(); Py_DECREF(k); return NULL; }
  if (!strcmp(ks, "n")) {
    if (PyList_Append(nodes, e) == 0) out = PyObject_GetAttr(e, s_atom_type);
  } else if (!strcmp(ks, "v")) {
    PyObject *n = PyObject_GetAttr(e, s_name);
    if (n) out = Py_BuildValue("(sN)", "v", n);
  } else if (!strcmp(ks, "tv")) {
    PyObject *n = PyObject_GetAttr(e, s_name), *t = n ? PyObject_GetAttr(e, s_type) : NULL;
    if (t) out = Py_BuildValue("(sNN)", "tv", n, t);
    else Py_XDECREF(n);
  } else if (!strcmp(ks, "l")) {
    PyObject *at = PyObject_GetAttr(e, s_atom_type), *od = at ? PyObject_GetAttr(e, s_ordered) : NULL;
    PyObject *ts = od ? PyObject_GetAttr(e, s_targets) : NULL;
    PyObject *seq = ts ? PySequence_Fast(ts, "targets") : NULL;
    int ok = seq != NULL;
    if (ok) {
      const int un = PySet_Contains(unordered, at);
      ok = un == 0;
    }
    PyObject *tup = NULL;
    if (ok) {
      const Py_ssize_t m = PySequence_Fast_GET_SIZE(seq);
      int all_nodes = 1;
      tup = PyTuple_New(m);
      for (Py_ssize_t i = 0; tup && i < m; ++i) {
        PyObject *t = PySequence_Fast_GET_ITEM(seq, i);
        PyObject *tk = PyObject_GetAttr(t, s_k);
        if (!tk) { ok = 0; break; }
        const char *tks = PyUnicode_Check(tk) ? PyUnicode_AsUTF8(tk) : NULL;
        if (!tks || strcmp(tks, "n")) all_nodes = 0;
        Py_DECREF(tk);
        PyObject *x = shape_of(t, nodes, unordered, depth + 1);
        if (!x) { ok = 0; break; }
        PyTuple_SET_ITEM(tup, i, x);
      }
      if (!tup || all_nodes) ok = 0;
    }
    if (ok) {
      out = PyTuple_Pack(4, PyTuple_GET_ITEM(s_tags, 0), at, od, tup);
    }
    Py_XDECREF(tup);
    Py_XDECREF(seq);
    Py_XDECREF(ts);
    Py_XDECREF(od);
    Py_XDECREF(at);
  } else if (!strcmp(ks, "t")) {
    PyObject *lt = PyObject_GetAttr(e, s_link_type), *od = lt ? PyObject_GetAttr(e, s_ordered) : NULL;
    PyObject *ts = od ? PyObject_GetAttr(e, s_targets) : NULL;
    PyObject *seq = ts ? PySequence_Fast(ts, "targets") : NULL;
    PyObject *tup = seq ? PyTuple_New(PySequence_Fast_GET_SIZE(seq)) : NULL;
    int ok = tup != NULL;
    for (Py_ssize_t i = 0; ok && i < PyTuple_GET_SIZE(tup); ++i) {
      PyObject *v = PySequence_Fast_GET_ITEM(seq, i);
      PyObject *n = PyObject_GetAttr(v, s_name), *t = n ? PyObject_GetAttr(v, s_type) : NULL;
      if (!t) { Py_XDECREF(n); ok = 0; break; }
      PyObject *pair = PyTuple_New(2);
      if (!pair) { Py_DECREF(n); Py_DECREF(t); ok = 0; break; }
      PyTuple_SET_ITEM(pair, 0, n);
      PyTuple_SET_ITEM(pair, 1, t);
      PyTuple_SET_ITEM(tup, i, pair);
    }
    if (ok) out = PyTuple_Pack(4, PyTuple_GET_ITEM(s_tags, 1), lt, od, tup);
    Py_XDECREF(tup);
    Py_XDECREF(seq);
    Py_XDECREF(ts);
    Py_XDECREF(od);
    Py_XDECREF(lt);
  } else if (!strcmp(ks, "x")) {
    PyObject *t = PyObject_GetAttr(e, s_term);
    PyObject *x = t ? shape_of(t, nodes, unordered, depth + 1) : NULL;
    if (x) out = PyTuple_Pack(2, PyTuple_GET_ITEM(s_tags, 2), x);
    Py_XDECREF(x);
    Py_XDECREF(t);
  } else if (!strcmp(ks, "a") || !strcmp(ks, "o")) {
    PyObject *ts = PyObject_GetAttr(e, s_terms);
    PyObject *seq = ts ? PySequence_Fast(ts, "terms") : NULL;
    PyObject *tup = seq ? PyTuple_New(PySequence_Fast_GET_SIZE(seq)) : NULL;
    int ok = tup != NULL;
    for (Py_ssize_t i = 0; ok && i < PyTuple_GET_SIZE(tup); ++i) {
      PyObject *x = shape_of(PySequence_Fast_GET_ITEM(seq, i), nodes, unordered, depth + 1);
      if (!x) { ok = 0; break; }
      PyTuple_SET_ITEM(tup, i, x);
    }
    if (ok) out = PyTuple_Pack(2, k, tup);
    Py_XDECREF(tup);
    Py_XDECREF(seq);
    Py_XDECREF(ts);
  }
  Py_DECREF(k);
  if (!out) PyErr_Clear();
  return out;
}

/* plan_words(expr, shapes, no_overload, node_handles, handle_cache, node_dir,
 * unordered[, get_node_handle]) -> a copy of the cached words of expr's query shape with its
 * nodes' atom ids patched in, or None: pattern_matcher._lower's shape-cache
 * hit, restated (the caller takes its Python path on None -- a shape not
 * cached yet, a node whose handle (without get_node_handle) or id is not
 * cached, a node absent). */
static PyObject *plan_words(PyObject *self, PyObject *args) {
  PyObject *e, *shapes, *no_overload, *node_handles, *cache, *node_dir, *unordered, *hfun = NULL;
  if (!PyArg_ParseTuple(args, "OO!OO!O!OO|O", &e, &PyDict_Type, &shapes, &no_overload, &PyDict_Type, &node_handles,
                        &PyDict_Type, &cache, &node_dir, &unordered, &hfun))
    return NULL;
  if (!PyAnySet_Check(unordered)) { PyErr_SetString(PyExc_TypeError, "unordered: a set"); return NULL; }
  PyObject *nodes = PyList_New(0);
  if (!nodes) return NULL;
  PyObject *shape = shape_of(e, nodes, unordered, 0), *res = NULL;
  PyObject *key = shape ? PyTuple_Pack(2, no_overload, shape) : NULL;
  PyObject *hit = key ? PyDict_GetItemWithError(shapes, key) : NULL;   /* borrowed */
  Py_XDECREF(key);
  Py_XDECREF(shape);
  if (!hit || !PyTuple_Check(hit) || PyTuple_GET_SIZE(hit) != 2) goto done;
  {
    const Py_ssize_t nn = PyList_GET_SIZE(nodes);
    uint32_t ids_small[64];
    if (nn > 64) goto done;
    for (Py_ssize_t i = 0; i < nn; ++i) {
      PyObject *n = PyList_GET_ITEM(nodes, i);
      PyObject *h = PyObject_GetAttr(n, s_handle);
      if (!h) { PyErr_Clear(); goto done; }
      if (!PyObject_IsTrue(h)) {
        Py_DECREF(h);
        PyObject *t = PyObject_GetAttr(n, s_atom_type), *nm = t ? PyObject_GetAttr(n, s_name) : NULL;
        PyObject *tk = nm ? PyTuple_Pack(2, t, nm) : NULL;
        Py_XDECREF(t);
        Py_XDECREF(nm);
        h = tk ? PyDict_GetItemWithError(node_handles, tk) : NULL;
        if (h) {
          Py_INCREF(h);
        } else if (tk && !PyErr_Occurred() && hfun && hfun != Py_None) {
          /* a fresh anchor: its handle from the DB's own (memoising) get_node_handle */
          h = PyObject_CallObject(hfun, tk);
        }
        Py_XDECREF(tk);
        if (!h) { PyErr_Clear(); goto done; }
        if (PyObject_SetAttr(n, s_handle, h) < 0) { Py_DECREF(h); PyErr_Clear(); goto done; }
      }
      PyObject *r = PyDict_GetItemWithError(cache, h);              /* (id, category, arity) */
      if (!r && !PyErr_Occurred() && node_dir != Py_None && PyDict_Check(node_dir)) {
        PyObject *nid = PyDict_GetItemWithError(node_dir, h);
        if (nid) {
          PyObject *v = Py_BuildValue("(Oii)", nid, 1, 0);
          if (v && PyDict_SetItem(cache, h, v) == 0) r = v;
          Py_XDECREF(v);                                              /* the dict holds it */
        }
      }
      Py_DECREF(h);
      if (!r || !PyTuple_Check(r) || PyTuple_GET_SIZE(r) < 2) { PyErr_Clear(); goto done; }
      const long aid = PyLong_AsLong(PyTuple_GET_ITEM(r, 0)), cat = PyLong_AsLong(PyTuple_GET_ITEM(r, 1));
      if (PyErr_Occurred()) { PyErr_Clear(); goto done; }
      if (aid < 0 || cat != 1) goto done;                            /* not a node of the KB */
      ids_small[i] = (uint32_t)aid;
    }
    PyObject *w = PyObject_CallMethodObjArgs(PyTuple_GET_ITEM(hit, 0), s_copy, NULL);
    if (!w) { PyErr_Clear(); goto done; }
    Py_buffer wb;
    if (PyObject_GetBuffer(w, &wb, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0 || wb.itemsize != 4) {
      PyErr_Clear();
      Py_DECREF(w);
      goto done;
    }
    uint32_t *wp = (uint32_t *)wb.buf;
    const Py_ssize_t nw = wb.len / 4;
    PyObject *patches = PySequence_Fast(PyTuple_GET_ITEM(hit, 1), "patches");
    int ok = patches != NULL;
    for (Py_ssize_t i = 0; ok && i < PySequence_Fast_GET_SIZE(patches); ++i) {
      PyObject *pr = PySequence_Fast_GET_ITEM(patches, i);
      if (!PyTuple_Check(pr) || PyTuple_GET_SIZE(pr) != 2) { ok = 0; break; }
      const Py_ssize_t wi = PyLong_AsSsize_t(PyTuple_GET_ITEM(pr, 0)), ki = PyLong_AsSsize_t(PyTuple_GET_ITEM(pr, 1));
      if (PyErr_Occurred() || wi < 0 || wi >= nw || ki < 0 || ki >= nn) { ok = 0; break; }
      wp[wi] = ids_small[ki];
    }
    Py_XDECREF(patches);
    PyBuffer_Release(&wb);
    if (!ok) { PyErr_Clear(); Py_DECREF(w); goto done; }
    res = w;
  }
done:
  Py_DECREF(nodes);
  if (PyErr_Occurred()) PyErr_Clear();
  if (res) return res;
  Py_RETURN_NONE;
}

static PyObject *fast_hash_enabled(PyObject *self, PyObject *noargs);

static PyMethodDef methods[] = {
    {"plan_words", plan_words, METH_VARARGS, "Cached plan words of an expression's query shape, node ids patched."},
    {"seed", seed, METH_VARARGS, "Seed the handle cache with (id, 2, arity) per new link handle."},
    {"add_rows", add_rows, METH_VARARGS, "Add Assignment objects built from a binding table to a set."},
    {"format_set", format_set, METH_VARARGS, "str() of a set of assignments."},
    {"hex_list", hex_list, METH_VARARGS, "Handle strs of n atoms (digest table + ids, or gathered digests)."},
    {"hex_pairs", hex_pairs, METH_VARARGS, "[(link, targets)] handle rows of k id columns."},
    {"fast_hash_enabled", fast_hash_enabled, METH_NOARGS, "True when the C restatement of the hashes is in use."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_assign", NULL, -1, methods};

/* fast_hash_ok: the restated hashes equal the interpreter's on sample rows */
static void check_fast_hash(void) {
  fast_hash_ok = 0;
  for (int k = 1; k <= 4; ++k)
    for (int trial = 0; trial < 8; ++trial) {
      PyObject *d = PyDict_New();
      Py_uhash_t lanes[4];
      for (int c = 0; c < k; ++c) {
        PyObject *key = PyUnicode_FromFormat("$v%d_%d", c, trial);
        PyObject *val = PyUnicode_FromFormat("%032x", 7919 * (trial + 1) * (c + 3));
        if (!key || !val || PyDict_SetItem(d, key, val) < 0) {
          PyErr_Clear();
          Py_XDECREF(key); Py_XDECREF(val); Py_DECREF(d);
          return;
        }
        lanes[c] = pair_hash((Py_uhash_t)PyObject_Hash(key), (Py_uhash_t)PyObject_Hash(val));
        Py_DECREF(key);
        Py_DECREF(val);
      }
      const Py_hash_t want = items_hash(d);
      Py_DECREF(d);
      if (want == -1) { PyErr_Clear(); return; }
      if (small_frozenset_hash(lanes, k) != want) return;
    }
  fast_hash_ok = 1;
}

static PyObject *fast_hash_enabled(PyObject *self, PyObject *noargs) { return PyBool_FromLong(fast_hash_ok); }

PyMODINIT_FUNC PyInit__assign(void) {
  check_fast_hash();
  s_variables = PyUnicode_InternFromString("variables");
  s_hash = PyUnicode_InternFromString("hash");
  s_frozen = PyUnicode_InternFromString("frozen");
  s_mapping = PyUnicode_InternFromString("mapping");
  s_values = PyUnicode_InternFromString("values");
  s_symbols = PyUnicode_InternFromString("symbols");
  s_k = PyUnicode_InternFromString("_k");
  s_atom_type = PyUnicode_InternFromString("atom_type");
  s_name = PyUnicode_InternFromString("name");
  s_type = PyUnicode_InternFromString("type");
  s_ordered = PyUnicode_InternFromString("ordered");
  s_targets = PyUnicode_InternFromString("targets");
  s_link_type = PyUnicode_InternFromString("link_type");
  s_term = PyUnicode_InternFromString("term");
  s_terms = PyUnicode_InternFromString("terms");
  s_handle = PyUnicode_InternFromString("handle");
  s_copy = PyUnicode_InternFromString("copy");
  s_tags = Py_BuildValue("(sss)", "l", "t", "x");
  return PyModule_Create(&module);
}
