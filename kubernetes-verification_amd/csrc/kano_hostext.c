/* Host interning at C speed (CPython C API): the two per-pod loops of the
 * drop-in build_matrix / user_crosscheck that dominated its cold time
 * (C3, 10^5 pods: 0.41 s of a 0.44 s build_matrix in Python).
 *
 *   intern_column(labels, key, ids, out) -> next_id
 *       kano/_intern.py _ValueIndex.pod_id over one key's column: for each
 *       label dict (exact dicts only), ABSENT (-1) where the key is missing,
 *       NEVER_MATCH (-3) where v != v (NaN-like, checked first, as pod_id
 *       does), else the id of v's equality class in `ids` (a dict, value ->
 *       id, filled in first-seen order).  `out` is a writable int32 buffer of
 *       len(labels).  Raises TypeError on an unhashable value (the caller's
 *       per-pod loop then handles the column, unhashables included) and
 *       ValueError on a non-dict label map.
 *   group_ids(containers, cls, label, out) -> number of groups
 *       kano/_intern.py group_ids: gid[i] = dense id (first appearance) of
 *       containers[i].labels.get(label, "") -- getValueOrDefault of the
 *       reference's Container (kano_py/kano/model.py:25-29,
 *       algorithm.py:20-24); every container must be exactly `cls` with a
 *       dict `labels` (ValueError otherwise: the caller's loop runs instead).
 *
 * No state, no GPU: plumbing for the host side of the drop-in boundary. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>
#include <stdint.h>

#define ABSENT (-1)
#define NEVER_MATCH (-3)

/* Python's `v != v` (PyObject_RichCompareBool would shortcut on identity and
 * call a NaN equal to itself); an exception counts as False, as in pod_id. */
static int self_ne(PyObject* v) {
  PyObject* r = PyObject_RichCompare(v, v, Py_NE);
  if (r == NULL) {
    PyErr_Clear();
    return 0;
  }
  int t = PyObject_IsTrue(r);
  Py_DECREF(r);
  if (t < 0) {
    PyErr_Clear();
    t = 0;
  }
  return t;
}

/* The byte offset of a __slots__ member of type cls (a member descriptor),
 * or -1: reading it directly skips the generic attribute lookup. */
static Py_ssize_t slot_offset(PyObject* cls, const char* name) {
  if (!PyType_Check(cls)) return -1;
  PyObject* d = PyObject_GetAttrString(cls, name);
  if (d == NULL) {
    PyErr_Clear();
    return -1;
  }
  Py_ssize_t off = -1;
  if (Py_TYPE(d) == &PyMemberDescr_Type) {
    PyMemberDef* m = ((PyMemberDescrObject*)d)->d_member;
    if (m->type == T_OBJECT_EX || m->type == T_OBJECT) off = m->offset;
  }
  Py_DECREF(d);
  return off;
}

/* a slot's value (new reference), AttributeError when unset */
static PyObject* slot_get(PyObject* o, Py_ssize_t off, PyObject* name) {
  if (off < 0) return PyObject_GetAttr(o, name);
  PyObject* v = *(PyObject**)((char*)o + off);
  if (v == NULL) {
    PyErr_SetObject(PyExc_AttributeError, name);
    return NULL;
  }
  Py_INCREF(v);
  return v;
}

static int get_out(PyObject* obj, Py_buffer* view, Py_ssize_t n) {
  if (PyObject_GetBuffer(obj, view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0) return -1;
  if (view->len != n * (Py_ssize_t)sizeof(int32_t)) {
    PyBuffer_Release(view);
    PyErr_SetString(PyExc_ValueError, "out: an int32 buffer of len(items) expected");
    return -1;
  }
  return 0;
}

static PyObject* intern_column(PyObject* self, PyObject* args) {
  PyObject *labels, *key, *ids, *outobj;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!OO!O", &PyList_Type, &labels, &key, &PyDict_Type, &ids, &outobj))
    return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(labels);
  Py_buffer view;
  if (get_out(outobj, &view, n) < 0) return NULL;
  int32_t* out = (int32_t*)view.buf;
  Py_ssize_t next = PyDict_GET_SIZE(ids);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* lab = PyList_GET_ITEM(labels, i);
    if (!PyDict_CheckExact(lab)) {
      PyErr_SetString(PyExc_ValueError, "labels: exact dicts expected");
      goto fail;
    }
    PyObject* v = PyDict_GetItemWithError(lab, key);   /* borrowed */
    if (v == NULL) {
      if (PyErr_Occurred()) goto fail;
      out[i] = ABSENT;
      continue;
    }
    /* pod_id: `if v != v` first (an exception there counts as False) */
    const int ne = self_ne(v);
    if (ne) {
      out[i] = NEVER_MATCH;
      continue;
    }
    PyObject* got = PyDict_GetItemWithError(ids, v);    /* TypeError if unhashable */
    if (got == NULL) {
      if (PyErr_Occurred()) goto fail;
      PyObject* id = PyLong_FromSsize_t(next);
      if (id == NULL) goto fail;
      const int rc = PyDict_SetItem(ids, v, id);
      Py_DECREF(id);
      if (rc < 0) goto fail;
      out[i] = (int32_t)next++;
    } else {
      out[i] = (int32_t)PyLong_AsLong(got);
    }
  }
  PyBuffer_Release(&view);
  return PyLong_FromSsize_t(next);
fail:
  PyBuffer_Release(&view);
  return NULL;
}

/* scan_labels(labels, cand, ids_list, out2d) -> keys
 *   One pass over the pods' label dicts: KEYS (every key any pod carries, a
 *   dict in first-seen order: the labelMap of kano_py/kano/model.py:127-133)
 *   and, for every candidate key cand[j], the column of value ids exactly as
 *   intern_column computes it into out2d[j] (ids_list[j] filled).  One pass
 *   instead of one per column: the label dicts are scattered over the heap,
 *   every visit is a cache miss.  Errors as intern_column. */
static PyObject* scan_labels(PyObject* self, PyObject* args) {
  PyObject *labels, *cand, *idsl, *outobj;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!O!O", &PyList_Type, &labels, &PyList_Type, &cand, &PyList_Type,
                        &idsl, &outobj))
    return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(labels), nc = PyList_GET_SIZE(cand);
  if (PyList_GET_SIZE(idsl) != nc) {
    PyErr_SetString(PyExc_ValueError, "ids_list: one dict per candidate key expected");
    return NULL;
  }
  for (Py_ssize_t j = 0; j < nc; ++j)
    if (!PyDict_CheckExact(PyList_GET_ITEM(idsl, j))) {
      PyErr_SetString(PyExc_ValueError, "ids_list: dicts expected");
      return NULL;
    }
  Py_buffer view;
  if (get_out(outobj, &view, n * nc) < 0) return NULL;
  int32_t* out = (int32_t*)view.buf;
  PyObject* keys = PyDict_New();
  if (keys == NULL) goto fail;
  Py_ssize_t* next = (Py_ssize_t*)PyMem_Calloc((size_t)(nc > 0 ? nc : 1), sizeof(Py_ssize_t));
  if (next == NULL) {
    PyErr_NoMemory();
    goto fail;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* lab = PyList_GET_ITEM(labels, i);
    if (!PyDict_CheckExact(lab)) {
      PyErr_SetString(PyExc_ValueError, "labels: exact dicts expected");
      goto fail_next;
    }
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(lab, &pos, &k, &v))
      if (PyDict_SetDefault(keys, k, Py_None) == NULL) goto fail_next;
    for (Py_ssize_t j = 0; j < nc; ++j) {
      int32_t* o = out + j * n + i;
      v = PyDict_GetItemWithError(lab, PyList_GET_ITEM(cand, j));
      if (v == NULL) {
        if (PyErr_Occurred()) goto fail_next;
        *o = ABSENT;
        continue;
      }
      const int ne = self_ne(v);
      if (ne) {
        *o = NEVER_MATCH;
        continue;
      }
      PyObject* ids = PyList_GET_ITEM(idsl, j);
      PyObject* got = PyDict_GetItemWithError(ids, v);
      if (got == NULL) {
        if (PyErr_Occurred()) goto fail_next;
        PyObject* id = PyLong_FromSsize_t(next[j]);
        if (id == NULL) goto fail_next;
        const int rc = PyDict_SetItem(ids, v, id);
        Py_DECREF(id);
        if (rc < 0) goto fail_next;
        *o = (int32_t)next[j]++;
      } else {
        *o = (int32_t)PyLong_AsLong(got);
      }
    }
  }
  PyMem_Free(next);
  PyBuffer_Release(&view);
  return keys;
fail_next:
  PyMem_Free(next);
fail:
  Py_XDECREF(keys);
  PyBuffer_Release(&view);
  return NULL;
}

/* A growable int32 / int64 array for the term CSRs. */
typedef struct {
  char* p;
  Py_ssize_t n, cap, w;
} Vec;

static int vec_push(Vec* v, int64_t x) {
  if (v->n == v->cap) {
    const Py_ssize_t cap = v->cap ? 2 * v->cap : 1024;
    char* q = (char*)PyMem_Realloc(v->p, (size_t)(cap * v->w));
    if (q == NULL) {
      PyErr_NoMemory();
      return -1;
    }
    v->p = q;
    v->cap = cap;
  }
  if (v->w == 8) ((int64_t*)v->p)[v->n++] = x;
  else ((int32_t*)v->p)[v->n++] = (int32_t)x;
  return 0;
}

static PyObject* vec_bytes(Vec* v) {
  return PyBytes_FromStringAndSize(v->p ? v->p : "", v->n * v->w);
}

/* policy_terms(sides, default, keys, cand_index, scan_ids, expr_cls)
 *     -> (col_keys, sel_off, sel_col, sel_val, alw_off, alw_col, alw_val)
 *   kano/_intern.py intern's term loop for the common case -- every policy's
 *   matcher the default equality (default[p] true) and no LabelExpression
 *   value: per policy, per side (working selector, working allow: exact
 *   dicts), per (k, rule) in insertion order: dropped when no pod carries k
 *   (k not in keys: quirk Q1, kano_py/kano/model.py:143,146), else (column of
 *   k -- numbered by first use --, rule_id(rule)) where rule_id is
 *   _ValueIndex.rule_id: NO_MATCH (-2) if rule != rule, else the id of rule's
 *   equality class in scan_ids[cand_index[k]], NO_MATCH when absent or
 *   unhashable (scan_labels saw no unhashable value in a scanned column).
 *   Raises LookupError when the case does not apply (a custom matcher, an
 *   expression, a non-dict side, a key not scanned): the caller's loop runs. */
#define NO_MATCH_RULE (-2)
static PyObject* policy_terms(PyObject* self, PyObject* args) {
  PyObject *sides, *deflt, *keys, *cidx, *sids, *ecls;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!O!O!O!O", &PyList_Type, &sides, &PyList_Type, &deflt,
                        &PyDict_Type, &keys, &PyDict_Type, &cidx, &PyList_Type, &sids, &ecls))
    return NULL;
  const Py_ssize_t P = PyList_GET_SIZE(sides);
  if (PyList_GET_SIZE(deflt) != P) {
    PyErr_SetString(PyExc_ValueError, "default: one flag per policy expected");
    return NULL;
  }
  PyObject* col_of = PyDict_New();      /* key -> column */
  PyObject* col_keys = PyList_New(0);
  PyObject* ids_of_col = PyList_New(0);
  Vec off[2] = {{NULL, 0, 0, 8}, {NULL, 0, 0, 8}};
  Vec col[2] = {{NULL, 0, 0, 4}, {NULL, 0, 0, 4}};
  Vec val[2] = {{NULL, 0, 0, 4}, {NULL, 0, 0, 4}};
  PyObject* res = NULL;
  if (col_of == NULL || col_keys == NULL || ids_of_col == NULL) goto done;
  for (int w = 0; w < 2; ++w)
    if (vec_push(&off[w], 0) < 0) goto done;
  for (Py_ssize_t p = 0; p < P; ++p) {
    PyObject* t = PyList_GET_ITEM(sides, p);
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) < 2 || PyList_GET_ITEM(deflt, p) != Py_True) {
      PyErr_SetString(PyExc_LookupError, "not the default-matcher case");
      goto done;
    }
    for (int w = 0; w < 2; ++w) {
      PyObject* side = PyTuple_GET_ITEM(t, w);
      if (!PyDict_CheckExact(side)) {
        PyErr_SetString(PyExc_LookupError, "non-dict side");
        goto done;
      }
      Py_ssize_t pos = 0;
      PyObject *k, *rule;
      while (PyDict_Next(side, &pos, &k, &rule)) {
        const int isx = PyObject_IsInstance(rule, ecls);
        if (isx < 0) goto done;
        if (isx) {
          PyErr_SetString(PyExc_LookupError, "expression term");
          goto done;
        }
        const int has = PyDict_Contains(keys, k);
        if (has < 0) goto done;
        if (!has) continue;                                  /* quirk Q1 */
        PyObject* c = PyDict_GetItemWithError(col_of, k);
        Py_ssize_t ci;
        PyObject* ids;
        if (c == NULL) {
          if (PyErr_Occurred()) goto done;
          PyObject* j = PyDict_GetItemWithError(cidx, k);
          if (j == NULL) {
            if (!PyErr_Occurred()) PyErr_SetString(PyExc_LookupError, "key not scanned");
            goto done;
          }
          ids = PyList_GetItem(sids, PyLong_AsSsize_t(j));
          if (ids == NULL) goto done;
          ci = PyList_GET_SIZE(col_keys);
          PyObject* cobj = PyLong_FromSsize_t(ci);
          if (cobj == NULL) goto done;
          const int rc = PyDict_SetItem(col_of, k, cobj);
          Py_DECREF(cobj);
          if (rc < 0 || PyList_Append(col_keys, k) < 0 || PyList_Append(ids_of_col, ids) < 0)
            goto done;
        } else {
          ci = PyLong_AsSsize_t(c);
          ids = PyList_GET_ITEM(ids_of_col, ci);
        }
        /* rule_id */
        int64_t rid = NO_MATCH_RULE;
        const int ne = self_ne(rule);
        if (!ne) {
          PyObject* got = PyDict_GetItemWithError(ids, rule);
          if (got != NULL) rid = PyLong_AsLong(got);
          else if (PyErr_Occurred()) {
            if (!PyErr_ExceptionMatches(PyExc_TypeError)) goto done;
            PyErr_Clear();                                   /* unhashable rule */
          }
        }
        if (vec_push(&col[w], ci) < 0 || vec_push(&val[w], rid) < 0) goto done;
      }
      if (vec_push(&off[w], col[w].n) < 0) goto done;
    }
  }
  res = Py_BuildValue("(ONNNNNN)", col_keys, vec_bytes(&off[0]), vec_bytes(&col[0]),
                      vec_bytes(&val[0]), vec_bytes(&off[1]), vec_bytes(&col[1]),
                      vec_bytes(&val[1]));
done:
  for (int w = 0; w < 2; ++w) {
    PyMem_Free(off[w].p);
    PyMem_Free(col[w].p);
    PyMem_Free(val[w].p);
  }
  Py_XDECREF(col_of);
  Py_XDECREF(col_keys);
  Py_XDECREF(ids_of_col);
  return res;
}

static PyObject* group_ids(PyObject* self, PyObject* args) {
  PyObject *items, *cls, *label, *outobj;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!OOO", &PyList_Type, &items, &cls, &label, &outobj)) return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(items);
  Py_buffer view;
  if (get_out(outobj, &view, n) < 0) return NULL;
  int32_t* out = (int32_t*)view.buf;
  PyObject* groups = PyDict_New();
  PyObject* attr = PyUnicode_InternFromString("labels");
  PyObject* empty = PyUnicode_FromString("");
  if (groups == NULL || attr == NULL || empty == NULL) goto fail;
  /* (memory-latency bound: every container, its label dict, the dict's
   * table and the value are separate heap objects -- the containers are
   * prefetched PF_FAR ahead, their label dicts and tables PF_NEAR ahead) */
  enum { PF_FAR = 16, PF_NEAR = 8 };
  const Py_ssize_t loff = slot_offset(cls, "labels");
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (i + PF_FAR < n) __builtin_prefetch(PyList_GET_ITEM(items, i + PF_FAR));
    if (loff >= 0 && i + PF_NEAR < n) {
      PyObject* cn = PyList_GET_ITEM(items, i + PF_NEAR);
      if ((PyObject*)Py_TYPE(cn) == cls) {
        PyObject* ln = *(PyObject**)((char*)cn + loff);
        if (ln != NULL && PyDict_CheckExact(ln)) __builtin_prefetch(((PyDictObject*)ln)->ma_keys);
      }
    }
    PyObject* c = PyList_GET_ITEM(items, i);
    if ((PyObject*)Py_TYPE(c) != cls) {
      PyErr_SetString(PyExc_ValueError, "containers: exact Container objects expected");
      goto fail;
    }
    PyObject* lab = slot_get(c, loff, attr);            /* new reference */
    if (lab == NULL) goto fail;
    if (!PyDict_CheckExact(lab)) {
      Py_DECREF(lab);
      PyErr_SetString(PyExc_ValueError, "labels: exact dicts expected");
      goto fail;
    }
    PyObject* v = PyDict_GetItemWithError(lab, label);
    if (v == NULL && PyErr_Occurred()) {
      Py_DECREF(lab);
      goto fail;
    }
    if (v == NULL) v = empty;
    Py_INCREF(v);
    Py_DECREF(lab);
    PyObject* got = PyDict_GetItemWithError(groups, v);
    if (got == NULL) {
      if (PyErr_Occurred()) {
        Py_DECREF(v);
        goto fail;
      }
      const Py_ssize_t g = PyDict_GET_SIZE(groups);
      PyObject* id = PyLong_FromSsize_t(g);
      if (id == NULL) {
        Py_DECREF(v);
        goto fail;
      }
      const int rc = PyDict_SetItem(groups, v, id);
      Py_DECREF(id);
      if (rc < 0) {
        Py_DECREF(v);
        goto fail;
      }
      out[i] = (int32_t)g;
    } else {
      out[i] = (int32_t)PyLong_AsLong(got);
    }
    Py_DECREF(v);
  }
  {
    const Py_ssize_t ng = PyDict_GET_SIZE(groups);
    Py_DECREF(groups);
    Py_DECREF(attr);
    Py_DECREF(empty);
    PyBuffer_Release(&view);
    return PyLong_FromSsize_t(ng);
  }
fail:
  Py_XDECREF(groups);
  Py_XDECREF(attr);
  Py_XDECREF(empty);
  PyBuffer_Release(&view);
  return NULL;
}

/* pending_is(containers, cls, lists[, order]) -> bool
 *   kano/algorithm.py _fast_path's per-container test: every container is
 *   exactly `cls`, its own select list (_sel) is empty and its only pending
 *   entry is `lists` (the build's view) -- its select_policies is still
 *   exactly that build's list; with `order` (the build's container list),
 *   container i is also order[i] (the caller did not reorder its list). */
static PyObject* pending_is(PyObject* self, PyObject* args) {
  PyObject *items, *cls, *lists, *order = NULL;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!OO|O!", &PyList_Type, &items, &cls, &lists, &PyList_Type,
                        &order))
    return NULL;
  if (order != NULL && PyList_GET_SIZE(order) != PyList_GET_SIZE(items)) Py_RETURN_FALSE;
  PyObject* a_sel = PyUnicode_InternFromString("_sel");
  PyObject* a_pend = PyUnicode_InternFromString("_pending");
  if (a_sel == NULL || a_pend == NULL) {
    Py_XDECREF(a_sel);
    Py_XDECREF(a_pend);
    return NULL;
  }
  int ok = 1;
  const Py_ssize_t n = PyList_GET_SIZE(items);
  const Py_ssize_t soff = slot_offset(cls, "_sel"), poff = slot_offset(cls, "_pending");
  for (Py_ssize_t i = 0; i < n && ok; ++i) {
    PyObject* c = PyList_GET_ITEM(items, i);
    if ((PyObject*)Py_TYPE(c) != cls || (order != NULL && PyList_GET_ITEM(order, i) != c)) {
      ok = 0;
      break;
    }
    PyObject* sel = slot_get(c, soff, a_sel);
    PyObject* pend = sel ? slot_get(c, poff, a_pend) : NULL;
    if (pend == NULL) {
      Py_XDECREF(sel);
      Py_DECREF(a_sel);
      Py_DECREF(a_pend);
      return NULL;
    }
    const int sel_empty = PyList_CheckExact(sel) ? PyList_GET_SIZE(sel) == 0 : PyObject_Not(sel);
    ok = sel_empty == 1 && PyList_CheckExact(pend) && PyList_GET_SIZE(pend) == 1 &&
         PyList_GET_ITEM(pend, 0) == lists;
    Py_DECREF(sel);
    Py_DECREF(pend);
  }
  Py_DECREF(a_sel);
  Py_DECREF(a_pend);
  if (PyErr_Occurred()) return NULL;
  return PyBool_FromLong(ok);
}

/* pairs_list(buf, P) -> [(j, k), ...]
 *   policy_shadow's result as kano_py returns it (a list of int tuples,
 *   kano_py/kano/algorithm.py:58-80) from the engine's (T, 2) int32 pairs;
 *   the ints of policy ids 0..P-1 made once and shared. */
static PyObject* pairs_list(PyObject* self, PyObject* args) {
  PyObject* obj;
  Py_ssize_t P;
  (void)self;
  if (!PyArg_ParseTuple(args, "On", &obj, &P)) return NULL;
  Py_buffer view;
  if (PyObject_GetBuffer(obj, &view, PyBUF_C_CONTIGUOUS) < 0) return NULL;
  const Py_ssize_t T = view.len / (Py_ssize_t)(2 * sizeof(int32_t));
  const int32_t* v = (const int32_t*)view.buf;
  /* (68k tuples: the cyclic GC, run by the allocations, walked every live
   * container of the build, 12 of 14 ms on C3) */
  const int gc_was = PyGC_Disable();
  PyObject* ints = PyList_New(P > 0 ? P : 0);
  PyObject* out = ints ? PyList_New(T) : NULL;
  if (out == NULL) goto fail;
  for (Py_ssize_t p = 0; p < P; ++p) {
    PyObject* x = PyLong_FromSsize_t(p);
    if (x == NULL) goto fail;
    PyList_SET_ITEM(ints, p, x);
  }
  for (Py_ssize_t t = 0; t < T; ++t) {
    const int32_t a = v[2 * t], b = v[2 * t + 1];
    PyObject* pa = (a >= 0 && a < P) ? PyList_GET_ITEM(ints, a) : NULL;
    PyObject* pb = (b >= 0 && b < P) ? PyList_GET_ITEM(ints, b) : NULL;
    if (pa) Py_INCREF(pa); else if ((pa = PyLong_FromLong(a)) == NULL) goto fail;
    if (pb) Py_INCREF(pb); else if ((pb = PyLong_FromLong(b)) == NULL) { Py_DECREF(pa); goto fail; }
    PyObject* tup = PyTuple_New(2);
    if (tup == NULL) {
      Py_DECREF(pa);
      Py_DECREF(pb);
      goto fail;
    }
    PyTuple_SET_ITEM(tup, 0, pa);
    PyTuple_SET_ITEM(tup, 1, pb);
    PyList_SET_ITEM(out, t, tup);
  }
  Py_DECREF(ints);
  PyBuffer_Release(&view);
  if (gc_was) PyGC_Enable();
  return out;
fail:
  Py_XDECREF(ints);
  Py_XDECREF(out);
  PyBuffer_Release(&view);
  if (gc_was) PyGC_Enable();
  return NULL;
}

static PyMethodDef methods[] = {
    {"intern_column", intern_column, METH_VARARGS, "pod value ids of one key's column"},
    {"group_ids", group_ids, METH_VARARGS, "dense group ids of containers by one label"},
    {"scan_labels", scan_labels, METH_VARARGS, "KEYS and the candidate keys' value-id columns"},
    {"policy_terms", policy_terms, METH_VARARGS, "the working-term CSRs, default matchers"},
    {"pending_is", pending_is, METH_VARARGS, "every container's lists still the build's"},
    {"pairs_list", pairs_list, METH_VARARGS, "policy_shadow's pairs as a list of tuples"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_kano_host", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__kano_host(void) { return PyModule_Create(&module); }
