/* Host-side search loop of the engine-backed navigation planner (gym_cooking_amd/planner.py),
 * as a CPython extension: the bounded-RTDP sample trial of E2E_BRTDP.runSampleTrial
 * (navigation_planner/planners/e2e_brtdp.py:257-331) over the planner's own tables.
 *
 * Nothing here is approximated: the values are the same IEEE doubles the Python loop computes
 * (c + v[vk], a difference, a division by tau), in the same order, stored into the same dicts;
 * min keeps the first minimum as Python's min does; argmin consumes the tie-break generator
 * exactly as planner.argmin does (one random_sample() for a unique minimum that is not the
 * last entry, nothing for the last; for ties, numpy's legacy multinomial restated over the
 * generator's uniforms: binomial inversion per entry, tie_pick_c).  The loop runs while every state it meets is expanded and its successors'
 * values are initialised, and hands back to Python otherwise.
 *
 * An expanded state's entry (planner.E2E_BRTDP._expanded) is a list:
 *   [0] actions  [1] successor keys  [2] costs (floats)  [3] successor value keys
 *   [4] goal flags  [5] bounds  [6] successors initialised (bool)  [7] copy-crash action
 *   indices (set or None)  [8] this state's value key  [9] (entries built by expand) the
 *   hashes of [3]'s keys, of [8] and of the successors' (state key, subtask) _succ keys, as a
 *   bytes of 2n+1 Py_hash_t -- the loops below look values up with them instead of hashing a
 *   nested tuple per lookup (the dicts are the same; a hash is a pure function of the key).
 * expand interns the value keys it builds in the planner's key table, so that the keys stored
 * in v_l / v_u and the ones looked up are mostly one object (a dict compares those by identity).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

/* v[k] as a double; NULL (with KeyError set) when absent */
static int get_val(PyObject* d, PyObject* k, double* out) {
    PyObject* v = PyDict_GetItemWithError(d, k);
    if (v == NULL) {
        if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, k);
        return -1;
    }
    *out = PyFloat_AsDouble(v);
    if (*out == -1.0 && PyErr_Occurred()) return -1;
    return 0;
}

/* Known-hash dict calls and _PySet_NextEntry are CPython internals: 3.10's public headers (this
 * toolchain) still declare them, 3.13 moved them to the internal API.  From 3.13 on the public
 * calls stand in; they hash the key again but read and write the same dicts, keys and values. */
#if PY_VERSION_HEX >= 0x030D0000
#define OC_DICT_GET_KH(d, k, h) PyDict_GetItemWithError((d), (k))
#define OC_DICT_SET_KH(d, k, v, h) PyDict_SetItem((d), (k), (v))
#define OC_DICT_HAS_KH(d, k, h) PyDict_Contains((d), (k))
#else
#define OC_DICT_GET_KH(d, k, h) _PyDict_GetItem_KnownHash((d), (k), (h))
#define OC_DICT_SET_KH(d, k, v, h) _PyDict_SetItem_KnownHash((d), (k), (v), (h))
#define OC_DICT_HAS_KH(d, k, h) _PyDict_Contains_KnownHash((d), (k), (h))
#endif

/* The smallest int in a set of ints (*out = -1 when empty); -1 on error. */
static int set_min_index(PyObject* set, Py_ssize_t* out) {
    *out = -1;
#if PY_VERSION_HEX >= 0x030D0000
    PyObject* iter = PyObject_GetIter(set);
    if (iter == NULL) return -1;
    PyObject* it;
    while ((it = PyIter_Next(iter)) != NULL) {
        const Py_ssize_t v = PyLong_AsSsize_t(it);
        Py_DECREF(it);
        if (v == -1 && PyErr_Occurred()) { Py_DECREF(iter); return -1; }
        if (*out < 0 || v < *out) *out = v;
    }
    Py_DECREF(iter);
    return PyErr_Occurred() ? -1 : 0;
#else
    Py_ssize_t pos = 0;
    PyObject* it;
    Py_hash_t hh;
    while (_PySet_NextEntry(set, &pos, &it, &hh)) {
        const Py_ssize_t v = PyLong_AsSsize_t(it);
        if (v == -1 && PyErr_Occurred()) return -1;
        if (*out < 0 || v < *out) *out = v;
    }
    return 0;
#endif
}

static int set_val(PyObject* d, PyObject* k, double x) {
    PyObject* f = PyFloat_FromDouble(x);
    if (f == NULL) return -1;
    int r = PyDict_SetItem(d, k, f);
    Py_DECREF(f);
    return r;
}

/* hash i of an entry's hash table (NULL: none) */
static inline Py_hash_t hash_at(const char* h, Py_ssize_t i) {
    Py_hash_t v;
    memcpy(&v, h + (size_t)i * sizeof(Py_hash_t), sizeof v);
    return v;
}

/* An entry's precomputed hashes ([9], see above) for its n successors, or NULL for an entry
 * built in Python (planner._expanded). */
static const char* entry_hashes(PyObject* got, Py_ssize_t n) {
    if (PyList_GET_SIZE(got) < 10) return NULL;
    PyObject* h = PyList_GET_ITEM(got, 9);
    if (!PyBytes_Check(h) || PyBytes_GET_SIZE(h) != (Py_ssize_t)sizeof(Py_hash_t) * (2 * n + 1)) return NULL;
    return PyBytes_AS_STRING(h);
}

/* get_val / set_val with the key's hash known (h = NULL: hash it) */
static int get_val_h(PyObject* d, PyObject* k, const char* h, Py_ssize_t i, double* out) {
    if (h == NULL) return get_val(d, k, out);
    PyObject* v = OC_DICT_GET_KH(d, k, hash_at(h, i));
    if (v == NULL) {
        if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, k);
        return -1;
    }
    *out = PyFloat_AsDouble(v);
    if (*out == -1.0 && PyErr_Occurred()) return -1;
    return 0;
}

static int set_val_h(PyObject* d, PyObject* k, const char* h, Py_ssize_t i, double x) {
    if (h == NULL) return set_val(d, k, x);
    PyObject* f = PyFloat_FromDouble(x);
    if (f == NULL) return -1;
    int r = OC_DICT_SET_KH(d, k, f, hash_at(h, i));
    Py_DECREF(f);
    return r;
}

/* k in d, with the hash known (h = NULL: hash it); -1 on error */
static int has_key_h(PyObject* d, PyObject* k, const char* h, Py_ssize_t i) {
    return h == NULL ? PyDict_Contains(d, k) : OC_DICT_HAS_KH(d, k, hash_at(h, i));
}

/* numpy's bit-generator interface (numpy/random/bitgen.h): a legacy RandomState's
 * random_sample() returns next_double(state) of its bit generator. */
typedef struct {
    void* state;
    uint64_t (*next_uint64)(void* st);
    uint32_t (*next_uint32)(void* st);
    double (*next_double)(void* st);
    uint64_t (*next_raw)(void* st);
} bitgen_t;

/* One uniform double from the tie-break generator (RandomState.random_sample: MT19937's
 * next_double, the variate numpy's legacy binomial reads); -1 on error.  `sample` is the bound
 * random_sample, or the generator's "BitGenerator" capsule (planner._sampler), whose
 * next_double is the very function random_sample calls: the same stream without a Python call.
 * The capsule path does not take the bit generator's lock (random_sample does): it assumes, as
 * the planner guarantees, that no other thread uses the same RandomState while a search runs
 * (each planner owns its generator; the search holds the GIL throughout). */
static int uniform(PyObject* sample, double* u) {
    if (PyCapsule_CheckExact(sample)) {
        bitgen_t* bg = (bitgen_t*)PyCapsule_GetPointer(sample, "BitGenerator");
        if (bg == NULL) return -1;
        *u = bg->next_double(bg->state);
        return 0;
    }
    PyObject* r = PyObject_CallNoArgs(sample);
    if (r == NULL) return -1;
    *u = PyFloat_AsDouble(r);
    Py_DECREF(r);
    return (*u == -1.0 && PyErr_Occurred()) ? -1 : 0;
}

/* numpy's legacy binomial by inversion (random_binomial_inversion, distributions.c), n = 1 */
static int binomial_inversion1(PyObject* sample, double p, long* X) {
    const long n = 1;
    const double q = 1.0 - p, qn = exp((double)n * log(q)), np_ = (double)n * p;
    const double b = np_ + 10.0 * sqrt(np_ * q + 1);
    const long bound = (long)((double)n < b ? (double)n : b);
    double U, px = qn;
    long x = 0;
    if (uniform(sample, &U) < 0) return -1;
    while (U > px) {
        x++;
        if (x > bound) {
            x = 0;
            px = qn;
            if (uniform(sample, &U) < 0) return -1;
        } else {
            U -= px;
            px = ((double)(n - x + 1) * p * px) / ((double)x * q);
        }
    }
    *X = x;
    return 0;
}

/* numpy's legacy random_binomial(p, n = 1) (distributions.c): 0 for p == 0 without a variate,
 * inversion for p <= 0.5, else 1 - inversion(1 - p) */
static int binomial1(PyObject* sample, double p, long* X) {
    if (p == 0.0) {
        *X = 0;
        return 0;
    }
    if (p <= 0.5) return binomial_inversion1(sample, p, X);
    long y;
    if (binomial_inversion1(sample, 1.0 - p, &y) < 0) return -1;
    *X = 1 - y;
    return 0;
}

/* planner.argmin's tie-break, np.where(rng.multinomial(1, e / e.sum()))[0][0] for the 0/1
 * vector e of the minima (mtrand multinomial: a binomial(1, p_j / remaining) per entry until
 * the trial is used, the last entry takes what is left); -1 on error. */
static Py_ssize_t tie_pick_c(const char* is_min, Py_ssize_t n, PyObject* sample) {
    Py_ssize_t k = 0;
    for (Py_ssize_t i = 0; i < n; ++i) k += is_min[i] ? 1 : 0;
    double remaining = 1.0;
    for (Py_ssize_t j = 0; j + 1 < n; ++j) {
        const double pj = (is_min[j] ? 1.0 : 0.0) / (double)k;
        long x;
        if (binomial1(sample, pj / remaining, &x) < 0) return -1;
        if (x > 0) return j;
        remaining -= pj;
    }
    return n - 1;
}

/* tie_pick(minima, sample) -> index: tie_pick_c over a list of truth values (tests) */
static PyObject* tie_pick(PyObject* self, PyObject* args) {
    PyObject *lst, *sample;
    if (!PyArg_ParseTuple(args, "O!O", &PyList_Type, &lst, &sample)) return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(lst);
    if (n == 0) {
        PyErr_SetString(PyExc_ValueError, "tie_pick: no candidates");
        return NULL;
    }
    char* m = (char*)PyMem_Malloc((size_t)n + 1);
    if (m == NULL) return PyErr_NoMemory();
    for (Py_ssize_t i = 0; i < n; ++i) m[i] = (char)PyObject_IsTrue(PyList_GET_ITEM(lst, i));
    const Py_ssize_t r = tie_pick_c(m, n, sample);
    PyMem_Free(m);
    if (r < 0) return NULL;
    return PyLong_FromSsize_t(r);
}

/* min over i of costs[i] + v[vks[i]] (the first minimum), into *out; -1 on error */
static int min_q(PyObject* costs, PyObject* vks, const char* hs, PyObject* v, double* out) {
    const Py_ssize_t n = PyList_GET_SIZE(costs);
    double m = 0.0;
    if (n == 0) {  /* Python's min() of an empty sequence */
        PyErr_SetString(PyExc_ValueError, "min() arg is an empty sequence");
        return -1;
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
        double c = PyFloat_AsDouble(PyList_GET_ITEM(costs, i)), x;
        if (c == -1.0 && PyErr_Occurred()) return -1;
        if (get_val_h(v, PyList_GET_ITEM(vks, i), hs, i, &x) < 0) return -1;
        const double q = c + x;
        if (i == 0 || q < m) m = q;
    }
    *out = m;
    return 0;
}

/* value_init of every successor of an entry, in action order (planner.E2E_BRTDP._init_succ
 * past its copy-crash check; e2e_brtdp.py:678-729 through T): a key already in both tables is
 * kept; a goal gets 0.0 / 0.0; else lower = bound * tc must be > 0 (AssertionError "lower: x"
 * as the reference's assert, after the inserts before it), v_l = lower - 1.09,
 * v_u = lower * 5 * tc.  Sets the entry's initialised flag. */
static int init_entry(PyObject* got, PyObject* v_l, PyObject* v_u, double tc) {
    PyObject *vks = PyList_GET_ITEM(got, 3), *goals = PyList_GET_ITEM(got, 4), *lbs = PyList_GET_ITEM(got, 5);
    const Py_ssize_t n = PyList_GET_SIZE(vks);
    const char* hs = entry_hashes(got, n);
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* vk = PyList_GET_ITEM(vks, i);
        const int il = has_key_h(v_l, vk, hs, i);
        if (il < 0) return -1;
        if (il) {
            const int iu = has_key_h(v_u, vk, hs, i);
            if (iu < 0) return -1;
            if (iu) continue;
        }
        const int g = PyObject_IsTrue(PyList_GET_ITEM(goals, i));
        if (g < 0) return -1;
        if (g) {
            if (set_val_h(v_l, vk, hs, i, 0.0) < 0 || set_val_h(v_u, vk, hs, i, 0.0) < 0) return -1;
            continue;
        }
        const double lb = PyFloat_AsDouble(PyList_GET_ITEM(lbs, i));
        if (lb == -1.0 && PyErr_Occurred()) return -1;
        const double lower = lb * tc;
        if (!(lower > 0)) {
            PyObject* f = PyFloat_FromDouble(lower);
            if (f != NULL) {
                PyErr_Format(PyExc_AssertionError, "lower: %R", f);
                Py_DECREF(f);
            }
            return -1;
        }
        if (set_val_h(v_l, vk, hs, i, lower - 1.09) < 0 || set_val_h(v_u, vk, hs, i, lower * 5 * tc) < 0) return -1;
    }
    Py_INCREF(Py_True);
    PyList_SetItem(got, 6, Py_True);  /* steals; drops the old flag */
    return 0;
}

/* init_succ(entry, v_l, v_u, tc): init_entry for Python (_init_succ after its crash check) */
static PyObject* init_succ(PyObject* self, PyObject* args) {
    PyObject *got, *v_l, *v_u;
    double tc;
    if (!PyArg_ParseTuple(args, "O!O!O!d", &PyList_Type, &got, &PyDict_Type, &v_l, &PyDict_Type, &v_u, &tc))
        return NULL;
    if (PyList_GET_SIZE(got) < 9) {
        PyErr_SetString(PyExc_ValueError, "init_succ: not a _succ entry");
        return NULL;
    }
    if (init_entry(got, v_l, v_u, tc) < 0) return NULL;
    Py_RETURN_NONE;
}

/* backprop(v_u, v_l, traj, entries): the trial's backward pass (e2e_brtdp.py:320-331): pop
 * every state of traj and set both of its values to the min over its actions.  entries[t] is
 * traj[t]'s _succ entry (forward collects them), so no state is looked up again. */
static PyObject* backprop(PyObject* self, PyObject* args) {
    PyObject *v_u, *v_l, *traj, *ents;
    if (!PyArg_ParseTuple(args, "O!O!O!O!", &PyDict_Type, &v_u, &PyDict_Type, &v_l, &PyList_Type, &traj, &PyList_Type,
                          &ents))
        return NULL;
    if (PyList_GET_SIZE(ents) != PyList_GET_SIZE(traj)) {
        PyErr_SetString(PyExc_ValueError, "backprop: a trajectory state without its entry");
        return NULL;
    }
    for (Py_ssize_t t = PyList_GET_SIZE(ents) - 1; t >= 0; --t) {
        PyObject* got = PyList_GET_ITEM(ents, t);
        PyObject *costs = PyList_GET_ITEM(got, 2), *vks = PyList_GET_ITEM(got, 3), *rx = PyList_GET_ITEM(got, 8);
        const Py_ssize_t n = PyList_GET_SIZE(costs);
        const char* hs = entry_hashes(got, n);
        double mu, ml;
        if (min_q(costs, vks, hs, v_u, &mu) < 0 || set_val_h(v_u, rx, hs, n, mu) < 0) return NULL;
        if (min_q(costs, vks, hs, v_l, &ml) < 0 || set_val_h(v_l, rx, hs, n, ml) < 0) return NULL;
    }
    if (PyList_SetSlice(traj, 0, PyList_GET_SIZE(traj), NULL) < 0) return NULL;
    if (PyList_SetSlice(ents, 0, PyList_GET_SIZE(ents), NULL) < 0) return NULL;
    Py_RETURN_NONE;
}

/* forward(succ, v_u, v_l, x, sk, rs, cap, counter, tau, traj, sample, resume, entries, tc)
 *   -> (status, x, counter, i)
 * The forward loop of runSampleTrial (e2e_brtdp.py:257-318) from state x:
 *   counter += 1; stop past cap; traj.append(x); [x must be expanded]; initialise its
 *   successors' values if not yet (init_entry, with tc = time_cost + action_cost);
 *   v_u[x] = min_a Q(x, a, v_u); a = argmin_a Q(x, a, v_l); v_l[x] = Q(x, a, v_l);
 *   stop when v_u - v_l of a's successor <= (v_u - v_l of the start) / tau; else x = succ.
 * Every traj state's entry is appended to `entries` as it is found (backprop reads them).
 * status 0: the trial's forward pass is over (x, counter as reached);
 *         1: x is not expanded: x is already counted and in traj -- call again with resume=1
 *            once it is;
 *         2: a copy crash (i = the action index): the chosen action's successor, or, before
 *            x's successors are initialised, the first crashing one (_init_succ's raise). */
static PyObject* forward(PyObject* self, PyObject* args) {
    PyObject *succ, *v_u, *v_l, *x, *sk, *rs, *traj, *sample, *ents;
    long cap, counter;
    double tau, tc;
    int resume;
    if (!PyArg_ParseTuple(args, "O!O!O!OOOlldO!OpO!d", &PyDict_Type, &succ, &PyDict_Type, &v_u, &PyDict_Type, &v_l, &x,
                          &sk, &rs, &cap, &counter, &tau, &PyList_Type, &traj, &sample, &resume, &PyList_Type, &ents,
                          &tc))
        return NULL;
    const Py_hash_t rsh = PyObject_Hash(rs);
    if (rsh == -1) return NULL;
    char rsb[sizeof(Py_hash_t)];
    memcpy(rsb, &rsh, sizeof rsh);
    Py_hash_t xh = -1;  /* hash of (x, sk) when known from the parent's entry */
    Py_INCREF(x);
    for (;;) {
        if (!resume) {
            counter += 1;
            if (counter > cap) break;
            if (PyList_Append(traj, x) < 0) goto fail;
        }
        resume = 0;
        PyObject* key = PyTuple_Pack(2, x, sk);
        if (key == NULL) goto fail;
        PyObject* got = xh != -1 ? OC_DICT_GET_KH(succ, key, xh) : PyDict_GetItemWithError(succ, key);
        Py_DECREF(key);
        if (got == NULL && PyErr_Occurred()) goto fail;
        if (got == NULL) return Py_BuildValue("(iNli)", 1, x, counter, -1);
        if (PyList_Append(ents, got) < 0) goto fail;
        PyObject* crash = PyList_GET_ITEM(got, 7);
        if (PyList_GET_ITEM(got, 6) != Py_True) {
            if (crash != Py_None && PySet_GET_SIZE(crash) > 0) {  /* _init_succ raises on the first */
                Py_ssize_t first;
                if (set_min_index(crash, &first) < 0) goto fail;
                return Py_BuildValue("(iNli)", 2, x, counter, (int)first);
            }
            if (init_entry(got, v_l, v_u, tc) < 0) goto fail;
        }
        PyObject *costs = PyList_GET_ITEM(got, 2), *vks = PyList_GET_ITEM(got, 3), *rx = PyList_GET_ITEM(got, 8);
        const Py_ssize_t n = PyList_GET_SIZE(costs);
        const char* hs = entry_hashes(got, n);
        double mu;
        if (min_q(costs, vks, hs, v_u, &mu) < 0 || set_val_h(v_u, rx, hs, n, mu) < 0) goto fail;  /* n == 0 raises here */
        /* ql = [c + v_l[vk]]; argmin with planner.argmin's generator consumption */
        double ql_stack[32];
        double* ql = n <= 32 ? ql_stack : (double*)PyMem_Malloc(sizeof(double) * (size_t)n);
        if (ql == NULL) {
            PyErr_NoMemory();
            goto fail;
        }
        Py_ssize_t im = 0, nmin = 0;
        int err = 0;
        for (Py_ssize_t i = 0; i < n && !err; ++i) {
            double c = PyFloat_AsDouble(PyList_GET_ITEM(costs, i)), v;
            if ((c == -1.0 && PyErr_Occurred()) || get_val_h(v_l, PyList_GET_ITEM(vks, i), hs, i, &v) < 0) {
                err = 1;
                break;
            }
            ql[i] = c + v;
            if (i == 0 || ql[i] < ql[im]) {
                im = i;
                nmin = 1;
            } else if (ql[i] == ql[im]) {
                ++nmin;
            }
        }
        Py_ssize_t pick = im;
        if (!err && nmin == 1) {
            double u;
            if (im != n - 1 && uniform(sample, &u) < 0) err = 1;
        } else if (!err) {  /* ties: the multinomial draw of planner.argmin */
            char mins_stack[32];
            char* mins = n <= 32 ? mins_stack : (char*)PyMem_Malloc((size_t)n);
            if (mins == NULL) {
                PyErr_NoMemory();
                err = 1;
            }
            for (Py_ssize_t i = 0; i < n && !err; ++i) mins[i] = ql[i] == ql[im];
            if (!err) {
                pick = tie_pick_c(mins, n, sample);
                if (pick < 0) err = 1;
            }
            if (mins != NULL && mins != mins_stack) PyMem_Free(mins);
        }
        const double qi = err ? 0.0 : ql[pick];
        if (ql != ql_stack) PyMem_Free(ql);
        if (err || set_val_h(v_l, rx, hs, n, qi) < 0) goto fail;
        if (crash != Py_None && PySet_GET_SIZE(crash) > 0) {
            PyObject* pi = PyLong_FromSsize_t(pick);
            if (pi == NULL) goto fail;
            const int in = PySet_Contains(crash, pi);
            Py_DECREF(pi);
            if (in < 0) goto fail;
            if (in) return Py_BuildValue("(iNli)", 2, x, counter, (int)pick);
        }
        PyObject* vk = PyList_GET_ITEM(vks, pick);
        double a, b, c, d;
        if (get_val_h(v_u, vk, hs, pick, &a) < 0 || get_val_h(v_l, vk, hs, pick, &b) < 0 ||
            get_val_h(v_u, rs, rsb, 0, &c) < 0 || get_val_h(v_l, rs, rsb, 0, &d) < 0)
            goto fail;
        const double B = a - b, diff = (c - d) / tau;
        if (B <= diff) break;
        PyObject* nx = PyList_GET_ITEM(PyList_GET_ITEM(got, 1), pick);
        xh = hs != NULL ? hash_at(hs, n + 1 + pick) : -1;
        Py_INCREF(nx);
        Py_DECREF(x);
        x = nx;
    }
    return Py_BuildValue("(iNli)", 0, x, counter, -1);
fail:
    Py_DECREF(x);
    return NULL;
}

/* expand(rows, fl, lb, cand, key, sk, m0, K, A, cost, changed, keys[, succ, illegal_tbl])
 *   -> (entry, illegal), or None when it stores them itself
 * planner.E2E_BRTDP._expanded over one expansion's rollout rows (e2e_brtdp.py:103-206: T,
 * get_actions; value_init's inputs): rows = the successors' state bytes [n][NP] (a buffer),
 * fl = their u8 flags, lb = their f32 bounds, cand = the candidate joint actions in get_actions
 * order, key = (state bytes, group names, agents, Level).  A row whose item masks changed (a
 * chop or a merge) goes through changed(bytes, group names) -> (canonical bytes, group names)
 * in Python.  With `succ` and `illegal_tbl` (dicts) it stores the entry as succ[(key, sk)] and
 * the illegal candidates as illegal_tbl[(key, sk)] = (illegal, rows, NP, fl), as
 * planner._expanded_native does, and returns None.
 * keys: the planner's key table (a dict; None: no interning) -- every value key built here is
 * replaced by the table's equal key, if it has one.
 * Returns the _succ entry (without its initialised flag set; with its hashes, [9]) and
 * {action: row} of the illegal candidates (or None). */
static PyObject* expand(PyObject* self, PyObject* args) {
    PyObject *rows_o, *fl_o, *lb_o, *cand, *key, *sk, *cost, *changed, *keys, *store = Py_None, *ill_tbl = Py_None;
    Py_ssize_t m0, K, A;
    if (!PyArg_ParseTuple(args, "OOOO!O!OnnnO!OO|OO", &rows_o, &fl_o, &lb_o, &PyList_Type, &cand, &PyTuple_Type, &key,
                          &sk, &m0, &K, &A, &PyDict_Type, &cost, &changed, &keys, &store, &ill_tbl))
        return NULL;
    if ((store != Py_None && !PyDict_Check(store)) || (ill_tbl != Py_None && !PyDict_Check(ill_tbl)) ||
        ((store == Py_None) != (ill_tbl == Py_None))) {
        PyErr_SetString(PyExc_TypeError, "expand: succ and illegal_tbl must both be dicts or both be absent");
        return NULL;
    }
    if (keys != Py_None && !PyDict_Check(keys)) {
        PyErr_SetString(PyExc_TypeError, "expand: keys must be a dict or None");
        return NULL;
    }
    Py_buffer rb, fb, lbb;
    if (PyObject_GetBuffer(rows_o, &rb, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    if (PyObject_GetBuffer(fl_o, &fb, PyBUF_C_CONTIGUOUS) < 0) {
        PyBuffer_Release(&rb);
        return NULL;
    }
    if (PyObject_GetBuffer(lb_o, &lbb, PyBUF_C_CONTIGUOUS) < 0) {
        PyBuffer_Release(&rb);
        PyBuffer_Release(&fb);
        return NULL;
    }
    PyObject *actions = NULL, *succ = NULL, *costs = NULL, *vks = NULL, *goals = NULL, *lbs = NULL, *crash = NULL,
             *illegal = NULL, *out = NULL, *ra = NULL, *self_vk = NULL, *self_r = NULL, *hb = NULL;
    Py_hash_t* hv = NULL;  /* the value keys' hashes, then the _succ keys' */
    Py_ssize_t m = 0;      /* legal successors so far */
    PyObject *sb = PyTuple_GET_ITEM(key, 0), *groups = PyTuple_GET_ITEM(key, 1), *agents = PyTuple_GET_ITEM(key, 2),
             *lvl_o = PyTuple_GET_ITEM(key, 3);
    const Py_ssize_t n = PyList_GET_SIZE(cand);
    const Py_ssize_t NP = PyBytes_GET_SIZE(sb);
    const int lvl = PyObject_IsTrue(lvl_o);
    const unsigned char* raw = (const unsigned char*)rb.buf;
    const unsigned char* fl = (const unsigned char*)fb.buf;
    const float* lbv = (const float*)lbb.buf;
    const unsigned char* pm = (const unsigned char*)PyBytes_AS_STRING(sb) + m0;
    if (rb.len < n * NP || fb.len < n || lbb.len < n * (Py_ssize_t)sizeof(float)) {
        PyErr_SetString(PyExc_ValueError, "expand: row buffers shorter than the candidates");
        goto done;
    }
    hv = (Py_hash_t*)PyMem_Malloc(sizeof(Py_hash_t) * (size_t)(2 * n + 1));
    if (hv == NULL) {
        PyErr_NoMemory();
        goto done;
    }
    actions = PyList_New(0);
    succ = PyList_New(0);
    costs = PyList_New(0);
    vks = PyList_New(0);
    goals = PyList_New(0);
    lbs = PyList_New(0);
    if (!actions || !succ || !costs || !vks || !goals || !lbs) goto done;
    ra = (lvl || PyTuple_GET_SIZE(agents) == A) ? Py_None : agents;  /* _repr's agents entry */
    Py_INCREF(ra);
    for (Py_ssize_t r = 0; r < n; ++r) {
        PyObject* c = PyList_GET_ITEM(cand, r);
        const unsigned f = fl[r];
        if (!(f & 1u)) {  /* OC_ROLL_LEGAL */
            if (illegal == NULL && (illegal = PyDict_New()) == NULL) goto done;
            PyObject* ri = PyLong_FromSsize_t(r);
            if (ri == NULL || PyDict_SetItem(illegal, c, ri) < 0) {
                Py_XDECREF(ri);
                goto done;
            }
            Py_DECREF(ri);
            continue;
        }
        if (f & 4u) {  /* OC_ROLL_ASSERT: T raises (e2e_brtdp.py:143) */
            PyErr_Format(PyExc_AssertionError, "action %S led to co-located subtask agents", c);
            goto done;
        }
        const unsigned char* row = raw + r * NP;
        PyObject *ns, *ng;
        if (memcmp(row + m0, pm, (size_t)K) != 0) {  /* a chop or a merge */
            PyObject* b = PyBytes_FromStringAndSize((const char*)row, NP);
            if (b == NULL) goto done;
            PyObject* t = PyObject_CallFunctionObjArgs(changed, b, groups, NULL);
            Py_DECREF(b);
            if (t == NULL) goto done;
            ns = PyTuple_GetItem(t, 0);
            ng = PyTuple_GetItem(t, 1);
            if (ns == NULL || ng == NULL) {
                Py_DECREF(t);
                goto done;
            }
            Py_INCREF(ns);
            Py_INCREF(ng);
            Py_DECREF(t);
        } else {
            ns = PyBytes_FromStringAndSize((const char*)row, NP);
            if (ns == NULL) goto done;
            ng = groups;
            Py_INCREF(ng);
        }
        /* Keys of bytes, a frozenset of names, ints and strings: no tuple here can be part of a
         * reference cycle, so the collector is told not to walk them (CPython would untrack them
         * itself at its first pass over them, after walking each once; a search makes millions). */
        PyObject* nk = PyTuple_Pack(4, ns, ng, agents, lvl_o);
        PyObject* rep = PyTuple_Pack(3, ns, ng, ra);
        PyObject* vk = rep ? PyTuple_Pack(2, rep, sk) : NULL;
        if (nk) PyObject_GC_UnTrack(nk);
        if (rep) PyObject_GC_UnTrack(rep);
        if (vk) PyObject_GC_UnTrack(vk);
        Py_XDECREF(rep);
        const Py_hash_t h1 = vk != NULL ? PyObject_Hash(vk) : -1;
        if (nk != NULL && h1 != -1 && keys != Py_None) {  /* intern */
            PyObject* c = OC_DICT_GET_KH(keys, vk, h1);
            if (c != NULL) {
                Py_INCREF(c);
                Py_DECREF(vk);
                vk = c;
            } else if (PyErr_Occurred() || OC_DICT_SET_KH(keys, vk, vk, h1) < 0) {
                Py_CLEAR(vk);
            }
        }
        PyObject* sk2 = (nk != NULL && vk != NULL) ? PyTuple_Pack(2, nk, sk) : NULL;
        const Py_hash_t h2 = sk2 != NULL ? PyObject_Hash(sk2) : -1;
        Py_XDECREF(sk2);
        if (nk == NULL || vk == NULL || h2 == -1) {
            Py_XDECREF(nk);
            Py_XDECREF(vk);
            Py_DECREF(ns);
            Py_DECREF(ng);
            goto done;
        }
        hv[m] = h1;
        hv[n + 1 + m] = h2;
        ++m;
        if (lvl) {  /* _copy_crashes: two co-located agents that both hold */
            const unsigned char* q = (const unsigned char*)PyBytes_AS_STRING(ns);
            int hit = 0;
            for (Py_ssize_t i = 0; i < A && !hit; ++i) {
                if (q[2 * A + i] == 0xFF) continue;
                for (Py_ssize_t j = i + 1; j < A; ++j)
                    if (q[2 * A + j] != 0xFF && q[i] == q[j] && q[A + i] == q[A + j]) {
                        hit = 1;
                        break;
                    }
            }
            if (hit) {
                PyObject* ai = PyLong_FromSsize_t(PyList_GET_SIZE(actions));
                if (crash == NULL) crash = PySet_New(NULL);
                if (ai == NULL || crash == NULL || PySet_Add(crash, ai) < 0) {
                    Py_XDECREF(ai);
                    Py_DECREF(nk);
                    Py_DECREF(vk);
                    Py_DECREF(ns);
                    Py_DECREF(ng);
                    goto done;
                }
                Py_DECREF(ai);
            }
        }
        Py_DECREF(ns);
        Py_DECREF(ng);
        PyObject* cst = PyDict_GetItemWithError(cost, c);
        PyObject* lbf = PyFloat_FromDouble((double)lbv[r]);
        int bad = cst == NULL || lbf == NULL;
        if (cst == NULL && !PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, c);
        bad = bad || PyList_Append(actions, c) < 0 || PyList_Append(succ, nk) < 0 || PyList_Append(costs, cst) < 0 ||
              PyList_Append(vks, vk) < 0 || PyList_Append(goals, (f & 2u) ? Py_True : Py_False) < 0 ||
              PyList_Append(lbs, lbf) < 0;
        Py_DECREF(nk);
        Py_DECREF(vk);
        Py_XDECREF(lbf);
        if (bad) goto done;
    }
    self_r = PyTuple_Pack(3, sb, groups, ra);
    if (self_r == NULL || (self_vk = PyTuple_Pack(2, self_r, sk)) == NULL) goto done;
    if (keys != Py_None) {
        PyObject* c = PyDict_SetDefault(keys, self_vk, self_vk);
        if (c == NULL) goto done;
        Py_INCREF(c);
        Py_DECREF(self_vk);
        self_vk = c;
    }
    if ((hv[m] = PyObject_Hash(self_vk)) == -1) goto done;
    memmove(hv + m + 1, hv + n + 1, sizeof(Py_hash_t) * (size_t)m);  /* compact: [m value keys, self, m _succ keys] */
    hb = PyBytes_FromStringAndSize((const char*)hv, (Py_ssize_t)sizeof(Py_hash_t) * (2 * m + 1));
    if (hb == NULL) goto done;
    out = Py_BuildValue("([OOOOOOOOOO]O)", actions, succ, costs, vks, goals, lbs, Py_False, crash ? crash : Py_None,
                        self_vk, hb, illegal ? illegal : Py_None);
    if (out != NULL) {  /* the entry and its lists hold no reference back to a container: no cycles */
        PyObject* e = PyTuple_GET_ITEM(out, 0);
        for (Py_ssize_t i = 0; i < 6; ++i) PyObject_GC_UnTrack(PyList_GET_ITEM(e, i));
        PyObject_GC_UnTrack(e);
        PyObject_GC_UnTrack(self_vk);
    }
    if (out != NULL && store != Py_None) {  /* store them: succ[(key, sk)], illegal_tbl[(key, sk)] */
        PyObject* k2 = PyTuple_Pack(2, key, sk);
        if (k2 != NULL) PyObject_GC_UnTrack(k2);  /* (state key, subtask key): no cycle */
        int bad = k2 == NULL || PyDict_SetItem(store, k2, PyTuple_GET_ITEM(out, 0)) < 0;
        if (!bad && illegal != NULL) {
            PyObject* rec = Py_BuildValue("(OOnO)", illegal, rows_o, NP, fl_o);
            if (rec != NULL) PyObject_GC_UnTrack(rec);
            bad = rec == NULL || PyDict_SetItem(ill_tbl, k2, rec) < 0;
            Py_XDECREF(rec);
        }
        Py_XDECREF(k2);
        Py_CLEAR(out);
        if (!bad) {
            Py_INCREF(Py_None);
            out = Py_None;
        }
    }
done:
    Py_XDECREF(actions);
    Py_XDECREF(succ);
    Py_XDECREF(costs);
    Py_XDECREF(vks);
    Py_XDECREF(goals);
    Py_XDECREF(lbs);
    Py_XDECREF(crash);
    Py_XDECREF(illegal);
    Py_XDECREF(ra);
    Py_XDECREF(self_r);
    Py_XDECREF(self_vk);
    Py_XDECREF(hb);
    PyMem_Free(hv);
    PyBuffer_Release(&rb);
    PyBuffer_Release(&fb);
    PyBuffer_Release(&lbb);
    return out;
}

static PyMethodDef methods[] = {
    {"expand", expand, METH_VARARGS, "_expanded's successor lists from one expansion's rollout rows"},
    {"forward", forward, METH_VARARGS, "runSampleTrial's forward loop over expanded, initialised states"},
    {"backprop", backprop, METH_VARARGS, "runSampleTrial's backward pass"},
    {"init_succ", init_succ, METH_VARARGS, "value_init of an expanded state's successors"},
    {"tie_pick", tie_pick, METH_VARARGS, "argmin's multinomial tie-break over a list of minima flags"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_brtdp", "planner search loop (host)", -1, methods};

PyMODINIT_FUNC PyInit__brtdp(void) { return PyModule_Create(&module); }
