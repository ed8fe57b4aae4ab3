/* pyfast.c -- CPython fast path of qsmd.device.Context.check_arrays.
 *
 * The per-history drop-in makes one qsmd_check_batch call per history (the
 * reference's pattern: one `linearisable` call per history,
 * test/TicketDispenser.hs:320).  Through ctypes, the 13-argument call and
 * its four numpy pointer conversions cost ~10 us of host time per call; here
 * the buffers come through the buffer protocol and the call is a plain C
 * call of the function pointer qsmd/device.py hands over (the symbol of the
 * libqsmd.so ctypes already loaded: no second copy of the library, no link
 * dependency).  No search here: it only forwards to the C ABI.
 *
 *   check_batch(fn, ctx, model_id, hdr, events, model0_addr, flags,
 *               max_nodes, status, nodes, witness, totals) -> int
 * hdr / events: C-contiguous buffers of include/qsmd.h records; status /
 * nodes / totals: writable buffers (nodes, witness may be None);
 * fn, ctx, model0_addr: addresses as ints (model0_addr 0 = NULL).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

#include "qsmd.h"

typedef int (*check_fn)(qsmd_ctx*, uint32_t, const qsmd_hdr*, uint64_t, const qsmd_event*, uint64_t, const void*,
                        uint32_t, uint64_t, uint8_t*, uint64_t*, uint8_t*, qsmd_totals*);

static int get_buf(PyObject* o, Py_buffer* b, int writable, const char* what) {
    if (o == Py_None) {
        b->obj = NULL;
        b->buf = NULL;
        b->len = 0;
        return 0;
    }
    if (PyObject_GetBuffer(o, b, (writable ? PyBUF_WRITABLE : 0) | PyBUF_C_CONTIGUOUS) != 0) {
        PyErr_Format(PyExc_TypeError, "%s: a C-contiguous%s buffer", what, writable ? " writable" : "");
        return -1;
    }
    return 0;
}

static void rel(Py_buffer* b) {
    if (b->obj) PyBuffer_Release(b);
}

static PyObject* check_batch(PyObject* self, PyObject* args) {
    (void)self;
    unsigned long long fn, ctx, m0, max_nodes;
    unsigned int model_id, flags;
    PyObject *o_hdr, *o_ev, *o_st, *o_nd, *o_w, *o_tot;
    if (!PyArg_ParseTuple(args, "KKIOOKIKOOOO", &fn, &ctx, &model_id, &o_hdr, &o_ev, &m0, &flags, &max_nodes, &o_st,
                          &o_nd, &o_w, &o_tot))
        return NULL;
    Py_buffer hdr = {0}, ev = {0}, st = {0}, nd = {0}, w = {0}, tot = {0};
    int rc = 0;
    if (get_buf(o_hdr, &hdr, 0, "hdr") || get_buf(o_ev, &ev, 0, "events") || get_buf(o_st, &st, 1, "status") ||
        get_buf(o_nd, &nd, 1, "nodes") || get_buf(o_w, &w, 1, "witness") || get_buf(o_tot, &tot, 1, "totals")) {
        rc = -1;
    } else if ((size_t)hdr.len % sizeof(qsmd_hdr) || (size_t)ev.len % sizeof(qsmd_event) ||
               (tot.obj && (size_t)tot.len < sizeof(qsmd_totals))) {
        PyErr_SetString(PyExc_ValueError, "buffer sizes do not match include/qsmd.h records");
        rc = -1;
    } else {
        const uint64_t n = (uint64_t)hdr.len / sizeof(qsmd_hdr), n_ev = (uint64_t)ev.len / sizeof(qsmd_event);
        if ((uint64_t)st.len < n || (nd.obj && (uint64_t)nd.len < 8 * n) || (w.obj && (uint64_t)w.len < n_ev)) {
            PyErr_SetString(PyExc_ValueError, "output buffers shorter than the batch");
            rc = -1;
        } else {
            check_fn f = (check_fn)(uintptr_t)fn;
            Py_BEGIN_ALLOW_THREADS
            rc = f((qsmd_ctx*)(uintptr_t)ctx, model_id, (const qsmd_hdr*)hdr.buf, n, (const qsmd_event*)ev.buf, n_ev,
                   (const void*)(uintptr_t)m0, flags, max_nodes, (uint8_t*)st.buf, (uint64_t*)nd.buf,
                   (uint8_t*)w.buf, (qsmd_totals*)tot.buf);
            Py_END_ALLOW_THREADS
        }
    }
    rel(&hdr);
    rel(&ev);
    rel(&st);
    rel(&nd);
    rel(&w);
    rel(&tot);
    if (PyErr_Occurred()) return NULL;
    return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"check_batch", check_batch, METH_VARARGS, "qsmd_check_batch through the buffer protocol"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pyfast", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pyfast(void) { return PyModule_Create(&module); }
