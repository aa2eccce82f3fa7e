/*
 * fastcall.c -- CPython binding of MPI_Reduce_local for the Python side
 * (bench.py, tests): one METH_FASTCALL function that unpacks five integers and
 * calls the C ABI directly, ~0.1 us per call against ~1.2 us through ctypes.
 * The way mpi4py binds MPI (compiled, not libffi); no compute of its own.
 *
 *   _fastcall.reduce_local(inbuf_addr, inoutbuf_addr, count, datatype, op) -> int
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <limits.h>
#include <stdint.h>
#include <time.h>

#include "mpi_reduce_local.h"

static PyObject *fc_reduce_local(PyObject *self, PyObject *const *args, Py_ssize_t nargs)
{
    (void) self;
    if (nargs != 5) {
        PyErr_SetString(PyExc_TypeError, "reduce_local(inbuf, inoutbuf, count, datatype, op)");
        return NULL;
    }
    const void *in = PyLong_AsVoidPtr(args[0]);
    void *io = PyLong_AsVoidPtr(args[1]);
    const long count = PyLong_AsLong(args[2]);
    const long dt = PyLong_AsLong(args[3]);
    const long op = PyLong_AsLong(args[4]);
    int rc;
    if (PyErr_Occurred())
        return NULL;
    if (count < INT_MIN || count > INT_MAX) {
        PyErr_SetString(PyExc_OverflowError, "count does not fit the C int of MPI_Reduce_local");
        return NULL;
    }
    /* the call waits for the device (~130 us at 256 MiB, longer through the
     * pageable bounce path): other Python threads run meanwhile, as with
     * ctypes.  A Python user op (ctypes callback) takes the GIL back itself. */
    Py_BEGIN_ALLOW_THREADS
    rc = MPI_Reduce_local(in, io, (int) count, (MPI_Datatype) dt, (MPI_Op) op);
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

/* reduce_local_loop(arg_sets, start, k[, stamps]) -> int: k MPI_Reduce_local
 * calls in a C loop, call i with arg_sets[(start + i) % len(arg_sets)]
 * (5-tuples as for reduce_local), the way a C caller -- an MPICH schedule, an
 * OSU-style benchmark -- issues them: the k argument sets are unpacked first,
 * then the calls run back to back without the GIL.  `stamps`, a writable
 * buffer of at least k + 1 int64, receives CLOCK_MONOTONIC ns before the first
 * call and after each call (one clock read per call, ~20 ns: the calls'
 * distribution).  Returns the first nonzero error code (and stops
 * there), else 0. */
static PyObject *fc_reduce_local_loop(PyObject *self, PyObject *const *args, Py_ssize_t nargs)
{
    struct set {
        const void *in;
        void *io;
        int count, dt, op;
    } *sets;
    Py_ssize_t n, start, k, i, m;
    int rc = 0;
    Py_buffer view = { 0 };
    int64_t *stamps = NULL;
    struct timespec ts;
    (void) self;
    if ((nargs != 3 && nargs != 4) || !PyTuple_Check(args[0])) {
        PyErr_SetString(PyExc_TypeError, "reduce_local_loop(arg_sets: tuple of 5-tuples, start, k[, stamps])");
        return NULL;
    }
    n = PyTuple_GET_SIZE(args[0]);
    start = PyLong_AsSsize_t(args[1]);
    k = PyLong_AsSsize_t(args[2]);
    if (PyErr_Occurred())
        return NULL;
    if (n < 1 || k < 0 || start < 0) {
        PyErr_SetString(PyExc_ValueError, "need at least one argument set, k >= 0, start >= 0");
        return NULL;
    }
    if (nargs == 4 && args[3] != Py_None) {
        if (PyObject_GetBuffer(args[3], &view, PyBUF_WRITABLE) != 0)
            return NULL;
        if (view.len < (Py_ssize_t) sizeof(int64_t) * (k + 1)) {
            PyBuffer_Release(&view);
            PyErr_SetString(PyExc_ValueError, "stamps needs room for k + 1 int64");
            return NULL;
        }
        stamps = (int64_t *) view.buf;
    }
    /* the m = min(n, k) distinct sets the calls use, in call order: call i
     * takes sets[i % m] */
    m = n < k ? n : k;
    sets = PyMem_Malloc(sizeof(*sets) * (size_t) (m ? m : 1));
    if (!sets) {
        if (stamps)
            PyBuffer_Release(&view);
        return PyErr_NoMemory();
    }
    for (i = 0; i < m; i++) {
        PyObject *t = PyTuple_GET_ITEM(args[0], (start + i) % n);
        long count;
        if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 5) {
            PyMem_Free(sets);
            if (stamps)
                PyBuffer_Release(&view);
            PyErr_SetString(PyExc_TypeError, "each argument set is (inbuf, inoutbuf, count, datatype, op)");
            return NULL;
        }
        sets[i].in = PyLong_AsVoidPtr(PyTuple_GET_ITEM(t, 0));
        sets[i].io = PyLong_AsVoidPtr(PyTuple_GET_ITEM(t, 1));
        count = PyLong_AsLong(PyTuple_GET_ITEM(t, 2));
        sets[i].dt = (int) PyLong_AsLong(PyTuple_GET_ITEM(t, 3));
        sets[i].op = (int) PyLong_AsLong(PyTuple_GET_ITEM(t, 4));
        if (PyErr_Occurred() || count < INT_MIN || count > INT_MAX) {
            PyMem_Free(sets);
            if (stamps)
                PyBuffer_Release(&view);
            if (!PyErr_Occurred())
                PyErr_SetString(PyExc_OverflowError, "count does not fit the C int of MPI_Reduce_local");
            return NULL;
        }
        sets[i].count = (int) count;
    }
    Py_BEGIN_ALLOW_THREADS
    if (stamps) {
        clock_gettime(CLOCK_MONOTONIC, &ts);
        stamps[0] = (int64_t) ts.tv_sec * 1000000000 + ts.tv_nsec;
        for (i = 0; i < k && rc == 0; i++) {
            const struct set *s = &sets[i % m];
            rc = MPI_Reduce_local(s->in, s->io, s->count, (MPI_Datatype) s->dt, (MPI_Op) s->op);
            clock_gettime(CLOCK_MONOTONIC, &ts);
            stamps[i + 1] = (int64_t) ts.tv_sec * 1000000000 + ts.tv_nsec;
        }
    } else {
        for (i = 0; i < k && rc == 0; i++) {
            const struct set *s = &sets[i % m];
            rc = MPI_Reduce_local(s->in, s->io, s->count, (MPI_Datatype) s->dt, (MPI_Op) s->op);
        }
    }
    Py_END_ALLOW_THREADS
    PyMem_Free(sets);
    if (stamps)
        PyBuffer_Release(&view);
    return PyLong_FromLong(rc);
}

static PyMethodDef fc_methods[] = {
    {"reduce_local", (PyCFunction) (void (*)(void)) fc_reduce_local, METH_FASTCALL,
     "MPI_Reduce_local(inbuf, inoutbuf, count, datatype, op) on raw addresses; returns the MPI error code"},
    {"reduce_local_loop", (PyCFunction) (void (*)(void)) fc_reduce_local_loop, METH_FASTCALL,
     "k MPI_Reduce_local calls in a C loop over arg_sets[(start + i) % len] (optional stamps buffer of k + 1 int64 ns); "
     "returns the first error code"},
    {NULL, NULL, 0, NULL}
};

static struct PyModuleDef fc_module = {
    PyModuleDef_HEAD_INIT, "_fastcall", "Compiled binding of MPI_Reduce_local", -1, fc_methods,
    NULL, NULL, NULL, NULL
};

PyMODINIT_FUNC PyInit__fastcall(void)
{
    return PyModule_Create(&fc_module);
}
