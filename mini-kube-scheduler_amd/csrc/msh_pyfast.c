/* msh_pyfast.c — CPython fast-call bindings for the per-batch device entry points of
 * include/minisched_hip.h, for the Python host mirror (scheduler.DeviceContext) and bench.py.
 *
 * A device entry point costs ~2.6 us of host time (a HIP kernel launch, profiles/ab/
 * r2_submit_cost.jsonl); through ctypes the Python side added ~0.9 us per call on top (argument
 * conversion of eight parameters). These METH_FASTCALL wrappers take plain ints (the ctx handle,
 * device pointers, the stream handle) and call the C ABI directly. They do not replace the ABI:
 * everything else goes through ctypes (_native.py), and a cgo caller binds the C functions.
 * schedule_batch_host does the same for the host-buffer msh_schedule_batch, taking arrays by the
 * buffer protocol.
 * Build (mini-kube-scheduler_amd/build.py): gcc -shared against libminisched_hip.so. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "../../include/minisched_hip.h"

/* int (or None) -> pointer; -1 with a Python error set on failure */
static int as_ptr(PyObject* o, void** out) {
  if (o == Py_None) {
    *out = NULL;
    return 0;
  }
  *out = PyLong_AsVoidPtr(o);
  return PyErr_Occurred() ? -1 : 0;
}

static int as_i64(PyObject* o, long long* out) {
  *out = PyLong_AsLongLong(o);
  return PyErr_Occurred() ? -1 : 0;
}

static int want_args(Py_ssize_t n, Py_ssize_t want, const char* name) {
  if (n == want) return 0;
  PyErr_Format(PyExc_TypeError, "%s takes %zd arguments (%zd given)", name, want, n);
  return -1;
}

/* schedule_batch_device(ctx, p, d_pod_digit, d_pod_tol, d_out_idx, d_out_score, d_out_status,
 * stream) -> rc */
static PyObject* py_schedule_batch_device(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  void *ctx, *pd, *pt, *oi, *os, *ost, *st;
  long long p;
  if (want_args(n, 8, "schedule_batch_device") || as_ptr(a[0], &ctx) || as_i64(a[1], &p) ||
      as_ptr(a[2], &pd) || as_ptr(a[3], &pt) || as_ptr(a[4], &oi) || as_ptr(a[5], &os) ||
      as_ptr(a[6], &ost) || as_ptr(a[7], &st))
    return NULL;
  if (p < INT32_MIN || p > INT32_MAX) return PyErr_Format(PyExc_OverflowError, "pod count out of range");
  const int rc = msh_schedule_batch_device((msh_ctx*)ctx, (int32_t)p, (const int8_t*)pd, (const uint8_t*)pt,
                                           (int32_t*)oi, (int64_t*)os, (int32_t*)ost, st);
  return PyLong_FromLong(rc);
}

/* schedule_batch_device_steps(steps, k) -> rc: `steps` is a sequence of up to 16 argument tuples
 * of schedule_batch_device; call i (0 <= i < k) uses steps[i % len(steps)]. The loop a C or Go
 * caller runs when it submits k batches back to back: no interpreter between the launches.
 * Stops at the first failing call and returns its code. */
static PyObject* py_schedule_batch_device_steps(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  enum { MAXS = 16 };
  void *ctx[MAXS], *pd[MAXS], *pt[MAXS], *oi[MAXS], *os[MAXS], *ost[MAXS], *st[MAXS];
  long long p[MAXS], k;
  if (want_args(n, 2, "schedule_batch_device_steps") || as_i64(a[1], &k)) return NULL;
  PyObject* seq = PySequence_Fast(a[0], "steps must be a sequence of argument tuples");
  if (!seq) return NULL;
  const Py_ssize_t ns = PySequence_Fast_GET_SIZE(seq);
  if (ns < 1 || ns > MAXS) {
    Py_DECREF(seq);
    return PyErr_Format(PyExc_ValueError, "1 to %d argument tuples", MAXS);
  }
  for (Py_ssize_t i = 0; i < ns; ++i) {
    PyObject* t = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, i), "an argument tuple");
    if (!t) {
      Py_DECREF(seq);
      return NULL;
    }
    PyObject** v = PySequence_Fast_ITEMS(t);
    const int bad = PySequence_Fast_GET_SIZE(t) != 8 || as_ptr(v[0], &ctx[i]) || as_i64(v[1], &p[i]) ||
                    as_ptr(v[2], &pd[i]) || as_ptr(v[3], &pt[i]) || as_ptr(v[4], &oi[i]) ||
                    as_ptr(v[5], &os[i]) || as_ptr(v[6], &ost[i]) || as_ptr(v[7], &st[i]);
    Py_DECREF(t);
    if (bad || p[i] < INT32_MIN || p[i] > INT32_MAX) {
      Py_DECREF(seq);
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "an argument tuple of schedule_batch_device");
      return NULL;
    }
  }
  Py_DECREF(seq);
  int rc = 0;
  for (long long i = 0; i < k && rc == 0; ++i) {
    const int j = (int)(i % ns);
    rc = msh_schedule_batch_device((msh_ctx*)ctx[j], (int32_t)p[j], (const int8_t*)pd[j], (const uint8_t*)pt[j],
                                   (int32_t*)oi[j], (int64_t*)os[j], (int32_t*)ost[j], st[j]);
  }
  return PyLong_FromLong(rc);
}

/* ---- Submitter: batches submitted from several host threads ----------------------------------
 * One HIP launch costs ~2.6 us of host time, more than a C3 batch takes on the device with
 * batches in flight on several streams, so one submitting thread leaves the GPU waiting. The
 * launch path scales over threads that each own a stream (scripts/submit_mt.hip: 2.56 us per
 * launch from 1 thread, 1.49 from 2, 1.17 from 3), as a Go caller's goroutines would submit.
 * Submitter(device, lanes) starts one host thread per lane; a lane is an argument tuple of
 * schedule_batch_device with its OWN ctx (the ABI's one-ctx-per-thread rule), stream and buffers.
 * run(k) submits k batches, batch i by lane i % len(lanes) (the round robin of the single-thread
 * loop), each lane bracketing its launches with two HIP events on its stream, and returns when
 * every lane has submitted (not when the device is done). span_ms() (after the caller's
 * synchronize) = latest end event - earliest start event over the lanes of the last run. Idle
 * threads spin for a while after each run, then sleep on a condition variable. */
#include <pthread.h>
#include <stdatomic.h>
#include <time.h>

typedef void* hipEvent_t;
extern int hipSetDevice(int);
extern int hipEventCreate(hipEvent_t*);
extern int hipEventDestroy(hipEvent_t);
extern int hipEventRecord(hipEvent_t, void*);
extern int hipEventElapsedTime(float*, hipEvent_t, hipEvent_t);

enum { SUB_MAXT = 8 };
static const long long SUB_SPIN_NS = 2000000000LL;  // spin up to 2 s after a run, then sleep

enum { SUB_NT = 24 };  // host timestamps kept per lane and run (A/B probe)
typedef struct {
  void *ctx, *pd, *pt, *oi, *os, *ost, *st;
  long long p;
  hipEvent_t e0, e1;
  int ran;
  int nt;                 // timestamps taken in the last run
  long long ts[SUB_NT];   // wake, after the start event, after each launch..., after the end event
} SubLane;

typedef struct Submitter {
  PyObject_HEAD
  int nt, device, started;
  SubLane lane[SUB_MAXT];
  pthread_t th[SUB_MAXT];
  struct SubArg {
    struct Submitter* s;
    int t;
  } arg[SUB_MAXT];
  pthread_mutex_t mu;
  pthread_cond_t cv;
  atomic_int gen, done, stop, rc;
  long long k;
  long long t_go;  // CLOCK_MONOTONIC ns at the signal of the last run
} Submitter;

static long long mono_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (long long)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

static void* sub_thread(void* v) {
  struct SubArg* a = (struct SubArg*)v;
  Submitter* s = a->s;
  const int t = a->t;
  SubLane* l = &s->lane[t];
  (void)hipSetDevice(s->device);  // once: the ctx's DeviceGuard then never switches
  int seen = 0;
  for (;;) {
    const long long t0 = mono_ns();
    for (unsigned it = 1;; ++it) {  // spin, then sleep
      if (atomic_load_explicit(&s->gen, memory_order_acquire) != seen || atomic_load(&s->stop)) break;
      __builtin_ia32_pause();
      if ((it & 4095u) == 0 && mono_ns() - t0 > SUB_SPIN_NS) {
        pthread_mutex_lock(&s->mu);
        while (atomic_load(&s->gen) == seen && !atomic_load(&s->stop)) pthread_cond_wait(&s->cv, &s->mu);
        pthread_mutex_unlock(&s->mu);
        break;
      }
    }
    if (atomic_load(&s->stop)) break;
    seen = atomic_load_explicit(&s->gen, memory_order_acquire);
    const long long k = s->k;
    l->ran = t < k;
    l->nt = 0;
#define SUB_TS() \
  if (l->nt < SUB_NT) l->ts[l->nt++] = mono_ns()
    SUB_TS();
    if (l->ran) {
      int rc = hipEventRecord(l->e0, l->st) ? MSH_ERR_HIP : 0;
      SUB_TS();
      for (long long i = t; i < k && rc == 0; i += s->nt) {
        rc = msh_schedule_batch_device((msh_ctx*)l->ctx, (int32_t)l->p, (const int8_t*)l->pd, (const uint8_t*)l->pt,
                                       (int32_t*)l->oi, (int64_t*)l->os, (int32_t*)l->ost, l->st);
        SUB_TS();
      }
      if (rc == 0 && hipEventRecord(l->e1, l->st)) rc = MSH_ERR_HIP;
      SUB_TS();
      if (rc) {
        int zero = 0;
        atomic_compare_exchange_strong(&s->rc, &zero, rc);
      }
    }
    atomic_fetch_add_explicit(&s->done, 1, memory_order_release);
  }
  return NULL;
}

static void sub_stop(Submitter* s) {
  if (!s->started) return;
  pthread_mutex_lock(&s->mu);
  atomic_store(&s->stop, 1);
  pthread_cond_broadcast(&s->cv);
  pthread_mutex_unlock(&s->mu);
  for (int t = 0; t < s->started; ++t) pthread_join(s->th[t], NULL);
  s->started = 0;
}

static void sub_dealloc(Submitter* s) {
  sub_stop(s);
  for (int t = 0; t < s->nt; ++t) {
    if (s->lane[t].e0) (void)hipEventDestroy(s->lane[t].e0);
    if (s->lane[t].e1) (void)hipEventDestroy(s->lane[t].e1);
  }
  pthread_cond_destroy(&s->cv);
  pthread_mutex_destroy(&s->mu);
  Py_TYPE(s)->tp_free((PyObject*)s);
}

static PyObject* sub_new(PyTypeObject* type, PyObject* args, PyObject* kw) {
  (void)kw;
  int device;
  PyObject* lanes;
  if (!PyArg_ParseTuple(args, "iO", &device, &lanes)) return NULL;
  PyObject* seq = PySequence_Fast(lanes, "lanes must be a sequence of argument tuples");
  if (!seq) return NULL;
  const Py_ssize_t nt = PySequence_Fast_GET_SIZE(seq);
  if (nt < 1 || nt > SUB_MAXT) {
    Py_DECREF(seq);
    return PyErr_Format(PyExc_ValueError, "1 to %d lanes", SUB_MAXT);
  }
  Submitter* s = (Submitter*)type->tp_alloc(type, 0);
  if (!s) {
    Py_DECREF(seq);
    return NULL;
  }
  s->nt = (int)nt;
  s->device = device;
  pthread_mutex_init(&s->mu, NULL);
  pthread_cond_init(&s->cv, NULL);
  for (Py_ssize_t i = 0; i < nt; ++i) {
    SubLane* l = &s->lane[i];
    PyObject* t = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, i), "an argument tuple");
    if (!t) goto fail;
    PyObject** v = PySequence_Fast_ITEMS(t);
    const int bad = PySequence_Fast_GET_SIZE(t) != 8 || as_ptr(v[0], &l->ctx) || as_i64(v[1], &l->p) ||
                    as_ptr(v[2], &l->pd) || as_ptr(v[3], &l->pt) || as_ptr(v[4], &l->oi) || as_ptr(v[5], &l->os) ||
                    as_ptr(v[6], &l->ost) || as_ptr(v[7], &l->st);
    Py_DECREF(t);
    if (bad || l->p < 0 || l->p > INT32_MAX) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "an argument tuple of schedule_batch_device");
      goto fail;
    }
    for (Py_ssize_t j = 0; j < i; ++j)
      if (s->lane[j].ctx == l->ctx || s->lane[j].st == l->st) {
        PyErr_SetString(PyExc_ValueError, "every lane needs its own ctx and its own stream");
        goto fail;
      }
  }
  Py_DECREF(seq);
  seq = NULL;
  for (int t = 0; t < s->nt; ++t)  // the lanes are valid: now the device
    if (hipEventCreate(&s->lane[t].e0) || hipEventCreate(&s->lane[t].e1)) {
      PyErr_SetString(PyExc_RuntimeError, "hipEventCreate failed");
      goto fail;
    }
  for (int t = 0; t < s->nt; ++t) {
    s->arg[t].s = s;
    s->arg[t].t = t;
    if (pthread_create(&s->th[t], NULL, sub_thread, &s->arg[t])) {
      sub_dealloc(s);
      return PyErr_Format(PyExc_RuntimeError, "pthread_create failed");
    }
    s->started = t + 1;
  }
  return (PyObject*)s;
fail:
  Py_XDECREF(seq);
  sub_dealloc(s);
  return NULL;
}

/* run(k) -> rc: k batches over the lanes; returns once all are submitted */
static PyObject* sub_run(Submitter* s, PyObject* const* a, Py_ssize_t n) {
  long long k;
  if (want_args(n, 1, "run") || as_i64(a[0], &k)) return NULL;
  if (k < 0) return PyErr_Format(PyExc_ValueError, "negative step count");
  if (!s->started) return PyErr_Format(PyExc_RuntimeError, "submitter closed");
  Py_BEGIN_ALLOW_THREADS
  s->k = k;
  s->t_go = mono_ns();
  atomic_store(&s->done, 0);
  atomic_store(&s->rc, 0);
  pthread_mutex_lock(&s->mu);
  atomic_fetch_add_explicit(&s->gen, 1, memory_order_release);
  pthread_cond_broadcast(&s->cv);
  pthread_mutex_unlock(&s->mu);
  while (atomic_load_explicit(&s->done, memory_order_acquire) < s->nt) __builtin_ia32_pause();
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(atomic_load(&s->rc));
}

/* span_ms() -> float: latest end event - earliest start event of the last run (synchronize first) */
static PyObject* sub_span_ms(Submitter* s, PyObject* unused) {
  (void)unused;
  float best = -1.0f;
  for (int j = 0; j < s->nt; ++j) {
    if (!s->lane[j].ran) continue;
    for (int i = 0; i < s->nt; ++i) {
      float ms;
      if (!s->lane[i].ran) continue;
      if (hipEventElapsedTime(&ms, s->lane[j].e0, s->lane[i].e1))
        return PyErr_Format(PyExc_RuntimeError, "hipEventElapsedTime failed (synchronize first)");
      if (ms > best) best = ms;
    }
  }
  return PyFloat_FromDouble(best);
}

/* host_us() -> [[us, ...] per lane]: the lanes' host timestamps of the last run, relative to the
 * run's signal: wake, after the start event, after each launch, after the end event (A/B probe) */
static PyObject* sub_host_us(Submitter* s, PyObject* unused) {
  (void)unused;
  PyObject* out = PyList_New(s->nt);
  if (!out) return NULL;
  for (int t = 0; t < s->nt; ++t) {
    PyObject* row = PyList_New(s->lane[t].nt);
    if (!row) {
      Py_DECREF(out);
      return NULL;
    }
    for (int i = 0; i < s->lane[t].nt; ++i)
      PyList_SET_ITEM(row, i, PyFloat_FromDouble((double)(s->lane[t].ts[i] - s->t_go) * 1e-3));
    PyList_SET_ITEM(out, t, row);
  }
  return out;
}

/* events_ms() -> [(start, end) per lane] in ms relative to lane 0's start event (synchronize first) */
static PyObject* sub_events_ms(Submitter* s, PyObject* unused) {
  (void)unused;
  PyObject* out = PyList_New(0);
  if (!out || !s->lane[0].ran) return out;
  for (int t = 0; t < s->nt; ++t) {
    if (!s->lane[t].ran) continue;
    float a = 0, b = 0;
    if (hipEventElapsedTime(&a, s->lane[0].e0, s->lane[t].e0) || hipEventElapsedTime(&b, s->lane[0].e0, s->lane[t].e1)) {
      Py_DECREF(out);
      return PyErr_Format(PyExc_RuntimeError, "hipEventElapsedTime failed (synchronize first)");
    }
    PyObject* pr = Py_BuildValue("(dd)", (double)a, (double)b);
    if (!pr || PyList_Append(out, pr)) {
      Py_XDECREF(pr);
      Py_DECREF(out);
      return NULL;
    }
    Py_DECREF(pr);
  }
  return out;
}

static PyObject* sub_close(Submitter* s, PyObject* unused) {
  (void)unused;
  sub_stop(s);
  Py_RETURN_NONE;
}

static PyMethodDef sub_methods[] = {
    {"run", (PyCFunction)(void (*)(void))sub_run, METH_FASTCALL, "run(k) -> rc: submit k batches over the lanes"},
    {"span_ms", (PyCFunction)sub_span_ms, METH_NOARGS, "device span of the last run in ms (synchronize first)"},
    {"host_us", (PyCFunction)sub_host_us, METH_NOARGS, "the lanes' host timestamps of the last run (A/B probe)"},
    {"events_ms", (PyCFunction)sub_events_ms, METH_NOARGS, "per lane (start, end) event times vs lane 0's start"},
    {"close", (PyCFunction)sub_close, METH_NOARGS, "stop the lane threads"},
    {NULL, NULL, 0, NULL},
};

static PyTypeObject SubmitterType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "_msh_fast.Submitter",
    .tp_basicsize = sizeof(Submitter),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "Submitter(device, lanes): batches submitted from one host thread per lane",
    .tp_new = sub_new,
    .tp_dealloc = (destructor)sub_dealloc,
    .tp_methods = sub_methods,
};

/* schedule_sequential_device(ctx, p, d_pod_digit, d_pod_tol, max_pods_per_node, d_out_idx,
 * d_out_score, d_out_status, stream) -> rc */
static PyObject* py_schedule_sequential_device(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  void *ctx, *pd, *pt, *oi, *os, *ost, *st;
  long long p, cap;
  if (want_args(n, 9, "schedule_sequential_device") || as_ptr(a[0], &ctx) || as_i64(a[1], &p) ||
      as_ptr(a[2], &pd) || as_ptr(a[3], &pt) || as_i64(a[4], &cap) || as_ptr(a[5], &oi) ||
      as_ptr(a[6], &os) || as_ptr(a[7], &ost) || as_ptr(a[8], &st))
    return NULL;
  if (p < INT32_MIN || p > INT32_MAX || cap < INT32_MIN || cap > INT32_MAX)
    return PyErr_Format(PyExc_OverflowError, "argument out of range");
  const int rc = msh_schedule_sequential_device((msh_ctx*)ctx, (int32_t)p, (const int8_t*)pd, (const uint8_t*)pt,
                                                (int32_t)cap, (int32_t*)oi, (int64_t*)os, (int32_t*)ost, st);
  return PyLong_FromLong(rc);
}

/* shard_keys_device(ctx, p, d_pod_digit, d_pod_tol, node_base, d_keys, stream) -> rc */
static PyObject* py_shard_keys_device(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  void *ctx, *pd, *pt, *keys, *st;
  long long p, base;
  if (want_args(n, 7, "shard_keys_device") || as_ptr(a[0], &ctx) || as_i64(a[1], &p) || as_ptr(a[2], &pd) ||
      as_ptr(a[3], &pt) || as_i64(a[4], &base) || as_ptr(a[5], &keys) || as_ptr(a[6], &st))
    return NULL;
  if (p < INT32_MIN || p > INT32_MAX) return PyErr_Format(PyExc_OverflowError, "pod count out of range");
  const int rc = msh_shard_keys_device((msh_ctx*)ctx, (int32_t)p, (const int8_t*)pd, (const uint8_t*)pt,
                                       (int64_t)base, (int32_t*)keys, st);
  return PyLong_FromLong(rc);
}

/* decode_keys_device(ctx, p, d_pod_digit, d_pod_tol, d_keys, d_out_idx, d_out_score,
 * d_out_status, stream) -> rc */
static PyObject* py_decode_keys_device(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  void *ctx, *pd, *pt, *keys, *oi, *os, *ost, *st;
  long long p;
  if (want_args(n, 9, "decode_keys_device") || as_ptr(a[0], &ctx) || as_i64(a[1], &p) || as_ptr(a[2], &pd) ||
      as_ptr(a[3], &pt) || as_ptr(a[4], &keys) || as_ptr(a[5], &oi) || as_ptr(a[6], &os) || as_ptr(a[7], &ost) ||
      as_ptr(a[8], &st))
    return NULL;
  if (p < INT32_MIN || p > INT32_MAX) return PyErr_Format(PyExc_OverflowError, "pod count out of range");
  const int rc = msh_decode_keys_device((msh_ctx*)ctx, (int32_t)p, (const int8_t*)pd, (const uint8_t*)pt,
                                        (const int32_t*)keys, (int32_t*)oi, (int64_t*)os, (int32_t*)ost, st);
  return PyLong_FromLong(rc);
}

/* ---- host-buffer calls: numpy arrays (or any C-contiguous buffer) by the buffer protocol ----
 * Taking an array's address through numpy's ctypes interface costs ~3 us per array in Python,
 * five per call; PyObject_GetBuffer costs ~0.1 us. The GIL is released during the call. */
static int get_buf(PyObject* o, Py_buffer* b, int writable, Py_ssize_t itemsize, const char* what) {
  if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | (writable ? PyBUF_WRITABLE : 0)) < 0) return -1;
  if (b->itemsize != itemsize) {
    PyBuffer_Release(b);
    PyErr_Format(PyExc_ValueError, "%s: item size %zd, expected %zd", what, b->itemsize, itemsize);
    return -1;
  }
  return 0;
}

/* The pod columns and the three output arrays of a host-buffer call; outputs may be longer. */
typedef struct {
  Py_buffer pd, pt, oi, os, ost;
  int n;
} HostBufs;

static void release_bufs(HostBufs* h) {
  Py_buffer* all[5] = {&h->pd, &h->pt, &h->oi, &h->os, &h->ost};
  for (int i = 0; i < h->n; ++i)
    if (all[i]->obj) PyBuffer_Release(all[i]);  // (an absent out_score holds no buffer)
}

static int get_host_bufs(PyObject* const* a, HostBufs* h, Py_ssize_t* p) {
  h->n = 0;
  if (get_buf(a[0], &h->pd, 0, 1, "pod_digit")) return -1;
  h->n = 1;
  if (get_buf(a[1], &h->pt, 0, 1, "pod_tol")) goto fail;
  h->n = 2;
  if (get_buf(a[2], &h->oi, 1, 4, "out_idx")) goto fail;
  h->n = 3;
  if (a[3] == Py_None) {  // optional: scores not written
    h->os.buf = NULL;
    h->os.len = 0;
    h->os.obj = NULL;
  } else if (get_buf(a[3], &h->os, 1, 8, "out_score")) {
    goto fail;
  }
  h->n = 4;
  if (get_buf(a[4], &h->ost, 1, 4, "out_status")) goto fail;
  h->n = 5;
  *p = h->pd.len;
  if (h->pt.len != *p || h->oi.len < 4 * *p || (h->os.buf && h->os.len < 8 * *p) || h->ost.len < 4 * *p ||
      *p > INT32_MAX) {
    PyErr_SetString(PyExc_ValueError, "pod_digit / pod_tol lengths differ, or an output array is too short");
    goto fail;
  }
  return 0;
fail:
  release_bufs(h);
  return -1;
}

/* schedule_batch_host(ctx, pod_digit, pod_tol, out_idx, out_score or None, out_status) -> rc */
static PyObject* py_schedule_batch_host(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  void* ctx;
  HostBufs h;
  Py_ssize_t p;
  if (want_args(n, 6, "schedule_batch_host") || as_ptr(a[0], &ctx) || get_host_bufs(a + 1, &h, &p)) return NULL;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = msh_schedule_batch((msh_ctx*)ctx, (int32_t)p, (const int8_t*)h.pd.buf, (const uint8_t*)h.pt.buf,
                          (int32_t*)h.oi.buf, (int64_t*)h.os.buf, (int32_t*)h.ost.buf);
  Py_END_ALLOW_THREADS
  release_bufs(&h);
  return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"schedule_batch_device_steps", (PyCFunction)(void (*)(void))py_schedule_batch_device_steps, METH_FASTCALL,
     "k msh_schedule_batch_device calls from C, cycling over the given argument tuples -> first rc"},
    {"schedule_batch_host", (PyCFunction)(void (*)(void))py_schedule_batch_host, METH_FASTCALL,
     "msh_schedule_batch(ctx, pod_digit, pod_tol, out_idx, out_score, out_status) -> rc (buffer protocol)"},
    {"schedule_batch_device", (PyCFunction)(void (*)(void))py_schedule_batch_device, METH_FASTCALL,
     "msh_schedule_batch_device(ctx, p, pod_digit, pod_tol, out_idx, out_score, out_status, stream) -> rc"},
    {"schedule_sequential_device", (PyCFunction)(void (*)(void))py_schedule_sequential_device, METH_FASTCALL,
     "msh_schedule_sequential_device(ctx, p, pod_digit, pod_tol, max_pods_per_node, out_idx, out_score, "
     "out_status, stream) -> rc"},
    {"shard_keys_device", (PyCFunction)(void (*)(void))py_shard_keys_device, METH_FASTCALL,
     "msh_shard_keys_device(ctx, p, pod_digit, pod_tol, node_base, keys, stream) -> rc"},
    {"decode_keys_device", (PyCFunction)(void (*)(void))py_decode_keys_device, METH_FASTCALL,
     "msh_decode_keys_device(ctx, p, pod_digit, pod_tol, keys, out_idx, out_score, out_status, stream) -> rc"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_msh_fast",
                                    "Fast-call bindings of the per-batch device entry points", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__msh_fast(void) {
  if (PyType_Ready(&SubmitterType) < 0) return NULL;
  PyObject* m = PyModule_Create(&module);
  if (!m) return NULL;
  Py_INCREF(&SubmitterType);
  if (PyModule_AddObject(m, "Submitter", (PyObject*)&SubmitterType) < 0) {
    Py_DECREF(&SubmitterType);
    Py_DECREF(m);
    return NULL;
  }
  return m;
}
