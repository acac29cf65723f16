// Native launch path for the HIP kernel library (_C_hip.so).
//
// Every exported launcher `pa_*` gets a METH_FASTCALL CPython entry point generated from the signature
// table in paddlepaddle_amd/ops/_loader.py (tools/build_native.py writes dispatch_gen.inc). An entry point
// unpacks its arguments straight from the Python objects the op layer already holds:
//   pointer args : torch.Tensor (-> data_ptr), None (-> nullptr), int, a ctypes pointer / struct, or the
//                  current-stream sentinel (-> the caller's current HIP stream, read from c10 without
//                  creating a Python stream object),
//   int / float  : Python int / float / numpy scalars (ctypes scalars accepted too).
// This replaces the ctypes marshalling (per-arg c_void_p objects, torch.cuda.current_stream(), argtype
// conversion) on the eager launch path; the kernels and their C ABI are unchanged, so the ctypes path
// stays available as a fallback when this module is not built.
#include <Python.h>

#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>

namespace {

PyObject* g_cur_stream = nullptr;  // sentinel object: "the current stream of the current device"

bool arg_ptr(PyObject* o, void** out);

bool ptr_from_attr(PyObject* o, const char* attr, void** out) {
  PyObject* v = PyObject_GetAttrString(o, attr);
  if (v == nullptr) {
    PyErr_Clear();
    return false;
  }
  bool ok = arg_ptr(v, out);
  Py_DECREF(v);
  return ok;
}

bool arg_ptr(PyObject* o, void** out) {
  if (THPVariable_Check(o)) {
    *out = THPVariable_Unpack(o).data_ptr();
    return true;
  }
  if (o == Py_None) {
    *out = nullptr;
    return true;
  }
  if (o == g_cur_stream) {
    *out = static_cast<void*>(c10::hip::getCurrentHIPStream().stream());
    return true;
  }
  if (PyLong_Check(o)) {
    *out = PyLong_AsVoidPtr(o);
    return !PyErr_Occurred();
  }
  // ctypes: c_void_p / c_int64 (.value), byref(struct) (._obj), Structure / Array (buffer protocol)
  if (ptr_from_attr(o, "value", out) || ptr_from_attr(o, "_obj", out)) return true;
  if (PyErr_Occurred()) return false;
  Py_buffer b;
  if (PyObject_GetBuffer(o, &b, PyBUF_SIMPLE) == 0) {
    *out = b.buf;
    PyBuffer_Release(&b);
    return true;
  }
  PyErr_Clear();
  PyErr_Format(PyExc_TypeError, "cannot pass a %s as a pointer argument", Py_TYPE(o)->tp_name);
  return false;
}

bool scalar_value(PyObject* o, PyObject** v) {
  *v = PyObject_GetAttrString(o, "value");  // ctypes scalar
  if (*v == nullptr) {
    PyErr_Clear();
    PyErr_Format(PyExc_TypeError, "expected a number, got %s", Py_TYPE(o)->tp_name);
    return false;
  }
  return true;
}

bool arg_i64(PyObject* o, int64_t* out) {
  if (PyLong_Check(o)) {
    *out = PyLong_AsLongLong(o);
    return !(*out == -1 && PyErr_Occurred());
  }
  PyObject* i = PyNumber_Index(o);
  if (i != nullptr) {
    *out = PyLong_AsLongLong(i);
    Py_DECREF(i);
    return !(*out == -1 && PyErr_Occurred());
  }
  PyErr_Clear();
  PyObject* v;
  if (!scalar_value(o, &v)) return false;
  bool ok = arg_i64(v, out);
  Py_DECREF(v);
  return ok;
}

bool arg_i32(PyObject* o, int* out) {
  int64_t v;
  if (!arg_i64(o, &v)) return false;
  *out = static_cast<int>(v);
  return true;
}

bool arg_u64(PyObject* o, uint64_t* out) {
  if (PyLong_Check(o)) {
    *out = PyLong_AsUnsignedLongLongMask(o);
    return !PyErr_Occurred();
  }
  int64_t v;
  if (!arg_i64(o, &v)) return false;
  *out = static_cast<uint64_t>(v);
  return true;
}

bool arg_f32(PyObject* o, float* out) {
  double d = PyFloat_AsDouble(o);
  if (d == -1.0 && PyErr_Occurred()) {
    PyErr_Clear();
    PyObject* v;
    if (!scalar_value(o, &v)) return false;
    d = PyFloat_AsDouble(v);
    Py_DECREF(v);
    if (d == -1.0 && PyErr_Occurred()) return false;
  }
  *out = static_cast<float>(d);
  return true;
}

PyObject* bad_nargs(const char* name, Py_ssize_t want, Py_ssize_t got) {
  PyErr_Format(PyExc_TypeError, "%s takes %zd arguments (%zd given)", name, want, got);
  return nullptr;
}

}  // namespace

#include "dispatch_gen.inc"

namespace {

PyObject* set_stream_sentinel(PyObject*, PyObject* o) {
  Py_XDECREF(g_cur_stream);
  Py_INCREF(o);
  g_cur_stream = o;
  Py_RETURN_NONE;
}

PyObject* current_stream(PyObject*, PyObject*) {
  return PyLong_FromVoidPtr(static_cast<void*>(c10::hip::getCurrentHIPStream().stream()));
}

std::vector<PyMethodDef>& methods() {
  static std::vector<PyMethodDef> m = [] {
    std::vector<PyMethodDef> v(std::begin(kGenMethods), std::end(kGenMethods));
    v.push_back({"set_stream_sentinel", set_stream_sentinel, METH_O, "register the current-stream sentinel"});
    v.push_back({"current_stream", current_stream, METH_NOARGS, "current HIP stream handle as an int"});
    v.push_back({nullptr, nullptr, 0, nullptr});
    return v;
  }();
  return m;
}

PyModuleDef g_module = {PyModuleDef_HEAD_INIT, "_C_dispatch", "native launch path of the HIP kernels", -1,
                        nullptr, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__C_dispatch() {
  g_module.m_methods = methods().data();
  return PyModule_Create(&g_module);
}
