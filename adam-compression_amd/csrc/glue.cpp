// Host glue of DistributedOptimizer(batch=True) (dgc/horovod/batched.py): the loops over
// every parameter that the grouped step runs each optimizer step, in C++ instead of
// Python — on the GPU box's host they cost ~0.2 ms per step for ResNet-50's 161 tensors
// in Python, as much as the whole device step.
//
//   grad_table(params, table_addr, align)   p.grad's data pointer of every parameter into
//       a ctypes array (the K1 / dense kernels' pointer tables); returns the positions
//       whose gradient the kernels cannot read in place (none; not contiguous; or not
//       `align`-byte aligned) for the Python fallback to handle.
//   release_grads(params)   p.grad = None for every parameter: torch's
//       zero_grad(set_to_none=True) without its per-parameter Python.
//   bind_grads(params, views)   p.grad = views[i] where it is not that tensor already —
//       the reference's p.grad.set_(decompressed) (dgc/horovod/optimizer.py:181-187).
//       The views are the batched step's own output views, built with each parameter's
//       shape, dtype and device (what the Python p.grad setter checks).
//
// Plumbing only: no arithmetic and nothing of the DGC path; the kernels stay behind the
// C ABI of libdgc_hip.so.
#include <Python.h>

#include <cstdint>

#include <torch/csrc/autograd/python_variable.h>
#include <torch/csrc/autograd/variable.h>

namespace {

bool is_list(PyObject* o) { return PyList_Check(o); }

// ATen calls below can throw c10::Error (a tensor without storage, ...): the exception
// becomes a Python RuntimeError instead of crossing the CPython frame (std::terminate)
#define GLUE_TRY try {
#define GLUE_CATCH                                                  \
    }                                                               \
    catch (const std::exception& e) {                               \
        PyErr_SetString(PyExc_RuntimeError, e.what());              \
        return nullptr;                                             \
    }

PyObject* grad_table(PyObject*, PyObject* args) {
    PyObject* params;
    unsigned long long addr;
    long long align;
    if (!PyArg_ParseTuple(args, "OKL", &params, &addr, &align)) return nullptr;
    if (!is_list(params) || addr == 0 || align < 1) {
        PyErr_SetString(PyExc_TypeError, "grad_table(params: list, table_addr: int, align: int)");
        return nullptr;
    }
    auto* table = reinterpret_cast<void**>(static_cast<uintptr_t>(addr));
    PyObject* fallback = PyList_New(0);
    if (!fallback) return nullptr;
    const Py_ssize_t n = PyList_GET_SIZE(params);
    GLUE_TRY
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* p = PyList_GET_ITEM(params, i);
        if (!THPVariable_Check(p)) {
            Py_DECREF(fallback);
            PyErr_SetString(PyExc_TypeError, "grad_table: not a tensor");
            return nullptr;
        }
        const at::Tensor& g = THPVariable_Unpack(p).grad();
        // a sparse (nn.Embedding(sparse=True)) or otherwise non-strided gradient has no
        // data pointer: the Python fallback handles it (or raises a Python error)
        const bool strided = g.defined() && g.layout() == at::kStrided && g.has_storage();
        void* ptr = strided ? g.data_ptr() : nullptr;
        if (!strided || !g.is_contiguous() || (reinterpret_cast<uintptr_t>(ptr) % (uintptr_t)align) != 0) {
            PyObject* idx = PyLong_FromSsize_t(i);
            if (!idx || PyList_Append(fallback, idx) != 0) {
                Py_XDECREF(idx);
                Py_DECREF(fallback);
                return nullptr;
            }
            Py_DECREF(idx);
            table[i] = nullptr;
            continue;
        }
        table[i] = ptr;
    }
    } catch (const std::exception& e) {
        Py_DECREF(fallback);
        PyErr_SetString(PyExc_RuntimeError, e.what());
        return nullptr;
    }
    return fallback;
}

PyObject* bind_grads(PyObject*, PyObject* args) {
    PyObject *params, *views;
    if (!PyArg_ParseTuple(args, "OO", &params, &views)) return nullptr;
    if (!is_list(params) || !is_list(views) || PyList_GET_SIZE(params) != PyList_GET_SIZE(views)) {
        PyErr_SetString(PyExc_TypeError, "bind_grads(params: list, views: list) of equal length");
        return nullptr;
    }
    const Py_ssize_t n = PyList_GET_SIZE(params);
    GLUE_TRY
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* p = PyList_GET_ITEM(params, i);
        PyObject* v = PyList_GET_ITEM(views, i);
        if (!THPVariable_Check(p) || !THPVariable_Check(v)) {
            PyErr_SetString(PyExc_TypeError, "bind_grads: not a tensor");
            return nullptr;
        }
        const at::Tensor& view = THPVariable_Unpack(v);
        at::Tensor& grad = const_cast<at::Tensor&>(THPVariable_Unpack(p)).mutable_grad();
        if (!grad.is_same(view)) grad = view;
    }
    GLUE_CATCH
    Py_RETURN_NONE;
}

PyObject* release_grads(PyObject*, PyObject* args) {
    PyObject* params;
    if (!PyArg_ParseTuple(args, "O", &params)) return nullptr;
    if (!is_list(params)) {
        PyErr_SetString(PyExc_TypeError, "release_grads(params: list)");
        return nullptr;
    }
    const Py_ssize_t n = PyList_GET_SIZE(params);
    GLUE_TRY
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* p = PyList_GET_ITEM(params, i);
        if (!THPVariable_Check(p)) {
            PyErr_SetString(PyExc_TypeError, "release_grads: not a tensor");
            return nullptr;
        }
        const_cast<at::Tensor&>(THPVariable_Unpack(p)).mutable_grad().reset();
    }
    GLUE_CATCH
    Py_RETURN_NONE;
}

PyMethodDef methods[] = {
    {"release_grads", release_grads, METH_VARARGS, "p.grad = None for every parameter (zero_grad(set_to_none=True))"},
    {"grad_table", grad_table, METH_VARARGS, "p.grad data pointers into a ctypes table; returns fallback positions"},
    {"bind_grads", bind_grads, METH_VARARGS, "p.grad = views[i] for every parameter"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_dgc_glue", "DistributedOptimizer(batch=True) host glue", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__dgc_glue(void) { return PyModule_Create(&module); }
