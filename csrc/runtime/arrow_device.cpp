// Zero-copy hand-off of device-resident query results through the Arrow C
// Device Data Interface (ArrowDeviceArray, device type ROCm) as PyCapsules
// ("arrow_schema" / "arrow_device_array", the __arrow_c_device_array__
// protocol). The exported buffers ARE the engine's HBM column buffers: the
// capsule's private data holds references to the Python objects (torch
// tensors) that own them and a HIP event recorded after the producing
// kernels, released when the consumer calls the array's release callback.
//
// Reference parity: pyigloo is an empty cdylib there (reference
// pyigloo/src/lib.rs:1, Cargo.toml:11-19 with pyo3 commented out); SURVEY
// §7.1 asks for Arrow C Device / DLPack interop of results.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

namespace py = pybind11;

extern "C" {
// Arrow C data / device interface ABI (arrow/c/abi.h, stable since Arrow 1.0 / 14.0)
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};
struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif
#ifndef ARROW_C_DEVICE_DATA_INTERFACE
#define ARROW_C_DEVICE_DATA_INTERFACE
typedef int32_t ArrowDeviceType;
#define ARROW_DEVICE_CPU 1
#define ARROW_DEVICE_ROCM 10
struct ArrowDeviceArray {
  struct ArrowArray array;
  int64_t device_id;
  ArrowDeviceType device_type;
  void* sync_event;
  int64_t reserved[3];
};
#endif
}

namespace igloo {
namespace {

// ----------------------------------------------------------------- schema
struct SchemaPriv {
  std::string format, name;
  std::vector<ArrowSchema*> kids;
};

void release_schema(ArrowSchema* s) {
  if (s == nullptr || s->release == nullptr) return;
  auto* p = static_cast<SchemaPriv*>(s->private_data);
  for (ArrowSchema* k : p->kids) {
    if (k->release) k->release(k);
    delete k;
  }
  if (s->dictionary) {
    if (s->dictionary->release) s->dictionary->release(s->dictionary);
    delete s->dictionary;
  }
  delete p;
  s->release = nullptr;
}

// spec: (format, name, nullable, [child specs], dictionary spec | None)
void fill_schema(ArrowSchema* s, const py::tuple& spec) {
  auto* p = new SchemaPriv();
  p->format = spec[0].cast<std::string>();
  p->name = spec[1].cast<std::string>();
  s->format = p->format.c_str();
  s->name = p->name.c_str();
  s->metadata = nullptr;
  s->flags = spec[2].cast<bool>() ? ARROW_FLAG_NULLABLE : 0;
  py::list kids = spec[3].cast<py::list>();
  for (auto k : kids) {
    auto* c = new ArrowSchema();
    fill_schema(c, k.cast<py::tuple>());
    p->kids.push_back(c);
  }
  s->n_children = static_cast<int64_t>(p->kids.size());
  s->children = p->kids.empty() ? nullptr : p->kids.data();
  s->dictionary = nullptr;
  if (!spec[4].is_none()) {
    s->dictionary = new ArrowSchema();
    fill_schema(s->dictionary, spec[4].cast<py::tuple>());
  }
  s->private_data = p;
  s->release = &release_schema;
}

// ------------------------------------------------------------------ array
struct ArrayPriv {
  std::vector<const void*> buffers;
  std::vector<ArrowArray*> kids;
  py::object keep;        // owners of the buffers (torch tensors), released under the GIL
  hipEvent_t event = nullptr;
};

void release_array(ArrowArray* a) {
  if (a == nullptr || a->release == nullptr) return;
  auto* p = static_cast<ArrayPriv*>(a->private_data);
  for (ArrowArray* k : p->kids) {
    if (k->release) k->release(k);
    delete k;
  }
  if (a->dictionary) {
    if (a->dictionary->release) a->dictionary->release(a->dictionary);
    delete a->dictionary;
  }
  if (p->event) (void)hipEventDestroy(p->event);
  {
    py::gil_scoped_acquire gil;
    p->keep = py::object();
  }
  delete p;
  a->release = nullptr;
}

// spec: (length, null_count, [buffer addresses], [child specs], dictionary spec | None, keepalive)
void fill_array(ArrowArray* a, const py::tuple& spec) {
  auto* p = new ArrayPriv();
  for (auto b : spec[2].cast<py::list>()) p->buffers.push_back(reinterpret_cast<const void*>(b.cast<uintptr_t>()));
  for (auto k : spec[3].cast<py::list>()) {
    auto* c = new ArrowArray();
    fill_array(c, k.cast<py::tuple>());
    p->kids.push_back(c);
  }
  p->keep = spec[5];
  a->length = spec[0].cast<int64_t>();
  a->null_count = spec[1].cast<int64_t>();
  a->offset = 0;
  a->n_buffers = static_cast<int64_t>(p->buffers.size());
  a->buffers = p->buffers.empty() ? nullptr : p->buffers.data();
  a->n_children = static_cast<int64_t>(p->kids.size());
  a->children = p->kids.empty() ? nullptr : p->kids.data();
  a->dictionary = nullptr;
  if (!spec[4].is_none()) {
    a->dictionary = new ArrowArray();
    fill_array(a->dictionary, spec[4].cast<py::tuple>());
  }
  a->private_data = p;
  a->release = &release_array;
}

void schema_capsule_dtor(PyObject* cap) {
  auto* s = static_cast<ArrowSchema*>(PyCapsule_GetPointer(cap, "arrow_schema"));
  if (s == nullptr) {
    PyErr_Clear();
    return;
  }
  if (s->release) s->release(s);
  delete s;
}

void device_capsule_dtor(PyObject* cap) {
  auto* d = static_cast<ArrowDeviceArray*>(PyCapsule_GetPointer(cap, "arrow_device_array"));
  if (d == nullptr) {
    PyErr_Clear();
    return;
  }
  if (d->array.release) {
    // the GIL is held here; release_array re-acquires it (recursive-safe)
    d->array.release(&d->array);
  }
  delete d;
}

void array_capsule_dtor(PyObject* cap) {
  auto* a = static_cast<ArrowArray*>(PyCapsule_GetPointer(cap, "arrow_array"));
  if (a == nullptr) {
    PyErr_Clear();
    return;
  }
  if (a->release) a->release(a);
  delete a;
}

// (schema capsule, device array capsule); device_id < 0: CPU memory
py::tuple export_device(const py::tuple& schema_spec, const py::tuple& array_spec, int device_id,
                        uintptr_t stream) {
  auto* s = new ArrowSchema();
  fill_schema(s, schema_spec);
  auto* d = new ArrowDeviceArray();
  fill_array(&d->array, array_spec);
  d->device_id = device_id < 0 ? -1 : device_id;
  d->device_type = device_id < 0 ? ARROW_DEVICE_CPU : ARROW_DEVICE_ROCM;
  d->sync_event = nullptr;
  if (device_id >= 0) {
    // consumers wait on this event before touching the buffers (the
    // producing kernels were enqueued on `stream`)
    auto* p = static_cast<ArrayPriv*>(d->array.private_data);
    if (hipEventCreateWithFlags(&p->event, hipEventDisableTiming) == hipSuccess &&
        hipEventRecord(p->event, reinterpret_cast<hipStream_t>(stream)) == hipSuccess) {
      d->sync_event = &p->event;
    }
  }
  py::capsule sc(s, "arrow_schema", &schema_capsule_dtor);
  py::capsule dc(d, "arrow_device_array", &device_capsule_dtor);
  return py::make_tuple(sc, dc);
}

// host memory: (schema capsule, array capsule), the __arrow_c_array__ protocol
py::tuple export_host(const py::tuple& schema_spec, const py::tuple& array_spec) {
  auto* s = new ArrowSchema();
  fill_schema(s, schema_spec);
  auto* a = new ArrowArray();
  fill_array(a, array_spec);
  return py::make_tuple(py::capsule(s, "arrow_schema", &schema_capsule_dtor),
                        py::capsule(a, "arrow_array", &array_capsule_dtor));
}

// introspection for tests: the exported struct's fields
py::dict describe_device_array(py::capsule cap) {
  auto* d = static_cast<ArrowDeviceArray*>(cap.get_pointer());
  py::dict out;
  out["device_type"] = d->device_type;
  out["device_id"] = d->device_id;
  out["length"] = d->array.length;
  out["null_count"] = d->array.null_count;
  out["n_children"] = d->array.n_children;
  out["has_event"] = d->sync_event != nullptr;
  py::list kids;
  for (int64_t i = 0; i < d->array.n_children; ++i) {
    ArrowArray* c = d->array.children[i];
    py::list bufs;
    for (int64_t b = 0; b < c->n_buffers; ++b) bufs.append(reinterpret_cast<uintptr_t>(c->buffers[b]));
    py::dict k;
    k["length"] = c->length;
    k["buffers"] = bufs;
    k["has_dictionary"] = c->dictionary != nullptr;
    kids.append(k);
  }
  out["children"] = kids;
  return out;
}

}  // namespace

void register_arrow_device(py::module_& m) {
  m.def("arrow_export_device", &export_device, py::arg("schema"), py::arg("array"), py::arg("device_id"),
        py::arg("stream") = 0, "ArrowSchema + ArrowDeviceArray PyCapsules over existing buffers (zero copy)");
  m.def("arrow_export_host", &export_host, py::arg("schema"), py::arg("array"));
  m.def("arrow_describe_device_array", &describe_device_array);
}

}  // namespace igloo
