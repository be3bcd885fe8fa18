// Conversion of the native SQL AST into plain Python dicts for the binder.
#pragma once

#include <pybind11/pybind11.h>

#include "ast.h"

namespace igloo {
namespace sql {

inline pybind11::object to_python(const NodeP& n) {
  namespace py = pybind11;
  if (!n) return py::none();
  py::dict d;
  d["k"] = n->kind;
  d["s"] = n->str;
  d["pos"] = n->pos;
  py::list kids;
  for (auto& c : n->kids) kids.append(to_python(c));
  d["c"] = kids;
  for (auto& kv : n->attrs) d[py::str(kv.first)] = to_python(kv.second);
  for (auto& kv : n->flags) d[py::str(kv.first)] = kv.second;
  return std::move(d);
}

}  // namespace sql
}  // namespace igloo
