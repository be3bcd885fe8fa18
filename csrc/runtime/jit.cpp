// Query-specialised kernels: HIP source generated per plan shape
// (igloo_amd/ops/jit.py), compiled for gfx950 in-process with hiprtc, loaded
// as a code object and launched with a flat kernarg buffer.
//
// Why: the descriptor-driven fused scan kernels (kernels/fused.hip) interpret
// their filter terms / aggregate factors per row; rocprofv3 counters on TPC-H
// Q1 at SF100 showed ~1.3 SALU + 1 VALU instruction per row-lane of pure
// interpretation (303k SALU and 229k VALU per wave) at 7% of HBM bandwidth.
// A kernel generated for the plan has the column widths, literals, group
// layout and aggregate shapes as compile-time constants. The reference builds
// its operators from DataFusion's physical plan at run time (reference
// crates/engine/src/lib.rs:55-56); here the physical plan's scan fragments
// become machine code.
//
// compile() is host-only (no HIP context: it runs on a background thread
// while the interpreted kernel serves the first executions); load() and
// launch() run on the query thread.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace igloo {
namespace {

std::string rtc_error(hiprtcProgram p, hiprtcResult r, const char* what) {
  std::string msg = std::string("jit ") + what + ": " + hiprtcGetErrorString(r);
  size_t n = 0;
  if (p && hiprtcGetProgramLogSize(p, &n) == HIPRTC_SUCCESS && n > 1) {
    std::string log(n, '\0');
    hiprtcGetProgramLog(p, log.data());
    msg += "\n" + log;
  }
  return msg;
}

// hipcc-equivalent options for the generated sources (no includes: the
// generator emits its own prelude)
std::vector<std::string> rtc_options(const std::string& arch) {
  return {"--offload-arch=" + arch, "-O3", "-std=c++17", "-munsafe-fp-atomics", "-ffast-math"};
}

py::bytes compile(const std::string& src, const std::string& name, const std::string& arch) {
  std::string code;
  {
    py::gil_scoped_release nogil;
    hiprtcProgram p = nullptr;
    hiprtcResult r = hiprtcCreateProgram(&p, src.c_str(), (name + ".hip").c_str(), 0, nullptr, nullptr);
    if (r != HIPRTC_SUCCESS) throw std::runtime_error(rtc_error(p, r, "create"));
    const auto opts = rtc_options(arch);
    std::vector<const char*> argv;
    for (const auto& o : opts) argv.push_back(o.c_str());
    r = hiprtcCompileProgram(p, (int)argv.size(), argv.data());
    if (r != HIPRTC_SUCCESS) {
      const std::string msg = rtc_error(p, r, "compile");
      hiprtcDestroyProgram(&p);
      throw std::runtime_error(msg);
    }
    size_t n = 0;
    hiprtcGetCodeSize(p, &n);
    code.resize(n);
    hiprtcGetCode(p, code.data());
    hiprtcDestroyProgram(&p);
  }
  return py::bytes(code);
}

struct Loaded {
  hipModule_t mod;
  hipFunction_t fn;
};
std::mutex g_mu;
std::vector<Loaded> g_loaded;  // modules stay loaded for the process lifetime (a handful per plan shape)

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("jit ") + what + ": " + hipGetErrorString(e));
}

int64_t load(const std::string& code, const std::string& name) {
  hipModule_t m = nullptr;
  check(hipModuleLoadData(&m, code.data()), "hipModuleLoadData");
  hipFunction_t f = nullptr;
  const hipError_t e = hipModuleGetFunction(&f, m, name.c_str());
  if (e != hipSuccess) {
    hipModuleUnload(m);
    check(e, "hipModuleGetFunction");
  }
  std::lock_guard<std::mutex> g(g_mu);
  g_loaded.push_back({m, f});
  return (int64_t)g_loaded.size() - 1;
}

struct KernArgs {
  std::vector<uint64_t> buf;
  size_t size;
};
// kernarg buffers of captured launches (stable addresses: deque push_back)
static std::deque<KernArgs> g_captured_args;

// args: the kernel's parameters in order, each one 8-byte slot (pointers and
// 64-bit integers: the generator declares nothing narrower)
void launch(int64_t h, uint32_t grid, uint32_t block, uint32_t shmem, uintptr_t stream,
            const std::vector<uint64_t>& args) {
  hipFunction_t f;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (h < 0 || h >= (int64_t)g_loaded.size()) throw std::runtime_error("jit launch: bad kernel handle");
    f = g_loaded[h].fn;
  }
  if (grid == 0 || block == 0 || block > 1024) throw std::runtime_error("jit launch: bad geometry");
  // Under stream capture (query graphs, igloo_amd/exec/graphs.py) the kernel
  // node may keep referring to the kernarg buffer passed through `extra`
  // rather than copying it, so a captured launch gets a buffer that lives as
  // long as the process (a few hundred bytes per captured launch); graph
  // replays read garbage arguments otherwise. Eager launches use the stack.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing((hipStream_t)stream, &cap);
  KernArgs local{args, args.size() * sizeof(uint64_t)};
  KernArgs* ka = &local;
  if (cap != hipStreamCaptureStatusNone) {
    std::lock_guard<std::mutex> g(g_mu);
    g_captured_args.push_back(local);
    ka = &g_captured_args.back();
  }
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, ka->buf.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &ka->size,
                   HIP_LAUNCH_PARAM_END};
  check(hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, shmem, (hipStream_t)stream, nullptr, extra),
        "hipModuleLaunchKernel");
}

// resource usage of a loaded kernel (tests / EXPLAIN): registers, LDS, scratch
py::dict attributes(int64_t h) {
  hipFunction_t f;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (h < 0 || h >= (int64_t)g_loaded.size()) throw std::runtime_error("jit: bad kernel handle");
    f = g_loaded[h].fn;
  }
  py::dict d;
  int v = 0;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_NUM_REGS, f) == hipSuccess) d["vgprs"] = v;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, f) == hipSuccess) d["lds"] = v;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, f) == hipSuccess) d["scratch"] = v;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, f) == hipSuccess) d["max_threads"] = v;
  return d;
}

}  // namespace

void register_jit(py::module_& m) {
  m.def("jit_compile", &compile, py::arg("src"), py::arg("name"), py::arg("arch") = "gfx950",
        "hiprtc: HIP source -> gfx950 code object (host only; releases the GIL)");
  m.def("jit_load", [](py::bytes code, const std::string& name) { return load(std::string(code), name); });
  m.def("jit_launch", &launch, py::arg("handle"), py::arg("grid"), py::arg("block"), py::arg("shmem"),
        py::arg("stream"), py::arg("args"));
  m.def("jit_attributes", &attributes);
}

}  // namespace igloo
