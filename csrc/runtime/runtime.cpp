// Device runtime helpers: launch checking, device inventory, pinned staging.
//
// Reference parity: the reference has no device runtime at all; its worker
// registers a bare {id, address} (reference crates/api/proto/coordinator.proto:11-14).
// Our workers report the GPU inventory gathered here.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/common.h"
#include "runtime.h"

namespace igloo {
namespace kern {

static int sync_check_mode() {
  static int mode = debug_flag("sync_check") ? 1 : 0;
  return mode;
}

void check_launch(const char* what, hipStream_t stream) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    throw std::runtime_error(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
  if (sync_check_mode()) {
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess)
      throw std::runtime_error(std::string("kernel execution failed (") + what + "): " + hipGetErrorString(e));
  }
}

}  // namespace kern

namespace rt {

DeviceInfo device_info(int device) {
  DeviceInfo d;
  hipDeviceProp_t p;
  IGLOO_HIP_CHECK(hipGetDeviceProperties(&p, device));
  d.device = device;
  d.name = p.name;
  d.arch = p.gcnArchName;
  d.total_mem = p.totalGlobalMem;
  d.cu_count = p.multiProcessorCount;
  d.lds_per_block = p.sharedMemPerBlock;
  d.wave_size = p.warpSize;
  d.clock_khz = p.clockRate;
  d.l2_bytes = p.l2CacheSize;
  size_t free_b = 0, total_b = 0;
  int prev = 0;
  IGLOO_HIP_CHECK(hipGetDevice(&prev));
  IGLOO_HIP_CHECK(hipSetDevice(device));
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) d.free_mem = free_b;
  IGLOO_HIP_CHECK(hipSetDevice(prev));
  return d;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ---------------------------------------------------------------- pinned pool
// Size-bucketed pool of page-locked host buffers used as H2D/D2H staging for
// scans and result materialisation. Buffers are recycled
// instead of hipHostMalloc'd per batch because pinning is expensive.
struct PinnedPool::Impl {
  std::mutex mu;
  std::vector<std::pair<size_t, void*>> free_list;
  size_t cached = 0, limit = 0;
};

PinnedPool::PinnedPool(size_t limit_bytes) : impl_(new Impl) { impl_->limit = limit_bytes; }

PinnedPool::~PinnedPool() {
  for (auto& f : impl_->free_list) (void)hipHostFree(f.second);
  delete impl_;
}

void* PinnedPool::acquire(size_t bytes, size_t* got) {
  size_t want = 1;
  while (want < bytes) want <<= 1;
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    for (size_t i = 0; i < impl_->free_list.size(); ++i) {
      if (impl_->free_list[i].first == want) {
        void* p = impl_->free_list[i].second;
        impl_->free_list.erase(impl_->free_list.begin() + i);
        impl_->cached -= want;
        *got = want;
        return p;
      }
    }
  }
  void* p = nullptr;
  IGLOO_HIP_CHECK(hipHostMalloc(&p, want, hipHostMallocDefault));
  *got = want;
  return p;
}

void PinnedPool::release(void* p, size_t bytes) {
  std::lock_guard<std::mutex> g(impl_->mu);
  if (impl_->cached + bytes > impl_->limit) {
    (void)hipHostFree(p);
    return;
  }
  impl_->free_list.emplace_back(bytes, p);
  impl_->cached += bytes;
}

size_t PinnedPool::cached_bytes() const { return impl_->cached; }

}  // namespace rt
}  // namespace igloo
