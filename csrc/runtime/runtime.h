#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace igloo {
namespace rt {

struct DeviceInfo {
  int device = 0;
  std::string name, arch;
  size_t total_mem = 0, free_mem = 0, lds_per_block = 0, l2_bytes = 0;
  int cu_count = 0, wave_size = 0, clock_khz = 0;
};

DeviceInfo device_info(int device);
int device_count();

class PinnedPool {
 public:
  explicit PinnedPool(size_t limit_bytes);
  ~PinnedPool();
  void* acquire(size_t bytes, size_t* got);
  void release(void* p, size_t bytes);
  size_t cached_bytes() const;

 private:
  struct Impl;
  Impl* impl_;
};

}  // namespace rt
}  // namespace igloo
