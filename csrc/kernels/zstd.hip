// GPU ZSTD decompression of Parquet pages (csrc/kernels/zstd_decode.h holds
// the decoder, written once for a wave of W lanes).
//
// pq_zstd_kernel: one 64-lane workgroup per compressed page (grid-strided
// over the page jobs, the grid capped by the per-workgroup literal buffers
// the caller allocates); pages of another codec are skipped, so the same job
// list feeds pq_snappy and pq_zstd. ZSTD is the default codec of DataFusion's
// and Iceberg's Parquet writers; the reference reads it on the host through
// parquet-rs (reference crates/engine/src/operators/parquet_scan.rs:47-58,
// crates/connectors/iceberg/src/lib.rs:95-104).
#include <memory>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "zstd_decode.h"

namespace igloo {
namespace kern {

namespace {

struct DevWave {
  static constexpr int W = kWave;
  __device__ int lane() const { return (int)threadIdx.x; }
  __device__ void sync() const { __syncthreads(); }
  // this wave's earlier global stores complete and visible to its later loads
  __device__ void fence() const {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  __device__ bool any(bool b) const { return __ballot(b) != 0; }
  __device__ uint64_t ballot(bool b) const { return __ballot(b); }
  __device__ int64_t scan(int64_t v) const { return wave_inclusive_scan(v); }
  __device__ int64_t bcast(int64_t v, int k) const { return __shfl(v, k, kWave); }
  __device__ uint8_t ld(const uint8_t* p) const { return __builtin_nontemporal_load(p); }
  // wave-uniform values: scalar registers, so the entropy decode runs on the scalar ALU
  __device__ uint32_t uni(uint32_t v) const { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
  __device__ uint64_t uni64(uint64_t v) const {
    return (uint64_t)uni((uint32_t)v) | ((uint64_t)uni((uint32_t)(v >> 32)) << 32);
  }
};

struct HostWave {
  static constexpr int W = 1;
  int lane() const { return 0; }
  void sync() const {}
  void fence() const {}
  bool any(bool b) const { return b; }
  uint64_t ballot(bool b) const { return b ? 1ull : 0ull; }
  int64_t scan(int64_t v) const { return v; }
  int64_t bcast(int64_t v, int) const { return v; }
  uint8_t ld(const uint8_t* p) const { return *p; }
  uint32_t uni(uint32_t v) const { return v; }
  uint64_t uni64(uint64_t v) const { return v; }
};

__global__ __launch_bounds__(kWave) void pq_zstd_kernel(const PqSnappyJob* __restrict__ jobs, int64_t njobs,
                                                        const uint8_t* __restrict__ raw, uint8_t* __restrict__ dec,
                                                        uint8_t* __restrict__ lit_all, int* __restrict__ err) {
  __shared__ zstd::Scratch sc;
  DevWave wv;
  uint8_t* lit = lit_all + (int64_t)blockIdx.x * zstd::kMaxLit;
  for (int64_t j = blockIdx.x; j < njobs; j += gridDim.x) {
    const PqSnappyJob jb = jobs[j];
    if (jb.codec != PQ_CODEC_ZSTD) continue;
    zstd::Decoder<DevWave> d(wv, sc, raw + jb.src_off, jb.src_len, dec + jb.dst_off, jb.dst_len, lit);
    const int e = d.run();
    if (e && threadIdx.x == 0) atomicCAS(err, 0, e);
    __syncthreads();
  }
}

}  // namespace

int zstd_decompress_host(const uint8_t* src, int64_t slen, uint8_t* dst, int64_t dcap) {
  auto sc = std::make_unique<zstd::Scratch>();
  std::vector<uint8_t> lit(zstd::kMaxLit);
  HostWave wv;
  zstd::Decoder<HostWave> d(wv, *sc, src, slen, dst, dcap, lit.data());
  return d.run();
}

int64_t pq_zstd_slots(int64_t njobs) { return njobs < kZstdMaxSlots ? njobs : kZstdMaxSlots; }

void pq_zstd(const PqSnappyJob* jobs, int64_t njobs, const uint8_t* raw, uint8_t* dec, uint8_t* lit, int64_t slots,
             int* error, hipStream_t stream) {
  if (njobs <= 0 || slots <= 0) return;
  const unsigned grid = (unsigned)(slots < njobs ? slots : njobs);
  hipLaunchKernelGGL(pq_zstd_kernel, dim3(grid), dim3(kWave), 0, stream, jobs, njobs, raw, dec, lit, error);
  check_launch("pq_zstd", stream);
}

}  // namespace kern
}  // namespace igloo
