// HyperLogLog distinct-count sketches for join ordering.
//
// The reference leaves join ordering to DataFusion's statistics-based
// optimizer (reference crates/engine/src/lib.rs:55). Here the executor orders
// joins at run time from the actual inputs, which needs NDV(key) per input:
// an exact hash-table count costs a build + compaction per key, whereas a
// sketch is one streaming read of the key column.
//
// Layout: p = 12 -> m = 4096 one-byte registers. Each block keeps its own
// registers in LDS (32-bit slots for ds_max_u32; 16 KB), then writes them to
// its row of a [blocks x m] workspace; a second kernel max-reduces the rows.
// No global atomics, so the grid can be sized to fill all 256 CUs.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kItemsPerThread = 16;

template <typename K>
__global__ __launch_bounds__(kBlock) void hll_block_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                          int64_t n, uint8_t* __restrict__ block_regs) {
  __shared__ uint32_t regs[kHllRegisters];
  for (int i = threadIdx.x; i < kHllRegisters; i += kBlock) regs[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    if (valid && !valid[i]) continue;
    uint64_t h = mix64((uint64_t)(int64_t)keys[i] * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL);
    uint32_t idx = (uint32_t)(h >> (64 - kHllBits));
    uint64_t w = h << kHllBits;
    uint32_t rank = w == 0 ? (uint32_t)(64 - kHllBits + 1) : (uint32_t)__builtin_clzll(w) + 1;
    atomicMax(&regs[idx], rank);
  }
  __syncthreads();
  uint8_t* out = block_regs + (int64_t)blockIdx.x * kHllRegisters;
  for (int i = threadIdx.x; i < kHllRegisters; i += kBlock) out[i] = (uint8_t)regs[i];
}

__global__ __launch_bounds__(kBlock) void hll_reduce_kernel(const uint8_t* __restrict__ block_regs, int blocks,
                                                           uint8_t* __restrict__ regs) {
  int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= kHllRegisters) return;
  uint8_t m = 0;
  for (int b = 0; b < blocks; ++b) {
    uint8_t v = block_regs[(int64_t)b * kHllRegisters + r];
    m = v > m ? v : m;
  }
  regs[r] = m;
}

}  // namespace

int hll_blocks(int64_t n) {
  return (int)grid_for(n, kBlock * kItemsPerThread, kHllMaxBlocks);
}

void hll_sketch(const void* keys, bool key64, const uint8_t* valid, int64_t n, uint8_t* block_regs, uint8_t* regs,
                hipStream_t stream) {
  int blocks = hll_blocks(n);
  if (key64)
    hll_block_kernel<int64_t><<<blocks, kBlock, 0, stream>>>((const int64_t*)keys, valid, n, block_regs);
  else
    hll_block_kernel<int32_t><<<blocks, kBlock, 0, stream>>>((const int32_t*)keys, valid, n, block_regs);
  check_launch("hll_block", stream);
  hll_reduce_kernel<<<(kHllRegisters + kBlock - 1) / kBlock, kBlock, 0, stream>>>(block_regs, blocks, regs);
  check_launch("hll_reduce", stream);
}

}  // namespace kern
}  // namespace igloo
