// Shared device helpers for the PoseCNN MI355X kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include "../../include/posecnn_hip.h"

// Every float operation of the reference-parity arithmetic rounds separately:
// the build passes -ffp-contract=off, and this pragma pins it per TU.
#pragma clang fp contract(off)

#define PCNN_WAVE 64

#define PCNN_CHECK_LAUNCH()                                   \
  do {                                                        \
    hipError_t e_ = hipGetLastError();                        \
    if (e_ != hipSuccess) return PCNN_EHIP;                   \
  } while (0)

#define PCNN_REQUIRE(cond)               \
  do {                                   \
    if (!(cond)) return PCNN_EINVAL;     \
  } while (0)

namespace pcnn {

// per-device once-only host state (kernel attributes are set per device)
constexpr int kMaxDevices = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  int l = lane_id();
  return l == 0 ? 0ull : ((~0ull) >> (64 - l));
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Completion event of the next op (pcnn_set_completion_event): the op's LAST
// kernel launch records it through the kernel's own completion signal
// (hipExtLaunchKernel's stop event), so a stream forked off at that point
// waits on it without an event-record marker packet on the launching stream.
// Thread-local, consumed by the launch that takes it.
extern thread_local hipEvent_t t_done_event;
inline hipEvent_t take_done_event() {
  hipEvent_t e = t_done_event;
  t_done_event = nullptr;
  return e;
}

// The last kernel of an op: records the pending completion event, if any.
template <typename... KArgs, typename... Args>
inline void launch_last(void (*k)(KArgs...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t st, Args... args) {
  hipExtLaunchKernelGGL(k, grid, block, shmem, st, nullptr, take_done_event(), 0, args...);
}

// Bump allocator over a caller-provided workspace (no allocation on the hot path).
struct Carve {
  char* base;
  size_t off;
  __host__ explicit Carve(void* p) : base((char*)p), off(0) {}
  template <typename T>
  __host__ T* take(size_t n) {
    off = align_up(off, 256);
    T* p = (T*)(base ? base + off : nullptr);
    off += n * sizeof(T);
    return p;
  }
};

}  // namespace pcnn
