// Philox4x32-10 (Salmon et al., SC'11; Random123 constants) and TF's
// Uint32ToFloat keep test of tf.nn.dropout, shared by the keep-mask kernel
// (dropout.hip) and the GEMM reduce epilogue that draws the masks in place
// (pose_head.hip k_gemm_reduce, drop_gen).  Counter of element quad e of a
// dense (rows, cols) mask: (e lo, e hi, stream id, step); key = the seed.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace pcnn_philox {

struct U4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)a * b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__host__ __device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t h0, l0, h1, l1;
    mulhilo(M0, c.x, h0, l0);
    mulhilo(M1, c.z, h1, l1);
    c = U4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// TF's Uint32ToFloat (random_distributions.h): 23 random mantissa bits -> [1, 2) - 1
__device__ __forceinline__ float u01(uint32_t x) { return __uint_as_float((x & 0x7fffffu) | 0x3f800000u) - 1.0f; }

__device__ __forceinline__ uint32_t keep_bit(uint32_t x, float keep) {
  return floorf(keep + u01(x)) >= 1.0f ? 1u : 0u;
}

// the four keep bytes of element quad e, packed little-endian (byte j = element 4 e + j)
__device__ __forceinline__ uint32_t keep_quad(uint64_t e, uint32_t k0, uint32_t k1, uint32_t sid, uint32_t step,
                                              float keep) {
  const U4 o = philox4x32_10(U4{(uint32_t)e, (uint32_t)(e >> 32), sid, step}, k0, k1);
  return keep_bit(o.x, keep) | keep_bit(o.y, keep) << 8 | keep_bit(o.z, keep) << 16 | keep_bit(o.w, keep) << 24;
}

}  // namespace pcnn_philox
