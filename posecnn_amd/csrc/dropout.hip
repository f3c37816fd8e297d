// Dropout keep masks of the pose head (drop6 / drop7, vgg16_convs.py:189,191;
// Network.dropout -> tf.nn.dropout, network.py:574-577).  tf.nn.dropout draws
// U ~ [0, 1) per element, keeps floor(keep_prob + U) (the "binary tensor")
// and returns (x / keep_prob) * binary; the GEMM epilogues of fc6 / fc7 apply
// that product (gemm_common.h drop_epi), so this kernel only writes the
// binary tensor, one byte per element.
//
// The uniform draw is Philox4x32-10 (Salmon et al., SC'11 -- the generator TF
// uses for random_uniform on the GPU) with TF's uint32 -> float construction.
// Key = the caller's 64-bit seed; counter = (element quad index: 2 words,
// stream id, device-side step counter).  Each lane turns one Philox block into
// the 4 bytes of one element quad (one 32-bit store).  The step counter lives
// in device memory so that a captured HIP graph draws fresh masks on every
// replay (the caller bumps it once per step).
#include "pcnn_common.h"
#include "pcnn_philox.h"

namespace {

using namespace pcnn_philox;

__global__ void __launch_bounds__(256) k_dropout_mask(uint8_t* __restrict__ mask, int rows, int cols, int ld,
                                                      const int32_t* __restrict__ rows_dev, uint32_t k0, uint32_t k1,
                                                      const int64_t* __restrict__ step_dev, uint32_t stream_id,
                                                      float keep) {
  int R = rows;
  if (rows_dev) {
    const int v = *rows_dev;
    R = v < rows ? (v < 0 ? 0 : v) : rows;
  }
  const uint64_t step = step_dev ? (uint64_t)*step_dev : 0;
  const int q4 = cols >> 2;
  const int quads = R * q4;  // < 2^31 (checked by the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < quads; i += gridDim.x * blockDim.x) {
    const int r = i / q4, c = (i - r * q4) * 4;
    const uint64_t e = (uint64_t)i;  // element quad of a dense (rows, cols) mask: r * q4 + c / 4
    *(uint32_t*)(mask + (size_t)r * ld + c) = keep_quad(e, k0, k1, stream_id, (uint32_t)step, keep);
  }
}

__global__ void k_philox_check(const uint32_t* __restrict__ ctr, const uint32_t* __restrict__ key, int n,
                               uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const U4 o = philox4x32_10(U4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]}, key[2 * i],
                             key[2 * i + 1]);
  out[4 * i] = o.x;
  out[4 * i + 1] = o.y;
  out[4 * i + 2] = o.z;
  out[4 * i + 3] = o.w;
}

}  // namespace

extern "C" int pcnn_dropout_mask(uint8_t* mask, int rows, int cols, int ld, const int32_t* rows_dev, uint64_t seed,
                                 const int64_t* step_dev, int stream_id, float keep_prob, void* stream) {
  PCNN_REQUIRE(mask && rows >= 0 && cols > 0 && cols % 4 == 0 && ld >= cols && ld % 4 == 0 && ((uintptr_t)mask & 3) == 0);
  PCNN_REQUIRE(keep_prob > 0.f && keep_prob <= 1.f && stream_id >= 0 && (long)rows * (cols / 4) < (1l << 31));
  if (rows == 0) return PCNN_OK;
  const long quads = (long)rows * (cols / 4);
  long grid = (quads + 255) / 256;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(k_dropout_mask, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, mask, rows, cols, ld,
                     rows_dev, (uint32_t)seed, (uint32_t)(seed >> 32), step_dev, (uint32_t)stream_id, keep_prob);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_philox_check(const uint32_t* ctr, const uint32_t* key, int n, uint32_t* out, void* stream) {
  PCNN_REQUIRE(ctr && key && out && n >= 0);
  if (n == 0) return PCNN_OK;
  hipLaunchKernelGGL(k_philox_check, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, ctr, key, n, out);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
