// Depth backprojection for PoseCNN on MI355X (gfx950).
//
// Replaces BackprojectForwardLaucher / BackprojectBackwardLaucher
// (lib/backprojecting_layer/backprojecting_op_gpu.cu.cc:16-242).
//
// Forward: one thread per (voxel, lane-channel) with the channel innermost, so
// the voxel geometry and the (2k+1)^2 depth tests are wave-uniform and every
// feature read / output write is a coalesced channel sweep.  Label channels are
// handled by lanes c < NC of the same voxel (the reference loops them on the
// c == 0 thread only, cu.cc:62-66, :88-93, which also races with the other
// channel threads' writes of the same voxel); per-channel summation order over
// the neighbourhood (x outer, y inner) is the reference's.
// The output is write-bound: B*G^3*(2Ch+NC)*4 bytes.
#include "pcnn_common.h"
#include <math.h>

namespace {

__global__ void __launch_bounds__(256) k_bp_fwd(const float* __restrict__ data, const float* __restrict__ label,
                                                 const float* __restrict__ depth, const float* __restrict__ meta,
                                                 int num_meta, const float* __restrict__ label_3d, int B, int H, int W,
                                                 int Ch, int NC, int G, int ks, float threshold, int CL,
                                                 float* __restrict__ top_data, float* __restrict__ top_label,
                                                 float* __restrict__ top_flag) {
  const long total = (long)B * G * G * G * CL;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % CL);
    const long vox = idx / CL;
    const int w = (int)(vox % G), h = (int)((vox / G) % G), d = (int)((vox / ((long)G * G)) % G);
    const int n = (int)(vox / ((long)G * G * G));
    const float* m = meta + (size_t)n * num_meta;
    // voxel centre -> live frame -> image (cu.cc:43-60)
    const float X = (float)d * m[42] + m[45];
    const float Y = (float)h * m[43] + m[46];
    const float Z = (float)w * m[44] + m[47];
    const float X1 = m[18] * X + m[19] * Y + m[20] * Z + m[21];
    const float Y1 = m[22] * X + m[23] * Y + m[24] * Z + m[25];
    const float Z1 = m[26] * X + m[27] * Y + m[28] * Z + m[29];
    const float x1 = m[0] * X1 + m[1] * Y1 + m[2] * Z1;
    const float x2 = m[3] * X1 + m[4] * Y1 + m[5] * Z1;
    const float x3 = m[6] * X1 + m[7] * Y1 + m[8] * Z1;
    const int px = (int)roundf(x1 / x3);
    const int py = (int)roundf(x2 / x3);
    const bool do_data = c < Ch, do_label = c < NC;
    float sd = 0.f, sl = 0.f;
    int count = 0;
    for (long x = (long)px - ks; x <= (long)px + ks; x++)
      for (long y = (long)py - ks; y <= (long)py + ks; y++) {
        if (x >= 0 && x < W && y >= 0 && y < H) {
          const size_t ip = ((size_t)n * H + y) * W + x;
          const float dep = depth[ip];
          if (fabsf(dep - Z1) < threshold) {  // cu.cc:79
            count++;
            if (do_data) sd += data[ip * Ch + c];
            if (do_label) sl += label[ip * NC + c];
          }
        }
      }
    if (count == 0) {
      if (do_data) {
        top_data[vox * Ch + c] = 0.f;
        top_flag[vox * Ch + c] = 0.f;
      }
      if (do_label) top_label[vox * NC + c] = label_3d[vox * NC + c];
    } else {
      if (do_data) {
        top_data[vox * Ch + c] = sd / (float)count;
        top_flag[vox * Ch + c] = 1.f;
      }
      if (do_label) top_label[vox * NC + c] = sl / (float)count;
    }
  }
}

__global__ void __launch_bounds__(256) k_bp_bwd(const float* __restrict__ top_diff, const float* __restrict__ depth,
                                                 const float* __restrict__ meta, int num_meta, int B, int H, int W,
                                                 int Ch, int G, float* __restrict__ bottom_diff) {
  const long total = (long)B * H * W * Ch;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % Ch);
    const long pix = idx / Ch;
    const int w = (int)(pix % W), h = (int)((pix / W) % H), n = (int)(pix / ((long)W * H));
    const float* m = meta + (size_t)n * num_meta;
    const float dep = depth[pix];
    // pixel -> camera ray (Kinv) -> live2world -> voxel (cu.cc:188-210)
    const float RX = m[9] * (float)w + m[10] * (float)h + m[11];
    const float RY = m[12] * (float)w + m[13] * (float)h + m[14];
    const float RZ = m[15] * (float)w + m[16] * (float)h + m[17];
    const float X = dep * RX, Y = dep * RY, Z = dep * RZ;
    const float X1 = m[30] * X + m[31] * Y + m[32] * Z + m[33];
    const float Y1 = m[34] * X + m[35] * Y + m[36] * Z + m[37];
    const float Z1 = m[38] * X + m[39] * Y + m[40] * Z + m[41];
    const int vd = (int)roundf((X1 - m[45]) / m[42]);
    const int vh = (int)roundf((Y1 - m[46]) / m[43]);
    const int vw = (int)roundf((Z1 - m[47]) / m[44]);
    float g = 0.f;
    if (vd >= 0 && vd < G && vh >= 0 && vh < G && vw >= 0 && vw < G)
      g = top_diff[((((size_t)n * G + vd) * G + vh) * G + vw) * Ch + c];
    bottom_diff[idx] = g;
  }
}

}  // namespace

extern "C" int pcnn_backproject_fwd(const float* data, const float* label, const float* depth, const float* meta,
                                    int num_meta, const float* label_3d, int B, int H, int W, int Ch, int NC,
                                    int grid_size, int kernel_size, float threshold, float* top_data,
                                    float* top_label, float* top_flag, void* stream) {
  PCNN_REQUIRE(data && label && depth && meta && label_3d && top_data && top_label && top_flag);
  PCNN_REQUIRE(B > 0 && H > 0 && W > 0 && Ch > 0 && NC > 0 && grid_size > 0 && kernel_size >= 0 && num_meta >= 48);
  const int CL = Ch > NC ? Ch : NC;
  const long total = (long)B * grid_size * grid_size * grid_size * CL;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(k_bp_fwd, dim3(blocks), dim3(256), 0, (hipStream_t)stream, data, label, depth, meta, num_meta,
                     label_3d, B, H, W, Ch, NC, grid_size, kernel_size, threshold, CL, top_data, top_label, top_flag);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}

extern "C" int pcnn_backproject_bwd(const float* top_diff, const float* depth, const float* meta, int num_meta, int B,
                                    int H, int W, int Ch, int grid_size, float* bottom_diff, void* stream) {
  PCNN_REQUIRE(top_diff && depth && meta && bottom_diff && B > 0 && H > 0 && W > 0 && Ch > 0 && grid_size > 0);
  PCNN_REQUIRE(num_meta >= 48);
  const long total = (long)B * H * W * Ch;
  const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(k_bp_bwd, dim3(blocks), dim3(256), 0, (hipStream_t)stream, top_diff, depth, meta, num_meta, B,
                     H, W, Ch, grid_size, bottom_diff);
  PCNN_CHECK_LAUNCH();
  return PCNN_OK;
}
