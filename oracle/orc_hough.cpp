// ORACLE — TEST INFRASTRUCTURE ONLY (see orc_common.h).
//
// Restatement of the reference `Houghvotinggpu` op: HoughvotinggpuOp<GPU>::Compute
// (lib/hough_voting_gpu_layer/hough_voting_gpu_op.cc:321-429) driving
// HoughVotingLaucher (hough_voting_gpu_op.cu.cc:615-799) once per image.
//
// Canonical order (SURVEY.md finding 5): the reference builds per-class pixel
// lists with atomicAdd (cu.cc:182-184), so with skip_pixels > 1 the set of
// voters is scheduling dependent; multi-instance maxima and RoI rows are also
// appended with atomics (cu.cc:377, :414, :558).  This oracle fixes ONE legal
// execution: pixel lists in ascending raster order, maxima in ascending flat
// (slot, y, x) order, RoIs image-major.
//
// Equivalence transformations (results identical to the reference loops):
//  * the per-cell voter loop of compute_hough_kernel (cu.cc:269-294) is run
//    voter-major: every voter visits only the cells of its +-T box (cells
//    outside the box fail the box test of cu.cc:288 whatever the angle), in
//    ascending voter order, so each cell still accumulates its count and its
//    distance sum in the reference's voter order;
//  * hough_data (cu.cc:296-331) is evaluated lazily, only at the cells the
//    max selection / NMS consumes.
#include "orc_common.h"
#include <vector>
#include <algorithm>
#include <cstring>

namespace {

const int kMaxRoi = 128;  // cu.cc:14

// cu.cc:32-42
inline float angle_distance(int cx, int cy, int x, int y, float u, float v) {
  float dx = (float)(cx - x);
  float dy = (float)(cy - y);
  float n1 = sqrtf(u * u + v * v);
  float n2 = sqrtf(dx * dx + dy * dy);
  float dot = u * dx + v * dy;
  float distance = dot / (n1 * n2);
  return distance;
}

// cu.cc:84-120
inline float project_box(int cls, const float* extents, const float* meta, float distance, float factor) {
  float xHalf = (float)(extents[cls * 3 + 0] * 0.5);
  float yHalf = (float)(extents[cls * 3 + 1] * 0.5);
  float zHalf = (float)(extents[cls * 3 + 2] * 0.5);
  float bb3D[24] = {
       xHalf,  yHalf,  zHalf + distance,
      -xHalf,  yHalf,  zHalf + distance,
       xHalf, -yHalf,  zHalf + distance,
      -xHalf, -yHalf,  zHalf + distance,
       xHalf,  yHalf, -zHalf + distance,
      -xHalf,  yHalf, -zHalf + distance,
       xHalf, -yHalf, -zHalf + distance,
      -xHalf, -yHalf, -zHalf + distance};
  float fx = meta[0], fy = meta[4], px = meta[2], py = meta[5];
  float minX = 1e8f, maxX = -1e8f, minY = 1e8f, maxY = -1e8f;
  for (int i = 0; i < 8; i++) {
    float x = fx * (bb3D[i * 3] / bb3D[i * 3 + 2]) + px;
    float y = fy * (bb3D[i * 3 + 1] / bb3D[i * 3 + 2]) + py;
    minX = fminf(minX, x);
    minY = fminf(minY, y);
    maxX = fmaxf(maxX, x);
    maxY = fmaxf(maxY, y);
  }
  float width = maxX - minX + 1;
  float height = maxY - minY + 1;
  return fmaxf(width, height) * factor;
}

// cu.cc:73-82
inline float iou(const float* a, const float* b) {
  float left = fmaxf(a[0], b[0]), right = fminf(a[2], b[2]);
  float top = fmaxf(a[1], b[1]), bottom = fminf(a[3], b[3]);
  float width = fmaxf(right - left + 1, 0.f), height = fmaxf(bottom - top + 1, 0.f);
  float interS = width * height;
  float Sa = (a[2] - a[0] + 1) * (a[3] - a[1] + 1);
  float Sb = (b[2] - b[0] + 1) * (b[3] - b[1] + 1);
  return interS / (Sa + Sb - interS);
}

// cu.cc:123-172.  Eigen::Quaternionf(w,x,y,z).toRotationMatrix() restated with
// Eigen's formula; the 3x3 * 3x8 lazy product sums a0 + (a1 + a2) (Eigen
// redux_novec_unroller split).
inline float compute_box_overlap(int cls, const float* extents, const float* meta, const float* pose, const float* box) {
  float xHalf = (float)(extents[cls * 3 + 0] * 0.5);
  float yHalf = (float)(extents[cls * 3 + 1] * 0.5);
  float zHalf = (float)(extents[cls * 3 + 2] * 0.5);
  float b[8][3] = {{xHalf, yHalf, zHalf}, {-xHalf, yHalf, zHalf}, {xHalf, -yHalf, zHalf}, {-xHalf, -yHalf, zHalf},
                   {xHalf, yHalf, -zHalf}, {-xHalf, yHalf, -zHalf}, {xHalf, -yHalf, -zHalf}, {-xHalf, -yHalf, -zHalf}};
  float qw = pose[6], qx = pose[7], qy = pose[8], qz = pose[9];
  float tx = 2.f * qx, ty = 2.f * qy, tz = 2.f * qz;
  float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  float R[3][3] = {{1.f - (tyy + tzz), txy - twz, txz + twy},
                   {txy + twz, 1.f - (txx + tzz), tyz - twx},
                   {txz - twy, tyz + twx, 1.f - (txx + tyy)}};
  float fx = meta[0], fy = meta[4], px = meta[2], py = meta[5];
  float x1 = 1e8f, x2 = -1e8f, y1 = 1e8f, y2 = -1e8f;
  for (int i = 0; i < 8; i++) {
    float P[3];
    for (int r = 0; r < 3; r++) P[r] = R[r][0] * b[i][0] + (R[r][1] * b[i][1] + R[r][2] * b[i][2]);
    float X = P[0] + pose[10];
    float Y = P[1] + pose[11];
    float Z = P[2] + pose[12];
    float x = fx * (X / Z) + px;
    float y = fy * (Y / Z) + py;
    x1 = fminf(x1, x);
    y1 = fminf(y1, y);
    x2 = fmaxf(x2, x);
    y2 = fmaxf(y2, y);
  }
  float box_gt[4] = {x1, y1, x2, y2};
  return iou(box, box_gt);
}

struct Voter { int x, y; float u, v, d, T; };

struct ImageCtx {
  int H, W, C;
  const float* vert;
  const float* extents;
  const float* meta;
  float inlier;
};

// Lazily evaluated hough_data at one cell (cu.cc:296-331); count > 0 required.
inline void hough_data_at(const ImageCtx& ic, int cls, const std::vector<Voter>& voters, float count, float dsum,
                          int cx, int cy, float* out3) {
  float distance = dsum / count;  // cu.cc:298
  float bb_width = -1, bb_height = -1;
  for (const Voter& vt : voters) {  // cu.cc:302-325
    if (angle_distance(cx, cy, vt.x, vt.y, vt.u, vt.v) > ic.inlier) {
      float threshold = project_box(cls, ic.extents, ic.meta, distance, 0.6f);
      float dx = fabsf((float)(vt.x - cx));
      float dy = fabsf((float)(vt.y - cy));
      if (dx > bb_width && dx < threshold && dy < threshold) bb_width = dx;
      if (dy > bb_height && dx < threshold && dy < threshold) bb_height = dy;
    }
  }
  out3[0] = distance;
  out3[1] = 2 * bb_height;
  out3[2] = 2 * bb_width;
}

}  // namespace

// Vote accumulation for one class of one image: counts (float, as the
// reference's hough_space) and distance sums in voter order.
// Returns the number of voters.
static int vote_class(const ImageCtx& ic, const std::vector<int>& plist, int cls, int skip,
                      std::vector<Voter>& voters, float* counts, float* dsum) {
  const int H = ic.H, W = ic.W, C = ic.C;
  voters.clear();
  for (size_t i = 0; i < plist.size(); i += skip) {  // cu.cc:269
    int location = plist[i];
    Voter vt;
    vt.x = location % W;
    vt.y = location / W;
    size_t off = (size_t)3 * cls + (size_t)3 * C * ((size_t)vt.y * W + vt.x);  // cu.cc:277
    vt.u = ic.vert[off];
    vt.v = ic.vert[off + 1];
    vt.d = orc::exp_depth(ic.vert[off + 2]);  // cu.cc:280
    vt.T = project_box(cls, ic.extents, ic.meta, vt.d, 0.6f);  // cu.cc:285 (pure in (cls, d))
    voters.push_back(vt);
  }
  std::fill(counts, counts + (size_t)H * W, 0.f);
  std::fill(dsum, dsum + (size_t)H * W, 0.f);
  for (const Voter& vt : voters) {
    float T = vt.T;
    if (!(T > 0.f)) continue;  // |dx| < T is false for every cell
    double Tb = std::min((double)T, 1e7);
    int r = (int)std::ceil(Tb);
    int x0 = std::max(0, vt.x - r), x1 = std::min(W - 1, vt.x + r);
    int y0 = std::max(0, vt.y - r), y1 = std::min(H - 1, vt.y + r);
    for (int cy = y0; cy <= y1; cy++)
      for (int cx = x0; cx <= x1; cx++) {
        if (angle_distance(cx, cy, vt.x, vt.y, vt.u, vt.v) > ic.inlier) {  // cu.cc:283
          float dx = fabsf((float)(vt.x - cx));
          float dy = fabsf((float)(vt.y - cy));
          if (dx < T && dy < T) {  // cu.cc:288-292
            counts[(size_t)cy * W + cx] += 1.f;
            dsum[(size_t)cy * W + cx] += vt.d;
          }
        }
      }
  }
  return (int)voters.size();
}

// One image of compute_rois_kernel (cu.cc:386-576) for one kept max.
static void emit_rois(const ImageCtx& ic, int cls, int x, int y, float score, const float* hdata,
                      int is_train, int batch_index, const float* gt, int num_gt,
                      float* top_box, float* top_pose, float* top_target, float* top_weight, int* top_domain,
                      int& num_rois) {
  const int C = ic.C;
  float scale = 0.05f;
  const float* meta = ic.meta;
  float fx = meta[0], fy = meta[4], px = meta[2], py = meta[5];
  float rx = ((float)x - px) / fx;
  float ry = ((float)y - py) / fy;
  float bb_distance = hdata[0], bb_height = hdata[1], bb_width = hdata[2];
  if (is_train) {
    int roi_index = num_rois;
    num_rois += 9;
    float* b = top_box + (size_t)roi_index * 7;
    b[0] = (float)batch_index;
    b[1] = (float)cls;
    b[2] = (float)((double)x - (double)bb_width * (0.5 + (double)scale));
    b[3] = (float)((double)y - (double)bb_height * (0.5 + (double)scale));
    b[4] = (float)((double)x + (double)bb_width * (0.5 + (double)scale));
    b[5] = (float)((double)y + (double)bb_height * (0.5 + (double)scale));
    b[6] = score;
    for (int i = 0; i < 9; i++) {
      float* p = top_pose + (size_t)(roi_index + i) * 7;
      p[0] = 1; p[1] = 0; p[2] = 0; p[3] = 0;
      p[4] = rx * bb_distance;
      p[5] = ry * bb_distance;
      p[6] = bb_distance;
      top_domain[roi_index + i] = (num_gt == 0) ? 1 : 0;
    }
    for (int i = 0; i < num_gt; i++) {  // cu.cc:440-466
      int gt_batch = (int)gt[i * 13 + 0];
      int gt_id = (int)gt[i * 13 + 1];
      if (cls == gt_id && batch_index == gt_batch) {
        float overlap = compute_box_overlap(cls, ic.extents, meta, gt + (size_t)i * 13, b + 2);
        if ((double)overlap > 0.2) {
          for (int j = 0; j < 9; j++) {
            float* t = top_target + (size_t)(roi_index + j) * 4 * C + 4 * cls;
            float* w = top_weight + (size_t)(roi_index + j) * 4 * C + 4 * cls;
            for (int q = 0; q < 4; q++) { t[q] = gt[i * 13 + 6 + q]; w[q] = 1; }
          }
          break;
        }
      }
    }
    // jittered boxes (cu.cc:468-554): (dx, dy) multipliers in reference order
    const int jit[8][2] = {{-1, -1}, {1, -1}, {-1, 1}, {1, 1}, {0, -1}, {-1, 0}, {0, 1}, {1, 0}};
    float x1 = b[2], y1 = b[3], x2 = b[4], y2 = b[5];
    float ww = x2 - x1, hh = y2 - y1;
    for (int k = 0; k < 8; k++) {
      float* bj = top_box + (size_t)(roi_index + 1 + k) * 7;
      bj[0] = (float)batch_index;
      bj[1] = (float)cls;
      double sx = jit[k][0] == 0 ? 0.0 : (jit[k][0] < 0 ? -0.05 * (double)ww : 0.05 * (double)ww);
      double sy = jit[k][1] == 0 ? 0.0 : (jit[k][1] < 0 ? -0.05 * (double)hh : 0.05 * (double)hh);
      bj[2] = jit[k][0] == 0 ? x1 : (float)((double)x1 + sx);
      bj[3] = jit[k][1] == 0 ? y1 : (float)((double)y1 + sy);
      bj[4] = bj[2] + ww;
      bj[5] = bj[3] + hh;
      bj[6] = score;
    }
  } else {
    int roi_index = num_rois;
    num_rois += 1;
    float* b = top_box + (size_t)roi_index * 7;
    b[0] = (float)batch_index;
    b[1] = (float)cls;
    b[2] = (float)((double)x - (double)bb_width * (0.5 + (double)scale));
    b[3] = (float)((double)y - (double)bb_height * (0.5 + (double)scale));
    b[4] = (float)((double)x + (double)bb_width * (0.5 + (double)scale));
    b[5] = (float)((double)y + (double)bb_height * (0.5 + (double)scale));
    b[6] = score;
    float* p = top_pose + (size_t)roi_index * 7;
    p[0] = 1; p[1] = 0; p[2] = 0; p[3] = 0;
    p[4] = rx * bb_distance;
    p[5] = ry * bb_distance;
    p[6] = bb_distance;
  }
}

// Full op over a batch.  Outputs are capacity-sized (cap rows, zero-filled by
// the caller as reset_outputs does, cu.cc:579-588).  batch_base rebases the
// box batch column (sharded runs); global_batch sets index_size =
// MAX_ROI / global_batch (cu.cc:734).  Returns the number of RoI rows
// (0 means the op emits one all-zero dummy row, hough_voting_gpu_op.cc:382-383).
ORC_API int orc_hough_voting(const int* label, const float* vertex, const float* extents, const float* meta,
                             int num_meta, const float* gt, int num_gt, int B, int H, int W, int C,
                             int batch_base, int global_batch, int is_train, float inlier_thr, int label_thr,
                             float vote_thr, float per_thr, int skip, float* top_box, float* top_pose,
                             float* top_target, float* top_weight, int* top_domain, int cap) {
  int num_rois = 0;
  const int index_size = kMaxRoi / global_batch;
  std::vector<float> counts((size_t)H * W), dsum((size_t)H * W);
  std::vector<Voter> voters;
  for (int n = 0; n < B; n++) {
    const int* lab = label + (size_t)n * H * W;
    ImageCtx ic{H, W, C, vertex + (size_t)n * H * W * 3 * C, extents, meta + (size_t)n * num_meta, inlier_thr};
    std::vector<std::vector<int>> plist(C);
    for (int p = 0; p < H * W; p++) {  // cu.cc:174-187 in canonical order
      int cls = lab[p];
      if (cls > 0 && cls < C) plist[cls].push_back(p);
    }
    std::vector<int> class_indexes;  // cu.cc:653-664
    for (int c = 1; c < C; c++)
      if ((int)plist[c].size() > label_thr) class_indexes.push_back(c);
    int count = (int)class_indexes.size();
    if (count == 0) continue;  // cu.cc:666-671
    const int batch_index = batch_base + n;

    if (vote_thr > 0) {
      // multi-instance path: compute_max_indexes_kernel (cu.cc:335-383)
      std::vector<std::vector<float>> cmaps(count), dmaps(count);
      std::vector<std::vector<Voter>> vlist(count);
      for (int ind = 0; ind < count; ind++) {
        cmaps[ind].resize((size_t)H * W);
        dmaps[ind].resize((size_t)H * W);
        vote_class(ic, plist[class_indexes[ind]], class_indexes[ind], skip, vlist[ind], cmaps[ind].data(), dmaps[ind].data());
      }
      std::vector<long> kept;
      std::vector<float> kept_data;
      for (int ind = 0; ind < count && (int)kept.size() < index_size; ind++) {
        const float* hs = cmaps[ind].data();
        for (int cy = 0; cy < H && (int)kept.size() < index_size; cy++)
          for (int cx = 0; cx < W && (int)kept.size() < index_size; cx++) {
            float c0 = hs[(size_t)cy * W + cx];
            if (!(c0 > vote_thr)) continue;
            float hd[3] = {0.f, 0.f, 0.f};
            hough_data_at(ic, class_indexes[ind], vlist[ind], c0, dmaps[ind][(size_t)cy * W + cx], cx, cy, hd);
            float bb_height = hd[1], bb_width = hd[2];
            if (!(bb_height > 0 && bb_width > 0)) continue;
            int flag = 0;
            for (int x = cx - 3; x <= cx + 3 && !flag; x++)
              for (int y = cy - 3; y <= cy + 3; y++)
                if (x >= 0 && x < W && y >= 0 && y < H && hs[(size_t)y * W + x] > c0) { flag = 1; break; }
            if (c0 / (bb_height * bb_width) < per_thr) flag = 1;
            if (flag == 0) {
              kept.push_back((long)ind * H * W + (long)cy * W + cx);
              kept_data.insert(kept_data.end(), hd, hd + 3);
            }
          }
      }
      for (size_t k = 0; k < kept.size(); k++) {
        int ind = (int)(kept[k] / ((long)H * W));
        int cell = (int)(kept[k] % ((long)H * W));
        if (num_rois + (is_train ? 9 : 1) > cap) return -1;
        emit_rois(ic, class_indexes[ind], cell % W, cell / W, cmaps[ind][cell], &kept_data[3 * k], is_train,
                  batch_index, gt, num_gt, top_box, top_pose, top_target, top_weight, top_domain, num_rois);
      }
    } else {
      // default path: thrust::max_element per class (cu.cc:751-764); the first
      // index_size classes survive the num_max cap (cu.cc:775-776)
      int num_max = std::min(count, index_size);
      for (int ind = 0; ind < num_max; ind++) {
        int cls = class_indexes[ind];
        vote_class(ic, plist[cls], cls, skip, voters, counts.data(), dsum.data());
        size_t best = 0;
        for (size_t p = 1; p < (size_t)H * W; p++)
          if (counts[p] > counts[best]) best = p;  // first maximum
        float hd[3] = {0.f, 0.f, 0.f};  // memset-zero hough_data for count == 0
        int cx = (int)(best % W), cy = (int)(best / W);
        if (counts[best] > 0) hough_data_at(ic, cls, voters, counts[best], dsum[best], cx, cy, hd);
        if (num_rois + (is_train ? 9 : 1) > cap) return -1;
        emit_rois(ic, cls, cx, cy, counts[best], hd, is_train, batch_index, gt, num_gt, top_box, top_pose,
                  top_target, top_weight, top_domain, num_rois);
      }
    }
  }
  return num_rois;
}

// Debug/parity helper: the vote counts map and hough_data at one cell for one
// (image, class), exactly as the reference's hough_space slice.
ORC_API int orc_hough_class_counts(const int* label, const float* vertex, const float* extents, const float* meta,
                                   int H, int W, int C, int cls, float inlier_thr, int skip, float* counts_out,
                                   float* dsum_out) {
  ImageCtx ic{H, W, C, vertex, extents, meta, inlier_thr};
  std::vector<int> plist;
  for (int p = 0; p < H * W; p++)
    if (label[p] == cls) plist.push_back(p);
  std::vector<Voter> voters;
  return vote_class(ic, plist, cls, skip, voters, counts_out, dsum_out);
}

ORC_API void orc_hough_data_at(const int* label, const float* vertex, const float* extents, const float* meta, int H,
                               int W, int C, int cls, float inlier_thr, int skip, int cx, int cy, float count,
                               float dsum, float* out3) {
  ImageCtx ic{H, W, C, vertex, extents, meta, inlier_thr};
  std::vector<int> plist;
  for (int p = 0; p < H * W; p++)
    if (label[p] == cls) plist.push_back(p);
  std::vector<Voter> voters;
  for (size_t i = 0; i < plist.size(); i += skip) {
    int location = plist[i];
    Voter vt;
    vt.x = location % W;
    vt.y = location / W;
    size_t off = (size_t)3 * cls + (size_t)3 * C * ((size_t)vt.y * W + vt.x);
    vt.u = vertex[off];
    vt.v = vertex[off + 1];
    vt.d = orc::exp_depth(vertex[off + 2]);
    vt.T = 0.f;
    voters.push_back(vt);
  }
  out3[0] = out3[1] = out3[2] = 0.f;
  if (count > 0) hough_data_at(ic, cls, voters, count, dsum, cx, cy, out3);
}
