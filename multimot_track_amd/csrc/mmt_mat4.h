// multimot_track_amd/csrc/mmt_mat4.h -- the float cv::Mat helpers of the tracker's pose
// bookkeeping, shared by host and device so the device-side motion-model matrix equals the host's
// bit for bit (double accumulation, float result; contraction is off in both compilations).
#pragma once
#include <hip/hip_runtime.h>

namespace mmt {

// cv::gemm, CV_32F: C = A B (4x4)
__host__ __device__ inline void mat4_mul(const float* A, const float* B, float* C) {
  float R[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      double s = 0;
      for (int k = 0; k < 4; k++) s += (double)A[4 * r + k] * (double)B[4 * k + c];
      R[4 * r + c] = (float)s;
    }
  for (int i = 0; i < 16; i++) C[i] = R[i];
}

// Tracking::InvMatrix: [R^T, -R^T t]
__host__ __device__ inline void inv_mat(const float* T, float* Ti) {
  float R[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) R[4 * r + c] = T[4 * c + r];
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (double)T[4 * k + r] * (double)T[4 * k + 3];
    R[4 * r + 3] = (float)(-s);
  }
  for (int i = 0; i < 16; i++) Ti[i] = R[i];
}

__host__ __device__ inline void mat4_eye(float* T) {
  for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.f : 0.f;
}

}  // namespace mmt
