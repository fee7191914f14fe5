// nc_frustum.hip -- frustum feature selection (ABI v4, nc_frustum_mask; SURVEY.md §8f
// row 3): Mapper.get_mask_from_c2w (src/Mapper.py:100-187) for one feature grid, one
// thread per voxel in the grid's [z][y][x] order (coalesced mask writes).
//
//   k_frustum_maxdepth  pass 1: every voxel's remapped depth, max over the grid
//                       (np.max(depths), Mapper.py:168) by wave reduction + one
//                       atomicMax per wave on the (non-negative) float bits
//   k_frustum_mask      pass 2: the same depth, zero -> max, and the mask
//
// cv2.remap(depth, u, v, INTER_LINEAR) is restated from OpenCV 4.5.5 (the version the
// reference pins, environment.yaml:159): coordinates to 5-bit fixed point by
// round-half-even (cvRound), integer cell = X >> 5 saturated to short, sub-pixel
// weights from the exact float table ((1-fy)(1-fx), (1-fy)fx, fy(1-fx), fy fx), the
// four taps summed left to right in float32, out-of-image taps = 0 (BORDER_CONSTANT).
// Compiled with -ffp-contract=off (no FMA contraction, like the baseline x86 build).
#include <math.h>

#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

struct FrustumPt {
  float u, v;     // pixel coordinates (float32, as uv.astype(np.float32))
  double negz;    // -(uv.z + 1e-5)
  bool near_cam;  // |p - c2w[:3,3]|^2 < 0.25
};

__device__ __forceinline__ FrustumPt frustum_project(const nc_frustum_args& a, int64_t x, int64_t y, int64_t z) {
  const float P[3] = {a.xs[x], a.ys[y], a.zs[z]};
  float cam[3];
#pragma unroll
  for (int r = 0; r < 3; ++r)  // w2c @ [p, 1] in float32, left to right
    cam[r] = ((a.w2c[4 * r] * P[0] + a.w2c[4 * r + 1] * P[1]) + a.w2c[4 * r + 2] * P[2]) + a.w2c[4 * r + 3] * 1.0f;
  cam[0] = -cam[0];
  const double c0 = cam[0], c1 = cam[1], c2 = cam[2];
  const double u = (a.fx * c0 + 0.0 * c1) + a.cx * c2;  // K @ cam in float64
  const double v = (0.0 * c0 + a.fy * c1) + a.cy * c2;
  const double w = (0.0 * c0 + 0.0 * c1) + 1.0 * c2;
  const double zz = w + 1e-5;
  FrustumPt o;
  o.u = (float)(u / zz);
  o.v = (float)(v / zz);
  o.negz = -zz;
  const float dx = P[0] - a.cam_o[0], dy = P[1] - a.cam_o[1], dz = P[2] - a.cam_o[2];
  o.near_cam = ((dx * dx + dy * dy) + dz * dz) < 0.25f;
  return o;
}

// saturate_cast<int>(float) = cvRound: round half to even; out of range / NaN -> INT_MIN
__device__ __forceinline__ int cv_round(float f) {
  if (!(fabsf(f) < 2147483520.0f)) return (int)0x80000000;
  return (int)__builtin_rintf(f);
}
__device__ __forceinline__ int sat_short(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

__device__ __forceinline__ float cv_remap_linear(const nc_frustum_args& a, float u, float v) {
  const int X = cv_round(u * 32.0f), Y = cv_round(v * 32.0f);
  const int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
  const int fxi = X & 31, fyi = Y & 31;
  if (sx >= a.W || sx + 1 < 0 || sy >= a.H || sy + 1 < 0) return 0.0f;
  const float tx1 = (float)fxi * (1.0f / 32.0f), ty1 = (float)fyi * (1.0f / 32.0f);
  const float tx0 = 1.0f - tx1, ty0 = 1.0f - ty1;
  const float w0 = ty0 * tx0, w1 = ty0 * tx1, w2 = ty1 * tx0, w3 = ty1 * tx1;
  auto tap = [&](int xx, int yy) -> float {
    return (xx >= 0 && xx < a.W && yy >= 0 && yy < a.H)
               ? a.depth[(int64_t)yy * a.depth_stride[0] + (int64_t)xx * a.depth_stride[1]]
               : 0.0f;
  };
  const float v0 = tap(sx, sy), v1 = tap(sx + 1, sy), v2 = tap(sx, sy + 1), v3 = tap(sx + 1, sy + 1);
  return ((v0 * w0 + v1 * w1) + v2 * w2) + v3 * w3;
}

__global__ void __launch_bounds__(256) k_frustum_maxdepth(const nc_frustum_args a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = a.nx * a.ny * a.nz;
  float d = 0.f;
  if (t < n) {
    const int64_t x = t % a.nx, y = (t / a.nx) % a.ny, z = t / (a.nx * a.ny);
    const FrustumPt p = frustum_project(a, x, y, z);
    d = cv_remap_linear(a, p.u, p.v);
  }
  for (int o = 32; o > 0; o >>= 1) d = fmaxf(d, __shfl_xor(d, o));
  if ((threadIdx.x & 63) == 0 && d > 0.f) atomicMax(a.scratch, __float_as_uint(d));
}

__global__ void __launch_bounds__(256) k_frustum_mask(const nc_frustum_args a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = a.nx * a.ny * a.nz;
  if (t >= n) return;
  const int64_t x = t % a.nx, y = (t / a.nx) % a.ny, z = t / (a.nx * a.ny);
  const FrustumPt p = frustum_project(a, x, y, z);
  float d = cv_remap_linear(a, p.u, p.v);
  if (d == 0.0f) d = __uint_as_float(*a.scratch);
  const bool in_img = (p.u < (float)a.W) && (p.u > 0.0f) && (p.v < (float)a.H) && (p.v > 0.0f);
  const bool depth_ok = (0.0 <= p.negz) && (p.negz <= (double)(d + 0.5f));
  a.mask[t] = ((in_img && depth_ok) || p.near_cam) ? 1 : 0;
}

int launch_frustum_mask(const nc_frustum_args& a, hipStream_t s) {
  const int64_t n = a.nx * a.ny * a.nz;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (hipError_t e = hipMemsetAsync(a.scratch, 0, sizeof(uint32_t), s)) return (int)e;
  hipLaunchKernelGGL(k_frustum_maxdepth, grid, dim3(256), 0, s, a);
  if (hipError_t e = hipGetLastError()) return (int)e;
  hipLaunchKernelGGL(k_frustum_mask, grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Masked grid rows (nc_grid_rows): the Mapper's val[mask] / val[mask] = val_grad /
// grad[mask] (Mapper.py:393-404, :491-500, :633-642) as copies between the grid's voxel
// rows and the packed [C][n] tensor.  Channels-last grids (channel stride 1, C = 32): a
// workgroup moves 64 rows; a row is 8 float4 loads (one 128-B line), the [C][64] side is
// 64-float runs per channel; the transpose goes through LDS (row pitch 33: conflict-free).
// Other strides: one thread per (channel, row), plain strided copies.
// ---------------------------------------------------------------------------
constexpr int GR_ROWS = 64;

__global__ void __launch_bounds__(256) k_grid_rows_cl(const nc_grid_rows_args a) {
  __shared__ float tile[GR_ROWS][33];
  const int64_t r0 = (int64_t)blockIdx.x * GR_ROWS;
  const int t = threadIdx.x;
  const int64_t n = a.n_rows;
  if (a.op == NC_ROWS_GATHER) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // 64 rows x 8 float4
      const int q = t + 256 * k, r = q >> 3, c4 = (q & 7) * 4;
      if (r0 + r < n) {
        const int64_t v = a.rows[r0 + r];
        const float4 x = *reinterpret_cast<const float4*>(a.grid + v * a.stride[3] + c4);
        tile[r][c4] = x.x; tile[r][c4 + 1] = x.y; tile[r][c4 + 2] = x.z; tile[r][c4 + 3] = x.w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // 32 channels x 64 rows, lane = row
      const int c = (t >> 6) + 4 * k, r = t & 63;
      if (r0 + r < n) a.packed[(int64_t)c * n + r0 + r] = tile[r][c];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = (t >> 6) + 4 * k, r = t & 63;
      if (r0 + r < n) tile[r][c] = a.op == NC_ROWS_ZERO ? 0.f : a.packed[(int64_t)c * n + r0 + r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = t + 256 * k, r = q >> 3, c4 = (q & 7) * 4;
      if (r0 + r < n) {
        const int64_t v = a.rows[r0 + r];
        *reinterpret_cast<float4*>(a.grid + v * a.stride[3] + c4) =
            float4{tile[r][c4], tile[r][c4 + 1], tile[r][c4 + 2], tile[r][c4 + 3]};
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_grid_rows_any(const nc_grid_rows_args a) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (c, i), i fastest
  const int64_t n = a.n_rows;
  if (e >= n * a.channels) return;
  const int64_t c = e / n, i = e - c * n;
  const int64_t v = a.rows[i];
  const int64_t H = a.dims[1], W = a.dims[2];
  const int64_t x = v % W, y = (v / W) % H, z = v / (W * H);
  float* g = a.grid + c * a.stride[0] + z * a.stride[1] + y * a.stride[2] + x * a.stride[3];
  if (a.op == NC_ROWS_GATHER) a.packed[e] = *g;
  else *g = a.op == NC_ROWS_ZERO ? 0.f : a.packed[e];
}

static bool grid_rows_cl(const nc_grid_rows_args& a) {
  const int64_t H = a.dims[1], W = a.dims[2];
  return a.channels == 32 && a.stride[0] == 1 && a.stride[3] == 32 && a.stride[2] == 32 * W &&
         a.stride[1] == 32 * W * H && (reinterpret_cast<uintptr_t>(a.grid) & 15u) == 0;
}

int launch_grid_rows(const nc_grid_rows_args& a, hipStream_t s) {
  if (a.n_rows == 0) return 0;
  if (grid_rows_cl(a))
    hipLaunchKernelGGL(k_grid_rows_cl, dim3((unsigned)((a.n_rows + GR_ROWS - 1) / GR_ROWS)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_grid_rows_any, dim3((unsigned)((a.n_rows * a.channels + 255) / 256)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace nc
