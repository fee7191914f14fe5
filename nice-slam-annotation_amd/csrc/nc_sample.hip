// nc_sample.hip -- training-ray sampling over a batch of camera frames (ABI v4,
// nc_sample_rays_forward / _backward).
//
//   k_sample_rays      thread = ray: region pixel (i, j) of the drawn flat index
//                      (get_sample_uv's meshgrid of torch.linspace over integer
//                      endpoints = exact integers), dirs and rays (get_rays_from_uv,
//                      common.py:74-89), the depth / colour gather (select_uv,
//                      common.py:92-108) and the bbox pre-filter of the Tracker /
//                      Mapper (Tracker.py:100-107, Mapper.py:580-591) in float64.
//   k_sample_pose_grad one workgroup per frame: d c2w[f][r][c] = sum_rays g_d[r] dirs[c]
//                      (c < 3), d c2w[f][r][3] = sum_rays g_o[r]; fixed-order tree sum.
// Compiled with -ffp-contract=off: the products and the 3-term sums keep torch's
// association (sum(dirs * R, -1) = (p0 + p1) + p2 over materialised products).
#include <math.h>

#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

template <typename T>
__device__ __forceinline__ T cam_at(const nc_sample_args& a, int64_t f, int k) {
  return reinterpret_cast<const T*>(a.cam)[f * a.cam_stride[0] + k * a.cam_stride[1]];
}

// quad2rotation's P_ab (R_ab = 1 - s P_ab on the diagonal, s P_ab off it; s = 2 / |q|^2),
// q = (qr, qi, qj, qk) -- src/common.py:137-160 term by term
template <typename T>
__device__ __forceinline__ void quad_terms(const T (&q)[4], T (&P)[3][3]) {
  const T qr = q[0], qi = q[1], qj = q[2], qk = q[3];
  P[0][0] = qj * qj + qk * qk; P[0][1] = qi * qj - qk * qr; P[0][2] = qi * qk + qj * qr;
  P[1][0] = qi * qj + qk * qr; P[1][1] = qi * qi + qk * qk; P[1][2] = qj * qk - qi * qr;
  P[2][0] = qi * qk - qj * qr; P[2][1] = qj * qk + qi * qr; P[2][2] = qi * qi + qj * qj;
}

// c2w rows 0..2 of frame f: the caller's matrix, or get_camera_from_tensor(cam[f])
// (common.py:163-176: [quad2rotation(q) | t]).  quad2rotation writes R into a float32
// tensor (common.py:150) whatever the quaternion's dtype: R is rounded to float (a no-op
// for T = float), t keeps T.
template <typename T>
__device__ __forceinline__ void pose_rows(const nc_sample_args& a, int64_t f, T (&M)[3][4]) {
  if (a.cam) {
    T q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = cam_at<T>(a, f, k);
    const T s = (T)2 / (((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
    T P[3][3];
    quad_terms(q, P);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) M[r][c] = (T)(float)(r == c ? (T)1 - s * P[r][c] : s * P[r][c]);
      M[r][3] = cam_at<T>(a, f, 4 + r);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        M[r][c] = reinterpret_cast<const T*>(a.c2w)[f * a.c2w_stride[0] + r * a.c2w_stride[1] + c * a.c2w_stride[2]];
  }
}

// d loss / d cam from d loss / d c2w (G: 3 x 4): the chain rule through quad2rotation --
// dR_ab/dq_m = sigma_ab (ds/dq_m P_ab + s dP_ab/dq_m), ds/dq_m = -s 2 q_m / |q|^2.  The
// rotation's gradient passes the reference's float32 rot_mat: rounded to float first.
template <typename T>
__device__ __forceinline__ void cam_grad(const T (&q)[4], const T (&G)[12], T (&gc)[7]) {
  const T n = ((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3];
  const T s = (T)2 / n;
  T P[3][3];
  quad_terms(q, P);
  const T qr = q[0], qi = q[1], qj = q[2], qk = q[3];
  // dP_ab/dq_m for m = r, i, j, k
  const T dP[3][3][4] = {
      {{0, 0, 2 * qj, 2 * qk}, {-qk, qj, qi, -qr}, {qj, qk, qr, qi}},
      {{qk, qj, qi, qr}, {0, 2 * qi, 0, 2 * qk}, {-qi, -qr, qk, qj}},
      {{-qj, qk, -qr, qi}, {qi, qr, qk, qj}, {0, 2 * qi, 2 * qj, 0}}};
  T gsP = 0;  // sum_ab sigma_ab G_ab P_ab
  T gdP[4] = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const T gr = (T)(float)G[r * 4 + c];
      const T sg = r == c ? -gr : gr;
      gsP += sg * P[r][c];
#pragma unroll
      for (int m = 0; m < 4; ++m) gdP[m] += sg * dP[r][c][m];
    }
#pragma unroll
  for (int m = 0; m < 4; ++m) gc[m] = (-s * (T)2 * q[m] / n) * gsP + s * gdP[m];
#pragma unroll
  for (int r = 0; r < 3; ++r) gc[4 + r] = G[r * 4 + 3];
}

// torch.max / torch.min over a dim propagate NaN
__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }
__device__ __forceinline__ double nan_min(double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }

template <typename T>
__global__ void __launch_bounds__(256) k_sample_rays(const nc_sample_args a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = a.n_frames * a.n_per_frame;
  if (r >= n) return;
  const int64_t f = r / a.n_per_frame;
  const int64_t img = a.frame_ids ? a.frame_ids[f] : f;
  int64_t col = 0, row = 0;
  float fi, fj;
  if (a.pix_i) {
    fi = a.pix_i[r];
    fj = a.pix_j[r];
  } else {
    const int64_t rw = a.W1 - a.W0;
    const int64_t k = a.indices[r];
    col = a.W0 + k % rw;
    row = a.H0 + k / rw;
    fi = (float)col;
    fj = (float)row;
  }
  // dirs in float32, as torch computes them from the float32 meshgrid
  const float di = (fi - a.cx) / a.fx;
  const float dj = -((fj - a.cy) / a.fy);
  const float dk = -1.f;
  const T d[3] = {(T)di, (T)dj, (T)dk};
  T M[3][4];
  pose_rows<T>(a, f, M);
  T o[3], rd[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const T p0 = d[0] * M[q][0];
    const T p1 = d[1] * M[q][1];
    const T p2 = d[2] * M[q][2];
    rd[q] = (p0 + p1) + p2;
    o[q] = M[q][3];
  }
  T* ro = reinterpret_cast<T*>(a.rays_o) + r * 3;
  T* rdd = reinterpret_cast<T*>(a.rays_d) + r * 3;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    ro[q] = o[q];
    rdd[q] = rd[q];
  }
  float dep = 0.f;
  if (a.depth) {
    dep = a.depth[img * a.depth_stride[0] + row * a.depth_stride[1] + col * a.depth_stride[2]];
    a.gt_depth[r] = dep;
  }
  if (a.color) {
    const float* c = a.color + img * a.color_stride[0] + row * a.color_stride[1] + col * a.color_stride[2];
#pragma unroll
    for (int q = 0; q < 3; ++q) a.gt_color[r * 3 + q] = c[q * a.color_stride[3]];
  }
  if (a.bound && a.inside) {
    // the reference filters the float32 rays (Mapper: after .float()) in float64
    double t = INFINITY;
    bool first = true;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const double oo = (double)(float)o[q], dd = (double)(float)rd[q];
      const double t0 = (a.bound[2 * q] - oo) / dd, t1 = (a.bound[2 * q + 1] - oo) / dd;
      const double m = nan_max(t0, t1);
      t = first ? m : nan_min(t, m);
      first = false;
    }
    a.inside[r] = (t >= (double)dep) ? 1 : 0;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_sample_pose_grad(const nc_sample_args a) {
  const int64_t f = blockIdx.x;
  const int64_t rw = a.W1 - a.W0;
  const T* go = reinterpret_cast<const T*>(a.g_rays_o);
  const T* gd = reinterpret_cast<const T*>(a.g_rays_d);
  T acc[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) acc[q] = (T)0;
  for (int64_t s = threadIdx.x; s < a.n_per_frame; s += blockDim.x) {
    const int64_t r = f * a.n_per_frame + s;
    float fi, fj;
    if (a.pix_i) {
      fi = a.pix_i[r];
      fj = a.pix_j[r];
    } else {
      const int64_t k = a.indices[r];
      fi = (float)(a.W0 + k % rw);
      fj = (float)(a.H0 + k / rw);
    }
    const float di = (fi - a.cx) / a.fx;
    const float dj = -((fj - a.cy) / a.fy);
    const T d[3] = {(T)di, (T)dj, (T)-1.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const T g = gd ? gd[r * 3 + q] : (T)0;
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[q * 4 + c] = acc[q * 4 + c] + g * d[c];
      acc[q * 4 + 3] = acc[q * 4 + 3] + (go ? go[r * 3 + q] : (T)0);
    }
  }
  __shared__ T red[12][256];
#pragma unroll
  for (int q = 0; q < 12; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
#pragma unroll
      for (int q = 0; q < 12; ++q) red[q][threadIdx.x] = red[q][threadIdx.x] + red[q][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (a.g_c2w && threadIdx.x < 12) reinterpret_cast<T*>(a.g_c2w)[f * 12 + threadIdx.x] = red[threadIdx.x][0];
  if (a.cam && threadIdx.x == 0) {  // d cam (get_camera_from_tensor's backward) in the same launch
    T q[4], G[12], gc[7];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = cam_at<T>(a, f, k);
#pragma unroll
    for (int k = 0; k < 12; ++k) G[k] = red[k][0];
    cam_grad(q, G, gc);
#pragma unroll
    for (int k = 0; k < 7; ++k) reinterpret_cast<T*>(a.g_cam)[f * 7 + k] = gc[k];
  }
}

int launch_sample_rays(const nc_sample_args& a, hipStream_t s) {
  const int64_t n = a.n_frames * a.n_per_frame;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (a.pose_dtype == NC_POSE_F64) hipLaunchKernelGGL(k_sample_rays<double>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_sample_rays<float>, grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int launch_sample_pose_grad(const nc_sample_args& a, hipStream_t s) {
  const dim3 grid((unsigned)a.n_frames);
  if (a.pose_dtype == NC_POSE_F64) hipLaunchKernelGGL(k_sample_pose_grad<double>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_sample_pose_grad<float>, grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace nc
