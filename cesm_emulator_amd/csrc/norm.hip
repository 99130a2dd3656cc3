// Channel LayerNorm, forward and backward (GroupNorm lives in gn.hip).
//
// GroupNorm: video_net.py:216-227 (Block: GroupNorm(8, C) eps 1e-5 affine -> x*(scale+1)+shift
// -> SiLU) and :265 (ResnetBlock residual add, fused into the apply pass).  Statistics are per
// sample over (C/G channels x F frames x H x W); activations are channels-last with the
// sample's F*H*W voxels contiguous, so a sample is a contiguous [rows][C] matrix.
//
// LayerNorm: video_net.py:78-87 — per voxel over C, biased variance, eps 1e-5, gamma only.
#include "common.h"
#include "cesm_hip.h"

namespace {

// ---------------------------------------------------------------- LayerNorm
// pixel-major row of voxel v = (b*F + f)*HW + p: (b*HW + p)*F + f (pf = 0: identity)
__device__ __forceinline__ int64_t ln_perm(int64_t v, int pf, int phw) {
  if (!pf) return v;
  const int64_t fhw = (int64_t)pf * phw;
  const int64_t b = v / fhw, r = v - b * fhw;
  const int f = (int)(r / phw), p = (int)(r - (int64_t)f * phw);
  return (b * phw + p) * pf + f;
}
// lanes per voxel L = C/8 (8..64, power of two); each lane 8 channels
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                     T* __restrict__ out, float* __restrict__ mr, int64_t V, int C,
                                                     float eps, int pf, int phw) {
  const int L = C / 8;
  const int64_t gt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t v = gt / L;
  const int sub = (int)(gt % L);
  const bool ok = v < V;
  float a[8];
  if (ok) load8(x + v * C + sub * 8, a);
  else for (int i = 0; i < 8; ++i) a[i] = 0.f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  s = group_sum(s, L);
  const float mean = s / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) { const float d = a[i] - mean; q = fmaf(d, d, q); }
  q = group_sum(q, L);
  const float rstd = 1.f / sqrtf(q / C + eps);
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (a[i] - mean) * rstd * gamma[sub * 8 + i];
  store8(out + ln_perm(v, pf, phw) * C + sub * 8, a);
  if (sub == 0 && mr) { mr[v * 2] = mean; mr[v * 2 + 1] = rstd; }
}

// dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma ; part[blk][c] = sum dy*xhat
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ mr, const float* __restrict__ gamma,
                                                     const T* __restrict__ dres, T* __restrict__ dx,
                                                     float* __restrict__ part, int64_t V, int C, int pf, int phw) {
  const int L = C / 8;
  const int vpb = 256 / L;  // voxels per block-iteration
  const int sub = threadIdx.x % L, vl = threadIdx.x / L;
  float ga[8], pg[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { ga[i] = gamma[sub * 8 + i]; pg[i] = 0.f; }
  const int64_t niter = (V + vpb - 1) / vpb;
  for (int64_t it = blockIdx.x; it < niter; it += gridDim.x) {
    const int64_t v = it * vpb + vl;
    const bool ok = v < V;
    float a[8], d[8];
    float mean = 0.f, rstd = 0.f;
    if (ok) {
      load8(x + v * C + sub * 8, a);
      load8(dy + ln_perm(v, pf, phw) * C + sub * 8, d);
      mean = mr[v * 2];
      rstd = mr[v * 2 + 1];
    } else {
      for (int i = 0; i < 8; ++i) { a[i] = 0.f; d[i] = 0.f; }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = (a[i] - mean) * rstd;  // xhat
      const float g = d[i] * ga[i];
      s1 += g;
      s2 = fmaf(g, a[i], s2);
      pg[i] = fmaf(d[i], a[i], pg[i]);
    }
    s1 = group_sum(s1, L) / C;
    s2 = group_sum(s2, L) / C;
    if (ok) {
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = rstd * (d[i] * ga[i] - s1 - a[i] * s2);
      if (dres) {
        float r[8];
        load8(dres + v * C + sub * 8, r);
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] += r[i];
      }
      store8(dx + v * C + sub * 8, d);
    }
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int i = 0; i < 8; ++i) red[threadIdx.x][i] = pg[i];
  __syncthreads();
  if ((int)threadIdx.x < L) {
    float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < vpb; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] += red[k * L + threadIdx.x][i];
#pragma unroll
    for (int i = 0; i < 8; ++i) part[(int64_t)blockIdx.x * C + threadIdx.x * 8 + i] = t[i];
  }
}

// one 64-lane wave per channel, fixed-order reduction
__global__ void sum_rows_kernel(const float* __restrict__ part, float* __restrict__ dst, int nrows, int C,
                                int accumulate) {
  const int c = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nrows; k += 64) s += part[(int64_t)k * C + c];
  s = wave_sum(s);
  if (threadIdx.x == 0) dst[c] = accumulate ? dst[c] + s : s;
}

template <typename F>
static int dispatch_dt(int dtype, F&& f) {
  if (dtype == CESM_DT_BF16) { f((bf16*)nullptr); return CESM_OK; }
  if (dtype == CESM_DT_F32) { f((float*)nullptr); return CESM_OK; }
  return CESM_EINVAL;
}

}  // namespace

extern "C" {

// x,out: [V][C]; mr: [V][2] (mean, rstd) saved for backward (may be null).  perm_f > 0: V = B * perm_f * perm_hw
// voxels in [B][F][HW] order, out rows written pixel-major ([B][HW][F]); mr in x's order
int cesm_ln_fwd(int dtype, const void* x, const float* gamma, void* out, float* mr, int64_t V, int C, float eps,
                int perm_f, int perm_hw, hipStream_t stream) {
  if (C % 8 || C / 8 > 64 || ((C / 8) & (C / 8 - 1))) return CESM_EINVAL;
  if (perm_f < 0 || (perm_f && (perm_hw < 1 || V % ((int64_t)perm_f * perm_hw)))) return CESM_EINVAL;
  const int64_t threads = V * (C / 8);
  const unsigned grid = (unsigned)cdiv(threads, 256);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    ln_fwd_kernel<T><<<grid, 256, 0, stream>>>((const T*)x, gamma, (T*)out, mr, V, C, eps, perm_f, perm_hw);
  });
  if (rc) return rc;
  return cesm_launch_status();
}

// part: nblk*C floats; perm_f > 0: dy rows pixel-major (as cesm_ln_fwd's permuted out), x / dres / dx not
int cesm_ln_bwd(int dtype, const void* dy, const void* x, const float* mr, const float* gamma, const void* dres,
                void* dx, float* dgamma, float* part, int nblk, int64_t V, int C, int accumulate, int perm_f, int perm_hw,
                hipStream_t stream) {
  if (C % 8 || C / 8 > 64 || ((C / 8) & (C / 8 - 1)) || nblk <= 0) return CESM_EINVAL;
  if (perm_f < 0 || (perm_f && (perm_hw < 1 || V % ((int64_t)perm_f * perm_hw)))) return CESM_EINVAL;
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    ln_bwd_kernel<T><<<nblk, 256, 0, stream>>>((const T*)dy, (const T*)x, mr, gamma, (const T*)dres, (T*)dx, part, V, C,
                                               perm_f, perm_hw);
  });
  if (rc) return rc;
  if (dgamma) sum_rows_kernel<<<C, 64, 0, stream>>>(part, dgamma, nblk, C, accumulate);
  return cesm_launch_status();
}

}  // extern "C"
