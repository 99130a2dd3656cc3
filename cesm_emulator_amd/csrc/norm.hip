// GroupNorm(+scale/shift+SiLU+residual) and channel LayerNorm, forward and backward.
//
// GroupNorm: video_net.py:216-227 (Block: GroupNorm(8, C) eps 1e-5 affine -> x*(scale+1)+shift
// -> SiLU) and :265 (ResnetBlock residual add, fused into the apply pass).  Statistics are per
// sample over (C/G channels x F frames x H x W); activations are channels-last with the
// sample's F*H*W voxels contiguous, so a sample is a contiguous [rows][C] matrix.
//
// LayerNorm: video_net.py:78-87 — per voxel over C, biased variance, eps 1e-5, gamma only.
#include "common.h"

namespace {

// ---------------------------------------------------------------- GroupNorm forward
// part[b][chunk][g] = (sum, sumsq) as double
template <typename T>
__global__ __launch_bounds__(256) void gn_stats_kernel(const T* __restrict__ y, double* __restrict__ part,
                                                       int64_t rows_b, int C, int G, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8;                // threads per row
  const int rl = 256 / cv;             // rows per iteration
  const int tid = threadIdx.x;
  const int c8 = tid % cv, rr = tid / cv;
  const int gsz = C / G;
  const int grp = (c8 * 8) / gsz;
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const T* base = y + (int64_t)b * rows_b * C;
  float s = 0.f, ss = 0.f;
  if (rr < rl) {
    for (int64_t r = r0 + rr; r < r1; r += rl) {
      float v[8];
      load8(base + r * C + c8 * 8, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s += v[i]; ss = fmaf(v[i], v[i], ss); }
    }
  }
  __shared__ double red[256][2];
  red[tid][0] = s;
  red[tid][1] = ss;
  __syncthreads();
  if (tid < G) {
    double a = 0.0, q = 0.0;
    for (int t = 0; t < rl * cv; ++t) {
      const int tc8 = t % cv;
      if ((tc8 * 8) / gsz == tid) { a += red[t][0]; q += red[t][1]; }
    }
    double* o = part + (((int64_t)b * nchunk + chunk) * G + tid) * 2;
    o[0] = a;
    o[1] = q;
  }
}

// stats[b][g] = (mean, rstd)
__global__ void gn_finalize_kernel(const double* __restrict__ part, float* __restrict__ stats, int B, int G,
                                   int nchunk, double count, float eps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * G) return;
  const int b = i / G, g = i - b * G;
  double a = 0.0, q = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const double* p = part + (((int64_t)b * nchunk + k) * G + g) * 2;
    a += p[0];
    q += p[1];
  }
  const double mean = a / count;
  double var = q / count - mean * mean;
  if (var < 0) var = 0;
  stats[i * 2] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// out = silu( ((y-mean)*rstd*gamma + beta) * (1+scale) + shift ) + res
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ y, const float* __restrict__ stats,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       const float* __restrict__ ss, const T* __restrict__ res,
                                                       T* __restrict__ out, int64_t rows_b, int B, int C, int G) {
  const int64_t total = (int64_t)B * rows_b * (C / 8);
  const int gsz = C / G;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % (C / 8));
    const int64_t row = e / (C / 8);
    const int b = (int)(row / rows_b);
    const int c0 = c8 * 8;
    const int g = c0 / gsz;
    const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
    float v[8], r[8];
    load8(y + row * C + c0, v);
    if (res) load8(res + row * C + c0, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float a = (v[i] - mean) * rstd * gamma[c0 + i] + beta[c0 + i];
      if (ss) a = a * (ss[(int64_t)b * 2 * C + c0 + i] + 1.f) + ss[(int64_t)b * 2 * C + C + c0 + i];
      a = silu_p(a);
      v[i] = res ? a + r[i] : a;
    }
    store8(out + row * C + c0, v);
  }
}

// ---------------------------------------------------------------- GroupNorm backward
// part[b][chunk][c] = (S1 = sum da, S2 = sum da*xhat)
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_reduce_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                            const float* __restrict__ stats,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ ss, float* __restrict__ part,
                                                            int64_t rows_b, int C, int G, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int tid = threadIdx.x;
  const int c8 = tid % cv, rr = tid / cv;
  const int c0 = c8 * 8;
  const int g = c0 / (C / G);
  const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
  float ga[8], be[8], sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ga[i] = gamma[c0 + i];
    be[i] = beta[c0 + i];
    sc[i] = ss ? ss[(int64_t)b * 2 * C + c0 + i] + 1.f : 1.f;
    sh[i] = ss ? ss[(int64_t)b * 2 * C + C + c0 + i] : 0.f;
  }
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < rl) {
    for (int64_t r = r0 + rr; r < r1; r += rl) {
      float v[8], d[8];
      load8(y + off + r * C + c0, v);
      load8(dout + off + r * C + c0, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (v[i] - mean) * rstd;
        const float a = (xh * ga[i] + be[i]) * sc[i] + sh[i];
        const float da = d[i] * dsilu_p(a);
        s1[i] += da;
        s2[i] = fmaf(da, xh, s2[i]);
      }
    }
  }
  __shared__ float red[256][17];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[tid][i] = s1[i]; red[tid][8 + i] = s2[i]; }
  __syncthreads();
  if (tid < cv) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < rl; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) { a[i] += red[k * cv + tid][i]; q[i] += red[k * cv + tid][8 + i]; }
    float* o = part + (((int64_t)b * nchunk + chunk) * C + tid * 8) * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) { o[i * 2] = a[i]; o[i * 2 + 1] = q[i]; }
  }
}

// per sample b (one block): S1,S2 over chunks -> dss[b] (d scale | d shift), per-b param
// contributions pb[b][c] = ((1+scale)*S2, (1+scale)*S1), coef[b][g] = (A_g, B_g)
__global__ __launch_bounds__(256) void gn_bwd_finalize_kernel(const float* __restrict__ part,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              const float* __restrict__ ss, float* __restrict__ dss,
                                                              float* __restrict__ pb, float* __restrict__ coef, int C,
                                                              int G, int nchunk, double count) {
  const int b = blockIdx.x;
  __shared__ float ga_[1024], gb_[1024];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s1 = 0.f, s2 = 0.f;
    for (int k = 0; k < nchunk; ++k) {
      const float* p = part + (((int64_t)b * nchunk + k) * C + c) * 2;
      s1 += p[0];
      s2 += p[1];
    }
    const float sc = ss ? ss[(int64_t)b * 2 * C + c] + 1.f : 1.f;
    if (dss) {
      dss[(int64_t)b * 2 * C + c] = gamma[c] * s2 + beta[c] * s1;  // d scale
      dss[(int64_t)b * 2 * C + C + c] = s1;                        // d shift
    }
    pb[((int64_t)b * C + c) * 2] = sc * s2;      // dgamma contribution
    pb[((int64_t)b * C + c) * 2 + 1] = sc * s1;  // dbeta contribution
    ga_[c] = gamma[c] * sc * s1;
    gb_[c] = gamma[c] * sc * s2;
  }
  __syncthreads();
  if ((int)threadIdx.x < G) {
    const int gsz = C / G;
    double a = 0.0, q = 0.0;
    for (int c = threadIdx.x * gsz; c < (int)(threadIdx.x + 1) * gsz; ++c) { a += ga_[c]; q += gb_[c]; }
    coef[(b * G + threadIdx.x) * 2] = (float)(a / count);
    coef[(b * G + threadIdx.x) * 2 + 1] = (float)(q / count);
  }
}

// dgamma/dbeta (+)= sum_b pb[b]
__global__ void gn_param_grad_kernel(const float* __restrict__ pb, float* __restrict__ dgamma,
                                     float* __restrict__ dbeta, int B, int C, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, q = 0.f;
  for (int b = 0; b < B; ++b) { a += pb[((int64_t)b * C + c) * 2]; q += pb[((int64_t)b * C + c) * 2 + 1]; }
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + a : a;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + q : q;
}

// dy = rstd * (dxhat - A_g - xhat*B_g), dxhat = da*(1+scale)*gamma
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                           const float* __restrict__ stats,
                                                           const float* __restrict__ coef,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ ss, T* __restrict__ dy,
                                                           int64_t rows_b, int B, int C, int G) {
  const int64_t total = (int64_t)B * rows_b * (C / 8);
  const int gsz = C / G;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % (C / 8));
    const int64_t row = e / (C / 8);
    const int b = (int)(row / rows_b);
    const int c0 = c8 * 8;
    const int g = c0 / gsz;
    const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
    const float A = coef[(b * G + g) * 2], Bc = coef[(b * G + g) * 2 + 1];
    float v[8], d[8];
    load8(y + row * C + c0, v);
    load8(dout + row * C + c0, d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sc = ss ? ss[(int64_t)b * 2 * C + c0 + i] + 1.f : 1.f;
      const float sh = ss ? ss[(int64_t)b * 2 * C + C + c0 + i] : 0.f;
      const float xh = (v[i] - mean) * rstd;
      const float a = (xh * gamma[c0 + i] + beta[c0 + i]) * sc + sh;
      const float dxh = d[i] * dsilu_p(a) * sc * gamma[c0 + i];
      v[i] = rstd * (dxh - A - xh * Bc);
    }
    store8(dy + row * C + c0, v);
  }
}

// ---------------------------------------------------------------- LayerNorm
// lanes per voxel L = C/8 (8..64, power of two); each lane 8 channels
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                     T* __restrict__ out, float* __restrict__ mr, int64_t V, int C,
                                                     float eps) {
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
  store8(out + v * C + sub * 8, a);
  if (sub == 0 && mr) { mr[v * 2] = mean; mr[v * 2 + 1] = rstd; }
}

// dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma ; part[blk][c] = sum dy*xhat
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ mr, const float* __restrict__ gamma,
                                                     const T* __restrict__ dres, T* __restrict__ dx,
                                                     float* __restrict__ part, int64_t V, int C) {
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
      load8(dy + v * C + sub * 8, d);
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

static int gn_nchunk(int64_t rows_b) {
  int64_t n = rows_b / 2048;
  if (n < 1) n = 1;
  if (n > 256) n = 256;
  return (int)n;
}

}  // namespace

extern "C" {

// y: [B][rows_b][C] (rows_b = F*H*W); writes stats[B][G][2] = (mean, rstd); ws >= B*256*G*2 doubles
int cesm_gn_stats(int dtype, const void* y, float* stats, double* ws, int B, int64_t rows_b, int C, int G, float eps,
                  hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || C % G || (C / G) % 8) return CESM_EINVAL;
  const int nchunk = gn_nchunk(rows_b);
  dim3 grid(nchunk, B);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_stats_kernel<T><<<grid, 256, 0, stream>>>((const T*)y, ws, rows_b, C, G, nchunk);
  });
  if (rc) return rc;
  gn_finalize_kernel<<<(unsigned)cdiv(B * G, 64), 64, 0, stream>>>(ws, stats, B, G, nchunk,
                                                                   (double)rows_b * (C / G), eps);
  return cesm_launch_status();
}

// ss: [B][2C] (scale | shift) or null; res: residual [B*rows_b][C] or null
int cesm_gn_apply(int dtype, const void* y, const float* stats, const float* gamma, const float* beta,
                  const float* ss, const void* res, void* out, int B, int64_t rows_b, int C, int G,
                  hipStream_t stream) {
  if (C % 8 || C % G) return CESM_EINVAL;
  const int64_t total = (int64_t)B * rows_b * (C / 8);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(total, 256), 16384);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_apply_kernel<T><<<grid, 256, 0, stream>>>((const T*)y, stats, gamma, beta, ss, (const T*)res, (T*)out, rows_b,
                                                 B, C, G);
  });
  if (rc) return rc;
  return cesm_launch_status();
}

// Backward of out = silu(GN(y)*(1+scale)+shift) (+res).  Writes dy, dss [B][2C] (if non-null),
// dgamma/dbeta (accumulate flag).  ws: float workspace >= B*256*C*2 + B*C*2 + B*G*2 floats.
int cesm_gn_bwd(int dtype, const void* dout, const void* y, const float* stats, const float* gamma,
                const float* beta, const float* ss, void* dy, float* dss, float* dgamma, float* dbeta, float* ws,
                int B, int64_t rows_b, int C, int G, int accumulate, hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || C % G || C > 1024) return CESM_EINVAL;
  const int nchunk = gn_nchunk(rows_b);
  float* part = ws;
  float* pb = part + (int64_t)B * nchunk * C * 2;
  float* coef = pb + (int64_t)B * C * 2;
  dim3 grid(nchunk, B);
  const int64_t total = (int64_t)B * rows_b * (C / 8);
  const unsigned g2 = (unsigned)std::min<int64_t>(cdiv(total, 256), 16384);
  const double count = (double)rows_b * (C / G);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_bwd_reduce_kernel<T><<<grid, 256, 0, stream>>>((const T*)dout, (const T*)y, stats, gamma, beta, ss, part,
                                                      rows_b, C, G, nchunk);
    gn_bwd_finalize_kernel<<<B, 256, 0, stream>>>(part, gamma, beta, ss, dss, pb, coef, C, G, nchunk, count);
    gn_bwd_apply_kernel<T><<<g2, 256, 0, stream>>>((const T*)dout, (const T*)y, stats, coef, gamma, beta, ss, (T*)dy,
                                                   rows_b, B, C, G);
  });
  if (rc) return rc;
  gn_param_grad_kernel<<<(unsigned)cdiv(C, 256), 256, 0, stream>>>(pb, dgamma, dbeta, B, C, accumulate);
  return cesm_launch_status();
}

// x,out: [V][C]; mr: [V][2] (mean, rstd) saved for backward (may be null)
int cesm_ln_fwd(int dtype, const void* x, const float* gamma, void* out, float* mr, int64_t V, int C, float eps,
                hipStream_t stream) {
  if (C % 8 || C / 8 > 64 || ((C / 8) & (C / 8 - 1))) return CESM_EINVAL;
  const int64_t threads = V * (C / 8);
  const unsigned grid = (unsigned)cdiv(threads, 256);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    ln_fwd_kernel<T><<<grid, 256, 0, stream>>>((const T*)x, gamma, (T*)out, mr, V, C, eps);
  });
  if (rc) return rc;
  return cesm_launch_status();
}

// part: nblk*C floats
int cesm_ln_bwd(int dtype, const void* dy, const void* x, const float* mr, const float* gamma, const void* dres,
                void* dx, float* dgamma, float* part, int nblk, int64_t V, int C, int accumulate, hipStream_t stream) {
  if (C % 8 || C / 8 > 64 || ((C / 8) & (C / 8 - 1)) || nblk <= 0) return CESM_EINVAL;
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    ln_bwd_kernel<T><<<nblk, 256, 0, stream>>>((const T*)dy, (const T*)x, mr, gamma, (const T*)dres, (T*)dx, part, V, C);
  });
  if (rc) return rc;
  if (dgamma) sum_rows_kernel<<<C, 64, 0, stream>>>(part, dgamma, nblk, C, accumulate);
  return cesm_launch_status();
}

}  // extern "C"
