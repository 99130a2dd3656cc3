// GroupNorm + scale/shift + SiLU (+ residual) — video_net.py:216-227 (Block) and :265 (ResnetBlock
// residual add) — forward and backward.
//
// Statistics are per sample over (C/G channels x F frames x H x W); the sample's voxels are a
// contiguous [rows][C] block of the channels-last activation.  Everything after the statistics
// is folded into per-(sample, channel) affine coefficients computed once per call:
//   forward   a = y*A1[b,c] + A0[b,c],  out = silu(a) + res
//   backward  da = dout * silu'(a),  S1 = sum da,  S3 = sum da*y   (per b,c; xhat never stored)
//             dy = da*E1[b,c] + y*E2[b,c] + E3[b,c]
// so the streaming kernels keep a thread on one 8-channel group (coefficients in registers)
// and touch HBM only for the activations.
#include "common.h"

namespace {

static int gn_nchunk(int64_t rows_b) {
  int64_t n = rows_b / 2048;
  if (n < 1) n = 1;
  if (n > 256) n = 256;
  return (int)n;
}

// part[b][chunk][g] = (sum, sumsq) as double
template <typename T>
__global__ __launch_bounds__(256) void gn_stats_kernel(const T* __restrict__ y, double* __restrict__ part,
                                                       int64_t rows_b, int C, int G, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int tid = threadIdx.x;
  const int c8 = tid % cv, rr = tid / cv;
  const int gsz = C / G;
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const T* base = y + (int64_t)b * rows_b * C;
  float s = 0.f, ss = 0.f;
  if (rr < rl) {
#pragma unroll 4
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
    const int g8 = gsz / 8;  // 8-channel groups per GroupNorm group (gsz % 8 == 0 checked on host)
    for (int k = 0; k < rl; ++k)
      for (int c = tid * g8; c < (tid + 1) * g8; ++c) { a += red[k * cv + c][0]; q += red[k * cv + c][1]; }
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

// coef[b][0][c] = A1, coef[b][1][c] = A0 :  a = y*A1 + A0
__global__ void gn_coef_kernel(const float* __restrict__ stats, const float* __restrict__ gamma,
                               const float* __restrict__ beta, const float* __restrict__ ss, float* __restrict__ coef,
                               int B, int C, int G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C;
  const int g = c / (C / G);
  const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
  const float sc = ss ? ss[(int64_t)b * 2 * C + c] + 1.f : 1.f;
  const float sh = ss ? ss[(int64_t)b * 2 * C + C + c] : 0.f;
  const float k = rstd * gamma[c];
  coef[((int64_t)b * 2) * C + c] = k * sc;
  coef[((int64_t)b * 2 + 1) * C + c] = (beta[c] - mean * k) * sc + sh;
}

__device__ __forceinline__ void load_coef8(const float* p, float* v) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

// grid (nchunk, B): thread = (8-channel group c8, row lane rr), rows strided by 256/(C/8)
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ y, const float* __restrict__ coef,
                                                       const T* __restrict__ res, T* __restrict__ out, int64_t rows_b,
                                                       int C, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int c8 = threadIdx.x % cv, rr = threadIdx.x / cv;
  if (rr >= rl) return;
  float A1[8], A0[8];
  load_coef8(coef + ((int64_t)b * 2) * C + c8 * 8, A1);
  load_coef8(coef + ((int64_t)b * 2 + 1) * C + c8 * 8, A0);
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C + c8 * 8;
#pragma unroll 4
  for (int64_t r = r0 + rr; r < r1; r += rl) {
    float v[8], rv[8];
    load8(y + off + r * C, v);
    if (res) load8(res + off + r * C, rv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float a = silu_t<T>(fmaf(v[i], A1[i], A0[i]));
      v[i] = res ? a + rv[i] : a;
    }
    store8(out + off + r * C, v);
  }
}

// part[b][chunk][c] = (S1 = sum da, S3 = sum da*y)
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_reduce_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                            const float* __restrict__ coef, float* __restrict__ part,
                                                            int64_t rows_b, int C, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int tid = threadIdx.x;
  const int c8 = tid % cv, rr = tid / cv;
  float A1[8], A0[8];
  load_coef8(coef + ((int64_t)b * 2) * C + c8 * 8, A1);
  load_coef8(coef + ((int64_t)b * 2 + 1) * C + c8 * 8, A0);
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C + c8 * 8;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < rl) {
#pragma unroll 4
    for (int64_t r = r0 + rr; r < r1; r += rl) {
      float v[8], d[8];
      load8(y + off + r * C, v);
      load8(dout + off + r * C, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float da = d[i] * dsilu_t<T>(fmaf(v[i], A1[i], A0[i]));
        s1[i] += da;
        s3[i] = fmaf(da, v[i], s3[i]);
      }
    }
  }
  __shared__ float red[256][17];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[tid][i] = s1[i]; red[tid][8 + i] = s3[i]; }
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

// per sample b (one block): S1, S2 = rstd*(S3 - mean*S1) -> dss[b] (d scale | d shift), param
// contributions pb[b][c] = ((1+scale)*S2, (1+scale)*S1), and the apply coefficients
// E[b][0..2][c]:  dy = da*E1 + y*E2 + E3
__global__ __launch_bounds__(256) void gn_bwd_finalize_kernel(const float* __restrict__ part,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              const float* __restrict__ ss, float* __restrict__ dss,
                                                              float* __restrict__ pb, float* __restrict__ E, int C,
                                                              int G, int nchunk, double count) {
  const int b = blockIdx.x;
  __shared__ float ga_[1024], gb_[1024];
  __shared__ float gA[64], gB[64];
  const int gsz = C / G;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s1 = 0.f, s3 = 0.f;
    for (int k = 0; k < nchunk; ++k) {
      const float* p = part + (((int64_t)b * nchunk + k) * C + c) * 2;
      s1 += p[0];
      s3 += p[1];
    }
    const int g = c / gsz;
    const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
    const float s2 = rstd * (s3 - mean * s1);  // sum da * xhat
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
    double a = 0.0, q = 0.0;
    for (int c = threadIdx.x * gsz; c < (int)(threadIdx.x + 1) * gsz; ++c) { a += ga_[c]; q += gb_[c]; }
    gA[threadIdx.x] = (float)(a / count);
    gB[threadIdx.x] = (float)(q / count);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / gsz;
    const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
    const float sc = ss ? ss[(int64_t)b * 2 * C + c] + 1.f : 1.f;
    // dy = rstd*(da*sc*gamma - A - (y-mean)*rstd*Bg)
    E[((int64_t)b * 3) * C + c] = rstd * sc * gamma[c];
    E[((int64_t)b * 3 + 1) * C + c] = -rstd * rstd * gB[g];
    E[((int64_t)b * 3 + 2) * C + c] = rstd * (mean * rstd * gB[g] - gA[g]);
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

template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                           const float* __restrict__ coef, const float* __restrict__ E,
                                                           T* __restrict__ dy, int64_t rows_b, int C, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int c8 = threadIdx.x % cv, rr = threadIdx.x / cv;
  if (rr >= rl) return;
  float A1[8], A0[8], E1[8], E2[8], E3[8];
  load_coef8(coef + ((int64_t)b * 2) * C + c8 * 8, A1);
  load_coef8(coef + ((int64_t)b * 2 + 1) * C + c8 * 8, A0);
  load_coef8(E + ((int64_t)b * 3) * C + c8 * 8, E1);
  load_coef8(E + ((int64_t)b * 3 + 1) * C + c8 * 8, E2);
  load_coef8(E + ((int64_t)b * 3 + 2) * C + c8 * 8, E3);
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C + c8 * 8;
#pragma unroll 4
  for (int64_t r = r0 + rr; r < r1; r += rl) {
    float v[8], d[8];
    load8(y + off + r * C, v);
    load8(dout + off + r * C, d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float da = d[i] * dsilu_t<T>(fmaf(v[i], A1[i], A0[i]));
      d[i] = fmaf(da, E1[i], fmaf(v[i], E2[i], E3[i]));
    }
    store8(dy + off + r * C, d);
  }
}

template <typename F>
static int dispatch_dt(int dtype, F&& f) {
  if (dtype == CESM_DT_BF16) { f((bf16*)nullptr); return CESM_OK; }
  if (dtype == CESM_DT_F32) { f((float*)nullptr); return CESM_OK; }
  return CESM_EINVAL;
}

static int gn_apply_chunks(int64_t rows_b, int C) {
  // ~16 row-iterations per thread
  const int rl = 256 / (C / 8);
  int64_t n = rows_b / (rl * 16);
  if (n < 1) n = 1;
  if (n > 4096) n = 4096;
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

// ss: [B][2C] (scale | shift) or null; res: residual [B*rows_b][C] or null; ws: >= 2*B*C floats
int cesm_gn_apply(int dtype, const void* y, const float* stats, const float* gamma, const float* beta,
                  const float* ss, const void* res, void* out, float* ws, int B, int64_t rows_b, int C, int G,
                  hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || C % G) return CESM_EINVAL;
  gn_coef_kernel<<<(unsigned)cdiv(B * C, 256), 256, 0, stream>>>(stats, gamma, beta, ss, ws, B, C, G);
  const int nch = gn_apply_chunks(rows_b, C);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_apply_kernel<T><<<dim3(nch, B), 256, 0, stream>>>((const T*)y, ws, (const T*)res, (T*)out, rows_b, C, nch);
  });
  if (rc) return rc;
  return cesm_launch_status();
}

// Backward of out = silu(GN(y)*(1+scale)+shift) (+res).  Writes dy, dss [B][2C] (if non-null),
// dgamma/dbeta (accumulate flag).  ws: float workspace >= B*256*C*2 + B*C*2 + B*C*5 floats.
int cesm_gn_bwd(int dtype, const void* dout, const void* y, const float* stats, const float* gamma,
                const float* beta, const float* ss, void* dy, float* dss, float* dgamma, float* dbeta, float* ws,
                int B, int64_t rows_b, int C, int G, int accumulate, hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || C % G || C > 1024 || G > 64) return CESM_EINVAL;
  const int nchunk = gn_nchunk(rows_b);
  float* part = ws;
  float* pb = part + (int64_t)B * nchunk * C * 2;
  float* coef = pb + (int64_t)B * C * 2;
  float* E = coef + (int64_t)B * C * 2;
  const double count = (double)rows_b * (C / G);
  gn_coef_kernel<<<(unsigned)cdiv(B * C, 256), 256, 0, stream>>>(stats, gamma, beta, ss, coef, B, C, G);
  const int nch = gn_apply_chunks(rows_b, C);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_bwd_reduce_kernel<T><<<dim3(nchunk, B), 256, 0, stream>>>((const T*)dout, (const T*)y, coef, part, rows_b, C,
                                                                 nchunk);
    gn_bwd_finalize_kernel<<<B, 256, 0, stream>>>(part, stats, gamma, beta, ss, dss, pb, E, C, G, nchunk, count);
    gn_bwd_apply_kernel<T><<<dim3(nch, B), 256, 0, stream>>>((const T*)dout, (const T*)y, coef, E, (T*)dy, rows_b, C,
                                                             nch);
  });
  if (rc) return rc;
  gn_param_grad_kernel<<<(unsigned)cdiv(C, 256), 256, 0, stream>>>(pb, dgamma, dbeta, B, C, accumulate);
  return cesm_launch_status();
}

}  // extern "C"
