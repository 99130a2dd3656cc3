// GroupNorm + scale/shift + SiLU (+ residual) — video_net.py:216-227 (Block) and :265 (ResnetBlock
// residual add) — forward and backward.
//
// Statistics are per sample over (C/G channels x F frames x H x W); the sample's voxels are a
// contiguous [rows][C] block of the channels-last activation.  Everything after the statistics
// is folded into per-(sample, channel) affine coefficients (computed in each streaming kernel's prologue
// for the thread's 8 channels):
//   forward   a = y*A1[b,c] + A0[b,c],  out = silu(a) + res
//   backward  da = dout * silu'(a),  S1 = sum da,  S3 = sum da*y,  Sy = sum y  (per b,c; xhat never
//             stored);  dy = da*E1[b,c] + y*E2[b,c] + E3[b,c], so the producing conv's bias gradient
//             sum dy = E1 S1 + E2 Sy + rows E3 comes out of the reduction without another pass over dy
// so the streaming kernels keep a thread on one 8-channel group (coefficients in registers)
// and touch HBM only for the activations.
#include "common.h"
#include "cesm_hip.h"

namespace {

// streaming activation accesses are non-temporal (bf16): measured at the level-0 bench shape stats 122 -> 107 us,
// apply (+ residual) 389 -> 370 us, backward 679 -> 631 us (tools/gn_time.py)
__device__ __forceinline__ void gl8(const bf16* p, float* v) { ldnt4(p, v); ldnt4(p + 4, v + 4); }
__device__ __forceinline__ void gl8(const float* p, float* v) { load8(p, v); }
__device__ __forceinline__ void gs8(bf16* p, const float* v) {
  bf16x8 a;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (bf16)v[i];
  stnt16(p, a);
}
__device__ __forceinline__ void gs8(float* p, const float* v) { store8(p, v); }

// row chunks per sample for the reduction kernels: >= ~8 row-iterations per thread, at most
// max(256, 1024 / B) chunks, so a B = 1 long window (F = 120: ~1M rows per sample) still launches 1024
// blocks = 4 per CU instead of 256 (measured: the 1-block-per-CU grid ran the bwd reduction at ~40 % of
// the apply kernel's bandwidth).  Workspaces hold max(B * 256, 1024) chunk partials (gn_ws_chunks).
constexpr int GN_SMALLB_CHUNKS = 1024;  // (256 = the round-2 fixed cap)
constexpr int GN_BIGB_CAP = 256;  // chunks per sample at B >= 4 (<= 1024: the workspace holds B * 1024 partials);
                                  // whole step 256 -> 512 / 1024: +0.2 / +0.5 ms (profiles/r3_gn_cap_ab.txt)
static int gn_nchunk(int64_t rows_b, int C, int B) {
  const int rl = 256 / (C / 8);
  const int cap = B >= GN_SMALLB_CHUNKS / 256 ? GN_BIGB_CAP : GN_SMALLB_CHUNKS / B;
  int64_t n = rows_b / (rl * 8);
  if (n < 1) n = 1;
  if (n > cap) n = cap;
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
      gl8(base + r * C + c8 * 8, v);
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

// stats[b][g] = (mean, rstd); one wave per (b, g)
__global__ __launch_bounds__(64) void gn_finalize_kernel(const double* __restrict__ part, float* __restrict__ stats,
                                                         int B, int G, int nchunk, double count, float eps) {
  const int i = blockIdx.x;
  const int b = i / G, g = i - b * G;
  double a = 0.0, q = 0.0;
  for (int k = threadIdx.x; k < nchunk; k += 64) {
    const double* p = part + (((int64_t)b * nchunk + k) * G + g) * 2;
    a += p[0];
    q += p[1];
  }
  a = wave_sum_d(a);
  q = wave_sum_d(q);
  if (threadIdx.x) return;
  const double mean = a / count;
  double var = q / count - mean * mean;
  if (var < 0) var = 0;
  stats[i * 2] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// stats[b][g] = (mean, rstd) from the producing conv's epilogue partials part[b][slot][C/4] (float2 per channel
// quad: sum, sum of squares; cesm_conv_fwd_gn): one GNP_T-thread block per (b, g), thread t takes the (slot, quad)
// pairs t, t + GNP_T, ... of the group in order and accumulates in double, then a fixed-order tree -> reproducible.
constexpr int GNP_T = 256;
__global__ __launch_bounds__(GNP_T) void gn_part_finalize_kernel(const float2* __restrict__ part, float* __restrict__ stats,
                                                                 int G, int64_t nslot, int nq, double count, float eps) {
  const int i = blockIdx.x;
  const int b = i / G, g = i - b * G;
  const int qpg = nq / G;
  const int64_t n = nslot * qpg;
  const float2* base = part + (int64_t)b * nslot * nq + g * qpg;
  double a = 0.0, q = 0.0;
  if ((qpg & (qpg - 1)) == 0 && n < (1ll << 31)) {  // uniform: power-of-two quads per group (C / 4G), 32-bit index
    const int sh = __ffs(qpg) - 1, nn = (int)n;
#pragma unroll 8
    for (int e = threadIdx.x; e < nn; e += GNP_T) {
      const int sl = e >> sh;
      const float2 v = base[(int64_t)sl * nq + (e & (qpg - 1))];
      a += v.x;
      q += v.y;
    }
  } else {
#pragma unroll 8
    for (int64_t e = threadIdx.x; e < n; e += GNP_T) {
      const int64_t sl = e / qpg;
      const float2 v = base[sl * nq + (e - sl * qpg)];
      a += v.x;
      q += v.y;
    }
  }
  __shared__ double red[2][GNP_T];
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = q;
  __syncthreads();
  for (int w = GNP_T / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x) return;
  const double mean = red[0][0] / count;
  double var = red[1][0] / count - mean * mean;
  if (var < 0) var = 0;
  stats[i * 2] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// Large sample (F = 120: ~60 k slots) in two stages, because G = 8 blocks per sample each striding over every
// 128-B slot row for their 16 B left the chip idle (38 us per call): stage 1, grid (S = nslot / 64, B): block j
// reduces slots [64 j, 64 j + 64) (the last block also the remainder) for ALL channel quads (coalesced rows),
// fixed-order tree over its row lanes, and writes (sum, sumsq) as doubles over its own first two slot rows (read
// by nobody else; the partials are scratch); stage 2: per (b, g) the S block sums in order.
constexpr int GNP_PER = 64;
__global__ __launch_bounds__(256) void gn_part_stage1_kernel(float2* __restrict__ part, int64_t nslot, int C4, int S) {
  const int b = blockIdx.y, j = blockIdx.x, tid = threadIdx.x;
  const int64_t s0 = (int64_t)j * GNP_PER, s1 = j == S - 1 ? nslot : s0 + GNP_PER;
  const int R = 256 / C4, qd = tid % C4, sr = tid / C4;
  float2* base = part + (int64_t)b * nslot * C4;
  double a = 0.0, q = 0.0;
  for (int64_t sl = s0 + sr; sl < s1; sl += R) {
    const float2 v = base[sl * C4 + qd];
    a += v.x;
    q += v.y;
  }
  __shared__ double red[2][256];
  red[0][tid] = a;
  red[1][tid] = q;
  __syncthreads();  // every read of this block's slots is done: its first two rows may be overwritten below
  for (int w = R >> 1; w > 0; w >>= 1) {
    if (sr < w) {
      red[0][tid] += red[0][tid + w * C4];
      red[1][tid] += red[1][tid + w * C4];
    }
    __syncthreads();
  }
  if (sr == 0) reinterpret_cast<double2*>(base + s0 * C4)[qd] = make_double2(red[0][tid], red[1][tid]);
}
__global__ __launch_bounds__(64) void gn_part_stage2_kernel(const float2* __restrict__ part, float* __restrict__ stats,
                                                             int G, int64_t nslot, int C4, int S, double count,
                                                             float eps) {
  const int i = blockIdx.x, b = i / G, g = i - b * G, qpg = C4 / G;
  const float2* base = part + (int64_t)b * nslot * C4;
  double a = 0.0, q = 0.0;
  for (int j = threadIdx.x; j < S; j += 64) {
    const double2* r = reinterpret_cast<const double2*>(base + (int64_t)j * GNP_PER * C4) + g * qpg;
    for (int k = 0; k < qpg; ++k) {
      a += r[k].x;
      q += r[k].y;
    }
  }
  a = wave_sum_d(a);
  q = wave_sum_d(q);
  if (threadIdx.x) return;
  const double mean = a / count;
  double var = q / count - mean * mean;
  if (var < 0) var = 0;
  stats[i * 2] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// coefficients: A1[b][c], A0[b][c] with a = y*A1 + A0 (gn_coef8 below)
__device__ __forceinline__ void load_coef8(const float* p, float* v) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

// The same coefficients computed in the streaming kernels' prologue for the thread's 8 channels (one
// group: C/G is a multiple of 8), which saves the coefficient kernel's launch per GroupNorm call.
struct GnAffine {
  const float* stats;  // [B][G][2] (mean, rstd)
  const float* gamma;
  const float* beta;
  const float* ss;     // [B][2C] (scale | shift) or null
  int G;
};
__device__ __forceinline__ void gn_coef8(const GnAffine& q, int b, int c0, int C, float* A1, float* A0) {
  const int g = c0 / (C / q.G);
  const float mean = q.stats[(b * q.G + g) * 2], rstd = q.stats[(b * q.G + g) * 2 + 1];
  float gm[8], bt[8], sc[8], sh[8];
  load_coef8(q.gamma + c0, gm);
  load_coef8(q.beta + c0, bt);
  if (q.ss) {
    load_coef8(q.ss + (int64_t)b * 2 * C + c0, sc);
    load_coef8(q.ss + (int64_t)b * 2 * C + C + c0, sh);
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] += 1.f;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) { sc[i] = 1.f; sh[i] = 0.f; }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float k = rstd * gm[i];
    A1[i] = k * sc[i];
    A0[i] = (bt[i] - mean * k) * sc[i] + sh[i];
  }
}

// (Round 3 measured two Infinity-Cache orders and removed them: the backward one sample at a time so gn_bwd_apply
// re-reads (dout, y) on-die -- whole step 132.0 -> 138.0 ms; gn_apply in reversed sample order -- neutral.)

// (Round 5: four rows per step with every load before the first store, GN_BATCH: whole step 61.58 / 61.83 ->
// 61.75 / 61.89 samples/s, inside the spread; removed -- profiles/r5j_gn_batch_ab.txt.)
// grid (nchunk, B): thread = (8-channel group c8, row lane rr), rows strided by 256/(C/8)
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ y, const GnAffine coef,
                                                       const T* __restrict__ res, T* __restrict__ out, int64_t rows_b,
                                                       int C, int nchunk) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int c8 = threadIdx.x % cv, rr = threadIdx.x / cv;
  if (rr >= rl) return;
  float A1[8], A0[8];
  gn_coef8(coef, b, c8 * 8, C, A1, A0);
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C + c8 * 8;
  int64_t r = r0 + rr;
#pragma unroll 4
  for (; r < r1; r += rl) {
    float v[8], rv[8];
    gl8(y + off + r * C, v);
    if (res) gl8(res + off + r * C, rv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float a = silu_t<T>(fmaf(v[i], A1[i], A0[i]));
      v[i] = res ? a + rv[i] : a;
    }
    gs8(out + off + r * C, v);
  }
}

// part[b][chunk][c] = (S1 = sum da, S3 = sum da*y, Sy = sum y)
template <typename T, bool NT = true>
__global__ __launch_bounds__(256) void gn_bwd_reduce_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                            const GnAffine coef, float* __restrict__ part,
                                                            int64_t rows_b, int C, int nchunk, int b0) {
  const int bl = blockIdx.y, b = bl + b0, chunk = blockIdx.x;
  const int cv = C / 8, rl = 256 / cv;
  const int tid = threadIdx.x;
  const int c8 = tid % cv, rr = tid / cv;
  float A1[8], A0[8];
  gn_coef8(coef, b, c8 * 8, C, A1, A0);
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C + c8 * 8;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s3[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sy[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < rl) {
#pragma unroll 4
    for (int64_t r = r0 + rr; r < r1; r += rl) {
      float v[8], d[8];
      if (NT) {
        gl8(y + off + r * C, v);
        gl8(dout + off + r * C, d);
      } else {  // default policy: the lines stay in the Infinity Cache for gn_bwd_apply's re-read
        load8(y + off + r * C, v);
        load8(dout + off + r * C, d);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float da = d[i] * dsilu_t<T>(fmaf(v[i], A1[i], A0[i]));
        s1[i] += da;
        s3[i] = fmaf(da, v[i], s3[i]);
        sy[i] += v[i];
      }
    }
  }
  // reduce over the lanes of a wave that share c8 (lane stride cv), then over the row groups in a
  // fixed order (deterministic)
  for (int o = cv; o < 64; o <<= 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s1[i] += __shfl_xor(s1[i], o, 64);
      s3[i] += __shfl_xor(s3[i], o, 64);
      sy[i] += __shfl_xor(sy[i], o, 64);
    }
  }
  __shared__ float red[3][1024];
  const int lane = tid & 63, wv = tid >> 6;
  const bool owner = lane < (cv < 64 ? cv : 64);          // holds the wave's sums for c8 = tid % cv
  const int ngroup = cv <= 64 ? 4 : 256 / cv;              // row groups left per c8
  const int grp = cv <= 64 ? wv : rr;
  for (int k = 0; k < ngroup; ++k) {
    if (owner && grp == k) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = c8 * 8 + i;
        if (k == 0) { red[0][c] = s1[i]; red[1][c] = s3[i]; red[2][c] = sy[i]; }
        else { red[0][c] += s1[i]; red[1][c] += s3[i]; red[2][c] += sy[i]; }
      }
    }
    __syncthreads();
  }
  float* o = part + ((int64_t)bl * nchunk + chunk) * C * 3;
  for (int c = tid; c < C; c += 256) {
    o[c * 3] = red[0][c];
    o[c * 3 + 1] = red[1][c];
    o[c * 3 + 2] = red[2][c];
  }
}

// grid (B, C/64), 256 threads = 64 channels x 4 chunk groups.  Per (b, c): S1, S3, Sy over the chunk
// partials; S2 = rstd*(S3 - mean*S1) = sum da*xhat -> dss[b] (d scale | d shift), parameter
// contributions pb[b][c] = ((1+scale)*S2, (1+scale)*S1, conv-bias sum dy), apply coefficients
// E[b][0..2][c]:  dy = da*E1 + y*E2 + E3.  Groups (C/G <= 64 channels) never straddle blocks.
constexpr int GNF_KG = 16;  // chunk groups of the bwd finalize (1024 threads: short partial-sum chains)
__global__ __launch_bounds__(1024) void gn_bwd_finalize_kernel(const float* __restrict__ part,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              const float* __restrict__ ss, float* __restrict__ dss,
                                                              float* __restrict__ pb, float* __restrict__ E, int C,
                                                              int G, int nchunk, double count, float rows_b, int b0) {
  const int bl = blockIdx.x, b = bl + b0;
  const int cl = threadIdx.x & 63, kg = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  __shared__ float red[GNF_KG][3][64];
  __shared__ float ga_[64], gb_[64];
  __shared__ float gA[64], gB[64];
  const int gsz = C / G;
  float s1 = 0.f, s3 = 0.f, sy = 0.f;
  if (c < C) {
    // four partials' loads in flight, summed in the same order as one at a time
    int k = kg;
    for (; k + 3 * GNF_KG < nchunk; k += 4 * GNF_KG) {
      float v[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* p = part + (((int64_t)bl * nchunk + k + u * GNF_KG) * C + c) * 3;
        v[u][0] = p[0];
        v[u][1] = p[1];
        v[u][2] = p[2];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s1 += v[u][0];
        s3 += v[u][1];
        sy += v[u][2];
      }
    }
    for (; k < nchunk; k += GNF_KG) {
      const float* p = part + (((int64_t)bl * nchunk + k) * C + c) * 3;
      s1 += p[0];
      s3 += p[1];
      sy += p[2];
    }
  }
  red[kg][0][cl] = s1;
  red[kg][1][cl] = s3;
  red[kg][2][cl] = sy;
  __syncthreads();
  float mean = 0.f, rstd = 0.f, sc = 1.f;
  if (kg == 0 && c < C) {
    s1 = s3 = sy = 0.f;
#pragma unroll
    for (int k = 0; k < GNF_KG; ++k) {  // fixed order (deterministic)
      s1 += red[k][0][cl];
      s3 += red[k][1][cl];
      sy += red[k][2][cl];
    }
    const int g = c / gsz;
    mean = stats[(b * G + g) * 2];
    rstd = stats[(b * G + g) * 2 + 1];
    const float s2 = rstd * (s3 - mean * s1);  // sum da * xhat
    sc = ss ? ss[(int64_t)b * 2 * C + c] + 1.f : 1.f;
    if (dss) {
      dss[(int64_t)b * 2 * C + c] = gamma[c] * s2 + beta[c] * s1;  // d scale
      dss[(int64_t)b * 2 * C + C + c] = s1;                        // d shift
    }
    pb[((int64_t)b * C + c) * 3] = sc * s2;      // dgamma contribution
    pb[((int64_t)b * C + c) * 3 + 1] = sc * s1;  // dbeta contribution
    ga_[cl] = gamma[c] * sc * s1;
    gb_[cl] = gamma[c] * sc * s2;
  }
  __syncthreads();
  const int ng = 64 / gsz;  // groups in this block (gsz <= 64)
  if ((int)threadIdx.x < ng && blockIdx.y * 64 + threadIdx.x * gsz < C) {
    double a = 0.0, q = 0.0;
    for (int j = threadIdx.x * gsz; j < (int)(threadIdx.x + 1) * gsz; ++j) { a += ga_[j]; q += gb_[j]; }
    gA[threadIdx.x] = (float)(a / count);
    gB[threadIdx.x] = (float)(q / count);
  }
  __syncthreads();
  if (kg == 0 && c < C) {
    const int gl = cl / gsz;
    // dy = rstd*(da*sc*gamma - A - (y-mean)*rstd*Bg)
    const float e1 = rstd * sc * gamma[c];
    const float e2 = -rstd * rstd * gB[gl];
    const float e3 = rstd * (mean * rstd * gB[gl] - gA[gl]);
    E[((int64_t)b * 3) * C + c] = e1;
    E[((int64_t)b * 3 + 1) * C + c] = e2;
    E[((int64_t)b * 3 + 2) * C + c] = e3;
    pb[((int64_t)b * C + c) * 3 + 2] = e1 * s1 + e2 * sy + rows_b * e3;  // sum over rows of dy
  }
}

// dgamma/dbeta/dbias (+)= sum_b pb[b] (fixed order over b), by one block of the apply kernel that follows the
// finalize (round 6: was its own launch, 38 per training step at 4.9 us)
struct GnParamGrad {
  const float* pb;
  float *dgamma, *dbeta, *dbias;
  int B, accumulate;
};
__device__ __forceinline__ void gn_param_grad_block(const GnParamGrad& pg, int C) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, q = 0.f, w = 0.f;
    for (int b = 0; b < pg.B; ++b) {
      a += pg.pb[((int64_t)b * C + c) * 3];
      q += pg.pb[((int64_t)b * C + c) * 3 + 1];
      w += pg.pb[((int64_t)b * C + c) * 3 + 2];
    }
    if (pg.dgamma) pg.dgamma[c] = pg.accumulate ? pg.dgamma[c] + a : a;
    if (pg.dbeta) pg.dbeta[c] = pg.accumulate ? pg.dbeta[c] + q : q;
    if (pg.dbias) pg.dbias[c] = pg.accumulate ? pg.dbias[c] + w : w;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                           const GnAffine coef, const float* __restrict__ E,
                                                           T* __restrict__ dy, int64_t rows_b, int C, int nchunk,
                                                           int b0, const GnParamGrad pg) {
  const int b = blockIdx.y + b0, chunk = blockIdx.x;
  if (blockIdx.x == 0 && blockIdx.y == 0) gn_param_grad_block(pg, C);
  const int cv = C / 8, rl = 256 / cv;
  const int c8 = threadIdx.x % cv, rr = threadIdx.x / cv;
  if (rr >= rl) return;
  float A1[8], A0[8], E1[8], E2[8], E3[8];
  gn_coef8(coef, b, c8 * 8, C, A1, A0);
  load_coef8(E + ((int64_t)b * 3) * C + c8 * 8, E1);
  load_coef8(E + ((int64_t)b * 3 + 1) * C + c8 * 8, E2);
  load_coef8(E + ((int64_t)b * 3 + 2) * C + c8 * 8, E3);
  const int64_t rpc = (rows_b + nchunk - 1) / nchunk;
  const int64_t r0 = chunk * rpc, r1 = min(rows_b, r0 + rpc);
  const int64_t off = (int64_t)b * rows_b * C + c8 * 8;
  int64_t r = r0 + rr;
#pragma unroll 4
  for (; r < r1; r += rl) {
    float v[8], d[8];
    gl8(y + off + r * C, v);
    gl8(dout + off + r * C, d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float da = d[i] * dsilu_t<T>(fmaf(v[i], A1[i], A0[i]));
      d[i] = fmaf(da, E1[i], fmaf(v[i], E2[i], E3[i]));
    }
    gs8(dy + off + r * C, d);
  }
}

template <typename F>
static int dispatch_dt(int dtype, F&& f) {
  if (dtype == CESM_DT_BF16) { f((bf16*)nullptr); return CESM_OK; }
  if (dtype == CESM_DT_F32) { f((float*)nullptr); return CESM_OK; }
  return CESM_EINVAL;
}

constexpr int GN_APPLY_ITERS = 8;  // row-iterations per thread of the streaming apply kernels: whole step 16 -> 8:
                                   // -0.5 ms (two calls, profiles/r3_gn_iters_ab.txt); 4 the same as 8, 32 +0.5 ms
static int gn_apply_chunks(int64_t rows_b, int C) {
  const int rl = 256 / (C / 8);
  int64_t n = rows_b / (rl * GN_APPLY_ITERS);
  if (n < 1) n = 1;
  if (n > 4096) n = 4096;
  return (int)n;
}

}  // namespace

extern "C" {

// y: [B][rows_b][C] (rows_b = F*H*W); writes stats[B][G][2] = (mean, rstd); ws >= max(B*256, 1024)*G*2 doubles
int cesm_gn_stats(int dtype, const void* y, float* stats, double* ws, int B, int64_t rows_b, int C, int G, float eps,
                  hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || C % G || (C / G) % 8) return CESM_EINVAL;
  const int nchunk = gn_nchunk(rows_b, C, B);
  dim3 grid(nchunk, B);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_stats_kernel<T><<<grid, 256, 0, stream>>>((const T*)y, ws, rows_b, C, G, nchunk);
  });
  if (rc) return rc;
  gn_finalize_kernel<<<B * G, 64, 0, stream>>>(ws, stats, B, G, nchunk, (double)rows_b * (C / G), eps);
  return cesm_launch_status();
}

// ss: [B][2C] (scale | shift) or null; res: residual [B*rows_b][C] or null; ws: >= 2*B*C floats
// part is consumed: at nslot >= 8192 the two-stage reduction writes its stage-1 block sums over the partials
int cesm_gn_stats_part(float* part, float* stats, int B, int64_t nslot, int C, int G, int64_t rows_b, float eps,
                       hipStream_t stream) {
  if (B <= 0 || G <= 0 || C % (4 * G) || nslot <= 0 || rows_b <= 0) return CESM_EINVAL;
  const int C4 = C / 4;
  if (nslot >= 8192 && C4 <= 256 && 256 % C4 == 0) {
    const int S = (int)(nslot / GNP_PER);  // >= 64 slots (>= 2 rows) per stage-1 block
    gn_part_stage1_kernel<<<dim3(S, B), 256, 0, stream>>>(reinterpret_cast<float2*>(part),
                                                          nslot, C4, S);
    gn_part_stage2_kernel<<<B * G, 64, 0, stream>>>(reinterpret_cast<const float2*>(part), stats, G, nslot, C4, S,
                                                    (double)rows_b * (C / G), eps);
    return cesm_launch_status();
  }
  gn_part_finalize_kernel<<<B * G, GNP_T, 0, stream>>>(reinterpret_cast<const float2*>(part), stats, G, nslot, C4,
                                                     (double)rows_b * (C / G), eps);
  return cesm_launch_status();
}

int cesm_gn_apply(int dtype, const void* y, const float* stats, const float* gamma, const float* beta,
                  const float* ss, const void* res, void* out, float* ws, int B, int64_t rows_b, int C, int G,
                  hipStream_t stream) {
  if (C % 8 || C / 8 > 256 || C % G) return CESM_EINVAL;
  const GnAffine aff{stats, gamma, beta, ss, G};
  (void)ws;
  const int nch = gn_apply_chunks(rows_b, C);
  int rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_apply_kernel<T><<<dim3(nch, B), 256, 0, stream>>>((const T*)y, aff, (const T*)res, (T*)out, rows_b, C, nch);
  });
  if (rc) return rc;
  return cesm_launch_status();
}

// Backward of out = silu(GN(y)*(1+scale)+shift) (+res).  Writes dy, dss [B][2C] (if non-null),
// dgamma/dbeta and the producing conv's bias gradient dbias = sum dy (each nullable; accumulate flag).
// ws: float workspace >= B*1024*C*3 + B*C*3 + B*C*5 floats.
int cesm_gn_bwd(int dtype, const void* dout, const void* y, const float* stats, const float* gamma,
                const float* beta, const float* ss, void* dy, float* dss, float* dgamma, float* dbeta, float* dbias,
                float* ws, int B, int64_t rows_b, int C, int G, int accumulate, hipStream_t stream) {
  if (C % 8 || C / 8 > 128 || C % G || C / G > 64 || 64 % (C / G) || G > 64) return CESM_EINVAL;
  const double count = (double)rows_b * (C / G);
  const GnAffine aff{stats, gamma, beta, ss, G};
  const int nch = gn_apply_chunks(rows_b, C);
  float* part = ws;
  int rc;
  const int nchunk = gn_nchunk(rows_b, C, B);
  float* pb = part + (int64_t)B * nchunk * C * 3;
  float* coef = pb + (int64_t)B * C * 3;
  float* E = coef + (int64_t)B * C * 2;
  rc = dispatch_dt(dtype, [&](auto* tp) {
    using T = std::remove_pointer_t<decltype(tp)>;
    gn_bwd_reduce_kernel<T><<<dim3(nchunk, B), 256, 0, stream>>>((const T*)dout, (const T*)y, aff, part, rows_b, C,
                                                                 nchunk, 0);
    gn_bwd_finalize_kernel<<<dim3(B, (unsigned)cdiv(C, 64)), 64 * GNF_KG, 0, stream>>>(part, stats, gamma, beta, ss, dss, pb,
                                                                               E, C, G, nchunk, count, (float)rows_b, 0);
    gn_bwd_apply_kernel<T><<<dim3(nch, B), 256, 0, stream>>>((const T*)dout, (const T*)y, aff, E, (T*)dy, rows_b, C,
                                                             nch, 0, GnParamGrad{pb, dgamma, dbeta, dbias, B, accumulate});
  });
  if (rc) return rc;
  return cesm_launch_status();
}

}  // extern "C"
