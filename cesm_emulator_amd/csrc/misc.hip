// Small ops of the training step:
//  * time embedding + small linears (video_net.py:101-113 SinusoidalPosEmb, :651-656 time_mlp,
//    :238-242 ResnetBlock.mlp = SiLU -> Linear) — M = batch rows, fp32
//  * diffusion q_sample + MSE loss and its gradient (model.py:196-208)
//  * global grad-norm clip (torch/nn/utils/clip_grad.py:165-180) + fused AdamW
//    (torch/optim/adam.py:417-547, decoupled weight decay) over one flat fp32 parameter buffer
//  * dtype casts and the training-window gather (dataset_single_member.py:168-196)
#include "common.h"
#include "cesm_hip.h"

namespace {

__global__ void sinusoidal_kernel(const int64_t* __restrict__ t, float* __restrict__ emb, int B, int dim) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int half = dim / 2;
  if (i >= B * half) return;
  const int b = i / half, k = i % half;
  const float step = logf(10000.f) / (float)(half - 1);
  const float fr = expf((float)k * -step);
  const float a = (float)t[b] * fr;
  emb[b * dim + k] = sinf(a);
  emb[b * dim + half + k] = cosf(a);
}

// y[r][o] = bias[o] + sum_i act(x[r][i]) * W[o][i]; act = silu if silu_in
// one wave per output feature o (coalesced W row), rows r looped (R = batch, small)
__global__ void linear_small_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                        const float* __restrict__ bias, float* __restrict__ y, int R, int I, int O,
                                        int silu_in) {
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= O) return;
  const float* wr = w + (int64_t)o * I;
  for (int r0 = 0; r0 < R; r0 += 8) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int i = lane; i < I; i += 64) {
      const float wv = wr[i];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (r0 + k < R) {
          const float xv = x[(int64_t)(r0 + k) * I + i];
          s[k] = fmaf(silu_in ? silu_p(xv) : xv, wv, s[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (r0 + k >= R) break;
      const float t = wave_sum(s[k]);
      if (lane == 0) y[(int64_t)(r0 + k) * O + o] = t + (bias ? bias[o] : 0.f);
    }
  }
}

// dx[r][i] (+)= act'(x) * sum_o dy[r][o] W[o][i]
// block = 4 waves x 64 lanes: lane <-> i (64 consecutive), wave <-> quarter of the o range
__global__ __launch_bounds__(256) void linear_small_dx_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ dy, float* __restrict__ dx,
                                                              int R, int I, int O, int silu_in, int accumulate) {
  // block = 16 inputs i x 16 slices of the O reduction (short dependent chains: O/16 FMAs per thread);
  // the 16 i of a slice read 64 consecutive bytes of each W row
  __shared__ float red[16][17];
  const int r = blockIdx.y;
  const int il = threadIdx.x & 15, os = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + il;
  float s = 0.f;
  if (i < I) {
#pragma unroll 8
    for (int o = os; o < O; o += 16) s = fmaf(dy[(int64_t)r * O + o], w[(int64_t)o * I + i], s);
  }
  red[os][il] = s;
  __syncthreads();
  if (os == 0 && i < I) {
    s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][il];
    const int64_t t = (int64_t)r * I + i;
    if (silu_in) s *= dsilu_p(x[t]);
    dx[t] = accumulate ? dx[t] + s : s;
  }
}

// dW[o][i] (+)= sum_r dy[r][o] act(x[r][i]); db[o] (+)= sum_r dy[r][o]
__global__ void linear_small_dw_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                       float* __restrict__ dw, float* __restrict__ db, int R, int I, int O,
                                       int silu_in, int accumulate) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < O * I) {
    const int o = t / I, i = t % I;
    float s = 0.f;
    for (int r = 0; r < R; ++r) {
      const float xv = silu_in ? silu_p(x[(int64_t)r * I + i]) : x[(int64_t)r * I + i];
      s = fmaf(dy[(int64_t)r * O + o], xv, s);
    }
    dw[t] = accumulate ? dw[t] + s : s;
  }
  if (db && t < O) {
    float s = 0.f;
    for (int r = 0; r < R; ++r) s += dy[(int64_t)r * O + t];
    db[t] = accumulate ? db[t] + s : s;
  }
}

// x_t = a[t_b] x0 + s[t_b] noise   (x0, noise, x_t: [B][HW] fp32)
__global__ void q_sample_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                const int64_t* __restrict__ t, const float* __restrict__ sa,
                                const float* __restrict__ s1a, float* __restrict__ xt, int B, int64_t HW) {
  const int64_t n = (int64_t)B * HW;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / HW);
    const int64_t ti = t[b];
    xt[e] = sa[ti] * x0[e] + s1a[ti] * noise[e];
  }
}

// DDPM ancestral step (model.py:168-183), fused:
//   x_{t-1} = r_t (x_t - (b_t / s1_t) eps) + sqrt(pv_t) z
// with the reference's operation order and no contraction (agrees with the eager torch expression to
// fp32 rounding).  pv_0 = 0 (alphas_cumprod_prev[0] = 1), so the t = 0 step adds no noise either way;
// z == nullptr skips the noise term (the reference's `(t == 0).all()` branch).  out may alias x.
__global__ void ddpm_step_kernel(const float* __restrict__ x, const float* __restrict__ eps,
                                 const float* __restrict__ z, const int64_t* __restrict__ t,
                                 const float* __restrict__ sra, const float* __restrict__ betas,
                                 const float* __restrict__ s1a, const float* __restrict__ pv, float* out, int B,
                                 int64_t HW) {
  const int64_t n = (int64_t)B * HW;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ti = t[e / HW];
    const float c = __fdiv_rn(betas[ti], s1a[ti]);
    float m = __fmul_rn(sra[ti], __fsub_rn(x[e], __fmul_rn(c, eps[e])));
    if (z) m = __fadd_rn(m, __fmul_rn(__fsqrt_rn(pv[ti]), z[e]));
    out[e] = m;
  }
}

// loss partials: part[blk] = sum (pred - noise)^2
__global__ void mse_partial_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                   float* __restrict__ part, int64_t n) {
  __shared__ float red[256];
  float s = 0.f;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const float d = pred[e] - tgt[e];
    s = fmaf(d, d, s);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void mse_final_kernel(const float* __restrict__ part, float* __restrict__ loss, int nblk, int64_t n) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int k = 0; k < nblk; ++k) s += part[k];
  loss[0] = (float)(s / (double)n);
}

// dpred = gscale[0] * 2 (pred - noise) / n
__global__ void mse_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                               const float* __restrict__ gscale, float* __restrict__ dpred, int64_t n) {
  const float c = 2.f * gscale[0] / (float)n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    dpred[e] = c * (pred[e] - tgt[e]);
}

// ---- grad norm + clip + AdamW over flat fp32 buffers
__global__ void sumsq_partial_kernel(const float* __restrict__ g, double* __restrict__ part, int64_t n) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const float v = g[e];
    s += (double)v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// info[0] = total norm, info[1] = clip coef (clamped to 1), info[2] = 1 if finite (norm & loss)
__global__ void clip_coef_kernel(const double* __restrict__ part, int nblk, float max_norm,
                                 const float* __restrict__ loss, float* __restrict__ info) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int k = 0; k < nblk; ++k) s += part[k];
  const float norm = (float)sqrt(s);
  info[0] = norm;
  float coef = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
  info[1] = coef < 1.f ? coef : 1.f;
  const bool fin = isfinite(norm) && (loss == nullptr || isfinite(loss[0]));
  info[2] = fin ? 1.f : 0.f;
}

// step counter kept on the device: advanced only when the step is finite (info[2]), so a skipped step
// leaves the bias corrections and the saved "step" consistent with exp_avg / exp_avg_sq (as
// torch.optim.AdamW, which never sees a skipped step).  info[3] = the step number this update uses.
__global__ void adamw_step_kernel(float* __restrict__ info, int* __restrict__ step) {
  if (threadIdx.x != 0) return;
  const int s = step[0] + ((info[2] != 0.f) ? 1 : 0);
  step[0] = s;
  info[3] = (float)s;
}

__global__ void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, const float* __restrict__ info, int64_t n, float lr, float b1,
                             float b2, float eps, float wd, int use_clip) {
  if (info[2] == 0.f) return;  // non-finite loss/grad: no update (train step raises)
  const float coef = use_clip ? info[1] : 1.f;
  const float st = info[3];
  const float bc1 = 1.f - powf(b1, st);
  const float bc2_sqrt = sqrtf(1.f - powf(b2, st));
  const float step_size = lr / bc1;
  const float decay = 1.f - lr * wd;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const float gr = g[e] * coef;
    if (use_clip) g[e] = gr;
    const float pv = p[e] * decay;
    const float mv = m[e] + (1.f - b1) * (gr - m[e]);
    const float vv = v[e] * b2 + (1.f - b2) * gr * gr;
    m[e] = mv;
    v[e] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    p[e] = pv - step_size * (mv / denom);
  }
}

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out, int64_t n8) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    float x[8], y[8];
    load8(a + e * 8, x);
    load8(b + e * 8, y);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] += y[i];
    store8(out + e * 8, x);
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    y[e] = from_f<TO>(to_f(x[e]));
}

// Training-window gather (dataset_single_member.py:168-196) from arrays resident in device or
// pinned host memory: cond/tgt [T][M][H][W] fp32.  Per item i: (t0, m, anchor, rev, ci, cj):
// cond_win[i][0][k][y][x] = cond[times[k]][m][ci+y][cj+x], x0[i][0][y][x] = tgt[anchor][m][..]
// times[k] = t0 + k, with the "reverse both halves around the centre" augmentation when rev.
__global__ void window_gather_kernel(const float* __restrict__ cond, const float* __restrict__ tgt,
                                     const int64_t* __restrict__ items, float* __restrict__ cwin,
                                     float* __restrict__ x0, int nitems, int K, int M, int H, int W, int h, int w,
                                     int center) {
  const int64_t per = (int64_t)(K + 1) * h * w;
  const int64_t total = per * nitems;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int it = (int)(e / per);
    int64_t r = e - (int64_t)it * per;
    const int k = (int)(r / ((int64_t)h * w));
    r -= (int64_t)k * h * w;
    const int y = (int)(r / w), x = (int)(r % w);
    const int64_t* d = items + it * 6;
    const int64_t t0 = d[0], m = d[1], anchor = d[2], rev = d[3], ci = d[4], cj = d[5];
    if (k < K) {
      int kk = k;
      if (rev) {
        if (center) {
          const int mid = K / 2;
          if (k < mid) kk = mid - 1 - k;
          else if (k > mid) kk = K - 1 - (k - mid - 1);
        } else {
          kk = K - 1 - k;
        }
      }
      const int64_t tt = t0 + kk;
      cwin[(((int64_t)it * K + k) * h + y) * w + x] = cond[(((tt * M + m) * H) + ci + y) * W + cj + x];
    } else {
      x0[((int64_t)it * h + y) * w + x] = tgt[(((anchor * M + m) * H) + ci + y) * W + cj + x];
    }
  }
}

// One-GPU stand-in for the RCCL all-reduce kernels of an overlapped data-parallel backward (a measurement aid,
// tools/overlap_sim.py): nblk blocks that each take a whole CU (the launch asks for the CU's full LDS) and idle on the
// real-time clock (100 MHz) for `ticks`, as an RCCL channel block holds its CU for a bucket's transfer time.
__global__ __launch_bounds__(64) void hold_cu_kernel(long long ticks) {
  extern __shared__ char hold_lds[];
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (ticks < 0) hold_lds[threadIdx.x] = 0;  // never taken: keeps the allocation referenced
}

}  // namespace

extern "C" {

// The header's CESM_ABI_VERSION this library was compiled against (hosts compare it with their own header)
int cesm_abi_version(void) { return CESM_ABI_VERSION; }

int cesm_hold_cus(int nblk, float usec, hipStream_t stream) {
  if (nblk < 1 || !(usec >= 0.f)) return CESM_EINVAL;
  constexpr int kLds = 160 * 1024;
  // the attribute is per device: set it on every call (cheap) rather than caching one process-wide flag, which left a
  // second device of the process without it
  if (hipFuncSetAttribute((const void*)hold_cu_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kLds) != hipSuccess)
    return CESM_ELAUNCH;
  hold_cu_kernel<<<nblk, 64, kLds, stream>>>((long long)(usec * 100.f));
  return cesm_launch_status();
}

int cesm_sinusoidal(const int64_t* t, float* emb, int B, int dim, hipStream_t stream) {
  sinusoidal_kernel<<<(unsigned)cdiv(B * (dim / 2), 256), 256, 0, stream>>>(t, emb, B, dim);
  return cesm_launch_status();
}

int cesm_linear_small_fwd(const float* x, const float* w, const float* bias, float* y, int R, int I, int O,
                          int silu_in, hipStream_t stream) {
  linear_small_fwd_kernel<<<(unsigned)cdiv(O, 4), 256, 0, stream>>>(x, w, bias, y, R, I, O, silu_in);
  return cesm_launch_status();
}

int cesm_linear_small_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, int R,
                          int I, int O, int silu_in, int accumulate_dx, int accumulate_w, hipStream_t stream) {
  if (dx)
    linear_small_dx_kernel<<<dim3((unsigned)cdiv(I, 16), R), 256, 0, stream>>>(x, w, dy, dx, R, I, O, silu_in,
                                                                               accumulate_dx);
  if (dw)
    linear_small_dw_kernel<<<(unsigned)cdiv((int64_t)O * I, 256), 256, 0, stream>>>(x, dy, dw, db, R, I, O, silu_in,
                                                                                    accumulate_w);
  return cesm_launch_status();
}

int cesm_q_sample(const float* x0, const float* noise, const int64_t* t, const float* sa, const float* s1a,
                  float* xt, int B, int64_t HW, hipStream_t stream) {
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv((int64_t)B * HW, 256), 4096);
  q_sample_kernel<<<grid, 256, 0, stream>>>(x0, noise, t, sa, s1a, xt, B, HW);
  return cesm_launch_status();
}

int cesm_ddpm_step(const float* x, const float* eps, const float* z, const int64_t* t, const float* sqrt_recip_alphas,
                   const float* betas, const float* sqrt_one_minus_ac, const float* posterior_variance, float* out,
                   int B, int64_t HW, hipStream_t stream) {
  if (B < 1 || HW < 1) return CESM_EINVAL;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv((int64_t)B * HW, 256), 4096);
  ddpm_step_kernel<<<grid, 256, 0, stream>>>(x, eps, z, t, sqrt_recip_alphas, betas, sqrt_one_minus_ac,
                                             posterior_variance, out, B, HW);
  return cesm_launch_status();
}

// loss[0] = mean((pred-tgt)^2); part: 512 floats
int cesm_mse(const float* pred, const float* tgt, float* loss, float* part, int64_t n, hipStream_t stream) {
  const int nblk = 512;
  mse_partial_kernel<<<nblk, 256, 0, stream>>>(pred, tgt, part, n);
  mse_final_kernel<<<1, 64, 0, stream>>>(part, loss, nblk, n);
  return cesm_launch_status();
}

int cesm_mse_bwd(const float* pred, const float* tgt, const float* gscale, float* dpred, int64_t n,
                 hipStream_t stream) {
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, 256), 4096);
  mse_bwd_kernel<<<grid, 256, 0, stream>>>(pred, tgt, gscale, dpred, n);
  return cesm_launch_status();
}

// info[3] (device): norm, clip coef, finite flag.  part: 1024 doubles.
int cesm_grad_norm(const float* g, int64_t n, float max_norm, const float* loss, double* part, float* info,
                   hipStream_t stream) {
  const int nblk = 1024;
  sumsq_partial_kernel<<<nblk, 256, 0, stream>>>(g, part, n);
  clip_coef_kernel<<<1, 64, 0, stream>>>(part, nblk, max_norm, loss, info);
  return cesm_launch_status();
}

int cesm_adamw(float* p, float* g, float* m, float* v, float* info, int* step, int64_t n, float lr, float b1,
               float b2, float eps, float wd, int use_clip, hipStream_t stream) {
  if (!info || !step) return CESM_EINVAL;
  adamw_step_kernel<<<1, 64, 0, stream>>>(info, step);
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, 256), 8192);
  adamw_kernel<<<grid, 256, 0, stream>>>(p, g, m, v, info, n, lr, b1, b2, eps, wd, use_clip);
  return cesm_launch_status();
}

int cesm_add(int dtype, const void* a, const void* b, void* out, int64_t n, hipStream_t stream) {
  if (n % 8) return CESM_EINVAL;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n / 8, 256), 8192);
  if (dtype == CESM_DT_BF16)
    add_kernel<bf16><<<grid, 256, 0, stream>>>((const bf16*)a, (const bf16*)b, (bf16*)out, n / 8);
  else if (dtype == CESM_DT_F32)
    add_kernel<float><<<grid, 256, 0, stream>>>((const float*)a, (const float*)b, (float*)out, n / 8);
  else
    return CESM_EINVAL;
  return cesm_launch_status();
}

int cesm_cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, hipStream_t stream) {
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n, 256), 8192);
  if (dtype_in == CESM_DT_F32 && dtype_out == CESM_DT_BF16)
    cast_kernel<float, bf16><<<grid, 256, 0, stream>>>((const float*)x, (bf16*)y, n);
  else if (dtype_in == CESM_DT_BF16 && dtype_out == CESM_DT_F32)
    cast_kernel<bf16, float><<<grid, 256, 0, stream>>>((const bf16*)x, (float*)y, n);
  else if (dtype_in == CESM_DT_F32 && dtype_out == CESM_DT_F32)
    cast_kernel<float, float><<<grid, 256, 0, stream>>>((const float*)x, (float*)y, n);
  else
    return CESM_EINVAL;
  return cesm_launch_status();
}

int cesm_window_gather(const float* cond, const float* tgt, const int64_t* items, float* cwin, float* x0,
                       int nitems, int K, int M, int H, int W, int h, int w, int center, hipStream_t stream) {
  const int64_t total = (int64_t)(K + 1) * h * w * nitems;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(total, 256), 8192);
  window_gather_kernel<<<grid, 256, 0, stream>>>(cond, tgt, items, cwin, x0, nitems, K, M, H, W, h, w, center);
  return cesm_launch_status();
}

}  // extern "C"
