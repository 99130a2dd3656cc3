// Implicit-GEMM convolutions on MFMA for the video_net U-Net (all convs are per-frame
// (1,k,k), so the frame axis folds into the batch: Nb = B*F "images").
//
// Activations are channels-last [Nb][H][W][C].  One generic forward kernel covers every
// conv in the net and every data-gradient (replaces ATen conv3d / conv_transpose3d at
// video_net.py:215 (Block.proj), :246 (res_conv), :61-62 (Downsample), :65-66 (Upsample),
// :380/:381 + :322/:323 (attention projections, as 1x1 convs), and their dgrads):
//
//   out[m=(n,oy,ox)][co] = bias[co] + res[m][co]
//                        + sum_{ky,kx,ci} W[co][ky*KW+kx][ci] * X[n][iy][ix][ci]
//   iy = (oy*S - P + ky) / U   (only when (oy*S - P + ky) % U == 0), likewise ix.
//
// U = 1 is an ordinary strided conv; U = 2 with flipped taps is a stride-2 transposed conv.
// The GEMM is computed transposed (D = W * X^T) so each lane's accumulator holds 4
// consecutive output channels of one pixel -> vectorised channels-last stores.
//
// Weight gradients use a second MFMA kernel (pixel axis = MFMA K) that writes fp32 split-K
// slabs, reduced deterministically by conv_wgrad_reduce into the PyTorch weight layout.
#include "common.h"
#include "cesm_hip.h"

namespace {

struct ConvGeom {
  int Nb, Hi, Wi, Ho, Wo;
  int C1, C2;       // input channels from source 1 / source 2 (concat on channel axis)
  int Cout, Co1;    // output channels; [0,Co1) -> y1, [Co1,Cout) -> y2
  int KH, KW, S, P, U;
  int wch = 0;      // packed weights in the chunked layout (wpk_chunked)
};

// Packed conv weights (cesm_conv_pack): row-major Wp[co][tap][ci], or -- bf16 3x3 / 4x4 weights with Cout % 64 == 0 and
// Cin % 32 == 0, the operands of the halo convs -- "chunked": one contiguous block per (64-co block, 32-channel chunk)
// holding [tap][co % 64][ci % 32]: the weight tile a halo conv stages per K step is one contiguous block (3x3) or
// 4-KB runs per live tap (4x4 stride-2), where the row-major layout gave 64-B pieces at a stride of Cin * 2 bytes.
// The halo conv micro ran 7-22 % faster at levels 1-3, the step's halo conv calls 2-8 % (profiles/r6late_h3_*.txt).
__host__ __device__ inline bool wpk_chunked(bool bf16_dtype, int Cout, int Cin, int KH, int KW) {
  return bf16_dtype && ((KH == 3 && KW == 3) || (KH == 4 && KW == 4)) && Cout % 64 == 0 && Cin % 32 == 0;
}
__host__ __device__ inline int64_t wpk_index(bool chunked, int co, int tap, int ci, int Cin, int NT) {
  if (!chunked) return ((int64_t)co * NT + tap) * Cin + ci;
  return ((((int64_t)(co >> 6) * (Cin >> 5) + (ci >> 5)) * NT + tap) * 64 + (co & 63)) * 32 + (ci & 31);
}

__device__ __forceinline__ bool tap_src(const ConvGeom& g, int oy, int ox, int ky, int kx, int& iy, int& ix) {
  int ny = oy * g.S - g.P + ky;
  int nx = ox * g.S - g.P + kx;
  if (g.U != 1) {
    if ((ny % g.U) != 0 || (nx % g.U) != 0) return false;  // negative remainders are non-zero too
    ny /= g.U;
    nx /= g.U;
  }
  iy = ny;
  ix = nx;
  return (unsigned)ny < (unsigned)g.Hi && (unsigned)nx < (unsigned)g.Wi;
}

// ----------------------------------------------------------------------------------------
// forward / dgrad kernel
// ----------------------------------------------------------------------------------------
constexpr int BK = 32;       // K per staging step (channels of one tap)
constexpr int BMP = 128;     // pixels per block

template <typename T> struct KCfg;
template <> struct KCfg<bf16> { static constexpr int VEC = 8; static constexpr int LDW = 40; };   // 80-B rows
template <> struct KCfg<float> { static constexpr int VEC = 4; static constexpr int LDW = 36; };  // 144-B rows

// PAR (U = 2, S = 1, even KH/KW, even Ho/Wo): parity-blocked transposed conv.  Output pixels with
// (oy, ox) = (2a + py, 2b + px) only receive taps ky = (P - py) mod 2 + 2i, kx = (P - px) mod 2 + 2j,
// so each block holds pixels of ONE parity class (blockIdx.y = parity * bpp + tile; M = pixels per
// class) and loops over its KH*KW/4 live taps instead of all KH*KW (3/4 of which gather zeros).
template <typename T, int BN, bool PAR = false>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const T* __restrict__ x1, const T* __restrict__ x2,
                                                       const T* __restrict__ w, const float* __restrict__ bias,
                                                       const T* __restrict__ res, const T* __restrict__ res2,
                                                       T* __restrict__ y1, T* __restrict__ y2, ConvGeom g,
                                                       int64_t M, int bpp = 0) {
  constexpr int VEC = KCfg<T>::VEC;
  constexpr int LDW = KCfg<T>::LDW;
  constexpr int VPR = BK / VEC;          // vectors per row
  constexpr int RPP = 256 / VPR;         // rows per pass
  constexpr int PX_PASS = BMP / RPP;     // pixel-tile passes per thread
  constexpr int W_PASS = BN / RPP;       // weight-tile passes per thread
  constexpr int TM = BN / 32;            // 16-row co tiles per wave (wave covers BN/2 co)
  constexpr int TN = 4;                  // 16-col pixel tiles per wave (wave covers 64 px)

  __shared__ __attribute__((aligned(16))) T lds[2][(BMP + BN) * LDW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  // grid.x = output-channel tile (fast): the Cout/BN blocks sharing one pixel tile run adjacently,
  // so the im2col tile is re-read from L2 instead of HBM
  const int par = PAR ? (int)blockIdx.y / bpp : 0;
  const int py = par >> 1, px = par & 1;
  const int64_t m0 = (int64_t)(PAR ? (int)blockIdx.y - par * bpp : (int)blockIdx.y) * BMP;
  const int n0 = blockIdx.x * BN;
  const int Cin = g.C1 + g.C2;
  const int csteps = Cin / BK;
  const int ntap = PAR ? (g.KH / 2) * (g.KW / 2) : g.KH * g.KW;
  const int ksteps = ntap * csteps;
  const int ky0 = PAR ? (((g.P - py) % 2) + 2) % 2 : 0;
  const int kx0 = PAR ? (((g.P - px) % 2) + 2) % 2 : 0;
  const int Wg = PAR ? g.Wo / 2 : g.Wo, Hg = PAR ? g.Ho / 2 : g.Ho;  // pixel grid enumerated by m

  // per-thread staging rows
  const int vrow = tid / VPR, vk = (tid % VPR) * VEC;
  int pn[PX_PASS], poy[PX_PASS], pox[PX_PASS];
  bool pval[PX_PASS];
#pragma unroll
  for (int p = 0; p < PX_PASS; ++p) {
    const int64_t m = m0 + vrow + p * RPP;
    pval[p] = m < M;
    const int64_t mm = pval[p] ? m : 0;
    pox[p] = (int)(mm % Wg);
    const int64_t t = mm / Wg;
    poy[p] = (int)(t % Hg);
    pn[p] = (int)(t / Hg);
    if constexpr (PAR) {
      poy[p] = 2 * poy[p] + py;
      pox[p] = 2 * pox[p] + px;
    }
  }

  float xr[PX_PASS][VEC];
  float wreg[W_PASS][VEC];

  auto gload = [&](int ks) {
    const int t = ks / csteps;
    const int c0 = (ks - t * csteps) * BK;
    int ky, kx;
    if constexpr (PAR) {
      const int hw = g.KW / 2;
      ky = ky0 + 2 * (t / hw);
      kx = kx0 + 2 * (t - (t / hw) * hw);
    } else {
      ky = t / g.KW;
      kx = t - ky * g.KW;
    }
    const int tap = ky * g.KW + kx;
    const T* src;
    int cs, cc;
    if (c0 < g.C1) { src = x1; cs = g.C1; cc = c0; } else { src = x2; cs = g.C2; cc = c0 - g.C1; }
#pragma unroll
    for (int p = 0; p < PX_PASS; ++p) {
      int iy, ix;
      if (pval[p] && tap_src(g, poy[p], pox[p], ky, kx, iy, ix)) {
        const T* ptr = src + ((((int64_t)pn[p] * g.Hi + iy) * g.Wi + ix) * cs + cc + vk);
        if constexpr (VEC == 8) load8(ptr, xr[p]); else load4(ptr, xr[p]);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) xr[p][i] = 0.f;
      }
    }
#pragma unroll
    for (int p = 0; p < W_PASS; ++p) {
      const int co = n0 + vrow + p * RPP;
      const T* ptr = w + wpk_index(g.wch, co, tap, c0 + vk, Cin, g.KH * g.KW);
      if constexpr (VEC == 8) load8(ptr, wreg[p]); else load4(ptr, wreg[p]);
    }
  };
  auto sstore = [&](int buf) {
    T* A = lds[buf];              // weights  [BN][LDW]
    T* B = lds[buf] + BN * LDW;   // pixels   [BMP][LDW]
#pragma unroll
    for (int p = 0; p < W_PASS; ++p) {
      T* d = A + (vrow + p * RPP) * LDW + vk;
      if constexpr (VEC == 8) store8(d, wreg[p]); else store4(d, wreg[p]);
    }
#pragma unroll
    for (int p = 0; p < PX_PASS; ++p) {
      T* d = B + (vrow + p * RPP) * LDW + vk;
      if constexpr (VEC == 8) store8(d, xr[p]); else store4(d, xr[p]);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();

  const int lr = lane & 15, lg = lane >> 4;
  for (int ks = 0; ks < ksteps; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < ksteps) gload(ks + 1);
    const T* A = lds[buf];
    const T* B = lds[buf] + BN * LDW;
    if constexpr (sizeof(T) == 2) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + (wr * (BN / 2) + i * 16 + lr) * LDW + lg * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(B + (wc * 64 + j * 16 + lr) * LDW + lg * 8);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      // fp32: lane holds k = 16h + 4*lg + s; the same permutation on both operands
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const f32x4*>(A + (wr * (BN / 2) + i * 16 + lr) * LDW + h * 16 + lg * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const f32x4*>(B + (wc * 64 + j * 16 + lr) * LDW + h * 16 + lg * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
      }
    }
    if (ks + 1 < ksteps) sstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds co = base + 4*lg + r (r=0..3) of pixel m
  const int Co2 = g.Cout - g.Co1;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int64_t m = m0 + wc * 64 + j * 16 + lr;
    if (m >= M) continue;
    if constexpr (PAR) {  // class-local index -> output pixel
      const int64_t b = m % Wg, t = m / Wg, a = t % Hg, n = t / Hg;
      m = (n * g.Ho + 2 * a + py) * g.Wo + 2 * b + px;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = n0 + wr * (BN / 2) + i * 16 + lg * 4;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bias[co + r];
      }
      if (co < g.Co1) {
        if (res) {
          float rv[4];
          load4(res + m * g.Co1 + co, rv);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += rv[r];
        }
        store4(y1 + m * g.Co1 + co, v);
      } else {
        if (res2) {
          float rv[4];
          load4(res2 + m * Co2 + (co - g.Co1), rv);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += rv[r];
        }
        store4(y2 + m * Co2 + (co - g.Co1), v);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// Conv epilogue loads, issued together and unpredicated.  Under lane predicates (pixel valid,
// channel half, residual present) every bias / residual load became a branch with its own
// vmcnt(0), i.e. one full memory round trip per (pixel group, channel tile) in sequence.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ void epi_bias(const float* __restrict__ bias, int co, float (&bv)[4]) {
  if (bias) {  // uniform (kernel argument)
    load4(bias + co, bv);
  } else {
    bv[0] = bv[1] = bv[2] = bv[3] = 0.f;
  }
}
// residual of output pixel m (ok: inside the image), channels co..co+3, from res (co < Co1) or res2;
// kept as raw bf16 (2 registers) until the epilogue adds it
__device__ __forceinline__ bf16x4 epi_res(const bf16* __restrict__ res, const bf16* __restrict__ res2, int64_t m, int co,
                                          int Co1, int Co2, bool ok) {
  const bool first = co < Co1;
  const bf16* rp = first ? res : res2;
  const bool use = ok && rp != nullptr;
  const bf16* base = use ? rp : (res ? res : res2);  // some valid address; the value is discarded
  const int64_t off = use ? (first ? m * Co1 + co : m * Co2 + (co - Co1)) : 0;
  const bf16x4 t = *reinterpret_cast<const bf16x4*>(base + off);
  return use ? t : bf16x4{};
}
__device__ __forceinline__ float b2f(bf16x4 v, int r) { return (float)v[r]; }

// ----------------------------------------------------------------------------------------
// bf16 generic implicit GEMM (strided down-sampling convs, transposed up-sampling convs in parity
// blocks, their data gradients, every conv the halo / 1x1 kernels do not take).  Same tiling and
// tap/parity enumeration as conv_fwd_kernel, but
//   * the im2col and weight tiles stay bf16 in registers (raw 16-B loads: no f32 round trip) and
//     are loaded TWO K-steps ahead (each step is only 16 MFMAs per wave, far shorter than a global
//     load's latency);
//   * LDS rows are 64 B with the 16-B chunk index XORed with bit 2 of the row (conflict-free
//     ds_read_b128 over any 16 consecutive rows; the 80-B padded rows ran 2-3-way conflicted).
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ int gx_off(int row, int ch) { return row * 32 + ((ch ^ ((row >> 1) & 2)) << 3); }

template <int BN, bool PAR = false>
__global__ __launch_bounds__(256) void conv_fwd_bf16_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                            const bf16* __restrict__ w, const float* __restrict__ bias,
                                                            const bf16* __restrict__ res, const bf16* __restrict__ res2,
                                                            bf16* __restrict__ y1, bf16* __restrict__ y2, ConvGeom g,
                                                            int64_t M, int bpp = 0) {
  constexpr int VPR = BK / 8;            // 16-B vectors per 32-channel row
  constexpr int RPP = 256 / VPR;         // rows per pass
  constexpr int PX_PASS = BMP / RPP;
  constexpr int W_PASS = BN / RPP;
  constexpr int TM = BN / 32;
  constexpr int TN = 4;
  __shared__ __attribute__((aligned(16))) bf16 lds[2][(BMP + BN) * 32];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int par = PAR ? (int)blockIdx.y / bpp : 0;
  const int py = par >> 1, px = par & 1;
  const int64_t m0 = (int64_t)(PAR ? (int)blockIdx.y - par * bpp : (int)blockIdx.y) * BMP;
  const int n0 = blockIdx.x * BN;
  const int Cin = g.C1 + g.C2;
  const int csteps = Cin / BK;
  const int ntap = PAR ? (g.KH / 2) * (g.KW / 2) : g.KH * g.KW;
  const int ksteps = ntap * csteps;
  const int ky0 = PAR ? (((g.P - py) % 2) + 2) % 2 : 0;
  const int kx0 = PAR ? (((g.P - px) % 2) + 2) % 2 : 0;
  const int Wg = PAR ? g.Wo / 2 : g.Wo, Hg = PAR ? g.Ho / 2 : g.Ho;

  const int vrow = tid / VPR, vch = tid % VPR;
  int pn[PX_PASS], poy[PX_PASS], pox[PX_PASS];
  bool pval[PX_PASS];
#pragma unroll
  for (int p = 0; p < PX_PASS; ++p) {
    const int64_t m = m0 + vrow + p * RPP;
    pval[p] = m < M;
    const int64_t mm = pval[p] ? m : 0;
    pox[p] = (int)(mm % Wg);
    const int64_t t = mm / Wg;
    poy[p] = (int)(t % Hg);
    pn[p] = (int)(t / Hg);
    if constexpr (PAR) {
      poy[p] = 2 * poy[p] + py;
      pox[p] = 2 * pox[p] + px;
    }
  }

  bf16x8 xr[2][PX_PASS], wreg[2][W_PASS];  // two K-steps in flight
  auto gload = [&](int ks, int slot) {
    const int t = ks / csteps;
    const int c0 = (ks - t * csteps) * BK;
    int ky, kx;
    if constexpr (PAR) {
      const int hw = g.KW / 2;
      ky = ky0 + 2 * (t / hw);
      kx = kx0 + 2 * (t - (t / hw) * hw);
    } else {
      ky = t / g.KW;
      kx = t - ky * g.KW;
    }
    const int tap = ky * g.KW + kx;
    const bf16* src;
    int cs, cc;
    if (c0 < g.C1) { src = x1; cs = g.C1; cc = c0; } else { src = x2; cs = g.C2; cc = c0 - g.C1; }
#pragma unroll
    for (int p = 0; p < PX_PASS; ++p) {
      int iy, ix;
      bf16x8 v = {};
      if (pval[p] && tap_src(g, poy[p], pox[p], ky, kx, iy, ix))
        v = *reinterpret_cast<const bf16x8*>(src + ((((int64_t)pn[p] * g.Hi + iy) * g.Wi + ix) * cs + cc + vch * 8));
      xr[slot][p] = v;
    }
#pragma unroll
    for (int p = 0; p < W_PASS; ++p) {
      const int co = n0 + vrow + p * RPP;
      wreg[slot][p] = *reinterpret_cast<const bf16x8*>(w + wpk_index(g.wch, co, tap, c0 + vch * 8, Cin, g.KH * g.KW));
    }
  };
  auto sstore = [&](int buf, int slot) {
    bf16* A = lds[buf];            // weights [BN][32]
    bf16* B = lds[buf] + BN * 32;  // pixels  [BMP][32]
#pragma unroll
    for (int p = 0; p < W_PASS; ++p) *reinterpret_cast<bf16x8*>(A + gx_off(vrow + p * RPP, vch)) = wreg[slot][p];
#pragma unroll
    for (int p = 0; p < PX_PASS; ++p) *reinterpret_cast<bf16x8*>(B + gx_off(vrow + p * RPP, vch)) = xr[slot][p];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  int aoff[TM], boff[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) aoff[i] = gx_off(wr * (BN / 2) + i * 16 + lr, lg);
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = BN * 32 + gx_off(wc * 64 + j * 16 + lr, lg);

  // K-steps in pairs so the register slots / LDS buffers are compile-time (a runtime slot index would
  // put the staging arrays in scratch memory)
  auto step = [&](int ks, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    // registers: slot buf held step ks (already in LDS), slot buf^1 holds step ks+1
    if (ks + 2 < ksteps) gload(ks + 2, buf);
    const bf16* L = lds[buf];
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(L + aoff[i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(L + boff[j]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (ks + 1 < ksteps) sstore(buf ^ 1, buf ^ 1);
    __syncthreads();
  };
  gload(0, 0);
  if (ksteps > 1) gload(1, 1);
  sstore(0, 0);
  __syncthreads();
  for (int ks = 0; ks < ksteps; ks += 2) {
    step(ks, std::integral_constant<int, 0>{});
    if (ks + 1 < ksteps) step(ks + 1, std::integral_constant<int, 1>{});
  }

  const int Co2 = g.Cout - g.Co1;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int64_t m = m0 + wc * 64 + j * 16 + lr;
    if (m >= M) continue;
    if constexpr (PAR) {
      const int64_t b = m % Wg, t = m / Wg, a = t % Hg, n = t / Hg;
      m = (n * g.Ho + 2 * a + py) * g.Wo + 2 * b + px;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = n0 + wr * (BN / 2) + i * 16 + lg * 4;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bias[co + r];
      }
      if (co < g.Co1) {
        if (res) {
          float rv[4];
          load4(res + m * g.Co1 + co, rv);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += rv[r];
        }
        store4(y1 + m * g.Co1 + co, v);
      } else {
        if (res2) {
          float rv[4];
          load4(res2 + m * Co2 + (co - g.Co1), rv);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += rv[r];
        }
        store4(y2 + m * Co2 + (co - g.Co1), v);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 conv (bf16): halo-tiled implicit GEMM.  Block = 8 x 32 output pixels of
// one image x 64 output channels.  Per 32-channel input chunk the (8+2) x (32+2) input halo and
// the 9 taps x 64 co weights are staged in LDS once and all 9 taps read shifted windows of the
// halo (9x fewer input loads than im2col).  The next chunk is prefetched into registers while the
// current one is consumed.  4 waves = 2 (co halves) x 2 (pixel halves of 4 rows).
// ----------------------------------------------------------------------------------------
constexpr int H3_TH = 8, H3_TW = 32;     // default tile (TH x TW is chosen per level, see c2_tile)
constexpr int H3_NPIX = 384;             // max halo pixels (TH+2)(TW+2) actually staged
constexpr int H3_P = 40;                 // LDS halo row pitch (pixels): >= TW+2, multiple of 8 (see below)
constexpr int H3_NROW = 10 * H3_P;       // LDS halo rows ((TH+2) <= 10 tile rows of H3_P pixels)
constexpr int H3_LD = 32;                // bf16 per LDS row: 32 channels = 64 B, no padding
constexpr int H3_BN = 64;
// element offset of 16-B chunk `ch` (8 channels) of LDS row `row`: 64-B rows, chunk index XORed with
// bit 2 of the row.  ds_read_b128 of 16 rows r0..r0+15 (lane = row, lane group = chunk) is then
// bank-conflict free for any r0 (the 80-B padded rows it replaces ran 2-3-way conflicted: PMC
// SQ_LDS_BANK_CONFLICT = 51 % of LDS cycles at level 3).  Steps of 8 rows keep the swizzle, so the
// tap offsets ky * H3_P and tap * 64 stay immediate.
__device__ __forceinline__ int h3_off(int row, int ch) { return row * H3_LD + ((ch ^ ((row >> 1) & 2)) << 3); }

// The halo conv's measured alternatives, removed in round 6 (profiles/r2_*, r3_*, r5_prio_ab.txt): staging
// through registers instead of LDS-DMA, the compiler's read -> MFMA tap order, 32 co x 128 px wave tiles, co-block-
// slowest (not XCD-grouped) block order, 256-pixel tiles only, and s_setprio around the MFMA phase.
// epilogue of the halo conv (conv3x3_bf16_kernel; a function since round 5's double-buffered variant): bias, residual, bf16 stores and the GroupNorm
// statistics partials; lane holds co = n0 + wr*32 + i*16 + 4*lg + r of pixel pyx[j] (packed (py << 16) | px, -1 past TH)
template <int NI, int NJ>
__device__ __forceinline__ void h3_epilogue(const f32x4 (&acc)[NI][NJ], const int (&pyx)[NJ], const ConvGeom& g,
                                            const float* __restrict__ bias, const bf16* __restrict__ res,
                                            const bf16* __restrict__ res2, bf16* __restrict__ y1, bf16* __restrict__ y2,
                                            float* __restrict__ gnp, int gn_fimg, int n, int tt, int ntile, int y0,
                                            int x0, int n0, int wr, int wc, int lane) {
  const int lr = lane & 15, lg = lane >> 4;
  const int Co2 = g.Cout - g.Co1;
  float bv[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i) epi_bias(bias, n0 + wr * 32 + i * 16 + lg * 4, bv[i]);
  int64_t mj[NJ];
  bool okj[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int oy = y0 + (pyx[j] >> 16), ox = x0 + (pyx[j] & 0xffff);
    okj[j] = pyx[j] >= 0 && oy < g.Ho && ox < g.Wo;
    mj[j] = okj[j] ? ((int64_t)n * g.Ho + oy) * g.Wo + ox : 0;
  }
  bf16x4 rv[NJ][NI];
  if (res || res2) {  // uniform
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < NI; ++i) rv[j][i] = epi_res(res, res2, mj[j], n0 + wr * 32 + i * 16 + lg * 4, g.Co1, Co2, okj[j]);
  } else {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < NI; ++i) rv[j][i] = bf16x4{};
  }
  // GroupNorm statistics partials (gnp: the Block conv feeding a GroupNorm): per channel quad (i, lg) the sum
  // and sum of squares of the stored bf16 output over this wave's valid pixels
  float gsum[NI], gsq[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) gsum[i] = gsq[i] = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (!okj[j]) continue;
    const int64_t m = mj[j];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int co = n0 + wr * 32 + i * 16 + lg * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv[i][r] + b2f(rv[j][i], r);
      if (gnp) {  // uniform: the statistics of the stored (bf16-rounded) y, which GroupNorm then normalises
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (float)(bf16)v[r];
      }
      if (co < g.Co1) store4(y1 + m * g.Co1 + co, v);
      else store4(y2 + m * Co2 + (co - g.Co1), v);
      if (gnp) {  // uniform
        gsum[i] += (v[0] + v[1]) + (v[2] + v[3]);
        gsq[i] += fmaf(v[3], v[3], fmaf(v[2], v[2], fmaf(v[1], v[1], v[0] * v[0])));
      }
    }
  }
  if (gnp) {
    const int b = n / gn_fimg, f = n - b * gn_fimg;
    constexpr int SPT = 4;  // GroupNorm slots per tile (= pixel ranges): h3_gn_slots
    const int64_t nslot = (int64_t)gn_fimg * ntile * SPT;
    const int64_t slot = ((int64_t)f * ntile + tt) * SPT + wc;
    float2* dst = reinterpret_cast<float2*>(gnp) + ((int64_t)b * nslot + slot) * (g.Cout / 4) + (n0 + wr * 32) / 4 + lg;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float a = row16_sum(gsum[i]), q = row16_sum(gsq[i]);
      if (lr == 0) dst[i * 4] = make_float2(a, q);
    }
  }
}

// (Round 3: double-buffered chunks at one block per CU measured slower, conv total 64.0 -> 68.2 ms per step: the
// second co-resident block hides the staging better than an in-block prefetch.  Removed.  Round 6: 16-channel stages in
// a double buffer at two blocks per CU, each K = 32 MFMA step taking two taps of a stage (so the K = 32 rate is kept,
// unlike round 5's K = 16 form), 44-pixel halo pitch with a conflict-free 32-B-row swizzle: correct, 385 vs 336 us per
// launch -- the extra zero-half step for the 9th tap, twice the barriers and the per-tap address VALU outweigh the
// overlap (profiles/r6o_tap_pair_conv_ab.txt).  Removed.  Also round 6: an L2 touch of chunk ch + 1's weight and
// halo lines (4 B per 128-B line, LDS-direct) issued while chunk ch computes -- the step's halo conv calls 1 % faster,
// the step 0.3 ms slower (profiles/r6late_h3_touch_ab.txt).  Removed.)
#ifndef H3_PW
#define H3_PW 1
#endif
#ifdef CESM_H3_STAMPS
__device__ uint64_t* g_h3_stamp_buf = nullptr;
__device__ int g_h3_stamp_blocks = 0;
#endif
template <int TW, int NJv = 4>
__global__ __launch_bounds__(256, 2) void conv3x3_bf16_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                              const bf16* __restrict__ w, const float* __restrict__ bias,
                                                              const bf16* __restrict__ res, const bf16* __restrict__ res2,
                                                              bf16* __restrict__ y1, bf16* __restrict__ y2, ConvGeom g,
                                                              int tiles_x, int TH, float* __restrict__ gnp = nullptr,
                                                              int gn_fimg = 1) {
  // NJv = 7: tiles of up to 448 pixels ((TH+2) <= 16 halo rows of H3_P), 64 co x 112 px per wave: 11
  // fragment reads per 28 MFMAs per tap (0.39 per MFMA instead of 0.5) and the 36-KiB weight chunk staged once
  // per 448 instead of 256 pixels; 77 KiB of LDS, still 2 blocks per CU
  static_assert(NJv == 4 || NJv == 7, "256- or 448-pixel tiles");
  constexpr int NROWS = (NJv == 7 ? 16 : 10) * H3_P;
  __shared__ __attribute__((aligned(16))) bf16 sh[NROWS * H3_LD];
  // the weight tile as three arrays of 3 taps each: distinct LDS objects, so the compiler's wait insertion can see that
  // reads of taps 0-2 do not depend on the DMA still landing taps 3-8 (H3_PW)
  __shared__ __attribute__((aligned(16))) bf16 sw0[3 * H3_BN * H3_LD];
  __shared__ __attribute__((aligned(16))) bf16 sw1[3 * H3_BN * H3_LD];
  __shared__ __attribute__((aligned(16))) bf16 sw2[3 * H3_BN * H3_LD];
  auto swt = [&](int k) { return k == 0 ? sw0 : (k == 1 ? sw1 : sw2); };  // k compile-time after unrolling
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // wave tile (round 3): 64 co x 16 NJv px = 4 x NJv MFMA tiles per wave (8 fragment reads per 16 MFMAs per
  // tap at NJv = 4); else 32 co x 128 px = 2 x 8 (10 reads per 16 MFMAs: the 4 waves' reads exceeded the LDS
  // array's 256 B/clk)
  constexpr int NI = 4, NJ = NJv;
  const int wr = 0, wc = wid;
  constexpr int PXW = 16 * NJ;  // pixels per wave
  // 1-D grid (h3_grid): the ncob co blocks of a (image, tile) run back to back on ONE XCD (linear id mod 8), so
  // its input halo is fetched into that XCD's L2 once (co-block-slowest order re-read every halo ncob times)
  const int ntile = tiles_x * ((g.Ho + TH - 1) / TH), ncob = g.Cout / H3_BN;
  const int L = blockIdx.x, jx = L >> 3;
  const int cb = jx % ncob;
  const int tflat = (jx / ncob) * 8 + (L & 7);
  if (tflat >= g.Nb * ntile) return;  // padded items (whole block)
  const int n = tflat / ntile, tt = tflat - n * ntile;
  const int ty = tt / tiles_x, tx = tt - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  constexpr int HWd = TW + 2;
  const int HP = (TH + 2) * HWd;
  const int n0 = cb * H3_BN;
  const int Cin = g.C1 + g.C2;
  const int nchunk = Cin / 32;

  // stage one 32-channel chunk by buffer-LDS-DMA (no registers, no address VALU per element beyond one per
  // 16-B piece): 1-KiB pieces of 16 LDS rows, each lane fetching the global chunk that the row swizzle puts in
  // its slot (chunk = slot ^ ((row >> 1) & 2)); halo rows outside the tile / image read as zeros (out-of-range
  // offset).  The second co-resident block computes while this one waits.
  auto stage = [&](int ch) {
    const int c0 = ch * 32;
    const bf16* src;
    int cs, cc;
    if (c0 < g.C1) { src = x1; cs = g.C1; cc = c0; } else { src = x2; cs = g.C2; cc = c0 - g.C1; }
    const int64_t img = (int64_t)g.Hi * g.Wi * cs;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + n * img + cc), (short)0, (int)(img * 2 - cc * 2), 0x00020000);
    // this (co block, chunk)'s weight tile: one contiguous [tap][co][32] block of the chunked pack (wpk_index)
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(w + ((int64_t)cb * nchunk + ch) * (9 * H3_BN * 32)), (short)0, 9 * H3_BN * 32 * 2, 0x00020000);
    const int prow = lane >> 2, pslot = lane & 3;
    constexpr int HPC = NROWS / 16;  // halo pieces (25 / 40)
    // NJv = 7: only the pieces the tile's halo rows span (pixels past the tile read row 0);
    // NJv = 4 at TW = 32 reads rows up to 9 for pixels past a short tile (discarded), so all 25 are staged
    const int hpc = NJv == 4 ? HPC : ((TH + 2) * H3_P + 15) >> 4;
#pragma unroll
    for (int k = 0; k < (HPC + 3) / 4; ++k) {
      const int q = wid + 4 * k;
      if (q < hpc) {  // wave-uniform
        const int row = 16 * q + prow;
        const int r = row / H3_P, col = row - r * H3_P;
        const int iy = y0 - 1 + r, ix = x0 - 1 + col;
        const bool in = r < TH + 2 && col < HWd && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
        const int chunk = pslot ^ ((row >> 1) & 2);
        const int vo = in ? ((iy * g.Wi + ix) * cs + chunk * 8) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(sh + q * 512), 16, vo, 0,
                                                 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {  // weights: 9 taps x 64 co rows = 36 pieces, each 1 KiB of the tile
      const int q = wid + 4 * k, row = 16 * q + prow;  // row = tap * 64 + co
      const int chunk = pslot ^ ((row >> 1) & 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(swt(k / 3) + (q - 12 * (k / 3)) * 512),
                                               16, (row * 32 + chunk * 8) * 2, 0, 0, 0);
    }
  };
#ifdef CESM_H3_STAMPS
  // diagnostic build only (tools/h3_stamps.py): per wave, cycles spent in each phase of the chunk loop
  uint64_t hs[8] = {}, hland[8] = {};
  const uint64_t h_t0 = __builtin_amdgcn_s_memtime();
  uint64_t h_t = h_t0;
  auto hstamp = [&](int k) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    hs[k] += t - h_t;
    h_t = t;
  };
#define H3STAMP(k) hstamp(k)
#else
#define H3STAMP(k)
#endif

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  // pixel group j of this wave: tile pixel p = wc*PXW + j*16 + lr -> halo row of tap (0,0)
  int hoff[NJ], pyx[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    int py, px;
    if constexpr (TW == 32 && NJ % 2 == 0) {  // rows of two 16-pixel groups: compile-time offsets per j
      py = wc * (NJ / 2) + (j >> 1);
      px = (j & 1) * 16 + lr;
    } else {
      const int p = wc * PXW + j * 16 + lr;
      py = p / TW;
      px = p - py * TW;
    }
    const bool in = py < TH;
    // TW == 32: rows past TH stay inside the LDS halo buffer (results discarded), no select needed
    hoff[j] = ((TW == 32 && NJ % 2 == 0) || in) ? py * H3_P + px : 0;
    pyx[j] = in ? (py << 16) | px : -1;
  }
  // fragment addresses for ky = 0 / tap = 0; the other taps add immediates (swizzle-preserving steps)
  int boff[NJ][3], aoff[NI];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) boff[j][kx] = h3_off(hoff[j] + kx, lg);
#pragma unroll
  for (int i = 0; i < NI; ++i) aoff[i] = h3_off(wr * 32 + i * 16 + lr, lg);
  for (int ch = 0; ch < nchunk; ++ch) {
    if (ch) __syncthreads();  // previous chunk fully consumed
    H3STAMP(0);
    stage(ch);
    H3STAMP(1);
#if H3_PW
    // progressive landing: each wave's 9 weight pieces are the youngest, piece k = tap k; wait for the halo and taps
    // 0-2 only, and for taps 3-5 / 6-8 at the tap loop's two later barriers
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    H3STAMP(2);
    __builtin_amdgcn_s_barrier();
#else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    H3STAMP(2);
    __syncthreads();
#endif
    H3STAMP(3);
#ifdef CESM_H3_STAMPS
    if (ch < 8) hland[ch] = h_t;
#endif
    // the 10 fragment reads of tap t+1 are issued between the 16 MFMAs of tap t (two register sets), so no
    // MFMA waits on a read issued just before it (the compiler's order was read -> wait -> 2 MFMAs)
    bf16x8 fa[2][NI], fb[2][NJ];
    auto rd = [&](int tap, int b) {
      const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        fa[b][i] = *reinterpret_cast<const bf16x8*>(swt(tap / 3) + aoff[i] + (tap % 3) * H3_BN * H3_LD);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[b][j] = *reinterpret_cast<const bf16x8*>(sh + boff[j][kx] + ky * H3_P * H3_LD);
    };
    rd(0, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int b = tap & 1;
      const bool gate = H3_PW && (tap == 2 || tap == 5);  // the next tap's weights land behind a barrier
      __builtin_amdgcn_sched_barrier(0);
      if (tap + 1 < 9 && !gate) rd(tap + 1, b ^ 1);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < NI; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[b][i], fb[b][j], acc[i][j], 0, 0, 0);
      if (gate) {
        __builtin_amdgcn_sched_barrier(0);
        if (tap == 2) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        rd(tap + 1, b ^ 1);
      } else if (tap + 1 < 9) {
#pragma unroll
        for (int q2 = 0; q2 < NI + NJ; ++q2) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NI * NJ - (NI + NJ), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    H3STAMP(4);
  }
  h3_epilogue<NI, NJ>(acc, pyx, g, bias, res, res2, y1, y2, gnp, gn_fimg, n, tt, ntile, y0, x0, n0, wr, wc, lane);
#ifdef CESM_H3_STAMPS
  H3STAMP(5);
  // record: [hw_id | xcc_id << 32, t0, t_end, hs[0..5], land[0..6]] -- vector stores from lane 0 to the diagnostic
  // buffer only
  if (g_h3_stamp_buf && lane == 0 && L < g_h3_stamp_blocks) {
    uint64_t* o = g_h3_stamp_buf + ((int64_t)L * 4 + wid) * 16;
    const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    o[0] = hwid | ((uint64_t)xcc << 32);
    o[1] = h_t0;
    o[2] = h_t;
#pragma unroll
    for (int k = 0; k < 6; ++k) o[3 + k] = hs[k];
#pragma unroll
    for (int k = 0; k < 7; ++k) o[9 + k] = hland[k];
  }
#endif
}
#undef H3STAMP



// ----------------------------------------------------------------------------------------
// 4x4 / stride-2 / pad-1 convs (Downsample, video_net.py:61-62) and their transposes (Upsample, :65-66;
// each is also the other's data gradient) as halo-tiled implicit GEMMs on the low-resolution grid.  Both
// are 3x3 stride-1 neighbourhoods in which only a 2x2 subset of the taps is live per parity:
//   DOWN  y[oy][ox] = sum_{ky,kx} W[ky*4+kx] . x[2oy-1+ky][2ox-1+kx]; split by the input parity (a, b)
//         (x_ab[Y][X] = x[2Y+a][2X+b]) the live taps are ky = (1-a) + 2t (t = 0, 1), read at halo row
//         offset (1-a) + t of the (TH+2) x (TW+2) halo of x_ab around the output tile;
//   UP    the transposed conv in its gather form (S = 1, U = 2, P = 2, taps flipped by the packing):
//         y[2Y+py][2X+px] = sum over ky = py + 2t, kx = px + 2u of W[ky*4+kx] . x[Y-1+py+t][X-1+px+u].
// The tap base (1-a or py) is a template parameter of the per-stage MFMA loop, so every LDS address stays
// compile-time + lane constant as in conv3x3_bf16_kernel (same 2 x 2 wave tiling, 64 co per block, two
// blocks per CU).  DOWN runs 4 parity stages per 32-channel chunk (consecutive stages touch the same input
// lines); UP gives each output parity its own blocks (blockIdx.z = parity * Cout/64 + co block).  The
// generic implicit GEMM it replaces gathered every (pixel, tap) pair from global memory, 16 K-steps of 8
// MFMAs per wave per chunk (190-260 TF/s on the bench shapes).
// ----------------------------------------------------------------------------------------
template <int TW, int BY, int BX>
__device__ __forceinline__ void s2_taps(const bf16* sh, const bf16* sw, const int (&boff)[8][3], const int (&aoff)[2],
                                        f32x4 (&acc)[2][8]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int oy = BY + (t >> 1), ox = BX + (t & 1);
    bf16x8 af[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sw + aoff[i] + t * H3_BN * H3_LD);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(sh + boff[j][ox] + oy * H3_P * H3_LD);
      acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bfr, acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bfr, acc[1][j], 0, 0, 0);
    }
  }
}
template <int TW, int BY, int BX>
__device__ __forceinline__ void s2_taps_pipe(const bf16* sh, const bf16* sw, const int (&boff)[8][3], const int (&aoff)[2],
                                        f32x4 (&acc)[2][8]) {
  // tap t+1's 10 fragment reads issued between tap t's 16 MFMAs (as conv3x3_bf16_kernel)
  bf16x8 fa[2][2], fb[2][8];
  auto rd = [&](int t, int b) {
    const int oy = BY + (t >> 1), ox = BX + (t & 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[b][i] = *reinterpret_cast<const bf16x8*>(sw + aoff[i] + t * H3_BN * H3_LD);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[b][j] = *reinterpret_cast<const bf16x8*>(sh + boff[j][ox] + oy * H3_P * H3_LD);
  };
  rd(0, 0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int b = t & 1;
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < 4) rd(t + 1, b ^ 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[b][0], fb[b][j], acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[b][1], fb[b][j], acc[1][j], 0, 0, 0);
    }
    if (t + 1 < 4) {
#pragma unroll
      for (int q2 = 0; q2 < 10; ++q2) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int TW, bool UP>
__global__ __launch_bounds__(256, 2) void convs2_bf16_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                             const float* __restrict__ bias, const bf16* __restrict__ res,
                                                             bf16* __restrict__ y, ConvGeom g, int tiles_x, int TH,
                                                             int Hl, int Wl) {
  __shared__ __attribute__((aligned(16))) bf16 sh[H3_NROW * H3_LD];
  __shared__ __attribute__((aligned(16))) bf16 sw[4 * H3_BN * H3_LD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int n = blockIdx.y;
  const int ty = blockIdx.x / tiles_x, tx = blockIdx.x - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;  // tile origin on the low-resolution grid
  constexpr int HWd = TW + 2;
  const int HP = (TH + 2) * HWd;
  const int ncob = g.Cout / H3_BN;
  const int par = UP ? (int)blockIdx.z / ncob : 0;
  const int n0 = ((int)blockIdx.z - par * ncob) * H3_BN;
  const int ppy = par >> 1, ppx = par & 1;
  const int Cin = g.C1;
  const int nchunk = Cin / 32;
  constexpr int WPT = 4 * H3_BN * 4 / 256;  // weight vectors per thread (4 taps x 64 co x 4 vectors)

  // stage s by buffer-LDS-DMA (as conv3x3_bf16_kernel): halo of the (parity sub-)image and the 4 live taps'
  // weights for one 32-channel chunk
  (void)WPT;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + (int64_t)n * g.Hi * g.Wi * Cin), (short)0, (int)((int64_t)g.Hi * g.Wi * Cin * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(w + (int64_t)n0 * 16 * Cin), (short)0, H3_BN * 16 * Cin * 2, 0x00020000);
  auto stage = [&](int ch, int a, int b, int by, int bx) {
    const int c0 = ch * 32;
    const int prow = lane >> 2, pslot = lane & 3;
    constexpr int HPC = H3_NROW / 16;
#pragma unroll
    for (int k = 0; k < (HPC + 3) / 4; ++k) {
      const int q = wid + 4 * k;
      if (q < HPC) {  // wave-uniform
        const int row = 16 * q + prow;
        const int r = row / H3_P, col = row - r * H3_P;
        const int Y = y0 - 1 + r, X = x0 - 1 + col;
        const int iy = UP ? Y : 2 * Y + a, ix = UP ? X : 2 * X + b;
        const bool in = r < TH + 2 && col < HWd && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
        const int chunk = pslot ^ ((row >> 1) & 2);
        const int vo = in ? ((iy * g.Wi + ix) * Cin + c0 + chunk * 8) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(sh + q * 512), 16, vo, 0,
                                                 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // 4 taps x 64 co rows = 16 pieces
      const int q = wid + 4 * k, row = 16 * q + prow;  // row = t * 64 + co
      const int t = row >> 6, co = row & 63;
      const int tap = (by + 2 * (t >> 1)) * 4 + bx + 2 * (t & 1);
      const int chunk = pslot ^ ((row >> 1) & 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(sw + q * 512), 16,
                                               (((ch * 16 + tap) * 64 + co) * 32 + chunk * 8) * 2, 0, 0, 0);  // chunked
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x4 acc[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  int hoff[8], pyx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = wc * 128 + j * 16 + lr;
    const int py = p / TW, px = p - py * TW;
    const bool in = py < TH;
    hoff[j] = in ? py * H3_P + px : 0;
    pyx[j] = in ? (py << 16) | px : -1;
  }
  int boff[8][3], aoff[2];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) boff[j][kx] = h3_off(hoff[j] + kx, lg);
#pragma unroll
  for (int i = 0; i < 2; ++i) aoff[i] = h3_off(wr * 32 + i * 16 + lr, lg);

  if constexpr (UP) {
    for (int ch = 0; ch < nchunk; ++ch) {
      if (ch) __syncthreads();  // previous chunk fully consumed
      stage(ch, 0, 0, ppy, ppx);
      __syncthreads();
      switch (par) {  // block-uniform
        case 0: s2_taps<TW, 0, 0>(sh, sw, boff, aoff, acc); break;
        case 1: s2_taps<TW, 0, 1>(sh, sw, boff, aoff, acc); break;
        case 2: s2_taps<TW, 1, 0>(sh, sw, boff, aoff, acc); break;
        default: s2_taps<TW, 1, 1>(sh, sw, boff, aoff, acc); break;
      }
    }
  } else {
    for (int ch = 0; ch < nchunk; ++ch) {
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const int a = ab >> 1, b = ab & 1;
        if (ch || ab) __syncthreads();
        stage(ch, a, b, 1 - a, 1 - b);
        __syncthreads();
        // (down: the software-pipelined taps; the up kernel keeps the plain loop, pipelined it spills)
        if (ab == 0) s2_taps_pipe<TW, 1, 1>(sh, sw, boff, aoff, acc);       // a = 0, b = 0
        else if (ab == 1) s2_taps_pipe<TW, 1, 0>(sh, sw, boff, aoff, acc);  // a = 0, b = 1
        else if (ab == 2) s2_taps_pipe<TW, 0, 1>(sh, sw, boff, aoff, acc);  // a = 1, b = 0
        else s2_taps_pipe<TW, 0, 0>(sh, sw, boff, aoff, acc);                // a = 1, b = 1
      }
    }
  }
  // epilogue: lane holds co = n0 + wr*32 + i*16 + 4*lg + r of tile pixel (py, px)
  float bv[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) epi_bias(bias, n0 + wr * 32 + i * 16 + lg * 4, bv[i]);
  int64_t mj[8];
  bool okj[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int Y = y0 + (pyx[j] >> 16), X = x0 + (pyx[j] & 0xffff);
    okj[j] = pyx[j] >= 0 && Y < Hl && X < Wl;
    const int oy = UP ? 2 * Y + ppy : Y, ox = UP ? 2 * X + ppx : X;
    mj[j] = okj[j] ? ((int64_t)n * g.Ho + oy) * g.Wo + ox : 0;
  }
  bf16x4 rv[8][2];
  if (res) {  // uniform
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) rv[j][i] = epi_res(res, nullptr, mj[j], n0 + wr * 32 + i * 16 + lg * 4, g.Cout, 0, okj[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) rv[j][i] = bf16x4{};
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (!okj[j]) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = n0 + wr * 32 + i * 16 + lg * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv[i][r] + b2f(rv[j][i], r);
      store4(y + mj[j] * g.Cout + co, v);
    }
  }
}

// ----------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 conv (bf16), v3 "wide wave": block = TH x TW (<= 512) output pixels of one
// image x 64 output channels; 4 waves, wave w owns tile pixels [128w, 128w + 128) (8 fragment groups
// of 16) x ALL 64 channels (32 accumulators): per tap 4 A + 8 B ds_read_b128 feed 32 MFMA (0.375
// reads / MFMA vs 0.625 for the 32-co wave tile of conv3x3_bf16_kernel), and the block's 512 pixels
// halve the weight staging per pixel.  Per 32-channel chunk the (TH+2)(TW+2) halo and the 9 x 64 x 32
// weight tile are staged by LDS-DMA (global_load_lds, no VGPR round trip) into 64-B rows whose
// 16-B chunk index is XORed with (row >> 1) & 2 - conflict-free for ds_read_b128 over any 16
// consecutive rows (exhaustive check over the four lane groups); the weight-fragment addresses are
// compile-time + lane constants.  76 KiB LDS -> two blocks per CU: one stages while the other
// computes.
// ----------------------------------------------------------------------------------------
constexpr int CW_HROWS = 640;                       // max halo rows (TH+2)(TW+2)
constexpr int CW_WROWS = 9 * 64;                    // weight rows (tap*64 + co)
constexpr int CW_HPIECE = CW_HROWS / 16;            // 1-KiB glds pieces
constexpr int CW_WPIECE = CW_WROWS / 16;
constexpr int CW_HPW = CW_HPIECE / 4;               // halo pieces per wave (10)
constexpr int CW_WPW = CW_WPIECE / 4;               // weight pieces per wave (9)
__device__ __attribute__((aligned(64))) bf16 cw_zero_page[32] = {};

__device__ __forceinline__ int cw_swz(int row) { return (row >> 1) & 2; }
__device__ __forceinline__ bf16x8 zero8_bf16() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}
// byte offset of 16-B chunk c (8 channels) of row `row`
__device__ __forceinline__ int cw_off(int row, int c) { return (row << 6) + ((c ^ cw_swz(row)) << 4); }

// the 9 taps of one staged 32-channel chunk: 4 A + 8 B fragments per tap, software-pipelined one
// tap ahead in registers (the reads of tap t+1 are issued before tap t's 32 MFMAs; sched_barrier
// pins the order so the scheduler cannot hoist every tap's reads and blow the register budget)
template <int TW>
__device__ __forceinline__ void cw_taps(const char* sh, const char* sw, const int (&hoff)[8], int lr, int lg,
                                        f32x4 (&acc)[4][8]) {
  constexpr int HWd = TW + 2;
  bf16x8 af[2][4], bfr[2][8];
  // weight rows tap*64 + i*16 + lr: swizzle bit = bit 2 of lr -> compile-time offset + a lane constant
  const int a_lane = (lr << 6) + ((lg ^ cw_swz(lr)) << 4);
  // opaque copies: keeps the (non-linear, swizzled) halo addresses from being hoisted out of the
  // chunk loop as 72 loop-invariant VGPRs
  int ho[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ho[j] = hoff[j];
    asm volatile("" : "+v"(ho[j]));
  }
  auto load = [&](int tap, int b) {
    const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[b][i] = *reinterpret_cast<const bf16x8*>(sw + a_lane + (tap * 64 + i * 16) * 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) bfr[b][j] = *reinterpret_cast<const bf16x8*>(sh + cw_off(ho[j] + ky * HWd + kx, lg));
  };
  load(0, 0);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int b = tap & 1;
    if (tap + 1 < 9) load(tap + 1, b ^ 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[b][i], bfr[b][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ----------------------------------------------------------------------------------------
// 3x3 conv (bf16), v4 "pipelined wide wave": the conv3x3w tile / wave layout / LDS image, but
// persistent (one block per CU) with TWO LDS stages: the buffer-LDS-DMA of step s+1 (next 32-channel
// chunk, or the next item's first chunk) is issued right after the barrier that opens step s and
// lands while step s's 288 MFMAs per wave run.  Steps run over the block's items (it = blockIdx.x +
// k * gridDim.x; item = (image, tile, 64-channel co block), co block fastest so the co blocks of a
// tile run concurrently and share its halo in L2).
// ----------------------------------------------------------------------------------------
constexpr int CP_STAGE = (CW_HROWS + CW_WROWS) * 64;  // 76 KiB
constexpr int CP_ELD = 68;                            // epilogue tile row (bf16): 136 B, conflict-free 8-B writes
constexpr int CP_PITCH = 40;                          // halo row pitch (pixels): multiple of 8
constexpr int CP_TH = 14;                             // max tile rows: (14 + 2) * 40 = 640 halo rows

// taps of one staged chunk for NG fragment groups per wave.  Halo rows use a pitch of 40 pixels, so a
// ky step (+40 rows) keeps bits 0..2 of the row and with them the chunk swizzle: the B address of
// (group j, ky, kx) = bad[j][kx] + ky * 40 * 64 -> immediate offsets, no per-read VALU.  Fragment reads
// of tap t+1 are interleaved with tap t's MFMAs (sched_group_barrier: 1 ds_read, 2 MFMA, ...).
struct NoHook {
  __device__ __forceinline__ void operator()(int) const {}
};

template <int NG, typename Hook = NoHook>
__device__ __forceinline__ void cp_taps(const char* sh, const char* sw, const int (&bad)[NG][3], int a_lane,
                                        f32x4 (&acc)[4][NG], const Hook& hook = Hook()) {
  bf16x8 af[2][4], bfr[2][NG];
  auto load = [&](int tap, int b) {
    const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[b][i] = *reinterpret_cast<const bf16x8*>(sw + a_lane + (tap * 64 + i * 16) * 64);
#pragma unroll
    for (int j = 0; j < NG; ++j)
      bfr[b][j] = *reinterpret_cast<const bf16x8*>(sh + bad[j][kx] + ky * CP_PITCH * 64);
  };
  load(0, 0);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int b = tap & 1;
    __builtin_amdgcn_sched_barrier(0);
    hook(tap);  // e.g. this tap's share of the next step's LDS-DMA, spread over the MFMA phase
    __builtin_amdgcn_sched_barrier(0);
    if (tap + 1 < 9) load(tap + 1, b ^ 1);
#pragma unroll
    for (int j = 0; j < NG; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[b][i], bfr[b][j], acc[i][j], 0, 0, 0);
    if (tap + 1 < 9) {
#pragma unroll
      for (int q = 0; q < 4 + NG; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * NG - 2 * (4 + NG), 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ----------------------------------------------------------------------------------------
// 3x3 conv (bf16), v4 "pipelined wide wave": persistent (one block per CU) with TWO LDS stages:
// the buffer-LDS-DMA of step s+1 (next 32-channel chunk, or the next item's first chunk) is issued
// right after the barrier that opens step s and lands while step s's MFMAs run.  Steps run over
// the block's items (it = blockIdx.x + k * gridDim.x; item = (image, TH x TW tile, 64-channel co
// block), co block fastest so a tile's co blocks run concurrently and share its halo in L2).
// Wave w owns tile pixels [16*NG*w, 16*NG*(w+1)) x all 64 co.  The epilogue stages (acc + bias) as
// bf16 in the stage just consumed and writes full 128-B pixel rows (+ residual) with exactly 2*NG
// buffer stores per wave, so the next step waits for its DMA with vmcnt(2*NG), not for the stores.
// ----------------------------------------------------------------------------------------
// Items are split statically (item it = blockIdx.x + k * gridDim.x): the kernel keeps no state between launches,
// so concurrent launches (two streams, graph branches, two model instances) are independent.  (Round 3 claimed
// items from a process-global atomic counter instead: 596.6 vs 599.1 us per launch, not worth the hidden state.)

template <int TW, int NG, bool RW, int NST = 2, int HPW = CW_HPW>
__global__ __launch_bounds__(256, 1) void conv3x3p_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                          const bf16* __restrict__ w, const float* __restrict__ bias,
                                                          const bf16* __restrict__ res, const bf16* __restrict__ res2,
                                                          bf16* __restrict__ y1, bf16* __restrict__ y2, ConvGeom g,
                                                          int tiles_x, int tiles_per_img, int TH, int ncob, int nitems,
                                                          float* __restrict__ gnp, int gn_fimg) {
  static_assert(TW + 2 <= CP_PITCH && NG <= 8 && HPW <= CW_HPW, "tile geometry");
  static_assert(NST == 2 || (NST == 3 && RW), "3 stages only with resident weights");
  // one LDS array (a second __shared__ object can make hipcc drain the DMA before ds_reads):
  // 2 stages | [RW: resident weights, all chunks] | bias [Cout <= 1024] fp32.  RW (Cin = Cout = 64):
  // a stage holds only the halo and the 2 x 36 KiB weight chunks are loaded once per block
  // NST = 3 (RW, short tiles): every wave issues exactly HPW halo pieces per step (rows past the halo
  // load zeros) so the step-start wait can leave the next step's pieces and the epilogue stores in
  // flight: vmcnt(HPW + 2*NG)
  constexpr int STG = RW ? HPW * 4 * 1024 : CP_STAGE;
  constexpr int WRES = RW ? 2 * CW_WROWS * 64 : 0;
  constexpr int BIASB = RW ? 256 : 4096;
  __shared__ __attribute__((aligned(1024))) char lds[NST * STG + WRES + BIASB + 16];
  char* wres = lds + NST * STG;
  float* sbias = reinterpret_cast<float*>(lds + NST * STG + WRES);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int HP = (TH + 2) * CP_PITCH;
  for (int c = tid; c < g.Cout; c += 256) sbias[c] = bias ? bias[c] : 0.f;
  const int hpieces = NST == 3 ? 4 * HPW : (HP + 15) >> 4;
  const int Cin = g.C1 + g.C2;
  const int nchunk = Cin / 32;
  const int prow = lane >> 2, pslot = lane & 3;
  const int nmine = nitems > (int)blockIdx.x ? (nitems - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nsteps = nmine * nchunk;

  // per-lane halo row -> tile-relative (hy, hx) of piece k (item independent); -1: zero row
  int hrel[HPW];
#pragma unroll
  for (int k = 0; k < HPW; ++k) {
    const int row = 16 * (wid + 4 * k) + prow;
    const int hy = row / CP_PITCH, hx = row - (row / CP_PITCH) * CP_PITCH;
    hrel[k] = (row < HP && hx < TW + 2) ? (hy << 16) | hx : -1;
  }
  // B-fragment addresses of tap (0, kx) per group; A lane constant
  int bad[NG][3];
#pragma unroll
  for (int j = 0; j < NG; ++j) {
    const int p = wid * 16 * NG + j * 16 + lr;
    const int h0 = p < TH * TW ? (p / TW) * CP_PITCH + (p - (p / TW) * TW) : 0;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) bad[j][kx] = cw_off(h0 + kx, lg);
  }
  const int a_lane = (lr << 6) + ((lg ^ cw_swz(lr)) << 4);

  auto item_geo = [&](int it, int& n, int& y0, int& x0, int& cob) {
    cob = it % ncob;
    const int t = it / ncob;
    n = t / tiles_per_img;
    const int r = t - n * tiles_per_img;
    const int ty = r / tiles_x;
    y0 = ty * TH;
    x0 = (r - ty * tiles_x) * TW;
  };
  // LDS-DMA of step s, piece by piece: piece k < CW_HPW = halo piece, else (!RW) weight piece.
  // Source descriptors of the step being prefetched (set by step_src):
  __amdgpu_buffer_rsrc_t dxrs, dwrs;
  int dcs = 0, dy0 = 0, dx0 = 0;
  char* dsh = lds;
  auto step_src = [&](int s, int it, int ch) {
    int n, cob;
    item_geo(it, n, dy0, dx0, cob);
    const int c0 = ch * 32;
    const bf16* src;
    int cc;
    if (c0 < g.C1) { src = x1; dcs = g.C1; cc = c0; } else { src = x2; dcs = g.C2; cc = c0 - g.C1; }
    const int64_t img_elems = (int64_t)g.Hi * g.Wi * dcs;
    dxrs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (int64_t)n * img_elems + cc), (short)0,
                                             (int)(img_elems * 2 - cc * 2), 0x00020000);
    dwrs = __builtin_amdgcn_make_buffer_rsrc((void*)(w + ((int64_t)cob * (Cin / 32) + ch) * (9 * 64 * 32)), (short)0,
                                             9 * 64 * 32 * 2, 0x00020000);  // chunked pack (wpk_index)
    dsh = lds + (s % NST) * STG;
  };
  auto issue_piece = [&](int k) {
    if (k < HPW) {
      const int q = wid + 4 * k;
      if (q < hpieces) {  // wave-uniform
        const int chunk = pslot ^ cw_swz(16 * q + prow);
        const int iy = dy0 - 1 + (hrel[k] >> 16), ix = dx0 - 1 + (hrel[k] & 0xffff);
        const bool in = hrel[k] >= 0 && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
        const int vo = in ? ((iy * g.Wi + ix) * dcs + chunk * 8) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dxrs, (__attribute__((address_space(3))) void*)(dsh + q * 1024), 16,
                                                 vo, 0, 0, 0);
      }
    } else if constexpr (!RW) {
      const int q = wid + 4 * (k - HPW);
      const int row = 16 * q + prow;  // tap*64 + co
      const int chunk = pslot ^ cw_swz(row);
      const int vo = (row * 32 + chunk * 8) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dwrs,
                                               (__attribute__((address_space(3))) void*)(dsh + CW_HROWS * 64 + q * 1024),
                                               16, vo, 0, 0, 0);
    }
  };
  constexpr int NPIECE = RW ? HPW : HPW + CW_WPW;  // per wave per step
  auto issue = [&](int s, int it, int ch) {
    step_src(s, it, ch);
#pragma unroll
    for (int k = 0; k < NPIECE; ++k) issue_piece(k);
  };
  if constexpr (RW) {  // the whole (64 co x 9 taps x 64 ci) weight, chunk-major, waited for by step 0
    const __amdgpu_buffer_rsrc_t wrs0 = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, 64 * 9 * 64 * 2, 0x00020000);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int k = 0; k < CW_WPW; ++k) {
        const int q = wid + 4 * k;
        const int row = 16 * q + prow;
        const int chunk = pslot ^ cw_swz(row);
        const int vo = (ch * 9 * 64 * 32 + row * 32 + chunk * 8) * 2;  // chunked pack (wpk_index)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wrs0, (__attribute__((address_space(3))) void*)(wres + ch * CW_WROWS * 64 + q * 1024), 16, vo, 0, 0, 0);
      }
  }

#pragma unroll
  for (int q = 0; q < NST - 1; ++q)
    if (q < nsteps) issue(q, (int)blockIdx.x + (q / nchunk) * (int)gridDim.x, q % nchunk);
  int s = 0;
  bool epi = false;
  int it = (int)blockIdx.x;
  for (int k = 0; it < nitems; ++k) {
    const int nxt = it + (int)gridDim.x;
    f32x4 acc[4][NG];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nchunk; ++ch, ++s) {
      // step s landed: after an epilogue only its 2*NG stores are younger than step s's DMA
      if constexpr (NST == 3) {
        // steady state (nchunk == 2): younger than step s's DMA are step s+1's HPW pieces and one
        // epilogue's 2*NG stores; the first two and the last two steps drain completely
        static_assert(HPW + 2 * NG == 15, "vmcnt immediate below");
        if (s >= 2 && s + 1 < nsteps && nchunk == 2) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (epi) {
        // younger than step s's DMA: the epilogue's 2*NG output stores (+ 4 GroupNorm partial stores)
        if (gnp) {
          if constexpr (NG == 8) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
        } else {
          if constexpr (NG == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        }
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      epi = false;
      __builtin_amdgcn_s_barrier();                     // ... for every wave; step s-1's reads are done
      const char* sh = lds + (s % NST) * STG;
      const char* sw = RW ? wres + ch * CW_WROWS * 64 : sh + CW_HROWS * 64;
      const int sp = s + NST - 1;  // step prefetched now, into the stage step s-1 used
      // its item / chunk: NST = 2: the next chunk of this item, or the next item's first chunk
      const int sp_it = NST == 2 ? (ch + 1 < nchunk ? it : nxt) : (int)blockIdx.x + (sp / nchunk) * (int)gridDim.x;
      const int sp_ch = NST == 2 ? (ch + 1 < nchunk ? ch + 1 : 0) : sp % nchunk;
      const bool pf = NST == 2 ? sp_it < nitems : sp < nsteps;
      if constexpr (!RW) {  // spreading the 19-piece (!RW) DMA over the taps spills at NG = 8
        if (pf) issue(sp, sp_it, sp_ch);
        cp_taps<NG>(sh, sw, bad, a_lane, acc);
      } else {
        // the prefetch DMA spread over this step's taps (issuing all of it up front stalls the wave on the
        // vector-memory queue before its first MFMA).  ONE tap loop for both cases (pf is a uniform branch inside
        // the hook): with a second, hook-less copy of the loop the compiler gave the two copies different
        // accumulator registers and copied all 112 of them AGPR -> VGPR -> AGPR at every step (224 v_accvgpr
        // moves per 252 MFMAs)
        if (pf) step_src(sp, sp_it, sp_ch);
        auto hook = [&](int tap) {
          if (pf) {
#pragma unroll
            for (int k = 0; k < NPIECE; ++k)
              if (k * 9 / NPIECE == tap) issue_piece(k);
          }
        };
        cp_taps<NG>(sh, sw, bad, a_lane, acc, hook);
      }
    }
    int n, y0, x0, cob;
    item_geo(it, n, y0, x0, cob);
    const int n0 = cob * 64;
    it = nxt;
    // epilogue through LDS, wave-private, in rounds of up to 4 fragment groups (64 px): (acc + bias)
    // -> bf16 rows [64 px][CP_ELD] in this wave's slice of the stage just consumed (barrier: every wave
    // is past its taps), then 8 lanes per pixel write full 128-B rows with 16-B buffer stores (+
    // residual read the same way); exactly 2*NG stores per wave (rows outside the image -> out-of-range
    // offset, dropped) so the next step waits for its DMA with vmcnt(2*NG), not for these stores
    __builtin_amdgcn_s_barrier();
    constexpr int RG = (4 * 16 * CP_ELD * 2 * 4 <= STG) ? 4 : 2;  // groups per epilogue round (fits the stage)
    bf16* so = reinterpret_cast<bf16*>(lds + ((s - 1) % NST) * STG) + wid * RG * 16 * CP_ELD;
    const bool first = n0 < g.Co1;
    const int cstride = first ? g.Co1 : g.Cout - g.Co1;
    const int cofs = (first ? n0 : n0 - g.Co1) + (lane & 7) * 8;
    const int64_t img = (int64_t)n * g.Ho * g.Wo * cstride;
    const int img_bytes = g.Ho * g.Wo * cstride * 2;
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)((first ? y1 : y2) + img), (short)0, img_bytes, 0x00020000);
    const bf16* rsrc = first ? res : res2;
    const __amdgpu_buffer_rsrc_t rrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)((rsrc ? rsrc : y1) + img), (short)0, img_bytes, 0x00020000);
    // GroupNorm statistics partials of this wave's pixels (gnp: the Block conv feeding a GroupNorm):
    // per channel quad (i, lg) the sum and sum of squares of bf16(acc + bias) over the valid pixels
    float gsum[4] = {0.f, 0.f, 0.f, 0.f}, gsq[4] = {0.f, 0.f, 0.f, 0.f};
    float gm[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int p = wid * 16 * NG + j * 16 + lr;
      const int oy = y0 + p / TW, ox = x0 + (p - (p / TW) * TW);
      gm[j] = (p < TH * TW && oy < g.Ho && ox < g.Wo) ? 1.f : 0.f;
    }
#pragma unroll
    for (int r0 = 0; r0 < NG; r0 += RG) {
      const int nj = NG - r0 < RG ? NG - r0 : RG;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = i * 16 + lg * 4;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + n0 + co);
#pragma unroll
        for (int jj = 0; jj < RG; ++jj) {
          if (jj < nj) {
            const int j = r0 + jj;
            float v[4] = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
            store4(so + (jj * 16 + lr) * CP_ELD + co, v);
            if (gnp) {  // uniform; statistics of the stored (bf16-rounded) y, which GroupNorm then normalises
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = (float)(bf16)v[r];
              const float sv = (v[0] + v[1]) + (v[2] + v[3]);
              const float qv = fmaf(v[3], v[3], fmaf(v[2], v[2], fmaf(v[1], v[1], v[0] * v[0])));
              gsum[i] = fmaf(gm[j], sv, gsum[i]);
              gsq[i] = fmaf(gm[j], qv, gsq[i]);
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own writes visible to the wave's other lanes
      // residual rows of the round in batches of CP_RB loads issued back to back (one load -> wait ->
      // add -> store chain per row made the residual-fused dgrads 1.7x slower than the plain ones);
      // the plain path keeps its own loop (uniform branch)
      constexpr int CP_RB = 4;
      if (!rsrc) {
        // all rows of the round read from LDS first, then stored (one ds_read -> wait -> store chain per row
        // exposed the LDS latency 14 times per item)
        bf16x8 rows[2 * RG];
#pragma unroll
        for (int u = 0; u < 2 * RG; ++u)
          if (u < 2 * nj) rows[u] = *reinterpret_cast<const bf16x8*>(so + (u * 8 + (lane >> 3)) * CP_ELD + (lane & 7) * 8);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2 * RG; ++u) {
          if (u < 2 * nj) {
            const int pl = u * 8 + (lane >> 3);  // row of the round
            const int p = wid * 16 * NG + r0 * 16 + pl;
            const int oy = y0 + p / TW, ox = x0 + (p - (p / TW) * TW);
            const bool ok = p < TH * TW && oy < g.Ho && ox < g.Wo;
            const int off = (ok ? oy * g.Wo + ox : 0) * cstride + cofs;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, rows[u]), yrs,
                                                   ok ? off * 2 : 0x7ffffff0, 0, 0);
          }
        }
      } else {
#pragma unroll
      for (int u0 = 0; u0 < 2 * RG; u0 += CP_RB) {
        int offs[CP_RB];
        bool oks[CP_RB];
        bf16x8 rv[CP_RB];
#pragma unroll
        for (int uu = 0; uu < CP_RB; ++uu) {
          const int u = u0 + uu;
          const int pl = u * 8 + (lane >> 3);  // row of the round
          const int p = wid * 16 * NG + r0 * 16 + pl;
          const int oy = y0 + p / TW, ox = x0 + (p - (p / TW) * TW);
          oks[uu] = u < 2 * nj && p < TH * TW && oy < g.Ho && ox < g.Wo;
          offs[uu] = (oks[uu] ? oy * g.Wo + ox : 0) * cstride + cofs;
          if (u < 2 * nj)
            rv[uu] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rrs, offs[uu] * 2, 0, 0));
        }
        bf16x8 rows[CP_RB];
#pragma unroll
        for (int uu = 0; uu < CP_RB; ++uu)
          if (u0 + uu < 2 * nj) rows[uu] = *reinterpret_cast<const bf16x8*>(so + ((u0 + uu) * 8 + (lane >> 3)) * CP_ELD + (lane & 7) * 8);
#pragma unroll
        for (int uu = 0; uu < CP_RB; ++uu) {
          const int u = u0 + uu;
          if (u < 2 * nj) {
            bf16x8 v = rows[uu];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)rv[uu][e]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, oks[uu] ? offs[uu] * 2 : 0x7ffffff0,
                                                   0, 0);
          }
        }
      }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next round overwrites
    }
    if (gnp) {  // after the output stores: exactly 4 more stores (the next step's vmcnt counts them)
      const int b = n / gn_fimg, f = n - b * gn_fimg;
      const int64_t nslot = (int64_t)gn_fimg * tiles_per_img * 4;
      const int64_t slot = ((int64_t)f * tiles_per_img + (y0 / TH) * tiles_x + x0 / TW) * 4 + wid;
      float2* dst = reinterpret_cast<float2*>(gnp) + ((int64_t)b * nslot + slot) * (g.Cout / 4) + n0 / 4 + lg;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = row16_sum(gsum[i]), q = row16_sum(gsq[i]);
        if (lr == 0) dst[i * 4] = make_float2(a, q);
      }
    }
    epi = true;
  }
}

// ----------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 conv (bf16), warp-specialized persistent kernel (round 4).  One block of 8 waves per CU
// (two per SIMD), static item split (item = (image, TH x TW tile of <= 256 px, 64-channel co block), the co blocks
// of a tile on blocks of one XCD):
//   waves 0-3 (compute): 64 co x 64 px each (4 x 4 MFMA tiles), the 9 taps of a 32-channel chunk from a halo +
//     weight stage in LDS (cp_taps: tap t+1's 8 fragment reads between tap t's 16 MFMAs); at an item's last chunk
//     they add the bias and write bf16 rows into a staging tile, and go straight on with the next item;
//   waves 4-7 (load / store): the buffer-LDS-DMA of the next step's stage while the compute waves consume the
//     current one, and the epilogue of the previous item from the staging tile -- residual (prefetched a step
//     ahead), GroupNorm partials, 16-B row stores.
// One s_barrier per step hands the stages over; the compute waves never wait on a load or a store, and the
// epilogue (~40 % of conv3x3p's time at one wave per SIMD, where it could not overlap the MFMAs) runs beside the next
// item's MFMAs.  Both roles pass exactly the same barriers.  LDS: 2 stages x 61 KiB + a 34 KiB staging tile.
// ----------------------------------------------------------------------------------------
// (Round 5, removed: s_setprio for the loader or the compute waves, within the spread -- profiles/r5_prio_ab.txt.)
constexpr int WS_PITCH = 40;                               // halo row pitch (pixels): ky steps keep the swizzle
constexpr int WS_MAXTH = 8;                                // tile rows: (8 + 2) * 40 = 400 halo rows
constexpr int WS_HROWS = (WS_MAXTH + 2) * WS_PITCH;        // 400
constexpr int WS_WROWS = 9 * 64;                           // weight rows (tap * 64 + co)
constexpr int WS_STAGE = (WS_HROWS + WS_WROWS) * 64;       // 62,464 B
constexpr int WS_PIX = 256;                                // pixels per item (4 waves x 4 groups of 16)
constexpr int WS_ELD = 68;                                 // staging row (bf16): 136 B, conflict-free 8-B writes
constexpr int WS_LDS = 2 * WS_STAGE + WS_PIX * WS_ELD * 2;  // 159,744 B
static_assert(WS_LDS + 1024 <= 160 * 1024, "warp-specialized conv LDS");
static_assert(2 * WS_WROWS * 64 + 2 * WS_HROWS * 64 == 2 * WS_STAGE, "resident-weight layout = the two stages");
constexpr int WS_HPMAX = (WS_HROWS / 16 + 3) / 4;          // halo pieces per loader wave (<= 7)
constexpr int WS_WP = WS_WROWS / 16 / 4;                   // weight pieces per loader wave (9)

__device__ __forceinline__ void ws_decode(int it, int ncob, int& tile, int& cb) {
  // co blocks of a tile 8 ids apart: the blocks b, b + 8, ... that take them share an XCD (round-robin placement).
  // (Round 4: items in per-XCD runs of vertically adjacent tiles, so tiles sharing halo rows meet in one L2, measured
  // 514-516 -> 548-552 us per launch in the step, profiles/r4c15_bench_ab.txt; removed.)
  const int g = it / (8 * ncob), r = it - g * 8 * ncob;
  cb = r >> 3;
  tile = g * 8 + (r & 7);
}

template <int TW, bool GN>
__global__ __launch_bounds__(512, 1) void conv3x3ws_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                           const bf16* __restrict__ w, const float* __restrict__ bias,
                                                           const bf16* __restrict__ res, const bf16* __restrict__ res2,
                                                           bf16* __restrict__ y1, bf16* __restrict__ y2, ConvGeom g,
                                                           int TH, int tiles_x, int tiles_per_img, int ncob,
                                                           int nitems_pad, float* __restrict__ gnp, int gn_fimg,
                                                           int* __restrict__ queue) {
  // + the touch loads' never-read rows (1 KiB) + 3 published item ids (dynamic claiming)
  __shared__ __attribute__((aligned(1024))) char lds[WS_LDS + 1024 + 16];
  bf16* stg = reinterpret_cast<bf16*>(lds + 2 * WS_STAGE);
  int* qslot = reinterpret_cast<int*>(lds + WS_LDS + 1024);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool loader = wid >= 4;  // wave-uniform role
  const int wl = wid & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int Cin = g.C1 + g.C2, nchunk = Cin / 32;
  const int ntile = g.Nb * tiles_per_img;
  const int G = (int)gridDim.x;
  // the block's valid items: it = blockIdx.x + k * G (k < nk), tile < ntile; steps = valid items x chunks
  auto next_valid = [&](int it) {
    for (; it < nitems_pad; it += G) {
      int tile, cb;
      ws_decode(it, ncob, tile, cb);
      if (tile < ntile) return it;
    }
    return nitems_pad;
  };
  // Item order.  Static (queue == null): item k of the block is the k-th valid id of blockIdx.x + j * G.  Dynamic
  // (round 5; a caller-owned counter, see cesm_conv_fwd): every item is claimed from queue[0] by one returning atomic
  // add -- a block slowed by co-running kernels (RCCL's, on the communication stream) or placed late takes fewer items
  // (none, if it starts after the queue has run dry) instead of leaving a static split's tail.  Claims run two items
  // ahead so every wave knows item k + 1 (the stage DMA, the L2 touch, the compute waves' bias and loop end) a full
  // item before it starts: loader wave 0 claims item k + 2 at item k's first step and publishes it in
  // qslot[(k + 2) % 3], which every wave reads at item k + 1's first step, a barrier later (the slot it overwrites
  // held item k - 1, read a barrier before); items 0 and 1 are claimed before a block barrier ahead of the loops.
  // The outputs do not depend on the order: an item is one block's whole 9 x Cin sum, and the GroupNorm partial slot
  // belongs to the tile.  Needs nchunk >= 2 (else the static order).  The last block to finish resets the counter,
  // so it is zero again for the next launch on the same stream.
  const bool dyn = queue != nullptr && nchunk >= 2;
  auto claim = [&]() {  // one lane; the next valid claimed id, or nitems_pad
    while (true) {
      const int it = atomicAdd(queue, 1);
      if (it >= nitems_pad) return nitems_pad;
      int tile, cb;
      ws_decode(it, ncob, tile, cb);
      if (tile < ntile) return it;
    }
  };
  auto publish = [&](int k, int val) {  // loader wave 0: item k's id into its slot (readers: after a barrier)
    if (lane == 0) qslot[k % 3] = val;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto finish_queue = [&]() {  // every block once, after its last claim: the last one resets the counter
    if (dyn && tid == 0) {  // (device-scope atomics: no fence, nothing else is published through the counter)
      if (atomicAdd(queue + 1, 1) == G - 1) {
        atomicExch(queue, 0);
        atomicExch(queue + 1, 0);
      }
    }
  };
  auto geo = [&](int it, int& n, int& y0, int& x0, int& cb, int& tile) {
    ws_decode(it, ncob, tile, cb);
    n = tile / tiles_per_img;
    const int r = tile - n * tiles_per_img, ty = r / tiles_x;
    y0 = ty * TH;
    x0 = (r - ty * tiles_x) * TW;
  };

  // ---------------- loader role state
  const int prow = lane >> 2, pslot = lane & 3;
  const int hpieces = ((TH + 2) * WS_PITCH + 15) >> 4;
  int hrel[WS_HPMAX];  // halo piece k of this loader wave: lane row -> (hy << 16 | hx), -1 outside the halo
#pragma unroll
  for (int k = 0; k < WS_HPMAX; ++k) {
    const int row = 16 * (wl + 4 * k) + prow;
    const int hy = row / WS_PITCH, hx = row - hy * WS_PITCH;
    hrel[k] = (hy < TH + 2 && hx < TW + 2) ? (hy << 16) | hx : -1;
  }
  // RW (resident weights): with 64 input channels and one co block the two weight chunks never change, so
  // they are staged once and the per-step DMA carries only the halo chunk (25 KB instead of 61 KB: the LDS-DMA
  // fill rate per CU, not HBM, bounded the step).  The layout is the same 156 KB rearranged: weight chunks 0 / 1 at
  // [0, 73728), halo stages at 73728 + st * 25600 (else stage st = halo + weights at st * WS_STAGE).
  const bool rw = Cin == 64 && ncob == 1;
  auto hbase = [&](int st) { return lds + (rw ? 2 * WS_WROWS * 64 + st * WS_HROWS * 64 : st * WS_STAGE); };
  auto wbase = [&](int st, int ch) { return rw ? lds + ch * WS_WROWS * 64 : lds + st * WS_STAGE + WS_HROWS * 64; };
  auto issue_w = [&](int cb, int ch, char* dst) {  // the weight chunk ch of co block cb
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(w + ((int64_t)cb * (Cin / 32) + ch) * (9 * 64 * 32)), (short)0, 9 * 64 * 32 * 2, 0x00020000);
#pragma unroll
    for (int k = 0; k < WS_WP; ++k) {  // one contiguous tile of the chunked pack (wpk_index)
      const int q = wl + 4 * k, row = 16 * q + prow;  // row = tap * 64 + co
      const int chunk = pslot ^ cw_swz(row);
      const int vo = (row * 32 + chunk * 8) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, vo,
                                               0, 0, 0);
    }
  };
  auto issue_stage = [&](int it, int ch, int st) {  // loader waves: chunk ch of item it -> stage st
    int n, y0, x0, cb, tile;
    geo(it, n, y0, x0, cb, tile);
    const int c0 = ch * 32;
    const bf16* src;
    int cs, cc;
    if (c0 < g.C1) { src = x1; cs = g.C1; cc = c0; } else { src = x2; cs = g.C2; cc = c0 - g.C1; }
    const int64_t img = (int64_t)g.Hi * g.Wi * cs;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + n * img + cc), (short)0, (int)(img * 2 - cc * 2), 0x00020000);
    char* dst = hbase(st);
#pragma unroll
    for (int k = 0; k < WS_HPMAX; ++k) {
      const int q = wl + 4 * k;
      if (q < hpieces) {  // wave-uniform
        const int chunk = pslot ^ cw_swz(16 * q + prow);
        const int iy = y0 - 1 + (hrel[k] >> 16), ix = x0 - 1 + (hrel[k] & 0xffff);
        const bool in = hrel[k] >= 0 && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
        const int vo = in ? ((iy * g.Wi + ix) * cs + chunk * 8) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, vo,
                                                 0, 0, 0);
      }
    }
    if (!rw) issue_w(cb, ch, wbase(st, ch));
  };
  // epilogue rows of loader wave wl: pixels 64 wl + 8 u + (lane >> 3), u = 0..7, channels (lane & 7) * 8 .. + 7
  bf16x8 resv[8];
  auto out_px = [&](int y0, int x0, int u, int& oy, int& ox, bool& ok) {
    const int p = 64 * wl + 8 * u + (lane >> 3);
    const int py = p / TW, px = p - py * TW;
    oy = y0 + py;
    ox = x0 + px;
    ok = py < TH && oy < g.Ho && ox < g.Wo;
  };
  auto out_rsrc = [&](int n, int cb, const bf16* a1, const bf16* a2, int& cofs, int& cstride) {
    const int n0 = cb * 64;
    const bool first = n0 < g.Co1;
    cstride = first ? g.Co1 : g.Cout - g.Co1;
    cofs = (first ? n0 : n0 - g.Co1) + (lane & 7) * 8;
    const bf16* base = first ? a1 : a2;
    const int64_t img = (int64_t)n * g.Ho * g.Wo * cstride;
    return __builtin_amdgcn_make_buffer_rsrc((void*)((base ? base : y1) + img), (short)0, g.Ho * g.Wo * cstride * 2,
                                             0x00020000);
  };
  auto load_res = [&](int it) {  // residual rows of item it (issued a step before its epilogue)
    int n, y0, x0, cb, tile;
    geo(it, n, y0, x0, cb, tile);
    int cofs, cstride;
    const __amdgpu_buffer_rsrc_t rrs = out_rsrc(n, cb, res, res2, cofs, cstride);
    const bool have = (cb * 64 < g.Co1 ? res : res2) != nullptr;  // this split's residual (none: loads return 0)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int oy, ox;
      bool ok;
      out_px(y0, x0, u, oy, ox, ok);
      const int off = have ? ((ok ? oy * g.Wo + ox : 0) * cstride + cofs) * 2 : 0x7ffffff0;
      resv[u] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rrs, off, 0, 0));
    }
  };
  const bool has_res = (res != nullptr) || (res2 != nullptr);
  // L2 touch of the next item's input halo: one 4-B load per halo pixel line of x1, issued at an item's
  // first step, so the stage DMA of that item -- a step later -- finds its lines in L2 instead of waiting out HBM
  // latency with one stage in flight.  Covers every channel of a pixel when C1 * 2 <= 128 B (level 0).  The loads
  // go LDS-direct into a never-read 256-B row per loader wave: no VGPRs held while they fly.
  auto touch = [&](int it) {
    int n, y0, x0, cb, tile;
    geo(it, n, y0, x0, cb, tile);
    const int64_t img = (int64_t)g.Hi * g.Wi * g.C1;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(x1 + n * img), (short)0, (int)(img * 2), 0x00020000);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = lane + 64 * (wl + 4 * k);
      const int hy = q / (TW + 2), hx = q - hy * (TW + 2);
      const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
      const bool in = hy < TH + 2 && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(lds + WS_LDS + wl * 256),
                                               4, in ? (iy * g.Wi + ix) * g.C1 * 2 : 0x7ffffff0, 0, 0, 0);
    }
  };
  // s_waitcnt vmcnt(n) for the counts the loader loop leaves in flight
  auto vm_wait = [&](int n) {
    switch (n) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
      case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
      case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
      case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
      case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
      case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
      case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  };
  // epilogue of item it from the staging tile; returns after issuing its stores (8 rows + GN partial)
  auto epilogue = [&](int it) {
    int n, y0, x0, cb, tile;
    geo(it, n, y0, x0, cb, tile);
    bf16x8 rows[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      rows[u] = *reinterpret_cast<const bf16x8*>(stg + (64 * wl + 8 * u + (lane >> 3)) * WS_ELD + (lane & 7) * 8);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int cofs, cstride;
    const __amdgpu_buffer_rsrc_t yrs = out_rsrc(n, cb, y1, y2, cofs, cstride);
    float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int oy, ox;
      bool ok;
      out_px(y0, x0, u, oy, ox, ok);
      bf16x8 v = rows[u];
      if (has_res) {  // uniform
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)resv[u][e]);
      }
      if constexpr (GN) {  // statistics of the stored bf16 y (a GroupNorm conv has no residual)
        const float m = ok ? 1.f : 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float a0 = (float)v[4 * h], a1 = (float)v[4 * h + 1], a2 = (float)v[4 * h + 2], a3 = (float)v[4 * h + 3];
          gs[h] = fmaf(m, (a0 + a1) + (a2 + a3), gs[h]);
          gq[h] = fmaf(m, fmaf(a3, a3, fmaf(a2, a2, fmaf(a1, a1, a0 * a0))), gq[h]);
        }
      }
      const int off = ok ? ((oy * g.Wo + ox) * cstride + cofs) * 2 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, off, 0, 0);
    }
    if constexpr (GN) {
      // lanes with equal (lane & 7) hold the same 8 channels: sum over lane bits 3..5 (fixed order)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {
          gs[h] += __shfl_xor(gs[h], o, 64);
          gq[h] += __shfl_xor(gq[h], o, 64);
        }
      }
      const int b = n / gn_fimg, f = n - b * gn_fimg;
      const int64_t nslot = (int64_t)gn_fimg * tiles_per_img * 4;
      const int64_t slot = ((int64_t)f * tiles_per_img + (tile - n * tiles_per_img)) * 4 + wl;
      // [B][nslot][C/4] float2: this wave's slot, the co block's 16 quads; lane c < 8 writes quads 2c, 2c + 1
      float* dst = gnp + (((int64_t)b * nslot + slot) * (g.Cout / 4) + cb * 16) * 2;
      const f32x4 v4 = {gs[0], gq[0], gs[1], gq[1]};
      const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, 128, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v4), grs, lane < 8 ? lane * 16 : 0x7ffffff0, 0,
                                             0);
    }
  };

  // ---------------- compute role state
  int bad[4][3];
  {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 64 * wl + 16 * j + lr;
      const int py = p / TW, px = p - py * TW;
      const int h0 = py < TH ? py * WS_PITCH + px : 0;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) bad[j][kx] = cw_off(h0 + kx, lg);
    }
  }
  const int a_lane = (lr << 6) + ((lg ^ cw_swz(lr)) << 4);
  f32x4 bv4[4];  // the item's bias (co = i * 16 + 4 lg + r), loaded at its first chunk, used at its last
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---------------- the step loops: one per role, the same sequence of steps and barriers (a loop per role keeps
  // the two roles' registers apart: one shared loop held the loader's residual rows live through the MFMAs)
  int it0;
  if (dyn) {  // items 0 and 1, claimed by loader wave 0 and published before a block barrier
    if (wid == 4) {
      int s0 = nitems_pad, s1 = nitems_pad;
      if (lane == 0) {
        s0 = claim();
        if (s0 < nitems_pad) s1 = claim();
      }
      publish(0, __builtin_amdgcn_readfirstlane(s0));
      publish(1, __builtin_amdgcn_readfirstlane(s1));
    }
    __syncthreads();
    it0 = qslot[0];
    if (it0 >= nitems_pad) {  // the queue ran dry before this block started (whole block)
      finish_queue();
      return;
    }
  } else {
    it0 = next_valid((int)blockIdx.x);
    if (it0 >= nitems_pad) return;  // whole block, before any barrier
  }
  // the item after `it` (item k): static order, or the published claim (read at item k's first step)
  auto successor = [&](int k, int it) { return dyn ? qslot[(k + 1) % 3] : next_valid(it + G); };
  if (loader) {
    if (rw) {
      issue_w(0, 0, wbase(0, 0));
      issue_w(0, 1, wbase(0, 1));
    }
    issue_stage(it0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int it = it0, ch = 0, s = 0, prev_it = -1, k = 0, succ = nitems_pad;
    const bool do_touch = g.C1 * 2 <= 128 && nchunk >= 2;
    while (true) {
      __builtin_amdgcn_s_barrier();  // stage s landed; stage s - 1 consumed; staging of prev_it written (ch == 0)
      if (ch == 0) {
        succ = successor(k, it);
        if (dyn && wid == 4) {  // claim item k + 2 (none once the queue has run dry)
          int s2 = nitems_pad;
          if (lane == 0 && succ < nitems_pad) s2 = claim();
          publish(k + 2, __builtin_amdgcn_readfirstlane(s2));
        }
      }
      const int nxt_ch = ch + 1 < nchunk ? ch + 1 : 0;
      const int nxt_it = ch + 1 < nchunk ? it : succ;
      const bool more = nxt_it < nitems_pad;
      const bool epi = ch == 0 && prev_it >= 0;
      if (epi) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // residual rows of prev_it
      if (more) issue_stage(nxt_it, nxt_ch, (s + 1) & 1);
      if (epi) epilogue(prev_it);
      // the next step ends item nxt_it (nchunk >= 2): its residual rows now, in registers at its epilogue
      const bool pre = more && has_res && nxt_ch == nchunk - 1;
      if (pre) load_res(nxt_it);
      // the item after next: its halo lines into L2 while this item's chunks run
      int tit = nitems_pad;
      if (do_touch && ch == 0) tit = succ;
      const bool tch = tit < nitems_pad;
      if (tch) touch(tit);
      // wait for this step's DMA only: the epilogue's stores (8 rows [+ 1 GN partial]), the residual loads (8) and
      // the touches (2) issued after it may stay in flight
      vm_wait((epi ? (GN ? 9 : 8) : 0) + (pre ? 8 : 0) + (tch ? 2 : 0));
      if (ch == nchunk - 1) {
        prev_it = it;
        ++k;
      }
      ch = nxt_ch;
      it = nxt_it;
      ++s;
      if (!more) break;
    }
    __builtin_amdgcn_s_barrier();  // the last item's staging rows written
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    epilogue(prev_it);
  } else {
    int it = it0, ch = 0, s = 0, k = 0, succ = nitems_pad;
    while (true) {
      __builtin_amdgcn_s_barrier();  // stage s landed; the staging tile free again (ch == 0)
      if (ch == 0) succ = successor(k, it);
      const int nxt_ch = ch + 1 < nchunk ? ch + 1 : 0;
      const int nxt_it = ch + 1 < nchunk ? it : succ;
      if (ch == 0) {
        int n, y0, x0, cb, tile;
        geo(it, n, y0, x0, cb, tile);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          bv4[i] = bias ? *reinterpret_cast<const f32x4*>(bias + cb * 64 + i * 16 + lg * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      cp_taps<4>(hbase(s & 1), wbase(s & 1, ch), bad, a_lane, acc);
      if (ch == nchunk - 1) {  // item end: (acc + bias) as bf16 rows of the staging tile
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = i * 16 + lg * 4;
          const f32x4 bv = bv4[i];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v[4] = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
            store4(stg + (64 * wl + 16 * j + lr) * WS_ELD + co, v);
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
        ++k;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging rows visible at the barrier
      ch = nxt_ch;
      it = nxt_it;
      ++s;
      if (it >= nitems_pad) break;
    }
    __builtin_amdgcn_s_barrier();  // pairs with the loaders' last barrier
  }
  finish_queue();
}

// ----------------------------------------------------------------------------------------
// 1x1 conv (bf16) as a GEMM: Y[m][co] = bias[co] + res[m][co] + sum_k X[m][k] W[co][k], X = [x1 | x2]
// concatenated on channels, Y = [y1 | y2] split at Co1.  Block = 128 pixels x BN output channels
// (the co blocks of a pixel tile run back to back on one XCD, sharing its X rows in L2); K in steps of 64
// through two LDS stages filled by buffer-LDS-DMA (128-B rows, 16-B chunk index XORed with row & 7,
// out-of-range rows -> zeros); 4 waves = 2 (co halves) x 2 (64-pixel halves).  The epilogue stages
// (acc + bias) as bf16 pixel rows in LDS and writes them (+ residual) with coalesced 16-B accesses.
// Replaces the generic implicit-GEMM path for every 1x1 conv: attention projections at levels with
// C >= 128, res_conv, and their data gradients.  NS = 1 (K = 64: one LDS stage, 35 KB) runs 4 blocks per
// CU instead of 2: the K = 64 projections (to_qkv 64 -> 768 of the long-window level 0) are output-store
// streams whose per-block load -> MFMA -> store phases need the extra blocks to overlap.  The X buffer
// resource covers the block's own 128 rows only, so M * K is not limited to 2^31 bytes.
// ----------------------------------------------------------------------------------------
constexpr int G1_BM = 128;
// (Measured and removed: non-temporal output stores -- GEMMs 5 % faster alone, whole step unchanged (round 3) and
// within the spread on the F = 120 leg (round 5, profiles/r5f_g1nt_f120_ab.txt); co-block-fastest block order.)
__device__ __forceinline__ int g1_off(int row, int chunk) { return (row << 7) + ((chunk ^ (row & 7)) << 4); }

template <int BN, int NS>
__global__ __launch_bounds__(256, NS == 1 ? 4 : 2) void gemm1x1_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                         const bf16* __restrict__ w, const float* __restrict__ bias,
                                                         const bf16* __restrict__ res, const bf16* __restrict__ res2,
                                                         bf16* __restrict__ y1, bf16* __restrict__ y2, int M, int C1,
                                                         int C2, int Cout, int Co1) {
  constexpr int STAGE = (G1_BM + BN) * 128;  // bytes
  constexpr int TM = BN / 32;                // 16-co fragments per wave
  constexpr int ELD = BN + 8;                // epilogue row (bf16)
  constexpr int LDSB = NS * STAGE > G1_BM * ELD * 2 ? NS * STAGE : G1_BM * ELD * 2;
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int K = C1 + C2, nk = K / 64;
  // 1-D grid: the ncb co blocks of a pixel tile are dealt to ONE XCD back to back (linear id mod 8 = XCD), so
  // the tile's X rows are fetched into that XCD's L2 once instead of into up to ncb different L2s
  const int ncb = Cout / BN, L = blockIdx.x, jx = L >> 3;
  const int cb = jx % ncb;
  const int tile = (jx / ncb) * 8 + (L & 7);
  if (tile * G1_BM >= M) return;  // padded tiles (whole block)
  const int m0 = tile * G1_BM, n0 = cb * BN;
  const int prow = lane >> 3, pslot = lane & 7;

  auto issue = [&](int ks) {
    const int c0 = ks * 64;
    const bf16* src;
    int cs, cc;
    if (c0 < C1) { src = x1; cs = C1; cc = c0; } else { src = x2; cs = C2; cc = c0 - C1; }
    const int rows = M - m0 < G1_BM ? M - m0 : G1_BM;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(src + (int64_t)m0 * cs + cc), (short)0, rows * cs * 2 - cc * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(w + (int64_t)n0 * K + c0), (short)0, BN * K * 2 - c0 * 2, 0x00020000);
    char* sx = lds + (NS == 2 ? (ks & 1) * STAGE : 0);
    char* sw = sx + G1_BM * 128;
#pragma unroll
    for (int k = 0; k < G1_BM / 32; ++k) {  // 8-row pieces, 4 per wave
      const int q = wid + 4 * k, row = 8 * q + prow;
      const int chunk = pslot ^ (row & 7);
      const int vo = m0 + row < M ? (row * cs + chunk * 8) * 2 : 0x7ffffff0;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (__attribute__((address_space(3))) void*)(sx + q * 1024), 16, vo, 0,
                                               0, 0);
    }
#pragma unroll
    for (int k = 0; k < BN / 32; ++k) {
      const int q = wid + 4 * k, row = 8 * q + prow;
      const int chunk = pslot ^ (row & 7);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(sw + q * 1024), 16,
                                               (row * K + chunk * 8) * 2, 0, 0, 0);
    }
  };

  f32x4 acc[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  for (int ks = 0; ks < nk; ++ks) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage ks landed for all waves; stage ks+1's previous reads (step ks-1) are done
    if (NS == 2 && ks + 1 < nk) issue(ks + 1);
    const char* sx = lds + (NS == 2 ? (ks & 1) * STAGE : 0);
    const char* sw = sx + G1_BM * 128;
#pragma unroll
    for (int k32 = 0; k32 < 2; ++k32) {
      const int chunk = k32 * 4 + lg;
      bf16x8 af[TM], bfr[4];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sw + g1_off(wr * (BN / 2) + i * 16 + lr, chunk));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sx + g1_off(wc * 64 + j * 16 + lr, chunk));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // all fragment reads done: reuse the stages for the output tile
  bf16* so = reinterpret_cast<bf16*>(lds);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = wr * (BN / 2) + i * 16 + lg * 4;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bias[n0 + co + r];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = wc * 64 + j * 16 + lr;
      float v[4] = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
      store4(so + p * ELD + co, v);
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per pixel row
  constexpr int NIT = G1_BM * CPR / 256;
  const int Co2 = Cout - Co1;
  // residual vectors of every iteration issued together, unpredicated (clamped address, selected
  // after): under the lane predicates each was a branch with its own vmcnt(0)
  bf16x8 rv[NIT];
  if (res || res2) {  // uniform
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = it * 256 + tid;
      const int p = e / CPR, c = e - p * CPR;
      const int m = m0 + p, co = n0 + c * 8;
      const bool first = co < Co1;
      const bf16* rp = first ? res : res2;
      const bool use = m < M && rp != nullptr;
      const int64_t off = use ? (first ? (int64_t)m * Co1 + co : (int64_t)m * Co2 + (co - Co1)) : 0;
      const bf16x8 t = *reinterpret_cast<const bf16x8*>((use ? rp : (res ? res : res2)) + off);
      rv[it] = use ? t : bf16x8{};
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = it * 256 + tid;
    const int p = e / CPR, c = e - p * CPR;
    const int m = m0 + p;
    if (m >= M) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(so + p * ELD + c * 8);
    const int co = n0 + c * 8;
    bf16* dst = co < Co1 ? y1 + (int64_t)m * Co1 + co : y2 + (int64_t)m * Co2 + (co - Co1);
    if (res || res2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = (bf16)((float)v[q] + (float)rv[it][q]);
    }
    *reinterpret_cast<bf16x8*>(dst) = v;  // (round 6: non-temporal here -- isolated 1x1 convs 9 % faster, the F = 12
                                          // step and the F = 120 leg unchanged, profiles/r6late_g1_nontemporal_ab.txt)
  }
}


// ----------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 conv (bf16), v2: persistent, software-pipelined halo conv.
// Work item = (TH x TW pixel tile of one image, 64 output channels); a block streams the
// (item, 32-channel chunk) sequence through two LDS stages filled by global_load_lds (LDS-DMA, no
// VGPR staging): the loads of step s+2 are issued as soon as step s's stage is released and stay in
// flight across the raw barriers (counted s_waitcnt vmcnt).  Stage = halo [(TH+2)(TW+2) <= 384 px]
// [32 ch] + weights [9 taps x 64 co][32 ci], 64-B rows with the 16-B chunk index XORed by
// (row >> 2) & 3 (conflict-free fragment reads).  Generic TW lets W = 36 / 72 / 144 levels use
// 36-wide tiles instead of wasting 25-44 % of a 32-wide tiling.  4 waves = 2 (co halves) x 2
// (pixel halves); wave tile 32 co x 128 px, 16 MFMA per tap.
// ----------------------------------------------------------------------------------------
constexpr int C2_HROWS = 384;                 // halo rows per stage (>= (TH+2)(TW+2))
constexpr int C2_HALO_B = C2_HROWS * 64;      // 24 KiB
constexpr int C2_W_B = 9 * 64 * 64;           // 36 KiB
constexpr int C2_STAGE_B = C2_HALO_B + C2_W_B;
constexpr int C2_NI = C2_HROWS / 16 + 9 * 64 / 16;  // wave-instructions per stage (60)
constexpr int C2_NPW = C2_NI / 4;                   // per wave (15)
static_assert(C2_NI % 4 == 0, "glds instructions must split evenly over the 4 waves");
__device__ __attribute__((aligned(16))) bf16 c2_zero_page[8] = {};

__device__ __forceinline__ int c2_swz(int row) { return (row >> 2) & 3; }

// tile shape for an Ho x Wo image: TW in {32, 36, 48}, TH*TW <= 256, (TH+2)(TW+2) <= 384; maximise
// useful / computed pixels (fewest tiles on ties)
static void c2_tile(int Ho, int Wo, int& TH, int& TW, bool only_32_36 = false) {
  double best = -1.0;
  int bt = 1 << 30;
  const int cands[3] = {32, 36, 48};
  for (int c = 0; c < (only_32_36 ? 2 : 3); ++c) {
    const int tw = cands[c];
    for (int th = 1; th * tw <= 256; ++th) {
      if ((th + 2) * (tw + 2) > C2_HROWS) break;
      const int ntile = (int)(cdiv(Ho, th) * cdiv(Wo, tw));
      const double util = (double)Ho * Wo / ((double)ntile * 256);
      // a non-32 width must buy > 10 % utilisation (32-wide tiles align with the fragment rows)
      const double u = tw == 32 ? util + 0.10 : util;
      if (u > best + 1e-9 || (u > best - 1e-9 && ntile < bt)) { best = u; bt = ntile; TH = th; TW = tw; }
    }
  }
}

// warp-specialized conv tile: TW in {32, 36} (halo width <= WS_PITCH), TH * TW <= 256; returns the pixel utilisation
static double ws_tile(int Ho, int Wo, int& TH, int& TW) {
  double best = -1.0;
  for (int tw : {32, 36}) {
    for (int th = 1; th <= WS_MAXTH && th * tw <= WS_PIX; ++th) {
      const double util = (double)Ho * Wo / ((double)cdiv(Ho, th) * cdiv(Wo, tw) * WS_PIX);
      if (util > best + 1e-9) { best = util; TH = th; TW = tw; }
    }
  }
  return best;
}

// halo-conv tile for the 448-pixel blocks (conv3x3_bf16_kernel<TW, 7>): TW in {32, 36}, TH*TW <= 448,
// TH + 2 <= 16 halo rows; the most useful / computed pixels, a 32-wide tile needs > 5 % better utilisation
static void h3_big_tile(int Ho, int Wo, int& TH, int& TW) {
  double best = -1.0;
  int bt = 1 << 30;
  for (int tw : {36, 32}) {
    for (int th = 1; th * tw <= 448 && th + 2 <= 16; ++th) {
      const int ntile = (int)(cdiv(Ho, th) * cdiv(Wo, tw));
      const double util = (double)Ho * Wo / ((double)ntile * 448);
      const double u = tw == 32 ? util - 0.05 : util;
      if (u > best + 1e-9 || (u > best - 1e-9 && ntile < bt)) { best = u; bt = ntile; TH = th; TW = tw; }
    }
  }
}

// ----------------------------------------------------------------------------------------
// weight-gradient kernel: slab[split][co][tap*Cin + ci] = sum over the split's pixels of
//   dY[m][co] * X(m, tap, ci)
// Pixel axis is the MFMA K.  Output tile 64 co x 64 K-columns (one tap, 64 channels).
// ----------------------------------------------------------------------------------------
constexpr int WG_BP = 32;   // pixels per step

template <typename T>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const T* __restrict__ x1, const T* __restrict__ x2,
                                                         const T* __restrict__ dy1, const T* __restrict__ dy2,
                                                         float* __restrict__ slab, ConvGeom g, int64_t M,
                                                         int64_t px_per_split) {
  // LDS tiles are [pixel][64] row-major; bf16 rows are XOR-swizzled in 8-byte chunks so the
  // transposed reads (ds_read_b64_tr_b16) are conflict free.
  constexpr int VEC = sizeof(T) == 2 ? 8 : 4;
  constexpr int ROW = 64;                    // elements per row
  constexpr int LDR = sizeof(T) == 2 ? 64 : 65;
  __shared__ __attribute__((aligned(16))) T tY[2][WG_BP * LDR];
  __shared__ __attribute__((aligned(16))) T tX[2][WG_BP * LDR];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;       // wave owns co [wr*32,+32) x kcol [wc*32,+32)
  const int Cin = g.C1 + g.C2;
  const int co0 = blockIdx.x * 64;
  const int kcol0 = blockIdx.y * 64;           // global K column (tap*Cin + ci)
  const int tap = kcol0 / Cin;
  const int ci0 = kcol0 - tap * Cin;
  const int ky = tap / g.KW, kx = tap - ky * g.KW;
  const int64_t pbeg = (int64_t)blockIdx.z * px_per_split;
  const int64_t pend = min(M, pbeg + px_per_split);

  const T* xs; int xcs, xcc;
  if (ci0 < g.C1) { xs = x1; xcs = g.C1; xcc = ci0; } else { xs = x2; xcs = g.C2; xcc = ci0 - g.C1; }
  const T* ys; int ycs, ycc;
  const int Co2 = g.Cout - g.Co1;
  if (co0 < g.Co1) { ys = dy1; ycs = g.Co1; ycc = co0; } else { ys = dy2; ycs = Co2; ycc = co0 - g.Co1; }

  constexpr int VPR = ROW / VEC;             // 8 (bf16) / 16 (f32) vectors per row
  constexpr int RPP = 256 / VPR;             // rows per pass: 32 / 16
  constexpr int NP = WG_BP / RPP;            // passes: 1 / 2
  const int vrow = tid / VPR, vcol = (tid % VPR) * VEC;

  float xr[NP][VEC], yr[NP][VEC];
  auto gload = [&](int64_t p0) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int64_t m = p0 + vrow + p * RPP;
      bool ok = m < pend;
      if (ok) {
        if constexpr (VEC == 8) load8(ys + m * ycs + ycc + vcol, yr[p]); else load4(ys + m * ycs + ycc + vcol, yr[p]);
        const int ox = (int)(m % g.Wo);
        const int64_t t = m / g.Wo;
        const int oy = (int)(t % g.Ho);
        const int n = (int)(t / g.Ho);
        int iy, ix;
        if (tap_src(g, oy, ox, ky, kx, iy, ix)) {
          const T* ptr = xs + ((((int64_t)n * g.Hi + iy) * g.Wi + ix) * xcs + xcc + vcol);
          if constexpr (VEC == 8) load8(ptr, xr[p]); else load4(ptr, xr[p]);
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) xr[p][i] = 0.f;
        }
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) { xr[p][i] = 0.f; yr[p][i] = 0.f; }
      }
    }
  };
  auto swz = [](int r) { return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3); };  // in 4-element chunks
  auto sstore = [&](int buf) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = vrow + p * RPP;
      if constexpr (sizeof(T) == 2) {
        const int ch = (vcol >> 2) ^ swz(r);
        store8(tY[buf] + r * LDR + ch * 4, yr[p]);
        store8(tX[buf] + r * LDR + ch * 4, xr[p]);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          tY[buf][r * LDR + vcol + i] = yr[p][i];
          tX[buf][r * LDR + vcol + i] = xr[p][i];
        }
      }
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (int)((pend - pbeg + WG_BP - 1) / WG_BP);
  if (nsteps > 0) {
    gload(pbeg);
    sstore(0);
  }
  __syncthreads();
  const int lr = lane & 15, lg = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) gload(pbeg + (int64_t)(s + 1) * WG_BP);
    if constexpr (sizeof(T) == 2) {
      // fragment (rows 0..15 of a 16-wide column block c0): lane group lg needs pixel rows
      // 8lg..8lg+7; tr read: lane 4q+p addresses row (8lg + q [+4]), columns c0 + 4p.
      const int q = lr >> 2, pp = lr & 3;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c0 = wr * 32 + i * 16;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int r = lg * 8 + half * 4 + q;
          const int ch = ((c0 >> 2) + pp) ^ swz(r);
          s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tY[buf] + r * LDR + ch * 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[i][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c0 = wc * 32 + j * 16;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int r = lg * 8 + half * 4 + q;
          const int ch = ((c0 >> 2) + pp) ^ swz(r);
          s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tX[buf] + r * LDR + ch * 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[j][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      // fp32 16x16x4: lane holds A[row lr][k = lg] and B[k = lg][col lr]; 8 k-steps of 4 pixels
#pragma unroll
      for (int kk = 0; kk < WG_BP / 4; ++kk) {
        const int r = kk * 4 + lg;
        float a0 = tY[buf][r * LDR + wr * 32 + lr];
        float a1 = tY[buf][r * LDR + wr * 32 + 16 + lr];
        float b0 = tX[buf][r * LDR + wc * 32 + lr];
        float b1 = tX[buf][r * LDR + wc * 32 + 16 + lr];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) sstore(buf ^ 1);
    __syncthreads();
  }
  // D[row = co][col = kcol]: lane holds col lr, rows 4lg + r
  const int K = g.KH * g.KW * Cin;
  float* out = slab + (int64_t)blockIdx.z * g.Cout * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kc = kcol0 + wc * 32 + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wr * 32 + i * 16 + lg * 4 + r;
        out[(int64_t)co * K + kc] = acc[i][j][r];
      }
    }
}

// ----------------------------------------------------------------------------------------
// bf16 weight gradient with wide output tiles: BM output channels x 64 K-columns (one tap, 64 input
// channels) per block, pixels split over grid.z.  Same MFMA scheme as conv_wgrad_kernel (pixels are
// the MFMA K axis, both operands read with ds_read_b64_tr_b16), but
//   * BM = 128/256 rows amortise each input tile over 2-4x more output channels (fewer x re-reads);
//   * the input pixel coordinates are advanced incrementally (no 64-bit div/mod per load);
//   * wave w owns rows [w*BM/4, +BM/4) x all 64 columns.
// ----------------------------------------------------------------------------------------
template <int BM>
__device__ __forceinline__ int wgb_swz(int r) {  // XOR on 4-element chunk index of a BM-wide row
  if constexpr (BM == 64) return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3);
  else return 4 * ((r & 3) | (((r >> 3) & 1) << 2));
}

// bslab (nullable): the conv bias gradient sum_px dY[px][co] comes out of the same K loop — the blocks
// of the first K tile multiply their dY fragments by a ones operand (MT extra MFMAs per step, no extra
// memory traffic) and write per-split partials bslab[z][co] (replaces a separate column-sum pass
// over dY, which re-read the whole tensor).
// (BIAS: compile-time, so the plain instantiation keeps its register count — the bias accumulators
// pushed the BM = 256 kernel past 128 VGPRs, a wave per SIMD fewer and 43 % slower.)
// (Round 3 measured an XCD-grouped 1-D grid for a pixel split's tiles: whole step 130.4 -> 131.5 ms; removed.)
// wgrad_wide: register allocation for >= 2 waves per SIMD (256 registers).  With the unconstrained 512-register
// budget the compiler kept the accumulators in VGPRs and copied each one into a[0:3] before its MFMA and back after
// (AGPR-form MFMAs: 64 v_accvgpr_write + 64 v_accvgpr_read + s_nop per 16 MFMAs in the BM = 256 loop, 244 + 40
// registers); capped: VGPR-form MFMAs, no copies, 178 / 122 / 68 registers at BM = 256 / 128 / 64.
template <int BM, bool BIAS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_wide_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                         const bf16* __restrict__ dy1, const bf16* __restrict__ dy2,
                                                         float* __restrict__ slab, float* __restrict__ bslab, ConvGeom g,
                                                         int M, int px_per_split) {
  constexpr int VPRY = BM / 8, RPPY = 256 / VPRY, NPY = WG_BP / RPPY;
  constexpr int MT = BM / 64;  // 16-row co tiles per wave
  __shared__ __attribute__((aligned(16))) bf16 tY[2][WG_BP * BM];
  __shared__ __attribute__((aligned(16))) bf16 tX[2][WG_BP * 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int Cin = g.C1 + g.C2;
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  const int co0 = bx * BM;
  const int kcol0 = by * 64;
  const int tap = kcol0 / Cin;
  const int ci0 = kcol0 - tap * Cin;
  const int ky = tap / g.KW, kx = tap - ky * g.KW;
  const int pbeg = bz * px_per_split;
  const int pend = min(M, pbeg + px_per_split);
  const bf16* xs; int xcs, xcc;
  if (ci0 < g.C1) { xs = x1; xcs = g.C1; xcc = ci0; } else { xs = x2; xcs = g.C2; xcc = ci0 - g.C1; }
  const bf16* ys; int ycs, ycc;
  const int Co2 = g.Cout - g.Co1;
  if (co0 < g.Co1) { ys = dy1; ycs = g.Co1; ycc = co0; } else { ys = dy2; ycs = Co2; ycc = co0 - g.Co1; }

  // x-tile role: one 8-channel vector of one pixel row per thread; its output coordinates advance by
  // WG_BP pixels per step
  const int xrow = tid >> 3, xcol = (tid & 7) * 8;
  int m = pbeg + xrow;
  int ox, oy, on;
  {
    const int hw = g.Ho * g.Wo;
    on = m / hw;
    const int rem = m - on * hw;
    oy = rem / g.Wo;
    ox = rem - oy * g.Wo;
  }
  const int yrow0 = tid / VPRY, ycol = (tid % VPRY) * 8;

  bf16x8 xr2[2], yr2[2][NPY];  // two steps in flight (register slot = step parity)
  auto gload = [&](int p0, auto slotc) {
    constexpr int slot = decltype(slotc)::value;
    bf16x8& xr = xr2[slot];
    bf16x8 (&yr)[NPY] = yr2[slot];
#pragma unroll
    for (int p = 0; p < NPY; ++p) {
      const int mm = p0 + yrow0 + p * RPPY;
      if (mm < pend) yr[p] = *reinterpret_cast<const bf16x8*>(ys + (int64_t)mm * ycs + ycc + ycol);
      else {
#pragma unroll
        for (int i = 0; i < 8; ++i) yr[p][i] = (bf16)0.f;
      }
    }
    int iy, ix;
    if (m < pend && tap_src(g, oy, ox, ky, kx, iy, ix))
      xr = *reinterpret_cast<const bf16x8*>(xs + (((int64_t)on * g.Hi + iy) * g.Wi + ix) * xcs + xcc + xcol);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) xr[i] = (bf16)0.f;
    }
    // advance this thread's pixel by one step
    m += WG_BP;
    ox += WG_BP;
    while (ox >= g.Wo) {
      ox -= g.Wo;
      if (++oy >= g.Ho) { oy = 0; ++on; }
    }
  };
  auto sstore = [&](auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    const bf16x8& xr = xr2[buf];
    const bf16x8 (&yr)[NPY] = yr2[buf];
#pragma unroll
    for (int p = 0; p < NPY; ++p) {
      const int r = yrow0 + p * RPPY;
      const int ch = (ycol >> 2) ^ wgb_swz<BM>(r);
      *reinterpret_cast<bf16x8*>(tY[buf] + r * BM + ch * 4) = yr[p];
    }
    const int ch = (xcol >> 2) ^ wgb_swz<64>(xrow);
    *reinterpret_cast<bf16x8*>(tX[buf] + xrow * 64 + ch * 4) = xr;
  };

  f32x4 acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool bias_blk = BIAS && by == 0;  // uniform
  f32x4 bacc[BIAS ? MT : 1];
#pragma unroll
  for (int i = 0; i < (BIAS ? MT : 1); ++i) bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;
  const int nsteps = (pend - pbeg + WG_BP - 1) / WG_BP;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (nsteps > 0) {
    gload(pbeg, I0{});
    if (nsteps > 1) gload(pbeg + WG_BP, I1{});
    sstore(I0{});
  }
  __syncthreads();
  const int q = lr >> 2, pp = lr & 3;
  // steps in pairs: LDS buffer and register slot are compile-time; step s+2 is loaded while step s runs
  auto step = [&](int s, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    if (s + 2 < nsteps) gload(pbeg + (s + 2) * WG_BP, bufc);
    bf16x8 af[MT], bfr[4];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int c0 = wid * (BM / 4) + i * 16;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int r = lg * 8 + half * 4 + q;
        const int ch = ((c0 >> 2) + pp) ^ wgb_swz<BM>(r);
        const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tY[buf] + r * BM + ch * 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) af[i][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int r = lg * 8 + half * 4 + q;
        const int ch = ((j * 16 >> 2) + pp) ^ wgb_swz<64>(r);
        const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tX[buf] + r * 64 + ch * 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) bfr[j][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if constexpr (BIAS) {
      if (bias_blk) {
#pragma unroll
        for (int i = 0; i < MT; ++i) bacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, bacc[i], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) sstore(std::integral_constant<int, buf ^ 1>{});
    __syncthreads();
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, I0{});
    if (s + 1 < nsteps) step(s + 1, I1{});
  }
  if (BIAS && bias_blk && lr == 0) {  // every output column holds the row sum: column 0 writes it
#pragma unroll
    for (int i = 0; i < (BIAS ? MT : 1); ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) bslab[(int64_t)bz * g.Cout + co0 + wid * (BM / 4) + i * 16 + lg * 4 + r] = bacc[i][r];
  }
  const int K = g.KH * g.KW * Cin;
  float* out = slab + (int64_t)bz * g.Cout * K;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kc = kcol0 + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wid * (BM / 4) + i * 16 + lg * 4 + r;
        out[(int64_t)co * K + kc] = acc[i][j][r];
      }
    }
}

// ----------------------------------------------------------------------------------------
// 1x1 weight gradient with square tiles (round 6): BM = 256 (or 64) output rows x BN = 256 (or 128) input channels per
// block, 8 waves (BM/64 row quarters x 8/(BM/64) column slices, 64 rows per wave).  wgrad_wide<256> reads the same 256-row dY slice
// once per 64 input channels: at the 768-channel qkv projections of the C = 256 / 512 levels that is 4-8 reads of the
// largest tensor, and the kernel is bound by those bytes (≈ 2 TB/s of loads at 0.15 of the MFMA peak).  Here dY is read
// once per (row tile, pixel split) and x once per row tile.  Loads through registers as wgrad_wide (two steps in
// flight), fragments by ds_read_b64_tr_b16 from the same XOR-swizzled rows.
// ----------------------------------------------------------------------------------------
template <int BM, int BN, bool BIAS = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_sq_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ slab, float* __restrict__ bslab, int M,
    int Cout, int Cin, int px_per_split) {
  // waves: WR row quarters of 64 rows x WC column slices of BN / WC columns
  constexpr int WR = BM / 64, WC = 8 / WR, MT = 4, NT = BN / (16 * WC);
  static_assert((BM == 256 || BM == 64) && NT >= 1, "wgrad_sq tiles");
  constexpr int TY = WG_BP * BM / 8, TX = WG_BP * BN / 8;  // 16-B vectors per step
  constexpr int NY = (TY + 511) / 512, NX = (TX + 511) / 512;
  __shared__ __attribute__((aligned(16))) bf16 tY[2][WG_BP * BM];
  __shared__ __attribute__((aligned(16))) bf16 tX[2][WG_BP * BN];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int wr = wid % WR, wc = wid / WR;
  const int co0 = blockIdx.x * BM, k0 = blockIdx.y * BN;
  const int pbeg = blockIdx.z * px_per_split;
  const int pend = min(M, pbeg + px_per_split);
  bf16x8 yr2[2][NY], xr2[2][NX];
  auto gload = [&](int p0, auto slotc) {
    constexpr int slot = decltype(slotc)::value;
#pragma unroll
    for (int u = 0; u < NY; ++u) {
      const int v = tid + 512 * u, r = v / (BM / 8), c = (v % (BM / 8)) * 8;
      const int m = p0 + r;
      yr2[slot][u] = m < pend && v < TY ? *reinterpret_cast<const bf16x8*>(dy + (int64_t)m * Cout + co0 + c) : bf16x8{};
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int v = tid + 512 * u, r = v / (BN / 8), c = (v % (BN / 8)) * 8;
      const int m = p0 + r;
      xr2[slot][u] = m < pend && v < TX ? *reinterpret_cast<const bf16x8*>(x + (int64_t)m * Cin + k0 + c) : bf16x8{};
    }
  };
  auto sstore = [&](auto bufc) {
    constexpr int buf = decltype(bufc)::value;
#pragma unroll
    for (int u = 0; u < NY; ++u) {
      const int v = tid + 512 * u, r = v / (BM / 8), c = (v % (BM / 8)) * 8;
      if (v < TY) *reinterpret_cast<bf16x8*>(tY[buf] + r * BM + (((c >> 2) ^ wgb_swz<BM>(r)) * 4)) = yr2[buf][u];
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int v = tid + 512 * u, r = v / (BN / 8), c = (v % (BN / 8)) * 8;
      if (v < TX) *reinterpret_cast<bf16x8*>(tX[buf] + r * BN + (((c >> 2) ^ wgb_swz<BN>(r)) * 4)) = xr2[buf][u];
    }
  };
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // BIAS: the conv bias gradient sum_px dY[px][co] from the same dY fragments times a ones operand, by the waves of the
  // first column slice of the first column block (as wgrad_wide<BM, true>); per-split partials bslab[z][co]
  const bool bias_w = BIAS && blockIdx.y == 0 && wc == 0;  // wave-uniform
  f32x4 bacc[BIAS ? MT : 1];
#pragma unroll
  for (int i = 0; i < (BIAS ? MT : 1); ++i) bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;
  const int nsteps = (pend - pbeg + WG_BP - 1) / WG_BP;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (nsteps > 0) {
    gload(pbeg, I0{});
    if (nsteps > 1) gload(pbeg + WG_BP, I1{});
    sstore(I0{});
  }
  __syncthreads();
  const int q = lr >> 2, pp = lr & 3;
  auto step = [&](int s, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    if (s + 2 < nsteps) gload(pbeg + (s + 2) * WG_BP, bufc);
    bf16x8 af[MT], bfr[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int c0 = wr * 64 + i * 16;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int r = lg * 8 + half * 4 + q;
        const int ch = ((c0 >> 2) + pp) ^ wgb_swz<BM>(r);
        const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tY[buf] + r * BM + ch * 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) af[i][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int c0 = wc * (BN / WC) + j * 16;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int r = lg * 8 + half * 4 + q;
        const int ch = ((c0 >> 2) + pp) ^ wgb_swz<BN>(r);
        const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tX[buf] + r * BN + ch * 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) bfr[j][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if constexpr (BIAS) {
      if (bias_w) {
#pragma unroll
        for (int i = 0; i < MT; ++i) bacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, bacc[i], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) sstore(std::integral_constant<int, buf ^ 1>{});
    __syncthreads();
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, I0{});
    if (s + 1 < nsteps) step(s + 1, I1{});
  }
  if (BIAS && bias_w && lr == 0) {  // every output column holds the row sum: column 0 writes it
#pragma unroll
    for (int i = 0; i < (BIAS ? MT : 1); ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) bslab[(int64_t)blockIdx.z * Cout + co0 + wr * 64 + i * 16 + lg * 4 + r] = bacc[i][r];
  }
  float* out = slab + (int64_t)blockIdx.z * Cout * Cin;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int kc = k0 + wc * (BN / WC) + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wr * 64 + i * 16 + lg * 4 + r;
        out[(int64_t)co * Cin + kc] = acc[i][j][r];
      }
    }
}

// ----------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 weight gradient (bf16), halo-tiled.  Block = (64 co) x (32 ci chunk) x
// all 9 taps, looping over 8x32-pixel tiles (its share of the split-K over pixels).  Per tile the
// dY tile [256 px][64 co] and the input halo [10x34 px][32 ci] are staged in LDS; pixels are the
// MFMA K axis, so both operands are read transposed with ds_read_b64_tr_b16 from XOR-swizzled
// rows (conflict-free).  Wave w: co tiles {2*(w>>1), 2*(w>>1)+1} x ci tile (w&1) x 9 taps.
// ----------------------------------------------------------------------------------------
constexpr int W3_TH = 8, W3_TW = 32;
constexpr int W3_HW = W3_TW + 2, W3_NPIX = (W3_TH + 2) * (W3_TW + 2);
// LDS pitch (pixels) of the input-halo rows of both 3x3 weight-gradient kernels: a multiple of 16, so
// a step of whole halo rows keeps bit 3 of the LDS row and with it the chunk swizzle (w3_swz_x) —
// the transposed fragment reads of all nine taps then share six per-lane offsets plus immediates
// instead of recomputing a swizzled address per read (the kernels were VALU-issue bound: 6-10 VALU
// per MFMA, mostly that address arithmetic).
constexpr int W3_P = 48;

__device__ __forceinline__ int w3_swz_dy(int r) { return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3); }
__device__ __forceinline__ int w3_swz_x(int r) { return ((r >> 3) & 1) << 2; }

// Same weight gradient with blocks of 64 co x 64 ci and 8 waves (one block per CU, two waves per SIMD; wave w:
// co tiles {2*(w>>2), 2*(w>>2)+1} x ci tile w&3).  The wgrad is bound by the per-CU load rate (~7.6 B/cycle
// with plain 16-B loads: 54 KB per 8 x 32 tile of a 64 x 32 block, the dY tile re-read by every ci block):
// 64 ci per block loads each dY tile once per 64 input channels (75 KB per tile for twice the MACs).  The
// input halo is kept as two 32-channel planes so the fragment reads are the 64-ci kernel's.
constexpr int W3_PLANE = (W3_TH + 2) * W3_P * 32;  // halo plane (bf16 elements)

// (Round 3 measured a 4-wave form -- one wave per SIMD, 144 accumulators, all four co tiles per wave -- as neutral,
// 63.69 vs 63.58 ms conv total per step: fewer LDS reads per MFMA, less latency hiding.  Removed.)
// 3x3 wgrad kernels: L2 touch of the tile after next (wgrad3x3c64 415 -> 389 us per launch in the step,
// profiles/r4c7b_bench_ab.txt)
constexpr int WG_NT = 512;  // threads per block
constexpr int WG_NI = 2;    // co tiles per wave
__global__ __launch_bounds__(WG_NT, 1) void wgrad3x3c64_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                             const bf16* __restrict__ dy1, const bf16* __restrict__ dy2,
                                                             float* __restrict__ slab, ConvGeom g, int tiles_x,
                                                             int ntiles) {
  __shared__ __attribute__((aligned(16))) bf16 sdy[W3_TH * W3_TW * 64];  // 32 KB, 128-B rows
  __shared__ __attribute__((aligned(16))) bf16 shx[2 * W3_PLANE];        // 2 x 30 KB, 64-B rows
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cot0 = (wid >> 2) * 2, cit = wid & 3;
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64;
  const int Cin = g.C1 + g.C2;
  const bf16* xs; int xcs, xcc;
  if (ci0 < g.C1) { xs = x1; xcs = g.C1; xcc = ci0; } else { xs = x2; xcs = g.C2; xcc = ci0 - g.C1; }
  const bf16* ys; int ycs, ycc;
  const int Co2 = g.Cout - g.Co1;
  if (co0 < g.Co1) { ys = dy1; ycs = g.Co1; ycc = co0; } else { ys = dy2; ycs = Co2; ycc = co0 - g.Co1; }
  const int tiles_per_img = tiles_x * ((g.Ho + W3_TH - 1) / W3_TH);

  f32x4 acc[WG_NI][9];
#pragma unroll
  for (int i = 0; i < WG_NI; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, pp = lr & 3;
  const bf16* shp = shx + (cit >> 1) * W3_PLANE;
  int aoff[WG_NI][2], boff[2][3];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lg * 8 + half * 4 + q;
#pragma unroll
    for (int i = 0; i < WG_NI; ++i) aoff[i][half] = r * 64 + ((((cot0 + i) * 4 + pp) ^ w3_swz_dy(r)) * 4);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) boff[half][kx] = (r + kx) * 32 + ((((cit & 1) * 4 + pp) ^ w3_swz_x(r + kx)) * 4);
  }
  // next tile's vectors in registers (unpredicated loads: clamped address + select), written to LDS after
  // the barrier that ends the current tile's reads
  constexpr int YV = 2048 / WG_NT, HV = (W3_NPIX * 8 + WG_NT - 1) / WG_NT;
  bf16x8 yv[YV], hv[HV];
  auto gload = [&](int tile) {
    const int n = tile / tiles_per_img;
    const int rem = tile - n * tiles_per_img;
    const int ty = rem / tiles_x, tx = rem - ty * tiles_x;
    const int y0 = ty * W3_TH, x0 = tx * W3_TW;
#pragma unroll
    for (int k = 0; k < YV; ++k) {      // dY: 256 px x 8 vectors
      const int e = tid + k * WG_NT;
      const int p = e >> 3, part = e & 7;
      const int oy = y0 + (p >> 5), ox = x0 + (p & 31);
      const bool ok = oy < g.Ho && ox < g.Wo;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(
          ys + (ok ? (((int64_t)n * g.Ho + oy) * g.Wo + ox) * ycs : 0) + ycc + part * 8);
      yv[k] = ok ? v : bf16x8{};
    }
#pragma unroll
    for (int k = 0; k < HV; ++k) {      // halo: 340 px x 8 vectors (64 ci)
      const int e = tid + k * WG_NT;
      const int hp = e >> 3, part = e & 7;
      const int r = hp / W3_HW, c = hp - r * W3_HW;
      const int iy = y0 - 1 + r, ix = x0 - 1 + c;
      const bool ok = e < W3_NPIX * 8 && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(
          xs + (ok ? (((int64_t)n * g.Hi + iy) * g.Wi + ix) * xcs : 0) + xcc + part * 8);
      hv[k] = ok ? v : bf16x8{};
    }
  };
  // L2 touch: the dY and input-halo lines of the tile after next, LDS-direct into a never-read row per wave
  // (4 B per 128-B pixel line), so the register prefetch of that tile a step later finds them in L2
  __shared__ __attribute__((aligned(16))) int tdump[WG_NT];
  auto touch = [&](int tile) {
    const int n = tile / tiles_per_img;
    const int rem = tile - n * tiles_per_img;
    const int ty = rem / tiles_x, tx = rem - ty * tiles_x;
    const int y0 = ty * W3_TH, x0 = tx * W3_TW;
    const int64_t yimg = (int64_t)g.Ho * g.Wo * ycs, ximg = (int64_t)g.Hi * g.Wi * xcs;
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(ys + n * yimg + ycc), (short)0, (int)(yimg * 2 - ycc * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(xs + n * ximg + xcc), (short)0, (int)(ximg * 2 - xcc * 2), 0x00020000);
    auto* dst = (__attribute__((address_space(3))) void*)(tdump + wid * 64);
    {  // dY: 256 pixels
      const int p = tid & 255;
      const int oy = y0 + (p >> 5), ox = x0 + (p & 31);
      const bool ok = tid < 256 && oy < g.Ho && ox < g.Wo;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yrs, dst, 4, ok ? (oy * g.Wo + ox) * ycs * 2 : 0x7ffffff0, 0, 0, 0);
    }
    {  // halo: 340 pixels (threads 256..511 and 0..83)
      const int hp = tid < 256 ? 256 + tid : tid - 256;
      const int r = hp / W3_HW, c = hp - r * W3_HW;
      const int iy = y0 - 1 + r, ix = x0 - 1 + c;
      const bool ok = hp < W3_NPIX && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, dst, 4, ok ? (iy * g.Wi + ix) * xcs * 2 : 0x7ffffff0, 0, 0, 0);
    }
  };
  if ((int)blockIdx.z < ntiles) gload(blockIdx.z);
  for (int tile = blockIdx.z; tile < ntiles; tile += gridDim.z) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < YV; ++k) {
      const int e = tid + k * WG_NT;
      const int p = e >> 3, part = e & 7;  // chunk pair (2part, 2part+1) of 8-B chunks
      const int ch = (part * 2) ^ w3_swz_dy(p);
      *reinterpret_cast<bf16x8*>(sdy + p * 64 + ch * 4) = yv[k];
    }
#pragma unroll
    for (int k = 0; k < HV; ++k) {
      const int e = tid + k * WG_NT;
      if (e < W3_NPIX * 8) {
        const int hp = e >> 3, part = e & 7;
        const int r = hp / W3_HW, row = r * W3_P + (hp - r * W3_HW);
        const int ch = ((part & 3) * 2) ^ w3_swz_x(row);
        *reinterpret_cast<bf16x8*>(shx + (part >> 2) * W3_PLANE + row * 32 + ch * 4) = hv[k];
      }
    }
    __syncthreads();
    if (tile + (int)gridDim.z < ntiles) gload(tile + gridDim.z);
    if (tile + 2 * (int)gridDim.z < ntiles) touch(tile + 2 * gridDim.z);
    // the fragment reads of pixel row py+1 (2 NI + 18) are issued between the 9 NI MFMAs of row py (two register
    // sets; 1 read : 1 MFMA via sched_group_barrier), so no row waits for its LDS reads
    bf16x8 fa[2][WG_NI], fb[2][9];
    auto rd = [&](int py, int b) {
#pragma unroll
      for (int i = 0; i < WG_NI; ++i)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(sdy + aoff[i][half] + py * 32 * 64));
#pragma unroll
          for (int e = 0; e < 4; ++e) fa[b][i][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (LDS_PTR(s16x4))(shp + boff[half][kx] + (py + ky) * W3_P * 32));
#pragma unroll
          for (int e = 0; e < 4; ++e) fb[b][tap][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
      }
    };
    auto mm = [&](int b) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int i = 0; i < WG_NI; ++i)
          acc[i][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[b][i], fb[b][tap], acc[i][tap], 0, 0, 0);
    };
    rd(0, 0);
#pragma unroll
    for (int py = 0; py < W3_TH; ++py) {
      const int b = py & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (py + 1 < W3_TH) rd(py + 1, b ^ 1);
      mm(b);
      if (py + 1 < W3_TH) {
        constexpr int NRD = 2 * WG_NI + 18, NMF = 9 * WG_NI;
        constexpr int NPAIR = NRD < NMF ? NRD : NMF;
#pragma unroll
        for (int q2 = 0; q2 < NPAIR; ++q2) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        }
        if (NRD > NPAIR) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NPAIR, 0);
        if (NMF > NPAIR) __builtin_amdgcn_sched_group_barrier(0x008, NMF - NPAIR, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const int K = 9 * Cin;
  float* out = slab + (int64_t)blockIdx.z * g.Cout * K;
#pragma unroll
  for (int i = 0; i < WG_NI; ++i)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ci = ci0 + cit * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + (cot0 + i) * 16 + lg * 4 + r;
        out[(int64_t)co * K + tap * Cin + ci] = acc[i][tap][r];
      }
    }
}

// Weight gradient of the 4x4 / stride-2 / pad-1 conv (Downsample; the Upsample's weight gradient is the same
// operation with dOut as the input and x as dY), halo-tiled like wgrad3x3c64_kernel on the low-resolution
// dY grid.  Block = (64 co) x (32 ci chunk) x one input parity (a, b) = its 4 live taps ky = (1-a) + 2t,
// kx = (1-b) + 2u, whose inputs are the (TH+2) x (TW+2) halo of x_ab[Y][X] = x[2Y+a][2X+b] at offsets
// (1-a+t, 1-b+u) - the forward's parity split (convs2_bf16_kernel).  Replaces the wide-tile wgrad, which
// gathered every (pixel, tap) pair (315 TF/s on the bench shapes).
template <int BY, int BX>
__device__ __forceinline__ void ws2_taps(const bf16* sdy, const bf16* shx, const int (&aoff)[2][2],
                                         const int (&boff)[2][3], f32x4 (&acc)[2][4]) {
#pragma unroll 1
  for (int py = 0; py < W3_TH; ++py) {
    bf16x8 af[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(sdy + aoff[i][half] + py * 32 * 64));
#pragma unroll
        for (int e = 0; e < 4; ++e) af[i][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int oy = BY + (t >> 1), ox = BX + (t & 1);
      bf16x8 bfr;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const s16x4 v =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(shx + boff[half][ox] + (py + oy) * W3_P * 32));
#pragma unroll
        for (int e = 0; e < 4; ++e) bfr[half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
      acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bfr, acc[0][t], 0, 0, 0);
      acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bfr, acc[1][t], 0, 0, 0);
    }
  }
}

__global__ __launch_bounds__(256, 2) void wgrads2_bf16_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                              float* __restrict__ slab, ConvGeom g, int tiles_x,
                                                              int ntiles) {
  __shared__ __attribute__((aligned(16))) bf16 sdy[W3_TH * W3_TW * 64];        // 32 KB, 128-B rows
  __shared__ __attribute__((aligned(16))) bf16 shx[(W3_TH + 2) * W3_P * 32];  // 30 KB, 64-B rows
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cot0 = (wid >> 1) * 2, cit = wid & 1;
  const int co0 = blockIdx.x * 64;
  const int ab = (int)blockIdx.y & 3, a = ab >> 1, b = ab & 1;
  const int ci0 = ((int)blockIdx.y >> 2) * 32;
  const int Cin = g.C1;
  const int tiles_per_img = tiles_x * ((g.Ho + W3_TH - 1) / W3_TH);

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, pp = lr & 3;
  int aoff[2][2], boff[2][3];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lg * 8 + half * 4 + q;
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i][half] = r * 64 + ((((cot0 + i) * 4 + pp) ^ w3_swz_dy(r)) * 4);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) boff[half][kx] = (r + kx) * 32 + (((cit * 4 + pp) ^ w3_swz_x(r + kx)) * 4);
  }
  for (int tile = blockIdx.z; tile < ntiles; tile += gridDim.z) {
    const int n = tile / tiles_per_img;
    const int rem = tile - n * tiles_per_img;
    const int ty = rem / tiles_x, tx = rem - ty * tiles_x;
    const int y0 = ty * W3_TH, x0 = tx * W3_TW;
    __syncthreads();
    {
      bf16x8 yv[8], hv[6];
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // dY: 256 px x 8 vectors
        const int e = tid + k * 256;
        const int p = e >> 3, part = e & 7;
        const int oy = y0 + (p >> 5), ox = x0 + (p & 31);
        bf16x8 v = {};
        if (oy < g.Ho && ox < g.Wo)
          v = *reinterpret_cast<const bf16x8*>(dy + (((int64_t)n * g.Ho + oy) * g.Wo + ox) * g.Cout + co0 + part * 8);
        yv[k] = v;
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {  // halo of x_ab: 340 px x 4 vectors
        const int e = tid + k * 256;
        bf16x8 v = {};
        if (e < W3_NPIX * 4) {
          const int hp = e >> 2, part = e & 3;
          const int r = hp / W3_HW, c = hp - r * W3_HW;
          const int iy = 2 * (y0 - 1 + r) + a, ix = 2 * (x0 - 1 + c) + b;
          if ((unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi)
            v = *reinterpret_cast<const bf16x8*>(x + (((int64_t)n * g.Hi + iy) * g.Wi + ix) * Cin + ci0 + part * 8);
        }
        hv[k] = v;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = tid + k * 256;
        const int p = e >> 3, part = e & 7;
        const int ch = (part * 2) ^ w3_swz_dy(p);
        *reinterpret_cast<bf16x8*>(sdy + p * 64 + ch * 4) = yv[k];
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int e = tid + k * 256;
        if (e < W3_NPIX * 4) {
          const int hp = e >> 2, part = e & 3;
          const int r = hp / W3_HW, row = r * W3_P + (hp - r * W3_HW);
          const int ch = (part * 2) ^ w3_swz_x(row);
          *reinterpret_cast<bf16x8*>(shx + row * 32 + ch * 4) = hv[k];
        }
      }
    }
    __syncthreads();
    switch (ab) {  // block-uniform: tap bases 1-a, 1-b
      case 0: ws2_taps<1, 1>(sdy, shx, aoff, boff, acc); break;
      case 1: ws2_taps<1, 0>(sdy, shx, aoff, boff, acc); break;
      case 2: ws2_taps<0, 1>(sdy, shx, aoff, boff, acc); break;
      default: ws2_taps<0, 0>(sdy, shx, aoff, boff, acc); break;
    }
  }
  // D[co][ci] per tap: lane col lr -> ci, rows 4lg+r -> co; tap = ky*4 + kx
  const int K = 16 * Cin;
  float* out = slab + (int64_t)blockIdx.z * g.Cout * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int tap = (1 - a + 2 * (t >> 1)) * 4 + (1 - b + 2 * (t & 1));
      const int ci = ci0 + cit * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + (cot0 + i) * 16 + lg * 4 + r;
        out[(int64_t)co * K + tap * Cin + ci] = acc[i][t][r];
      }
    }
}

// Same weight gradient on 8 x 36 pixel tiles (288 px = 9 K-chunks of 32 flat pixels): every U-Net
// level's width (288/144/72/36) is a multiple of 36, so no tile column is wasted (the 8 x 32 tiles
// above compute 36-px rows as two 32-px tiles: 56 % useful at 24 x 36).  A K-chunk may span two
// image rows: each lane derives its own halo row per chunk (the transposed ds_read takes per-lane
// addresses).
constexpr int W36_TH = 8, W36_TW = 36, W36_HW = W36_TW + 2, W36_NPIX = (W36_TH + 2) * W36_HW;  // 380 halo px
constexpr int W36_NP = W36_TH * W36_TW;                                                          // 288 px

// sum slabs over splits (fixed order) and scatter into the PyTorch weight layout
// dst[((d0*D1 + d1)*KH + kyt)*KW + kxt], with (d0,d1) = swap ? (ci,co) : (co,ci) and
// (kyt,kxt) = flip ? (KH-1-ky, KW-1-kx) : (ky,kx).
// 8 x 36 tiles (levels 2-3) with the 64 co x 64 ci / 8-wave blocking and the K-chunk software pipeline of
// wgrad3x3c64_kernel: each wave's 22 fragment reads of K-chunk kc+1 are issued between the 18 MFMAs of chunk kc
__global__ __launch_bounds__(WG_NT, 1) void wgrad3x3w36c64_kernel(const bf16* __restrict__ x1, const bf16* __restrict__ x2,
                                                                const bf16* __restrict__ dy1, const bf16* __restrict__ dy2,
                                                                float* __restrict__ slab, ConvGeom g, int tiles_x,
                                                                int ntiles) {
  __shared__ __attribute__((aligned(16))) bf16 sdy[W36_NP * 64];  // 36 KB, 128-B rows
  __shared__ __attribute__((aligned(16))) bf16 shx[2 * W3_PLANE];  // 2 x 30 KB, 64-B rows
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cot0 = (wid >> 2) * 2, cit = wid & 3;
  const int co0 = blockIdx.x * 64, ci0 = blockIdx.y * 64;
  const int Cin = g.C1 + g.C2;
  const bf16* xs; int xcs, xcc;
  if (ci0 < g.C1) { xs = x1; xcs = g.C1; xcc = ci0; } else { xs = x2; xcs = g.C2; xcc = ci0 - g.C1; }
  const bf16* ys; int ycs, ycc;
  const int Co2 = g.Cout - g.Co1;
  if (co0 < g.Co1) { ys = dy1; ycs = g.Co1; ycc = co0; } else { ys = dy2; ycs = Co2; ycc = co0 - g.Co1; }
  const int tiles_per_img = tiles_x * ((g.Ho + W36_TH - 1) / W36_TH);

  f32x4 acc[WG_NI][9];
#pragma unroll
  for (int i = 0; i < WG_NI; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4, q = lr >> 2, pp = lr & 3;
  const bf16* shp = shx + (cit >> 1) * W3_PLANE;
  const int cx = (cit & 1) * 4 + pp;
  int aoff[WG_NI][2];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int r = lg * 8 + half * 4 + q;
#pragma unroll
    for (int i = 0; i < WG_NI; ++i) aoff[i][half] = r * 64 + ((((cot0 + i) * 4 + pp) ^ w3_swz_dy(r)) * 4);
  }
  constexpr int YV = (W36_NP * 8 + WG_NT - 1) / WG_NT, HV = (W36_NPIX * 8 + WG_NT - 1) / WG_NT;
  bf16x8 yv[YV], hv[HV];
  auto gload = [&](int tile) {
    const int n = tile / tiles_per_img;
    const int rem = tile - n * tiles_per_img;
    const int ty = rem / tiles_x, tx = rem - ty * tiles_x;
    const int y0 = ty * W36_TH, x0 = tx * W36_TW;
#pragma unroll
    for (int k = 0; k < YV; ++k) {       // dY: 288 px x 8 vectors
      const int e = tid + k * WG_NT;
      const int p = e >> 3, part = e & 7;
      const int oy = y0 + p / W36_TW, ox = x0 + (p - (p / W36_TW) * W36_TW);
      const bool ok = e < W36_NP * 8 && oy < g.Ho && ox < g.Wo;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(
          ys + (ok ? (((int64_t)n * g.Ho + oy) * g.Wo + ox) * ycs : 0) + ycc + part * 8);
      yv[k] = ok ? v : bf16x8{};
    }
#pragma unroll
    for (int k = 0; k < HV; ++k) {       // halo: 380 px x 8 vectors (64 ci)
      const int e = tid + k * WG_NT;
      const int hp = e >> 3, part = e & 7;
      const int r = hp / W36_HW, c = hp - r * W36_HW;
      const int iy = y0 - 1 + r, ix = x0 - 1 + c;
      const bool ok = e < W36_NPIX * 8 && (unsigned)iy < (unsigned)g.Hi && (unsigned)ix < (unsigned)g.Wi;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(
          xs + (ok ? (((int64_t)n * g.Hi + iy) * g.Wi + ix) * xcs : 0) + xcc + part * 8);
      hv[k] = ok ? v : bf16x8{};
    }
  };
  if ((int)blockIdx.z < ntiles) gload(blockIdx.z);
  for (int tile = blockIdx.z; tile < ntiles; tile += gridDim.z) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < YV; ++k) {
      const int e = tid + k * WG_NT;
      if (e < W36_NP * 8) {
        const int p = e >> 3, part = e & 7;
        const int ch = (part * 2) ^ w3_swz_dy(p);
        *reinterpret_cast<bf16x8*>(sdy + p * 64 + ch * 4) = yv[k];
      }
    }
#pragma unroll
    for (int k = 0; k < HV; ++k) {
      const int e = tid + k * WG_NT;
      if (e < W36_NPIX * 8) {
        const int hp = e >> 3, part = e & 7;
        const int r = hp / W36_HW, row = r * W3_P + (hp - r * W36_HW);
        const int ch = ((part & 3) * 2) ^ w3_swz_x(row);
        *reinterpret_cast<bf16x8*>(shx + (part >> 2) * W3_PLANE + row * 32 + ch * 4) = hv[k];
      }
    }
    __syncthreads();
    if (tile + (int)gridDim.z < ntiles) gload(tile + gridDim.z);
    // flat pixel of this lane's two 4-pixel groups in K-chunk kc: P = kc*32 + r0[half] -> (row, col) of the
    // 36-wide tile (32 < 36: at most one wrap per chunk)
    int prow[2], pcol[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) { prow[half] = 0; pcol[half] = lg * 8 + half * 4 + q; }
    bf16x8 fa[2][WG_NI], fb[2][9];
    auto rd = [&](int kc, int b) {
#pragma unroll
      for (int i = 0; i < WG_NI; ++i)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(sdy + aoff[i][half] + kc * 32 * 64));
#pragma unroll
          for (int e = 0; e < 4; ++e) fa[b][i][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
      int bo[2][3];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int hb = prow[half] * W3_P + pcol[half];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) bo[half][kx] = (hb + kx) * 32 + ((cx ^ w3_swz_x(hb + kx)) * 4);
        pcol[half] += 32;
        if (pcol[half] >= W36_TW) { pcol[half] -= W36_TW; ++prow[half]; }
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(shp + bo[half][kx] + ky * W3_P * 32));
#pragma unroll
          for (int e = 0; e < 4; ++e) fb[b][tap][half * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
        }
      }
    };
    auto mm = [&](int b) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
        for (int i = 0; i < WG_NI; ++i)
          acc[i][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[b][i], fb[b][tap], acc[i][tap], 0, 0, 0);
      }
    };
    constexpr int NKC = W36_NP / 32;
    rd(0, 0);
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      const int b = kc & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (kc + 1 < NKC) rd(kc + 1, b ^ 1);
      mm(b);
      if (kc + 1 < NKC) {
        constexpr int NRD = 2 * WG_NI + 18, NMF = 9 * WG_NI;
        constexpr int NPAIR = NRD < NMF ? NRD : NMF;
#pragma unroll
        for (int q2 = 0; q2 < NPAIR; ++q2) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        }
        if (NRD > NPAIR) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NPAIR, 0);
        if (NMF > NPAIR) __builtin_amdgcn_sched_group_barrier(0x008, NMF - NPAIR, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const int K = 9 * Cin;
  float* out = slab + (int64_t)blockIdx.z * g.Cout * K;
#pragma unroll
  for (int i = 0; i < WG_NI; ++i)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ci = ci0 + cit * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + (cot0 + i) * 16 + lg * 4 + r;
        out[(int64_t)co * K + tap * Cin + ci] = acc[i][tap][r];
      }
    }
}

// dst (+)= sum over the nsplit slabs, remapped to the PyTorch layout.  Block = 64 consecutive slab
// elements x 4 split-groups (coalesced 256-B rows per split), fixed-order combine in LDS.
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dst,
                                                                int nsplit, int Cout, int Cin, int KH, int KW, int swap,
                                                                int flip, int accumulate) {
  const int64_t K = (int64_t)KH * KW * Cin;
  const int64_t total = (int64_t)Cout * K;
  const int64_t e = blockIdx.x * 64ll + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  float s = 0.f;
  if (e < total) {
    // 8 slab loads in flight, summed in the same order as one at a time (the loop waited out every load: 18.5 us per
    // call, 78 calls per step)
    int k = grp;
    for (; k + 28 < nsplit; k += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)(k + 4 * u) * total + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < nsplit; k += 4) s += slab[(int64_t)k * total + e];
  }
  __shared__ float red[4][64];
  red[grp][threadIdx.x & 63] = s;
  __syncthreads();
  if (grp != 0 || e >= total) return;
  s = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
  const int co = (int)(e / K);
  const int kc = (int)(e - (int64_t)co * K);
  const int tap = kc / Cin, ci = kc - tap * Cin;
  int ky = tap / KW, kx = tap - ky * KW;
  if (flip) { ky = KH - 1 - ky; kx = KW - 1 - kx; }
  const int d0 = swap ? ci : co, d1 = swap ? co : ci, D1 = swap ? Cout : Cin;
  const int64_t di = (((int64_t)d0 * D1 + d1) * KH + ky) * KW + kx;
  dst[di] = accumulate ? dst[di] + s : s;
}

// pack a PyTorch conv weight into the GEMM layout Wp[co][tap][ci] or its chunked form (wpk_index; cast to T)
template <typename T>
__global__ void conv_pack_kernel(const float* __restrict__ src, T* __restrict__ dst, int Cout, int Cin, int KH,
                                 int KW, int swap, int flip) {
  // 32-bit index math (a weight has < 2^31 elements, checked on the host): the 64-bit divisions per element
  // made this a 0.37 ms launch per optimizer step
  const int K = KH * KW * Cin;
  const int total = Cout * K;
  const bool chk = wpk_chunked(std::is_same<T, bf16>::value, Cout, Cin, KH, KW);
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int co = e / K;
    const int kc = e - co * K;
    const int tap = kc / Cin, ci = kc - tap * Cin;
    int ky = tap / KW, kx = tap - ky * KW;
    if (flip) { ky = KH - 1 - ky; kx = KW - 1 - kx; }
    const int d0 = swap ? ci : co, d1 = swap ? co : ci, D1 = swap ? Cout : Cin;
    dst[chk ? wpk_index(true, co, tap, ci, Cin, KH * KW) : e] = from_f<T>(src[((d0 * D1 + d1) * KH + ky) * KW + kx]);
  }
}

// batched repack after an optimizer step: job j = int64[8] {src, dst, Cout, Cin, KH, KW, swap, flip};
// One launch for every cached pack.  jobs: njobs rows of 8 int64 (src, dst, Cout, Cin, KH, KW, swap, flip), then njobs + 1
// block starts (the exclusive prefix of the per-job tile counts), then the job index of every block.  A block takes one
// (co, ci) tile of a job -- pb_co_t(T) output rows x 64 input channels x all T taps: it reads the tile's source runs
// contiguously (co-major rows of Cin*T floats, or ci-major rows of Cout*T when swap), transposes through LDS and writes
// dst[co][tap][ci] in 64-channel runs.  (Round 6: blockIdx.y = job with a fixed 512 blocks each dispatched ~92 k mostly
// empty blocks and gathered every element with a stride-T read -- 309 us per optimizer step.)
constexpr int PB_CI = 64;
constexpr int PB_TILE = 4096;  // floats of LDS per tile
__host__ __device__ inline int pb_co_t(int T) { const int c = PB_TILE / (T * PB_CI); return c < 1 ? 1 : (c > 64 ? 64 : c); }
// one (co, ci) tile; NTC = the tap count when known at compile time (1, 9, 16), else 0 (runtime NT)
template <typename T, int NTC>
__device__ __forceinline__ void pb_tile(float* tile, const float* __restrict__ src, T* __restrict__ dst, int Cout, int Cin,
                                        int NTr, int swap, int flip, int co0, int ci0, int nco, int ncc, bool chk) {
  const int NT = NTC ? NTC : NTr;
  const int run = swap ? nco * NT : ncc * NT;  // contiguous source floats per outer index
  const int nld = (swap ? ncc : nco) * run;
  float v[PB_TILE / 256];
#pragma unroll
  for (int u = 0; u < PB_TILE / 256; ++u) {  // every load of the tile issued before the LDS writes
    const int q = u * 256 + (int)threadIdx.x;
    const int qq = q < nld ? q : 0;
    const int o = qq / run, r = qq - o * run;
    const int inner = r / NT, t = r - inner * NT;
    const int co_l = swap ? inner : o, ci_l = swap ? o : inner;
    v[u] = src[swap ? ((ci0 + ci_l) * Cout + co0 + co_l) * NT + t : ((co0 + co_l) * Cin + ci0 + ci_l) * NT + t];
  }
#pragma unroll
  for (int u = 0; u < PB_TILE / 256; ++u) {
    const int q = u * 256 + (int)threadIdx.x;
    if (q < nld) {
      const int o = q / run, r = q - o * run;
      const int inner = r / NT, t = r - inner * NT;
      const int co_l = swap ? inner : o, ci_l = swap ? o : inner;
      tile[(co_l * NT + t) * PB_CI + ci_l] = v[u];
    }
  }
  __syncthreads();
  // store: dst[co][td][ci], 64-channel runs; flip reads the source tap NT - 1 - td
  const int nst = nco * NT * PB_CI;
#pragma unroll
  for (int u = 0; u < PB_TILE / 256; ++u) {
    const int q = u * 256 + (int)threadIdx.x;
    const int ci_l = q & (PB_CI - 1), ct = q / PB_CI, co_l = ct / NT, td = ct - co_l * NT;
    if (q < nst && ci_l < ncc) {
      const int ts = flip ? NT - 1 - td : td;
      dst[wpk_index(chk, co0 + co_l, td, ci0 + ci_l, Cin, NT)] = from_f<T>(tile[(co_l * NT + ts) * PB_CI + ci_l]);
    }
  }
}
template <typename T>
__global__ __launch_bounds__(256) void conv_pack_batch_kernel(const int64_t* __restrict__ jobs, int njobs) {
  __shared__ float tile[PB_TILE];
  const int64_t* start = jobs + (int64_t)njobs * 8;
  const int64_t nblocks = start[njobs];
  const int64_t* bjob = start + njobs + 1;  // job of every block (one load, not a search)
  for (int64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const int lo = (int)bjob[b];
    const int64_t* jb = jobs + (int64_t)lo * 8;
    const float* src = reinterpret_cast<const float*>(jb[0]);
    T* dst = reinterpret_cast<T*>(jb[1]);
    const int Cout = (int)jb[2], Cin = (int)jb[3], NT = (int)(jb[4] * jb[5]), swap = (int)jb[6], flip = (int)jb[7];
    const int cot = pb_co_t(NT), nci = (Cin + PB_CI - 1) / PB_CI;
    const int lb = (int)(b - start[lo]);
    const int co0 = (lb / nci) * cot, ci0 = (lb % nci) * PB_CI;
    const int nco = min(cot, Cout - co0), ncc = min(PB_CI, Cin - ci0);
    const bool chk = wpk_chunked(std::is_same<T, bf16>::value, Cout, Cin, (int)jb[4], (int)jb[5]);
    __syncthreads();  // the previous tile's LDS reads are done
    if (NT == 9) pb_tile<T, 9>(tile, src, dst, Cout, Cin, NT, swap, flip, co0, ci0, nco, ncc, chk);
    else if (NT == 1) pb_tile<T, 1>(tile, src, dst, Cout, Cin, NT, swap, flip, co0, ci0, nco, ncc, false);
    else if (NT == 16) pb_tile<T, 16>(tile, src, dst, Cout, Cin, NT, swap, flip, co0, ci0, nco, ncc, chk);
    else pb_tile<T, 0>(tile, src, dst, Cout, Cin, NT, swap, flip, co0, ci0, nco, ncc, false);
  }
}

// per-channel column sum over rows of a channels-last matrix: partial[split][c]
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ x, float* __restrict__ part, int64_t rows, int C,
                                      int64_t rows_per_split) {
  // block: 256 threads = (256/ (C/4)) row-lanes x (C/4) channel-quads  (C <= 1024, C % 4 == 0)
  const int cq = C / 4;
  const int rl = 256 / cq;
  const int tid = threadIdx.x;
  const int q = tid % cq, rr = tid / cq;
  __shared__ float red[256 * 4];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t r0 = blockIdx.x * rows_per_split;
  const int64_t r1 = min(rows, r0 + rows_per_split);
  if (rr < rl) {
    for (int64_t r = r0 + rr; r < r1; r += rl) {
      float v[4];
      load4(x + r * C + q * 4, v);
      s[0] += v[0]; s[1] += v[1]; s[2] += v[2]; s[3] += v[3];
    }
  }
  for (int i = 0; i < 4; ++i) red[tid * 4 + i] = s[i];
  __syncthreads();
  if (tid < cq) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < rl; ++k)
      for (int i = 0; i < 4; ++i) t[i] += red[(k * cq + tid) * 4 + i];
    for (int i = 0; i < 4; ++i) part[(int64_t)blockIdx.x * C + tid * 4 + i] = t[i];
  }
}

// one 64-lane wave per channel: lanes stride over the splits, then a fixed-order wave sum
__global__ void colsum_final_kernel(const float* __restrict__ part, float* __restrict__ dst, int nsplit, int C,
                                    int accumulate) {
  const int c = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nsplit; k += 64) s += part[(int64_t)k * C + c];
  s = wave_sum(s);
  if (threadIdx.x == 0) dst[c] = accumulate ? dst[c] + s : s;
}

// ----------------------------------------------------------------------------------------
// stem: Conv3d(2 -> Co, (1,7,7), pad 3) on cat([x_t broadcast over F, cond]) (video_net.py:595-600,
// :808-815).  Inputs are the boundary NCDHW fp32 tensors: xt [B][Fx][H][W] (Fx = 1 or F),
// cond [B][Fc][H][W].  Direct VALU conv (0.3 % of the MACs): block = 16x16 output pixels of
// one frame, 64 output channels (Co == 64 at the default base_ch; Co % 64 == 0 handled by grid.y).
// ----------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void stem_fwd_kernel(const float* __restrict__ xt, const float* __restrict__ cond,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       T* __restrict__ y, int B, int F, int Fx, int Fc, int H, int W,
                                                       int Co, int KS) {
  const int PAD = KS / 2;
  const int TS = 16;
  const int TW = TS + KS - 1;
  __shared__ float tin[2][22 * 22];
  __shared__ float tw[64 * 2 * 49];
  const int n = blockIdx.z;  // b*F + f
  const int b = n / F, f = n - b * F;
  const int ty0 = (blockIdx.x / ((W + TS - 1) / TS)) * TS;
  const int tx0 = (blockIdx.x % ((W + TS - 1) / TS)) * TS;
  const int cog = blockIdx.y * 64;
  const float* s0 = xt + ((int64_t)b * Fx + (Fx == 1 ? 0 : f)) * H * W;
  const float* s1 = cond + ((int64_t)b * Fc + (Fc == 1 ? 0 : f)) * H * W;
  for (int e = threadIdx.x; e < TW * TW; e += 256) {
    const int yy = ty0 - PAD + e / TW, xx = tx0 - PAD + e % TW;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    tin[0][e] = ok ? s0[(int64_t)yy * W + xx] : 0.f;
    tin[1][e] = ok ? s1[(int64_t)yy * W + xx] : 0.f;
  }
  for (int e = threadIdx.x; e < 64 * 2 * KS * KS; e += 256) tw[e] = w[(int64_t)cog * 2 * KS * KS + e];
  __syncthreads();
  const int py = threadIdx.x / TS, px = threadIdx.x % TS;
  const int oy = ty0 + py, ox = tx0 + px;
  float acc[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) acc[c] = bias[cog + c];
  for (int ci = 0; ci < 2; ++ci)
    for (int ky = 0; ky < KS; ++ky)
      for (int kx = 0; kx < KS; ++kx) {
        const float v = tin[ci][(py + ky) * TW + px + kx];
        const int wo = (ci * KS + ky) * KS + kx;
#pragma unroll
        for (int c = 0; c < 64; ++c) acc[c] = fmaf(tw[c * 2 * KS * KS + wo], v, acc[c]);
      }
  if (oy < H && ox < W) {
    T* dst = y + (((int64_t)n * H + oy) * W + ox) * Co + cog;
#pragma unroll
    for (int c = 0; c < 64; c += 4) store4(dst + c, acc + c);
  }
}

// bf16 stem on MFMA: the same 16x16 output tile / 22x22x2 fp32 input halo in LDS, as an implicit
// GEMM D[co][px] = W[co][k] X[k][px] with k = ci*KS*KS + ky*KS + kx padded to 128 (4 K-steps of 32).
// Wave w owns tile rows 4w..4w+3 (4 fragment groups of 16 px) x 64 co; B fragments are gathered
// straight from the LDS halo (8 taps per lane, converted to bf16), A fragments from the LDS weights.
// Replaces one LDS read per FMA of the VALU kernel (6272 per pixel) with ~100 per pixel.
// Persistent over tiles (round 2): the 64 x 98 weight is staged and converted to A fragments once per block
// (it was once per 256-pixel tile, which dominated: 1.13 ms per level-0 launch), then the block loops over its
// tiles (tile = blockIdx.x + k * gridDim.x) with the fragments in registers.
__global__ __launch_bounds__(256) void stem_fwd_mfma_kernel(const float* __restrict__ xt, const float* __restrict__ cond,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            bf16* __restrict__ y, int B, int F, int Fx, int Fc, int H,
                                                            int W, int Co, int KS, int ntiles) {
  constexpr int TS = 16, TWM = 22;  // tile and max halo width (KS <= 7)
  __shared__ float tin[2][TWM * TWM];
  __shared__ float tw[64 * 128];    // W[co][k], k padded to 128 with zeros
  const int PAD = KS / 2, TW = TS + KS - 1, KK = KS * KS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int cog = blockIdx.y * 64;
  const int tiles_x = (W + TS - 1) / TS, tiles_img = tiles_x * ((H + TS - 1) / TS);
  for (int e = tid; e < 64 * 128; e += 256) {
    const int co = e >> 7, k = e & 127;
    tw[e] = k < 2 * KK ? w[(int64_t)(cog + co) * 2 * KK + k] : 0.f;
  }
  __syncthreads();
  // A fragments: W[ct*16 + lr][ks*32 + lg*8 + e]
  bf16x8 af[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) af[ct][ks][e] = (bf16)tw[(ct * 16 + lr) * 128 + ks * 32 + lg * 8 + e];
  // per-lane LDS offset of tap k (relative to the pixel's (0,0) tap), -1 for padding taps
  int toff[4][8];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = ks * 32 + lg * 8 + e;
      const int ci = k / KK, r = k - ci * KK, ky = r / KS, kx = r - ky * KS;
      // padding taps (k >= 2 KK) read tap 0: their weights are zero and the halo holds finite values
      toff[ks][e] = k < 2 * KK ? ci * TWM * TWM + ky * TWM + kx : 0;
    }
  float bv[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[ct][r] = bias[cog + ct * 16 + lg * 4 + r];
  const float* tbase = &tin[0][0];
  // the next tile's halo values (TW*TW <= 484 <= 2 x 256) are loaded into registers while this tile computes
  float hv[2][2];
  auto fetch = [&](int tile_in) {
    // past the last tile: addresses of tile 0 (in bounds), values zeroed below
    const int tile = tile_in < ntiles ? tile_in : 0;
    const int n = tile / tiles_img, tr = tile - n * tiles_img;
    const int b = n / F, f = n - b * F;
    const int ty0 = (tr / tiles_x) * TS, tx0 = (tr - (tr / tiles_x) * tiles_x) * TS;
    const float* s0 = xt + ((int64_t)b * Fx + (Fx == 1 ? 0 : f)) * H * W;
    const float* s1 = cond + ((int64_t)b * Fc + (Fc == 1 ? 0 : f)) * H * W;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + q * 256;
      const int yy = ty0 - PAD + e / TW, xx = tx0 - PAD + e % TW;
      const bool ok = tile_in < ntiles && e < TW * TW && yy >= 0 && yy < H && xx >= 0 && xx < W;
      const int64_t o = ok ? (int64_t)yy * W + xx : 0;
      const float v0 = s0[o], v1 = s1[o];  // unpredicated loads, selected after
      hv[q][0] = ok ? v0 : 0.f;
      hv[q][1] = ok ? v1 : 0.f;
    }
  };
  if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tiles_img, tr = tile - n * tiles_img;
    const int ty0 = (tr / tiles_x) * TS, tx0 = (tr - (tr / tiles_x) * tiles_x) * TS;
    __syncthreads();  // previous tile's gathers done
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + q * 256;
      if (e < TW * TW) {
        tin[0][(e / TW) * TWM + e % TW] = hv[q][0];
        tin[1][(e / TW) * TWM + e % TW] = hv[q][1];
      }
    }
    __syncthreads();
    fetch(tile + gridDim.x);
    f32x4 acc[4][4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ct][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int py = wid * 4 + j, px = lr;  // group j = tile row py, pixel lr
      const int pbase = py * TWM + px;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 bfr;
#pragma unroll
        for (int e = 0; e < 8; ++e) bfr[e] = (bf16)tbase[pbase + toff[ks][e]];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct][ks], bfr, acc[ct][j], 0, 0, 0);
      }
    }
    // lane holds co = cog + ct*16 + lg*4 + r of pixel (wid*4 + j, lr)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oy = ty0 + wid * 4 + j, ox = tx0 + lr;
      if (oy >= H || ox >= W) continue;
      bf16* dst = y + (((int64_t)n * H + oy) * W + ox) * Co + cog;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int co = ct * 16 + lg * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[ct][j][r] + bv[ct][r];
        store4(dst + co, v);
      }
    }
  }
}

// stem weight gradient partials: part[blk][co][ci*KS*KS + ky*KS + kx]
template <typename T>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const float* __restrict__ xt, const float* __restrict__ cond,
                                                         const T* __restrict__ dy, float* __restrict__ part, int B,
                                                         int F, int Fx, int Fc, int H, int W, int Co, int KS,
                                                         int ntiles) {
  const int PAD = KS / 2;
  const int TH = 8, TWD = 32;
  const int IH = TH + KS - 1, IW = TWD + KS - 1;  // 14 x 38
  __shared__ float tin[2][14 * 38];
  __shared__ float tdy[TH * TWD * 65];
  const int KK = 2 * KS * KS;  // 98
  // thread -> (co, tap-group): 64 co x 4 groups
  const int co = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int tpg = (KK + 3) / 4;
  float acc[25];
  int toff[25];  // LDS offset of each of this thread's taps (-1: none), hoisted out of the pixel loop
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    acc[i] = 0.f;
    const int kk = grp * tpg + i;
    if (i < tpg && kk < KK) {
      const int ci = kk / (KS * KS), r = kk - ci * KS * KS;
      const int ky = r / KS, kx = r - ky * KS;
      toff[i] = ci * (14 * 38) + ky * IW + kx;
    } else {
      toff[i] = -1;
    }
  }
  const float* tinf = &tin[0][0];
  const int tx_tiles = (W + TWD - 1) / TWD, ty_tiles = (H + TH - 1) / TH;
  const int per_img = tx_tiles * ty_tiles;
  const int cog = blockIdx.y * 64;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / per_img;
    const int rem = tile - n * per_img;
    const int ty0 = (rem / tx_tiles) * TH, tx0 = (rem % tx_tiles) * TWD;
    const int b = n / F, f = n - b * F;
    const float* s0 = xt + ((int64_t)b * Fx + (Fx == 1 ? 0 : f)) * H * W;
    const float* s1 = cond + ((int64_t)b * Fc + (Fc == 1 ? 0 : f)) * H * W;
    __syncthreads();
    for (int e = threadIdx.x; e < IH * IW; e += 256) {
      const int yy = ty0 - PAD + e / IW, xx = tx0 - PAD + e % IW;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      tin[0][e] = ok ? s0[(int64_t)yy * W + xx] : 0.f;
      tin[1][e] = ok ? s1[(int64_t)yy * W + xx] : 0.f;
    }
    for (int e = threadIdx.x; e < TH * TWD * 64; e += 256) {
      const int p = e >> 6, c = e & 63;
      const int yy = ty0 + p / TWD, xx = tx0 + p % TWD;
      tdy[p * 65 + c] = (yy < H && xx < W) ? to_f(dy[(((int64_t)n * H + yy) * W + xx) * Co + cog + c]) : 0.f;
    }
    __syncthreads();
    for (int py = 0; py < TH; ++py)
      for (int px = 0; px < TWD; ++px) {
        const float g = tdy[(py * TWD + px) * 65 + co];
        const int base = py * IW + px;
#pragma unroll
        for (int i = 0; i < 25; ++i)
          if (toff[i] >= 0) acc[i] = fmaf(g, tinf[toff[i] + base], acc[i]);
      }
  }
  for (int i = 0; i < tpg; ++i) {
    const int kk = grp * tpg + i;
    if (kk < KK) part[((int64_t)blockIdx.x * Co + cog + co) * KK + kk] = acc[i];
  }
}

// bf16 stem dW on MFMA: dW[co][tap] = sum_px dy[px][co] * X[ci][y+ky-P][x+kx-P]  (tap = (ci,ky,kx)).
// Block = 8x32-pixel tiles (grid-stride), 4 waves = 4 output-channel tiles of 16 (Co slice of 64);
// each wave accumulates all <=7 tap tiles (98 taps padded to 112).  k-step = 32 pixels of one row.
//   A = dy^T fragment via ds_read_b64_tr_b16 from the [256 px][64 co] bf16 tile (XOR-swizzled chunks)
//   B = im2col fragment: 8 consecutive x of tap (ci,ky,kx) — read 16-B aligned from kx-shifted bf16
//       copies tin_k[kx][ci][row][32] of the input halo (so every tap's 8-pixel run is aligned)
constexpr int SW_TH = 8, SW_TW = 32;
__device__ __forceinline__ int sw_dy_off(int px, int co) {  // bf16 index in the [256][64] dy tile
  return px * 64 + ((((co >> 3) ^ (px & 7))) << 3) + (co & 7);
}
__global__ __launch_bounds__(256) void stem_wgrad_mfma_kernel(const float* __restrict__ xt, const float* __restrict__ cond,
                                                              const bf16* __restrict__ dy, float* __restrict__ part,
                                                              int F, int Fx, int Fc, int H, int W, int Co, int KS,
                                                              int ntiles) {
  const int PAD = KS / 2;
  const int IH = SW_TH + KS - 1, IW = SW_TW + KS - 1;  // <= 14 x 38
  const int NT = 2 * KS * KS;                          // taps (<= 98)
  __shared__ float tin[2 * 14 * 38];
  __shared__ __attribute__((aligned(16))) bf16 tink[7 * 2 * 14 * SW_TW];
  __shared__ __attribute__((aligned(16))) bf16 tdy[SW_TH * SW_TW * 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int cog = blockIdx.y * 64;
  // per-lane tap offsets into tink for each of the 7 tap tiles (-1: padded tap)
  int toff[7];
#pragma unroll
  for (int nt = 0; nt < 7; ++nt) {
    const int t = nt * 16 + lr;
    if (t < NT) {
      const int ci = t / (KS * KS), r = t - ci * KS * KS, ky = r / KS, kx = r - ky * KS;
      toff[nt] = ((kx * 2 + ci) * 14 + ky) * SW_TW + lg * 8;
    } else {
      toff[nt] = -1;
    }
  }
  f32x4 acc[7];
#pragma unroll
  for (int nt = 0; nt < 7; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tx_tiles = (W + SW_TW - 1) / SW_TW, ty_tiles = (H + SW_TH - 1) / SW_TH;
  const int per_img = tx_tiles * ty_tiles;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / per_img;
    const int rem = tile - n * per_img;
    const int ty0 = (rem / tx_tiles) * SW_TH, tx0 = (rem % tx_tiles) * SW_TW;
    const int b = n / F, f = n - b * F;
    const float* s0 = xt + ((int64_t)b * Fx + (Fx == 1 ? 0 : f)) * H * W;
    const float* s1 = cond + ((int64_t)b * Fc + (Fc == 1 ? 0 : f)) * H * W;
    __syncthreads();  // previous tile's readers done
    for (int e = tid; e < IH * IW; e += 256) {
      const int yy = ty0 - PAD + e / IW, xx = tx0 - PAD + e % IW;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      tin[e] = ok ? s0[(int64_t)yy * W + xx] : 0.f;
      tin[IH * IW + e] = ok ? s1[(int64_t)yy * W + xx] : 0.f;
    }
    for (int e = tid; e < SW_TH * SW_TW * 8; e += 256) {  // dy: 256 px x 8 chunks of 8 co
      const int px = e >> 3, ch = e & 7;
      const int yy = ty0 + px / SW_TW, xx = tx0 + px % SW_TW;
      bf16x8 v;
      if (yy < H && xx < W) v = *reinterpret_cast<const bf16x8*>(dy + (((int64_t)n * H + yy) * W + xx) * Co + cog + ch * 8);
      else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (bf16)0.f;
      }
      *reinterpret_cast<bf16x8*>(tdy + sw_dy_off(px, ch * 8)) = v;
    }
    __syncthreads();
    for (int e = tid; e < KS * 2 * IH * SW_TW; e += 256) {  // kx-shifted bf16 copies
      const int x = e % SW_TW, r = e / SW_TW;
      const int row = r % IH, r2 = r / IH, ci = r2 & 1, kx = r2 >> 1;
      tink[((kx * 2 + ci) * 14 + row) * SW_TW + x] = (bf16)tin[ci * IH * IW + row * IW + x + kx];
    }
    __syncthreads();
#pragma unroll 2
    for (int py = 0; py < SW_TH; ++py) {
      // A: dy^T[co = wid*16 + i][px = py*32 + 8g + e]
      bf16x8 a;
      const int q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int px = py * SW_TW + lg * 8 + hf * 4 + q;
        const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(tdy + sw_dy_off(px, wid * 16 + p4)));
#pragma unroll
        for (int e = 0; e < 4; ++e) a[hf * 4 + e] = __builtin_bit_cast(bf16, (short)v[e]);
      }
#pragma unroll
      for (int nt = 0; nt < 7; ++nt) {
        bf16x8 bb;
        if (toff[nt] >= 0) bb = *reinterpret_cast<const bf16x8*>(tink + toff[nt] + py * SW_TW);
        else {
#pragma unroll
          for (int i = 0; i < 8; ++i) bb[i] = (bf16)0.f;
        }
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[nt], 0, 0, 0);
      }
    }
  }
  // D[co = wid*16 + 4g + r][tap = nt*16 + i]
#pragma unroll
  for (int nt = 0; nt < 7; ++nt) {
    const int t = nt * 16 + lr;
    if (t >= NT) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = cog + wid * 16 + lg * 4 + r;
      part[((int64_t)blockIdx.x * Co + co) * NT + t] = acc[nt][r];
    }
  }
}

// dst[e] (+)= sum_k part[k][e]: block = 64 elements x 16 split groups (each thread sums every 16th split, the
// 16 group sums are added in a fixed order), so a few thousand elements over hundreds of splits still fill the
// chip (one thread per element ran 512 dependent loads: 120 us for the stem's 6272 x 512 partials)
__global__ __launch_bounds__(1024) void sum_partials_kernel(const float* __restrict__ part, float* __restrict__ dst,
                                                            int nsplit, int64_t n, int accumulate) {
  __shared__ float red[16][65];
  const int el = threadIdx.x & 63, kg = threadIdx.x >> 6;
  const int64_t e = blockIdx.x * (int64_t)64 + el;
  float s = 0.f;
  if (e < n)
    for (int k = kg; k < nsplit; k += 16) s += part[(int64_t)k * n + e];
  red[kg][el] = s;
  __syncthreads();
  if (kg == 0 && e < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][el];
    dst[e] = accumulate ? dst[e] + t : t;
  }
}

// ----------------------------------------------------------------------------------------
// head: Conv3d(C -> 1, 1) evaluated only on frame F//2 (the frame model.py:124-130 keeps).
// out[b][y][x] (fp32 [B,1,H,W]) = bias + sum_c w[c] * x[(b*F+mid)][y][x][c]
// ----------------------------------------------------------------------------------------
template <typename T>
__global__ void head_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                                float* __restrict__ out, int B, int F, int HW, int C) {
  // one 64-lane wave per 8 pixels: 8 lanes per pixel, each lane 8 channels (C <= 64*... looped)
  const int64_t gw = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 3;
  const int sub = threadIdx.x & 7;
  const int64_t total = (int64_t)B * HW;
  if (gw >= total) return;
  const int b = (int)(gw / HW);
  const int64_t p = gw - (int64_t)b * HW;
  const T* src = x + (((int64_t)b * F + F / 2) * HW + p) * C;
  float s = 0.f;
  for (int c = sub * 8; c < C; c += 64) {
    float v[8];
    load8(src + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) s = fmaf(v[i], w[c + i], s);
  }
  s = group_sum(s, 8);
  if (sub == 0) out[gw] = s + bias[0];
}

// dX = 0 everywhere except frame mid where dX[c] = dout * w[c]
template <typename T>
__global__ void head_dgrad_kernel(const float* __restrict__ dout, const float* __restrict__ w, T* __restrict__ dx,
                                  int B, int F, int HW, int C) {
  const int64_t total = (int64_t)B * F * HW * (C / 8);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int cq = (int)(e % (C / 8));
    const int64_t vox = e / (C / 8);
    const int64_t p = vox % HW;
    const int64_t nf = vox / HW;
    const int f = (int)(nf % F), b = (int)(nf / F);
    float v[8];
    const float g = (f == F / 2) ? dout[(int64_t)b * HW + p] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = g * w[cq * 8 + i];
    store8(dx + vox * C + cq * 8, v);
  }
}

// head weight/bias grads: part[blk][c] (c < C) and part[blk][C] = bias.  Thread = (pixel lane pl, 8-channel chunk
// sub): one coalesced pass over the mid frame (the per-channel strided loop it replaces read it C + 1 times:
// 0.5 ms per step); per-block sums over the 32 pixel lanes in a fixed order
template <typename T>
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ dout, const T* __restrict__ x,
                                                         float* __restrict__ part, int B, int F, int HW, int C,
                                                         int64_t px_per_blk) {
  __shared__ float red[32][65];
  const int64_t total = (int64_t)B * HW;
  const int64_t p0 = blockIdx.x * px_per_blk, p1 = min(total, p0 + px_per_blk);
  const int sub = threadIdx.x & 7, pl = threadIdx.x >> 3;
  for (int c0 = 0; c0 < C; c0 += 64) {
    const bool live = c0 + sub * 8 < C;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, gs = 0.f;
    for (int64_t q = p0 + pl; q < p1; q += 32) {
      const int b = (int)(q / HW);
      const int64_t p = q - (int64_t)b * HW;
      const float g = dout[q];
      gs += g;
      if (live) {
        float v[8];
        load8(x + (((int64_t)b * F + F / 2) * HW + p) * C + c0 + sub * 8, v);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(g, v[i], acc[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) red[pl][sub * 8 + i] = acc[i];
    if (sub == 0) red[pl][64] = gs;
    __syncthreads();
    if (threadIdx.x < 65) {
      const int c = threadIdx.x;
      float t = 0.f;
      for (int q = 0; q < 32; ++q) t += red[q][c];
      if (c < 64 && c0 + c < C) part[(int64_t)blockIdx.x * (C + 1) + c0 + c] = t;
      if (c == 64 && c0 == 0) part[(int64_t)blockIdx.x * (C + 1) + C] = t;
    }
    __syncthreads();
  }
}

__global__ void head_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw, float* __restrict__ db,
                                   int nblk, int C, int accumulate) {
  for (int c = threadIdx.x; c <= C; c += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += part[(int64_t)k * (C + 1) + c];
    float* d = (c == C) ? db : dw + c;
    *d = accumulate ? *d + s : s;
  }
}

// Kernel selection of cesm_conv_fwd (host only, no GPU work): every launch and the
// cesm_conv_fwd_variant query go through this one function, so tests can assert which kernel a shape reaches.
enum ConvFwdVariant {
  CFV_INVALID = -1,
  CFV_GEMM1X1_128 = 0, CFV_GEMM1X1_64, CFV_P32_RW, CFV_HALO36, CFV_HALO32, CFV_TCONV_PAR_128, CFV_TCONV_PAR_64, CFV_GEN_BF16_128, CFV_GEN_BF16_64,
  CFV_GEN_F32_128, CFV_GEN_F32_64, CFV_S2DOWN36, CFV_S2DOWN32, CFV_S2UP36, CFV_S2UP32, CFV_WS32, CFV_WS36, CFV_COUNT
};
static const char* const kConvFwdVariantName[CFV_COUNT] = {
    "gemm1x1_kernel<128>", "gemm1x1_kernel<64>", "conv3x3p_kernel<32,7,true>", "conv3x3_bf16_kernel<36>",
    "conv3x3_bf16_kernel<32>", "conv_fwd_bf16_kernel<128,true>", "conv_fwd_bf16_kernel<64,true>",
    "conv_fwd_bf16_kernel<128>", "conv_fwd_bf16_kernel<64>", "conv_fwd_kernel<float,128>",
    "conv_fwd_kernel<float,64>", "convs2_bf16_kernel<36,down>", "convs2_bf16_kernel<32,down>",
    "convs2_bf16_kernel<36,up>", "convs2_bf16_kernel<32,up>", "conv3x3ws_kernel<32>", "conv3x3ws_kernel<36>"};

struct ConvFwdPlan {
  ConvFwdVariant v = CFV_INVALID;
  int TH = 0, TW = 0;  // halo tile (conv3x3p / conv3x3ws / halo kernels)
};

static ConvFwdPlan conv_fwd_plan(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int Co1,
                                 int KH, int KW, int S, int P, int U) {
  ConvFwdPlan pl;
  if ((C1 % BK) || (C2 % BK) || (Cout % 64) || (Co1 % 16) || Co1 > Cout || C1 <= 0) return pl;
  if (dtype != CESM_DT_BF16 && dtype != CESM_DT_F32) return pl;
  const int64_t M = (int64_t)Nb * Ho * Wo;
  const int BN = (Cout % 128 == 0) ? 128 : 64;
  const bool halo3 = dtype == CESM_DT_BF16 && KH == 3 && KW == 3 && S == 1 && P == 1 && U == 1 && Ho == Hi &&
                     Wo == Wi && (Co1 % H3_BN) == 0;
  const bool g1x1 = dtype == CESM_DT_BF16 && KH == 1 && KW == 1 && S == 1 && P == 0 && U == 1 && Ho == Hi &&
                    Wo == Wi && (C1 % 64) == 0 && (C2 % 64) == 0 && (Co1 % 8) == 0 && M < (1ll << 31);
  int wth = 0, wtw = 0;
  // warp-specialized conv: by default for the level-0 64 -> 64 shape only (the conv3x3p case: 579 -> 518 us at
  // 96 x 192 x 288, profiles/r4c4_ws_check.txt); at 128 / 256 channels and for concat inputs it measured 0.85 - 1.01x
  // of the halo conv, so there it is opt-in (CESM_CONV_WS=1)
  const bool ws = halo3 && (C1 + C2) >= 64 && (getenv_flag("CESM_CONV_WS") || (C1 == 64 && C2 == 0 && Cout == 64));
  const double wutil = ws ? ws_tile(Ho, Wo, wth, wtw) : 0.0;
  if (g1x1) {
    pl.v = (Cout % 128 == 0) ? CFV_GEMM1X1_128 : CFV_GEMM1X1_64;
  } else if (wutil >= 0.9) {
    // warp-specialized persistent conv (round 4) where its 256-pixel tiles cover the image to >= 90 %
    pl.v = wtw == 36 ? CFV_WS36 : CFV_WS32;
    pl.TH = wth;
    pl.TW = wtw;
  } else if (halo3 && (C1 + C2) == 64 && Cout == 64 && (Wo % 32) == 0) {
    // v4 (persistent, resident weights) for the level-0 64 -> 64 convs the warp-specialized tiles do not cover
    // (the reference's 64 / 128-wide crops): TW = 32 -> TH = 14 (448 px = 4 waves x 7 groups).  (Round 6 removed the
    // env-selected alternatives: the halo conv here, this kernel everywhere, its 3-stage and streamed-weight forms,
    // and the round-1 v2 / v3 kernels -- all measured slower, profiles/r2_*, r3_conv_v4_everywhere_ab.txt.)
    pl.TW = 32;
    pl.TH = CP_TH;
    pl.v = CFV_P32_RW;
  } else if (halo3) {
    pl.TH = H3_TH; pl.TW = H3_TW;
    h3_big_tile(Ho, Wo, pl.TH, pl.TW);
    pl.v = pl.TW == 36 ? CFV_HALO36 : CFV_HALO32;
  } else if (dtype == CESM_DT_BF16 && KH == 4 && KW == 4 && C2 == 0 && Co1 == Cout && (Cout % H3_BN) == 0 &&
             ((S == 2 && P == 1 && U == 1 && Hi == 2 * Ho && Wi == 2 * Wo) ||
              (S == 1 && P == 2 && U == 2 && Ho == 2 * Hi && Wo == 2 * Wi))) {
    // stride-2 4x4 conv / its transpose: halo kernel on the low-resolution grid
    const bool up = U == 2;
    const int Hl = up ? Hi : Ho, Wl = up ? Wi : Wo;
    pl.TH = H3_TH; pl.TW = H3_TW;
    c2_tile(Hl, Wl, pl.TH, pl.TW, true);
    pl.v = up ? (pl.TW == 36 ? CFV_S2UP36 : CFV_S2UP32) : (pl.TW == 36 ? CFV_S2DOWN36 : CFV_S2DOWN32);
  } else if (dtype == CESM_DT_BF16 && U == 2 && S == 1 && KH % 2 == 0 && KW % 2 == 0 && Ho % 2 == 0 &&
             Wo % 2 == 0) {
    pl.v = BN == 128 ? CFV_TCONV_PAR_128 : CFV_TCONV_PAR_64;
  } else if (dtype == CESM_DT_BF16) {
    pl.v = BN == 128 ? CFV_GEN_BF16_128 : CFV_GEN_BF16_64;
  } else {
    pl.v = BN == 128 ? CFV_GEN_F32_128 : CFV_GEN_F32_64;
  }
  return pl;
}

}  // namespace

// ========================================================================================
// C ABI
// ========================================================================================
extern "C" {

const char* cesm_conv_fwd_variant(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout,
                                  int Co1, int KH, int KW, int S, int P, int U) {
  const ConvFwdPlan pl = conv_fwd_plan(dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P, U);
  return pl.v == CFV_INVALID ? "invalid" : kConvFwdVariantName[pl.v];
}

}  // extern "C"

namespace {
// GroupNorm statistics partial slots per sample that the halo conv of plan pl writes for Nb images in B samples:
// conv3x3p: (frame, tile, wave), conv3x3_bf16: (frame, tile, pixel half); 0 = this plan has no partials
int64_t conv_gn_nslot(const ConvFwdPlan& pl, int Nb, int Ho, int Wo, int B) {
  if (B <= 0 || Nb % B) return 0;
  const int64_t fimg = Nb / B;
  const int64_t tiles = (pl.TW > 0 && pl.TH > 0) ? cdiv(Wo, pl.TW) * cdiv(Ho, pl.TH) : 0;
  switch (pl.v) {
    case CFV_P32_RW: return fimg * tiles * 4;
    case CFV_HALO36: case CFV_HALO32: return fimg * tiles * 4;
    case CFV_WS32: case CFV_WS36: return fimg * tiles * 4;
    default: return 0;
  }
}

int conv_fwd_launch(int dtype, const void* x1, const void* x2, const void* wp, const float* bias, const void* res,
                    const void* res2, void* y1, void* y2, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo,
                    int Cout, int Co1, int KH, int KW, int S, int P, int U, float* gnp, int gn_fimg, int* queue,
                    hipStream_t stream) {
  const ConvFwdPlan pl = conv_fwd_plan(dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P, U);
  if (pl.v == CFV_INVALID) return CESM_EINVAL;
  ConvGeom g{Nb, Hi, Wi, Ho, Wo, C1, C2, Cout, Co1, KH, KW, S, P, U};
  g.wch = wpk_chunked(dtype == CESM_DT_BF16, Cout, C1 + C2, KH, KW);
  const int64_t M = (int64_t)Nb * Ho * Wo;
  const int BN = (Cout % 128 == 0) ? 128 : 64;
  dim3 grid(Cout / BN, (unsigned)cdiv(M, BMP));
  const bf16 *bx1 = (const bf16*)x1, *bx2 = (const bf16*)x2, *bwp = (const bf16*)wp, *br = (const bf16*)res,
             *br2 = (const bf16*)res2;
  bf16 *by1 = (bf16*)y1, *by2 = (bf16*)y2;
  const int TH = pl.TH, TW = pl.TW;
  switch (pl.v) {
    case CFV_GEMM1X1_128:
    case CFV_GEMM1X1_64: {
      const bool one = C1 + C2 == 64;  // single-stage K = 64 variant
#define G1L(BNv, NSv)                                                                                               \
  gemm1x1_kernel<BNv, NSv><<<dim3((unsigned)(Cout / BNv * 8 * cdiv(cdiv(M, G1_BM), 8))), 256, 0, stream>>>(      \
      bx1, bx2, bwp, bias, br, br2, by1, by2, (int)M, C1, C2, Cout, Co1)
      if (pl.v == CFV_GEMM1X1_128) {
        if (one) G1L(128, 1); else G1L(128, 2);
      } else {
        if (one) G1L(64, 1); else G1L(64, 2);
      }
#undef G1L
      break;
    }
    case CFV_P32_RW: {
      const int tx = (int)cdiv(Wo, TW), ty = (int)cdiv(Ho, TH);
      const int ncob = Cout / 64;
      const int nitems = Nb * tx * ty * ncob;
      const int nblk = std::min(nitems, cesm_num_cus());
      conv3x3p_kernel<32, 7, true><<<nblk, 256, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, tx, tx * ty, TH,
                                                             ncob, nitems, gnp, gn_fimg);
      break;
    }
    case CFV_WS32:
    case CFV_WS36: {
      const int tx = (int)cdiv(Wo, TW), ty = (int)cdiv(Ho, TH);
      const int ncob = Cout / 64;
      const int ntile = Nb * tx * ty;
      const int nitems_pad = (int)cdiv(ntile, 8) * 8 * ncob;
      const int nblk = std::min(nitems_pad, cesm_num_cus());
      // a stale count (a launch cut short, an aborted capture) would make every block of this launch find the queue
      // dry: zero it in stream order first (the kernel's last block also resets it)
      if (queue) (void)hipMemsetAsync(queue, 0, 2 * sizeof(int), stream);
#define WSL(TWv, GNv)                                                                                              \
  conv3x3ws_kernel<TWv, GNv><<<nblk, 512, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, TH, tx, tx * ty, ncob, \
                                                       nitems_pad, gnp, gn_fimg, queue)
      if (pl.v == CFV_WS36) { if (gnp) WSL(36, true); else WSL(36, false); }
      else { if (gnp) WSL(32, true); else WSL(32, false); }
#undef WSL
      break;
    }
    case CFV_HALO36:
    case CFV_HALO32: {
      const int tx = (int)cdiv(Wo, TW), ty = (int)cdiv(Ho, TH);
      const unsigned g3 = (unsigned)(Cout / H3_BN) * 8u * (unsigned)cdiv((int64_t)tx * ty * Nb, 8);
      const bool big = TH * TW > 256;  // h3_big_tile chose a 448-pixel tile
#define H3L(TWv, NJv)                                                                                                \
  conv3x3_bf16_kernel<TWv, NJv><<<g3, 256, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, tx, TH, gnp, gn_fimg)
      if (pl.v == CFV_HALO36) { if (big) H3L(36, 7); else H3L(36, 4); }
      else { if (big) H3L(32, 7); else H3L(32, 4); }
#undef H3L
      break;
    }
    case CFV_S2DOWN36:
    case CFV_S2DOWN32:
    case CFV_S2UP36:
    case CFV_S2UP32: {
      const bool up = pl.v == CFV_S2UP36 || pl.v == CFV_S2UP32;
      const int Hl = up ? Hi : Ho, Wl = up ? Wi : Wo;
      const int tx = (int)cdiv(Wl, TW), ty = (int)cdiv(Hl, TH);
      dim3 g3(tx * ty, Nb, (Cout / H3_BN) * (up ? 4 : 1));
      if (pl.v == CFV_S2DOWN36)
        convs2_bf16_kernel<36, false><<<g3, 256, 0, stream>>>(bx1, bwp, bias, br, by1, g, tx, TH, Hl, Wl);
      else if (pl.v == CFV_S2DOWN32)
        convs2_bf16_kernel<32, false><<<g3, 256, 0, stream>>>(bx1, bwp, bias, br, by1, g, tx, TH, Hl, Wl);
      else if (pl.v == CFV_S2UP36)
        convs2_bf16_kernel<36, true><<<g3, 256, 0, stream>>>(bx1, bwp, bias, br, by1, g, tx, TH, Hl, Wl);
      else
        convs2_bf16_kernel<32, true><<<g3, 256, 0, stream>>>(bx1, bwp, bias, br, by1, g, tx, TH, Hl, Wl);
      break;
    }
    case CFV_TCONV_PAR_128:
    case CFV_TCONV_PAR_64: {
      const int64_t Mp = (int64_t)Nb * (Ho / 2) * (Wo / 2);
      const int bpp = (int)cdiv(Mp, BMP);
      dim3 gp(Cout / BN, 4 * bpp);
      if (pl.v == CFV_TCONV_PAR_128)
        conv_fwd_bf16_kernel<128, true><<<gp, 256, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, Mp, bpp);
      else
        conv_fwd_bf16_kernel<64, true><<<gp, 256, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, Mp, bpp);
      break;
    }
    case CFV_GEN_BF16_128:
      conv_fwd_bf16_kernel<128><<<grid, 256, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, M);
      break;
    case CFV_GEN_BF16_64:
      conv_fwd_bf16_kernel<64><<<grid, 256, 0, stream>>>(bx1, bx2, bwp, bias, br, br2, by1, by2, g, M);
      break;
    case CFV_GEN_F32_128:
      conv_fwd_kernel<float, 128><<<grid, 256, 0, stream>>>((const float*)x1, (const float*)x2, (const float*)wp,
                                                            bias, (const float*)res, (const float*)res2, (float*)y1,
                                                            (float*)y2, g, M);
      break;
    case CFV_GEN_F32_64:
      conv_fwd_kernel<float, 64><<<grid, 256, 0, stream>>>((const float*)x1, (const float*)x2, (const float*)wp,
                                                           bias, (const float*)res, (const float*)res2, (float*)y1,
                                                           (float*)y2, g, M);
      break;
    default:
      return CESM_EINVAL;
  }
  return cesm_launch_status();
}
}  // namespace

extern "C" {

// Generic implicit-GEMM conv / dgrad.  Shapes: x1 [Nb][Hi][Wi][C1], x2 [Nb][Hi][Wi][C2] (may be
// null if C2 == 0), wp [Cout][KH*KW][C1+C2] packed, y1 [Nb][Ho][Wo][Co1], y2 [..][Cout-Co1].
int cesm_conv_fwd(int dtype, const void* x1, const void* x2, const void* wp, const float* bias, const void* res,
                  const void* res2, void* y1, void* y2, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int Co1,
                  int KH, int KW, int S, int P, int U, int* queue, hipStream_t stream) {
  if (Nb <= 0 || Ho <= 0 || Wo <= 0) return CESM_OK;
  return conv_fwd_launch(dtype, x1, x2, wp, bias, res, res2, y1, y2, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Co1, KH, KW, S, P,
                         U, nullptr, 1, queue, stream);
}

int64_t cesm_conv_gn_nslot(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int KH, int KW,
                           int S, int P, int U, int B) {
  const ConvFwdPlan pl = conv_fwd_plan(dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Cout, KH, KW, S, P, U);
  return conv_gn_nslot(pl, Nb, Ho, Wo, B);
}

int cesm_conv_fwd_gn(int dtype, const void* x1, const void* x2, const void* wp, const float* bias, void* y, float* gnpart,
                     int B, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int KH, int KW, int S,
                     int P, int U, int* queue, hipStream_t stream) {
  if (Nb <= 0 || Ho <= 0 || Wo <= 0) return CESM_OK;
  const ConvFwdPlan pl = conv_fwd_plan(dtype, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Cout, KH, KW, S, P, U);
  if (pl.v == CFV_INVALID) return CESM_EINVAL;
  if (!gnpart || conv_gn_nslot(pl, Nb, Ho, Wo, B) == 0) return CESM_EUNSUPPORTED;
  return conv_fwd_launch(dtype, x1, x2, wp, bias, nullptr, nullptr, y, nullptr, Nb, Hi, Wi, C1, C2, Ho, Wo, Cout, Cout,
                         KH, KW, S, P, U, gnpart, Nb / B, queue, stream);
}

}  // extern "C"

namespace {
// Kernel selection of cesm_conv_wgrad (host only)
enum WgradVariant { WGV_WIDE = 0, WGV_GEN, WGV_S2, WGV_W32C64, WGV_W36C64 };
// input-channel tile of wgrad_sq_kernel for a bf16 1x1 weight gradient it takes (0: the wide kernel's 64-column
// tiles): one source, one destination, no bias; Cout % 256 == 0 with BN = 256 when Cin % 256 == 0, else 128; or
// Cout = 64 with Cin % 256 == 0 (64 x 256 tiles)
static int wgrad_sq_bn(int KH, int KW, int S, int P, int U, int Hi, int Wi, int Ho, int Wo, int C1, int C2, int Cout,
                       int Co1, bool with_bias) {
  (void)with_bias;  // the bias gradient rides along (BIAS instantiations)
  if (KH != 1 || KW != 1 || S != 1 || P != 0 || U != 1 || Hi != Ho || Wi != Wo || C2 != 0 || Co1 != Cout) return 0;
  if (Cout == 64) return C1 % 256 == 0 ? 256 : 0;  // 64 x 256 tiles (the level-0 to_out: dY read once, not per 64 ci)
  if (Cout % 256 != 0) return 0;
  if (C1 % 256 == 0) return 256;
  if (C1 % 128 == 0) return 128;
  return 0;
}
static int wgrad_plan(int dtype, int64_t M, int Hi, int Wi, int Ho, int Wo, int KH, int KW, int S, int P, int U) {
  const bool halo3 = dtype == CESM_DT_BF16 && KH == 3 && KW == 3 && S == 1 && P == 1 && U == 1 && Ho == Hi &&
                     Wo == Wi;
  // 8 x 36 tiles only where 32-wide tiles waste >= 20 % of the columns (W = 36, 72); at W = 144 / 288
  // the 8 x 32 kernel's row-aligned K chunks are faster despite the partial last tile
  if (halo3 && (Wo % W36_TW) == 0 && 5 * Wo <= 4 * (int)cdiv(Wo, W3_TW) * W3_TW) return WGV_W36C64;
  if (halo3) return WGV_W32C64;  // (C1 % 64 == 0: cesm_conv_wgrad)
  // (32-wide pixel tiles: at Wo = 36 the second tile of a row is 8/9 empty and the wide kernel is faster)
  if (dtype == CESM_DT_BF16 && KH == 4 && KW == 4 && S == 2 && P == 1 && U == 1 && Hi == 2 * Ho && Wi == 2 * Wo &&
      Wo >= 64)
    return WGV_S2;
  if (dtype == CESM_DT_BF16 && M < (1ll << 31)) return WGV_WIDE;
  return WGV_GEN;
}
}  // namespace

extern "C" {

// input-channel tile of the square-tile 1x1 weight-gradient kernel for this shape (0: not taken); the caller sizes
// nsplit (and the slab) for Cout/256 x Cin/BN tiles when it is non-zero
int cesm_conv_wgrad_sq_bn(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int Co1, int KH,
                          int KW, int S, int P, int U, int with_bias) {
  const int64_t M = (int64_t)Nb * Ho * Wo;
  if (wgrad_plan(dtype, M, Hi, Wi, Ho, Wo, KH, KW, S, P, U) != WGV_WIDE) return 0;
  return wgrad_sq_bn(KH, KW, S, P, U, Hi, Wi, Ho, Wo, C1, C2, Cout, Co1, with_bias != 0);
}

const char* cesm_conv_wgrad_variant(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout,
                                    int Co1, int KH, int KW, int S, int P, int U, int with_bias) {
  const int64_t M = (int64_t)Nb * Ho * Wo;
  int wv = wgrad_plan(dtype, M, Hi, Wi, Ho, Wo, KH, KW, S, P, U);
  if (wv == WGV_S2 && (with_bias || C2 || Co1 != Cout)) wv = WGV_WIDE;  // (cesm_conv_wgrad's fallback)
  switch (wv) {
    case WGV_W32C64: return "wgrad3x3c64_kernel";
    case WGV_W36C64: return "wgrad3x3w36c64_kernel";
    case WGV_S2: return "wgrads2_bf16_kernel";
    case WGV_WIDE: {
      const int sq = wgrad_sq_bn(KH, KW, S, P, U, Hi, Wi, Ho, Wo, C1, C2, Cout, Co1, with_bias != 0);
      if (sq) {
        static const char* const sqn[6] = {"wgrad_sq_kernel<64,256>", "wgrad_sq_kernel<64,256,true>",
                                           "wgrad_sq_kernel<256,256>", "wgrad_sq_kernel<256,256,true>",
                                           "wgrad_sq_kernel<256,128>", "wgrad_sq_kernel<256,128,true>"};
        return sqn[(Cout == 64 ? 0 : sq == 256 ? 2 : 4) + (with_bias ? 1 : 0)];
      }
      const int bm = (Cout % 256 == 0 && Co1 % 256 == 0) ? 256 : ((Cout % 128 == 0 && Co1 % 128 == 0) ? 128 : 64);
      static const char* const names[6] = {"wgrad_wide_kernel<64,false>", "wgrad_wide_kernel<64,true>",
                                           "wgrad_wide_kernel<128,false>", "wgrad_wide_kernel<128,true>",
                                           "wgrad_wide_kernel<256,false>", "wgrad_wide_kernel<256,true>"};
      return names[(bm == 256 ? 4 : bm == 128 ? 2 : 0) + (with_bias ? 1 : 0)];
    }
    default: return dtype == CESM_DT_BF16 ? "conv_wgrad_kernel<__bf16>" : "conv_wgrad_kernel<float>";
  }
}

// Weight gradient of the conv whose forward launch had geometry (…, KH, KW, S, P, U).
// x = forward input (two sources), dy = forward output grad (two destinations, Co1 split).
// Result accumulated/written into the PyTorch weight tensor `dw` ([D0][D1][1][KH][KW] with the
// (swap, flip) mapping of the pack).  `slab` is an fp32 workspace of nsplit*Cout*K floats.
int cesm_conv_wgrad(int dtype, const void* x1, const void* x2, const void* dy1, const void* dy2, float* dw,
                    float* slab, float* db, float* bslab, int nsplit, int Nb, int Hi, int Wi, int C1, int C2, int Ho,
                    int Wo, int Cout, int Co1, int KH, int KW, int S, int P, int U, int swap, int flip, int accumulate,
                    hipStream_t stream) {
  if (db && !bslab) return CESM_EINVAL;
  const int Cin = C1 + C2;
  if ((Cin % 64) || (C1 % 64) || (Cout % 64) || (Co1 % 64) || nsplit <= 0) return CESM_EINVAL;
  ConvGeom g{Nb, Hi, Wi, Ho, Wo, C1, C2, Cout, Co1, KH, KW, S, P, U};
  const int64_t M = (int64_t)Nb * Ho * Wo;
  const int64_t pps = cdiv(cdiv(M, nsplit), WG_BP) * WG_BP;
  const int K = KH * KW * Cin;
  dim3 grid(Cout / 64, K / 64, nsplit);
  const int wv = wgrad_plan(dtype, M, Hi, Wi, Ho, Wo, KH, KW, S, P, U);
  if (wv == WGV_W36C64) {
    const int tx = Wo / W36_TW;
    const int ntiles = Nb * tx * (int)cdiv(Ho, W36_TH);
    dim3 g3(Cout / 64, Cin / 64, std::min(nsplit, ntiles));
    wgrad3x3w36c64_kernel<<<g3, WG_NT, 0, stream>>>((const bf16*)x1, (const bf16*)x2, (const bf16*)dy1,
                                                  (const bf16*)dy2, slab, g, tx, ntiles);
    nsplit = (int)g3.z;
  } else if (wv == WGV_W32C64) {
    const int tx = (int)cdiv(Wo, W3_TW);
    const int ntiles = Nb * tx * (int)cdiv(Ho, W3_TH);
    dim3 g3(Cout / 64, Cin / 64, std::min(nsplit, ntiles));
    wgrad3x3c64_kernel<<<g3, WG_NT, 0, stream>>>((const bf16*)x1, (const bf16*)x2, (const bf16*)dy1,
                                               (const bf16*)dy2, slab, g, tx, ntiles);
    nsplit = (int)g3.z;
  } else if (wv == WGV_S2 && C2 == 0 && Co1 == Cout && !db) {
    const int tx = (int)cdiv(Wo, W3_TW);
    const int ntiles = Nb * tx * (int)cdiv(Ho, W3_TH);
    dim3 g3(Cout / 64, (Cin / 32) * 4, std::min(nsplit, ntiles));
    wgrads2_bf16_kernel<<<g3, 256, 0, stream>>>((const bf16*)x1, (const bf16*)dy1, slab, g, tx, ntiles);
    nsplit = (int)g3.z;
  } else if (wv == WGV_WIDE && wgrad_sq_bn(KH, KW, S, P, U, Hi, Wi, Ho, Wo, C1, C2, Cout, Co1, db != nullptr) > 0) {
    // square 256 x BN tiles for the 1x1 convs whose dY would be re-read once per 64 input channels (the caller sized
    // nsplit for these tiles: cesm_conv_wgrad_sq_bn)
    const int bn = wgrad_sq_bn(KH, KW, S, P, U, Hi, Wi, Ho, Wo, C1, C2, Cout, Co1, db != nullptr);
    const int bm = Cout % 256 == 0 ? 256 : 64;
    const dim3 gq(Cout / bm, Cin / bn, nsplit);
    const bf16 *qx = (const bf16*)x1, *qy = (const bf16*)dy1;
#define SQL(BMv, BNv, Bv) \
  wgrad_sq_kernel<BMv, BNv, Bv><<<gq, 512, 0, stream>>>(qx, qy, slab, bslab, (int)M, Cout, Cin, (int)pps)
    if (bm == 64) { if (db) SQL(64, 256, true); else SQL(64, 256, false); }
    else if (bn == 256) { if (db) SQL(256, 256, true); else SQL(256, 256, false); }
    else { if (db) SQL(256, 128, true); else SQL(256, 128, false); }
#undef SQL
    if (db) colsum_final_kernel<<<Cout, 64, 0, stream>>>(bslab, db, nsplit, Cout, 1);
  } else if (wv == WGV_WIDE || wv == WGV_S2) {
    // wide-tile kernel; nsplit from the caller sized the slab for 64-row tiles, keep it
    const int bm = (Cout % 256 == 0 && Co1 % 256 == 0) ? 256 : ((Cout % 128 == 0 && Co1 % 128 == 0) ? 128 : 64);
    const int gx = Cout / bm, gy = (int)(K / 64);
    const dim3 gw(gx, gy, nsplit);
    auto launch = [&](auto bmc, auto biasc) {
      constexpr int BMv = decltype(bmc)::value;
      constexpr bool Bv = decltype(biasc)::value;
      wgrad_wide_kernel<BMv, Bv><<<gw, 256, 0, stream>>>((const bf16*)x1, (const bf16*)x2, (const bf16*)dy1,
                                                         (const bf16*)dy2, slab, bslab, g, (int)M, (int)pps);
    };
    using T0 = std::false_type;
    using T1 = std::true_type;
    if (bm == 256) { if (db) launch(std::integral_constant<int, 256>{}, T1{}); else launch(std::integral_constant<int, 256>{}, T0{}); }
    else if (bm == 128) { if (db) launch(std::integral_constant<int, 128>{}, T1{}); else launch(std::integral_constant<int, 128>{}, T0{}); }
    else { if (db) launch(std::integral_constant<int, 64>{}, T1{}); else launch(std::integral_constant<int, 64>{}, T0{}); }
    if (db) colsum_final_kernel<<<Cout, 64, 0, stream>>>(bslab, db, nsplit, Cout, 1);
  } else if (db) {
    return CESM_EUNSUPPORTED;  // the bias gradient rides only on the wide kernel (callers use cesm_colsum)
  } else if (dtype == CESM_DT_BF16)
    conv_wgrad_kernel<bf16><<<grid, 256, 0, stream>>>((const bf16*)x1, (const bf16*)x2, (const bf16*)dy1,
                                                      (const bf16*)dy2, slab, g, M, pps);
  else if (dtype == CESM_DT_F32)
    conv_wgrad_kernel<float><<<grid, 256, 0, stream>>>((const float*)x1, (const float*)x2, (const float*)dy1,
                                                       (const float*)dy2, slab, g, M, pps);
  else
    return CESM_EINVAL;
  const int64_t total = (int64_t)Cout * K;
  conv_wgrad_reduce_kernel<<<(unsigned)cdiv(total, 64), 256, 0, stream>>>(slab, dw, nsplit, Cout, Cin, KH, KW, swap,
                                                                          flip, accumulate);
  return cesm_launch_status();
}

int cesm_conv_pack(int dtype, const float* w, void* wp, int Cout, int Cin, int KH, int KW, int swap, int flip,
                   hipStream_t stream) {
  const int64_t total = (int64_t)Cout * KH * KW * Cin;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(total, 256), 4096);
  if (dtype == CESM_DT_BF16)
    conv_pack_kernel<bf16><<<grid, 256, 0, stream>>>(w, (bf16*)wp, Cout, Cin, KH, KW, swap, flip);
  else if (dtype == CESM_DT_F32)
    conv_pack_kernel<float><<<grid, 256, 0, stream>>>(w, (float*)wp, Cout, Cin, KH, KW, swap, flip);
  else
    return CESM_EINVAL;
  return cesm_launch_status();
}

int cesm_conv_pack_batch(int dtype, const int64_t* jobs, int njobs, int nblocks, hipStream_t stream) {
  if (njobs <= 0) return CESM_OK;
  const unsigned grid = (unsigned)std::max(1, nblocks);  // any grid is correct (block-stride loop)
  if (dtype == CESM_DT_BF16)
    conv_pack_batch_kernel<bf16><<<grid, 256, 0, stream>>>(jobs, njobs);
  else if (dtype == CESM_DT_F32)
    conv_pack_batch_kernel<float><<<grid, 256, 0, stream>>>(jobs, njobs);
  else
    return CESM_EINVAL;
  return cesm_launch_status();
}

// dst[c] (+)= sum_r x[r][c] ; part = workspace nsplit*C floats
int cesm_colsum(int dtype, const void* x, float* dst, float* part, int nsplit, int64_t rows, int C, int accumulate,
                hipStream_t stream) {
  if (C % 4 || C > 1024 || nsplit <= 0) return CESM_EINVAL;
  const int64_t rps = cdiv(rows, nsplit);
  if (dtype == CESM_DT_BF16)
    colsum_partial_kernel<bf16><<<nsplit, 256, 0, stream>>>((const bf16*)x, part, rows, C, rps);
  else if (dtype == CESM_DT_F32)
    colsum_partial_kernel<float><<<nsplit, 256, 0, stream>>>((const float*)x, part, rows, C, rps);
  else
    return CESM_EINVAL;
  colsum_final_kernel<<<C, 64, 0, stream>>>(part, dst, nsplit, C, accumulate);
  return cesm_launch_status();
}

int cesm_stem_fwd(int dtype, const float* xt, const float* cond, const float* w, const float* bias, void* y, int B,
                  int F, int Fx, int Fc, int H, int W, int Co, int KS, hipStream_t stream) {
  if (KS > 7 || Co % 64) return CESM_EINVAL;
  dim3 grid((unsigned)(cdiv(H, 16) * cdiv(W, 16)), Co / 64, B * F);
  if (dtype == CESM_DT_BF16 && 2 * KS * KS <= 128) {
    const int ntiles = (int)(cdiv(H, 16) * cdiv(W, 16)) * B * F;
    dim3 gp((unsigned)std::min(ntiles, 4 * cesm_num_cus()), Co / 64);
    stem_fwd_mfma_kernel<<<gp, 256, 0, stream>>>(xt, cond, w, bias, (bf16*)y, B, F, Fx, Fc, H, W, Co, KS, ntiles);
  } else if (dtype == CESM_DT_BF16)
    stem_fwd_kernel<bf16><<<grid, 256, 0, stream>>>(xt, cond, w, bias, (bf16*)y, B, F, Fx, Fc, H, W, Co, KS);
  else if (dtype == CESM_DT_F32)
    stem_fwd_kernel<float><<<grid, 256, 0, stream>>>(xt, cond, w, bias, (float*)y, B, F, Fx, Fc, H, W, Co, KS);
  else
    return CESM_EINVAL;
  return cesm_launch_status();
}

// stem dW (+ bias via cesm_colsum on dy); part: nblk*Co*2*KS*KS floats
int cesm_stem_wgrad(int dtype, const float* xt, const float* cond, const void* dy, float* dw, float* part, int nblk,
                    int B, int F, int Fx, int Fc, int H, int W, int Co, int KS, int accumulate, hipStream_t stream) {
  if (KS > 7 || Co % 64 || nblk <= 0) return CESM_EINVAL;
  const int ntiles = B * F * (int)cdiv(H, 8) * (int)cdiv(W, 32);
  dim3 grid(nblk, Co / 64);
  if (dtype == CESM_DT_BF16)
    stem_wgrad_mfma_kernel<<<grid, 256, 0, stream>>>(xt, cond, (const bf16*)dy, part, F, Fx, Fc, H, W, Co, KS, ntiles);
  else if (dtype == CESM_DT_F32)
    stem_wgrad_kernel<float><<<grid, 256, 0, stream>>>(xt, cond, (const float*)dy, part, B, F, Fx, Fc, H, W, Co, KS,
                                                       ntiles);
  else
    return CESM_EINVAL;
  const int64_t n = (int64_t)Co * 2 * KS * KS;
  sum_partials_kernel<<<(unsigned)cdiv(n, 64), 1024, 0, stream>>>(part, dw, nblk, n, accumulate);
  return cesm_launch_status();
}

int cesm_head_fwd(int dtype, const void* x, const float* w, const float* bias, float* out, int B, int F, int HW, int C,
                  hipStream_t stream) {
  if (C % 8) return CESM_EINVAL;
  const int64_t threads = (int64_t)B * HW * 8;
  const unsigned grid = (unsigned)cdiv(threads, 256);
  if (dtype == CESM_DT_BF16)
    head_fwd_kernel<bf16><<<grid, 256, 0, stream>>>((const bf16*)x, w, bias, out, B, F, HW, C);
  else if (dtype == CESM_DT_F32)
    head_fwd_kernel<float><<<grid, 256, 0, stream>>>((const float*)x, w, bias, out, B, F, HW, C);
  else
    return CESM_EINVAL;
  return cesm_launch_status();
}

// head backward: dx (full [B*F][HW][C]), dw[C], db[1] (via part: nblk*(C+1) floats)
int cesm_head_bwd(int dtype, const float* dout, const void* x, const float* w, void* dx, float* dw, float* db,
                  float* part, int nblk, int B, int F, int HW, int C, int accumulate, hipStream_t stream) {
  if (C % 8 || nblk <= 0) return CESM_EINVAL;
  const int64_t total = (int64_t)B * F * HW * (C / 8);
  const unsigned g1 = (unsigned)std::min<int64_t>(cdiv(total, 256), 8192);
  const int64_t ppb = cdiv((int64_t)B * HW, nblk);
  if (dtype == CESM_DT_BF16) {
    if (dx) head_dgrad_kernel<bf16><<<g1, 256, 0, stream>>>(dout, w, (bf16*)dx, B, F, HW, C);
    if (dw) head_wgrad_kernel<bf16><<<nblk, 256, 0, stream>>>(dout, (const bf16*)x, part, B, F, HW, C, ppb);
  } else if (dtype == CESM_DT_F32) {
    if (dx) head_dgrad_kernel<float><<<g1, 256, 0, stream>>>(dout, w, (float*)dx, B, F, HW, C);
    if (dw) head_wgrad_kernel<float><<<nblk, 256, 0, stream>>>(dout, (const float*)x, part, B, F, HW, C, ppb);
  } else {
    return CESM_EINVAL;
  }
  if (dw) head_reduce_kernel<<<1, 256, 0, stream>>>(part, dw, db, nblk, C, accumulate);
  return cesm_launch_status();
}

}  // extern "C"

#ifdef CESM_H3_STAMPS
// diagnostic build only (tools/h3_stamps.py): point the halo conv's phase stamps at buf (16 u64 per wave, 4 waves per
// block, blocks [0, nblocks)); buf = nullptr turns them off
extern "C" int cesm_diag_h3_stamps_set(void* buf, int nblocks) {
  uint64_t* p = static_cast<uint64_t*>(buf);
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_h3_stamp_buf), &p, sizeof(p)) != hipSuccess) return CESM_EINVAL;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_h3_stamp_blocks), &nblocks, sizeof(nblocks)) != hipSuccess) return CESM_EINVAL;
  return 0;
}
#endif
