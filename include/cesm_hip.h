/*
 * cesm_hip.h — C ABI of libcesm_hip.so, the gfx950 (MI355X) kernels behind the
 * cesm_emulator_amd drop-in for the reference's video_net training/inference hot path.
 *
 * The reference (kallenordling/cesm_emulator @ 2025-09-05) is pure Python: every entry point
 * below replaces one or more PyTorch-dispatched ATen/NCCL ops at the cited reference lines
 * (SURVEY.md §2.2).  Conventions:
 *   - all pointers are device pointers (hipMalloc / PyTorch caching allocator); kernels never
 *     allocate or free — workspaces are passed in by the caller;
 *   - activations are channels-last [N][H][W][C] with N = batch*frames, dtype = CESM_DT_F32
 *     (parity mode) or CESM_DT_BF16 (perf mode); parameters, statistics and grads are fp32;
 *   - every call is stream-ordered on `stream` and enqueue-only (no host sync, graph-capturable);
 *   - return 0 on success, negative CESM_E* on bad arguments or launch failure; the Python
 *     layer raises RuntimeError (mirroring model.py:99-132 / train.py:842-843 errors);
 *   - `accumulate` = 1 adds into the destination gradient (grad accumulation), 0 overwrites.
 */
#ifndef CESM_HIP_H
#define CESM_HIP_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CESM_DT_F32 0
#define CESM_DT_BF16 1

/* ABI version of this header.  Bumped whenever an entry point's argument list changes; a host binding compares it
 * with cesm_abi_version() before the first call (cesm_emulator_amd/_lib.py does), so an old header cannot silently
 * mis-call a newer library.  History:
 *   4 (round 4): cesm_ln_fwd / cesm_ln_bwd gained (perm_f, perm_hw), cesm_tflash_fwd / cesm_tflash_bwd gained
 *     qkv_pixel_major — each before the hipStream_t;
 *   5 (round 5): cesm_abi_version() itself; cesm_conv_fwd / cesm_conv_fwd_gn gained `queue` and cesm_tblock_bwd_dw
 *     gained `dwout`, each before the hipStream_t / after dgamma;
 *   6 (round 6): cesm_tblock_bwd_dw lost `dwout` again (the in-kernel to_out weight gradient measured slower than the
 *     forward's O write and was removed) and gained `o` after dx (O emitted by the backward); cesm_conv_pack_batch's
 *     job table gained per-job block starts and its fourth argument is the grid size;
 *     cesm_qkv_bwd / cesm_qkv_bwd_streams added. */
#define CESM_ABI_VERSION 6
int cesm_abi_version(void);
/* Measurement aid, not a training op: nblk blocks that each occupy one whole CU (full LDS) for `usec` microseconds on
 * `stream` -- the one-GPU stand-in for the RCCL kernels of an overlapped gradient all-reduce (tools/overlap_sim.py,
 * distributed.XgmiModelReducer). */
int cesm_hold_cus(int nblk, float usec, hipStream_t stream);

/* ---- convolutions (csrc/conv.hip) -------------------------------------------------------
 * Generic implicit-GEMM conv on MFMA. Replaces nn.Conv3d (1,k,k) at video_net.py:215 (Block.proj),
 * :246 (res_conv), :61-62 (Downsample), nn.ConvTranspose3d at :65-66 (Upsample), the attention
 * projections nn.Linear :380-381 and 1x1 nn.Conv2d :322-323, and all their data gradients.
 *   out[n,oy,ox,co] = bias[co] + res[..] + sum W[co][ky*KW+kx][ci] * X[n,(oy*S-P+ky)/U,(ox*S-P+kx)/U,ci]
 * Input may be the channel-concat of x1 (C1 ch) and x2 (C2 ch) (video_net.py:857, :868 torch.cat);
 * output channels [0,Co1) go to y1 and [Co1,Cout) to y2. */
int cesm_conv_fwd(int dtype, const void* x1, const void* x2, const void* wp, const float* bias, const void* res,
                  const void* res2, void* y1, void* y2, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int Co1,
                  int KH, int KW, int S, int P, int U, int* queue, hipStream_t stream);
/* cesm_conv_fwd (Co1 = Cout, no residual) that also writes the GroupNorm statistics partials of its output
 * y (the Block conv feeding GroupNorm, video_net.py:215-217): gnpart [B][nslot][Cout/4] float2 (sum, sum of
 * squares per channel quad over the pixels of one partial slot), every entry written once, no atomics;
 * nslot from cesm_conv_gn_nslot (0: the kernel for this shape has no partials -> CESM_EUNSUPPORTED here,
 * use cesm_gn_stats).  Nb = B * frames. */
int64_t cesm_conv_gn_nslot(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int KH, int KW,
                           int S, int P, int U, int B);
int cesm_conv_fwd_gn(int dtype, const void* x1, const void* x2, const void* wp, const float* bias, void* y, float* gnpart,
                     int B, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int KH, int KW, int S,
                     int P, int U, int* queue, hipStream_t stream);
/* name of the kernel cesm_conv_fwd launches for these arguments (host-only query, no GPU work; the
 * launcher itself selects through the same function).  "invalid" if cesm_conv_fwd would return EINVAL. */
const char* cesm_conv_fwd_variant(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout,
                                  int Co1, int KH, int KW, int S, int P, int U);
/* Input-channel tile (256 / 128) of the square-tile 1x1 weight-gradient kernel cesm_conv_wgrad runs for this shape, 0 if
 * it runs another kernel (host-only query).  When non-zero the caller sizes nsplit for Cout/256 x Cin/BN tiles. */
int cesm_conv_wgrad_sq_bn(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout, int Co1, int KH,
                          int KW, int S, int P, int U, int with_bias);
/* name of the kernel cesm_conv_wgrad launches (host-only query; with_bias: db != NULL) */
const char* cesm_conv_wgrad_variant(int dtype, int Nb, int Hi, int Wi, int C1, int C2, int Ho, int Wo, int Cout,
                                    int Co1, int KH, int KW, int S, int P, int U, int with_bias);
/* weight gradient of a cesm_conv_fwd launch; written in PyTorch layout [D0][D1][1][KH][KW] with the
 * (swap, flip) mapping of cesm_conv_pack.  slab: nsplit*Cout*KH*KW*(C1+C2) floats.
 * db (nullable): the conv bias gradient sum_px dY (+=), computed in the same pass (bslab: nsplit*Cout
 * floats); only on the bf16 wide-tile path (non-3x3, no dy2) — CESM_EUNSUPPORTED otherwise. */
int cesm_conv_wgrad(int dtype, const void* x1, const void* x2, const void* dy1, const void* dy2, float* dw,
                    float* slab, float* db, float* bslab, int nsplit, int Nb, int Hi, int Wi, int C1, int C2, int Ho,
                    int Wo, int Cout, int Co1, int KH, int KW, int S, int P, int U, int swap, int flip, int accumulate,
                    hipStream_t stream);
/* PyTorch conv weight (fp32) -> GEMM layout Wp[co][tap][ci] in dtype.  swap: GEMM co is dim 1 of
 * the torch tensor (transposed conv forward / conv dgrad); flip: taps reversed.  bf16 3x3 and 4x4 weights with
 * Cout % 64 == 0 and Cin % 32 == 0 are written "chunked" instead: element (co, tap, ci) at
 * (((co/64 * Cin/32 + ci/32) * KH*KW + tap) * 64 + co%64) * 32 + ci%32 -- one contiguous block per (64-co block,
 * 32-channel chunk), the tile the halo convs stage.  The pack is opaque to callers: cesm_conv_fwd reads either
 * layout by the same rule (same argument lists; round 6). */
int cesm_conv_pack(int dtype, const float* w, void* wp, int Cout, int Cin, int KH, int KW, int swap, int flip,
                   hipStream_t stream);
/* every cached pack of one dtype redone in ONE launch after an optimizer step: jobs = device
 * int64[njobs][8] {src fp32 ptr, dst ptr, Cout, Cin, KH, KW, swap, flip} (cesm_conv_pack semantics) followed by
 * int64[njobs + 1] block starts, the exclusive prefix sum of the per-job tile counts cdiv(Cout, cot) * cdiv(Cin, 64)
 * with cot = clamp(4096 / (KH * KW * 64), 1, 64), then int64[starts[njobs]] the job index of every block; nblocks = the grid
 * (the last start is the work; any nblocks >= 1 is correct).  ABI 6: the table gained the starts, the fourth
 * argument was blocks_per_job. */
int cesm_conv_pack_batch(int dtype, const int64_t* jobs, int njobs, int nblocks, hipStream_t stream);
/* dst[c] (+)= sum over rows of x[r][c]  (conv bias gradients) ; part: nsplit*C floats */
int cesm_colsum(int dtype, const void* x, float* dst, float* part, int nsplit, int64_t rows, int C, int accumulate,
                hipStream_t stream);
/* stem Conv3d(2->Co,(1,KS,KS),pad KS/2) on cat([x_t, cond]) read straight from the NCDHW fp32 boundary
 * tensors (video_net.py:595-600, :808-815; model.py:111-121 frame broadcast). */
int cesm_stem_fwd(int dtype, const float* xt, const float* cond, const float* w, const float* bias, void* y, int B,
                  int F, int Fx, int Fc, int H, int W, int Co, int KS, hipStream_t stream);
int cesm_stem_wgrad(int dtype, const float* xt, const float* cond, const void* dy, float* dw, float* part, int nblk,
                    int B, int F, int Fx, int Fc, int H, int W, int Co, int KS, int accumulate, hipStream_t stream);
/* head Conv3d(C->1,1) (video_net.py:763) evaluated on frame F//2 only (model.py:124-130). */
int cesm_head_fwd(int dtype, const void* x, const float* w, const float* bias, float* out, int B, int F, int HW, int C,
                  hipStream_t stream);
int cesm_head_bwd(int dtype, const float* dout, const void* x, const float* w, void* dx, float* dw, float* db,
                  float* part, int nblk, int B, int F, int HW, int C, int accumulate, hipStream_t stream);

/* ---- normalisation (csrc/norm.hip) -------------------------------------------------------
 * GroupNorm(G,C) eps, affine, then x*(scale+1)+shift, SiLU, + residual: video_net.py:216-227, :265. */
/* ws >= max(B*256, 1024)*G*2 doubles */
int cesm_gn_stats(int dtype, const void* y, float* stats, double* ws, int B, int64_t rows_b, int C, int G, float eps,
                  hipStream_t stream);
/* stats [B][G] (mean, rstd) from cesm_conv_fwd_gn's partials (replaces cesm_gn_stats' pass over y):
 * fixed-order double reduction, rows_b = voxels per sample.  part is scratch: for large nslot (>= 8192) the
 * two-stage reduction overwrites it with its block sums */
int cesm_gn_stats_part(float* part, float* stats, int B, int64_t nslot, int C, int G, int64_t rows_b, float eps,
                       hipStream_t stream);
int cesm_gn_apply(int dtype, const void* y, const float* stats, const float* gamma, const float* beta,
                  const float* ss, const void* res, void* out, float* ws, int B, int64_t rows_b, int C, int G,
                  hipStream_t stream);
/* backward; also writes the producing conv's bias gradient dbias (+)= sum dy (nullable) without another
 * pass over dy.  ws >= max(B*1024, 1024)*C*3 + B*C*3 + B*C*5 floats (max(B*256, 1024) suffices in the default
 * build; builds with -DGN_BIGB_CAP=512/1024 or -DGN_PER_SAMPLE=1 use up to 1024 chunk partials per sample). */
int cesm_gn_bwd(int dtype, const void* dout, const void* y, const float* stats, const float* gamma,
                const float* beta, const float* ss, void* dy, float* dss, float* dgamma, float* dbeta, float* dbias,
                float* ws, int B, int64_t rows_b, int C, int G, int accumulate, hipStream_t stream);
/* channel LayerNorm (biased var, gamma only): video_net.py:78-87.  perm_f > 0: x is [B][perm_f][perm_hw] voxels and
 * out is written pixel-major ([B][perm_hw][perm_f], the long-window qkv order); 0: same order as x */
int cesm_ln_fwd(int dtype, const void* x, const float* gamma, void* out, float* mr, int64_t V, int C, float eps,
                int perm_f, int perm_hw, hipStream_t stream);
/* dx = LN backward + dres (the Residual wrapper's pass-through gradient, video_net.py:75); perm_f > 0: dy is
 * pixel-major (as cesm_ln_fwd's permuted out) */
int cesm_ln_bwd(int dtype, const void* dy, const void* x, const float* mr, const float* gamma, const void* dres,
                void* dx, float* dgamma, float* part, int nblk, int64_t V, int C, int accumulate, int perm_f, int perm_hw,
                hipStream_t stream);

/* ---- attention (csrc/attn.hip) -----------------------------------------------------------
 * RoPE angle table (rotary_embedding.py:143-144, :275-278): rot[f][i] = (cos, sin)(f*freqs[i]). */
int cesm_rope_table(const float* freqs, float* rot, int F, hipStream_t stream);
/* RelativePositionBias (video_net.py:268-310): bias[h][i][j] = table[bucket(j-i)][h] and backward. */
int cesm_relpos_fwd(const float* table, float* bias, int F, int heads, int num_buckets, int max_distance,
                    hipStream_t stream);
int cesm_relpos_bwd(const float* part, int nparts_per_h, int B, float* dtable, float* ws, int F, int heads,
                    int num_buckets, int max_distance, int accumulate, hipStream_t stream);
/* temporal attention core (video_net.py:401-453 between to_qkv and to_out), qkv [V][768] -> out [V][256] */
int cesm_tattn_nblk(int F, int HW);
int cesm_tattn_fwd(int dtype, const void* qkv, const float* bias, const float* rot, void* out, float* lse, int B,
                   int F, int HW, float scale, hipStream_t stream);
int cesm_tattn_bwd(int dtype, const void* qkv, const void* o, const void* dout, const float* lse, const float* bias,
                   const float* rot, void* dqkv, float* dbias_part, int B, int F, int HW, float scale,
                   hipStream_t stream);
/* Temporal-attention core on MFMA (bf16, csrc/tflash.hip; F <= 128): same contract as cesm_tattn_fwd /
 * cesm_tattn_bwd (video_net.py:403-454) for the unfused path (long windows, C >= 256 levels).  fwd: qkv
 * [B*F*HW][768] -> out [..][256], lse [B][8][HW][F] (log2 units, nullable); bias [8][F][F], rot [F][16][2].
 * bwd: dqkv [..][768] from qkv, o (the forward's out), lse, dout [..][256]; dtable (+)= the rel-pos table
 * gradient (nullable).  Workspaces: dbuf B*8*HW*F, part B*8*cesm_tflash_nblk(HW)*(2F-1), off 8*(2F-1) floats.
 * Round 5 (same argument lists, CESM_ABI_VERSION unchanged): F >= 8 runs the one-pass fused backward (dbuf then
 * unused; CESM_TF_FUSED=0 in the environment restores the dq + dk / dv kernels), and cesm_tflash_nblk returns 128
 * for every HW (the fused kernel's pixel streams per (sample, head)) -- size part from it, not from a formula. */
int cesm_tflash_supported(int F);
int cesm_tflash_nblk(int HW);
/* name of the backward kernel (the fused one, or the dq kernel of the two-kernel form) cesm_tflash_bwd runs for
 * (F, HW) (host-only query) */
const char* cesm_tflash_bwd_variant(int F, int HW);
/* qkv_pixel_major (F > 16): qkv / dqkv rows ordered [B][HW][F] (a pixel's frames adjacent: the long-window path's
 * LN writes its output in that order, so the to_qkv GEMM produces it); out / dout / lse keep their layouts */
int cesm_tflash_fwd(const void* qkv, const float* bias, const float* rot, void* out, float* lse, int B, int F, int HW,
                    float scale, int qkv_pixel_major, hipStream_t stream);
int cesm_tflash_bwd(const void* qkv, const void* o, const void* dout, const float* lse, const float* bias,
                    const float* rot, void* dqkv, float* dtable, float* dbuf, float* part, float* off, int B, int F,
                    int HW, float scale, int num_buckets, int max_distance, int accumulate, int qkv_pixel_major,
                    hipStream_t stream);
/* Fused temporal-attention block forward, bf16 (csrc/tblock.hip): y = x + Residual(PreNorm(Attention))
 * (video_net.py:69-98, :350-454) with LN, QKV GEMM, RoPE, MFMA core, out-proj in one kernel; x,y
 * [B*F*HW][C], wqkv [768][C], wout [C][256] packed bf16; saves mr [B*F*HW][2] and lse [B][8][HW][F].
 * F <= 16, C in {64,128,256,512}. */
int cesm_tblock_fwd(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bias,
                    const float* rot, void* y, float* mr, float* lse, void* o, void* wimg, int B, int F, int HW, int C,
                    float scale, float eps, hipStream_t stream);
/* Fused temporal-attention block backward, dx path (bf16): recomputes LN/QKV/RoPE/softmax from mr and
 * lse, dO = dy.W_out, MFMA core backward, dxn = dqkv.W_qkv, LN backward + residual -> dx.  Emits
 * (nullable) dqkv [..][768], o [..][256], xn [..][C] bf16 for the to_qkv/to_out weight gradients,
 * dbias_part [B][8][nblk][F][F] (cesm_relpos_bwd layout) and dgamma (+)= sum dxn*xhat.
 * wqkv_t [C][768] and wout_t [256][C] are the swap-packed weights; nblk from cesm_tblock_bwd_nblk. */
int cesm_tblock_bwd_nblk(int B, int F, int HW, int C);
/* (cesm_tblock_fwd's o, nullable, C <= 256: the attention output O [..][256] bf16 before to_out, written
 * by the forward for the to_out weight gradient; the backward's o is then passed null.) */
int cesm_tblock_bwd(const void* x, const void* dy, const float* gamma, const float* mr, const float* lse,
                    const void* wqkv, const void* wqkv_t, const void* wout_t, const float* bias, const float* rot,
                    void* dx, void* dqkv, void* o, void* xn, float* dbias_part, float* dgamma, float* dgamma_part, void* wimg,
                    int nblk, int B, int F, int HW, int C, float scale, int accumulate, hipStream_t stream);
/* Fused temporal-attention block with in-kernel weight gradients (C = 64, 4F <= 48; csrc/tblock.hip):
 * cesm_tblock_fwd_fold is cesm_tblock_fwd with LN gamma folded into the QKV weights (wqkv_f32: the fp32
 * master weight [768][C]; wimg (768 + 256) * C bf16); cesm_tblock_bwd_dw is its backward: dx, and
 * dwqkv (+)= dW_qkv, dgamma (+)= the LN gamma gradient (nullable) without the 768-channel dqkv / xn
 * intermediates; dbias_part [8][nblk][F][F] (cesm_relpos_bwd, B = 1); slab nblk*768*C and tmp 768*C floats,
 * wimg (2*768 + 256) * C bf16; nblk from cesm_tblock_bwd_dw_nblk (0 = unsupported shape).  o (nullable) receives the
 * attention output O [..][256] bf16 recomputed from the backward's P (round 6: the forward then writes no O), the input
 * of the to_out weight gradient's wide GEMM.
 * Replaces video_net.py:368-454 (Attention) + :90-98 (PreNorm LN) + :69-75 (Residual) and the
 * to_qkv / to_out weight gradients of its backward. */
int cesm_tblock_bwd_dw_nblk(int B, int F, int HW, int C);
int cesm_tblock_fwd_fold(const void* x, const float* gamma, const float* wqkv_f32, const void* wout,
                         const float* bias, const float* rot, void* y, float* mr, float* lse, void* o, void* wimg,
                         int B, int F, int HW, int C, float scale, float eps, hipStream_t stream);
int cesm_tblock_bwd_dw(const void* x, const void* dy, const float* mr, const float* lse, const float* wqkv_f32,
                       const float* gamma, const void* wout_t, const float* bias, const float* rot, void* dx, void* o,
                       float* dwqkv, float* dgamma, float* dbias_part, float* slab, float* tmp, void* wimg,
                       int nblk, int B, int F, int HW, int C, float scale, int accumulate, hipStream_t stream);
/* Backward of the 768-channel qkv projection with dqkv read once (csrc/qkvbwd.hip, round 6): dx = dy . W (the LN
 * output's gradient, written) and dw (+)= dy^T . x in one pass -- replaces the dgrad GEMM + wide weight-gradient GEMM
 * pair of video_net.py:380-381 / :322-323 (to_qkv) on the unfused attention paths (long windows F > 16, C >= 256).
 * dy [M][768] bf16, x [M][C] bf16 (C = 64 .. 512, C % 64 == 0), wt [C][768] bf16 (wt[c][n] = W[n][c]), dx [M][C] bf16,
 * dw [768][C] fp32 (nullable), slab (C / 64) * streams * 768 * 64 floats with streams = cesm_qkv_bwd_streams (0 =
 * unsupported shape).  Rows may be in any order (pixel- or frame-major) as long as dy, x and dx agree. */
int cesm_qkv_bwd_streams(int64_t M, int N, int C);
int cesm_qkv_bwd(const void* dy, const void* x, const void* wt, void* dx, float* dw, float* slab, int64_t M, int N,
                 int C, int accumulate, hipStream_t stream);
/* spatial linear attention core (video_net.py:335-345 between to_qkv and to_out) */
int cesm_sla_nchunk(int HW);
int cesm_sla_fwd(int dtype, const void* qkv, void* out, float* ctx, float* ml, float* ws, int Nf, int HW, float scale,
                 hipStream_t stream);
int cesm_sla_bwd(int dtype, const void* qkv, const void* dout, const float* ctx, const float* ml, void* dqkv,
                 float* ws, int Nf, int HW, float scale, hipStream_t stream);

/* Fused spatial-linear-attention block (bf16, C = 64; csrc/sla_fused.hip): y = x + Residual(PreNorm(
 * SpatialLinearAttention)) (video_net.py:313-347) without per-pixel intermediates in HBM: online-softmax
 * context partials -> combine -> output.  Saves mz [Nf][8][32][2] (max, normaliser of k over pixels),
 * ctx32 [Nf][8][32][32] and the context as MFMA A fragments actT/actx [Nf][8][2][64][8] bf16.
 * o (nullable): the attention output before to_out [Nf][HW][256] bf16, for the to_out weight gradient
 * (training; the backward then need not emit it).
 * ws: cesm_slaf_nblk(Nf, HW) * Nf * 8 * 1088 floats. */
int cesm_slaf_nblk(int Nf, int HW);
int cesm_slaf_fwd(const void* x, const float* gamma, const void* wqkv, const void* wout, const float* bout, void* y,
                  void* o, float* mz, float* ctx32, void* actT, void* actx, float* ws, int Nf, int HW, int C,
                  float scale, float eps, hipStream_t stream);

/* Fused SLA block backward, dx path (bf16, C = 64): dctx partials -> combine (G_d = sum_e dctx ctx, dctx as
 * A fragments adc/adcT) -> dx (+ dy residual), dgamma (+)=; emits (nullable) dqkv [..][768], o [..][256],
 * xn [..][C] for the to_qkv / to_out weight gradients.  part: nblk*Nf*8*1024 floats, G: Nf*8*64*16 floats,
 * adc/adcT: Nf*8*2*64*8 bf16, dgp: cesm_slaf_bwd_nblk(Nf, HW, C)*C floats;
 * wimg: (2*768 + 256)*C bf16 (fragment images of the three weights, rebuilt per call). */
int cesm_slaf_bwd(const void* x, const void* dy, const float* gamma, const void* wqkv, const void* wqkv_t,
                  const void* wout_t, const float* mz, const float* ctx32, const void* actT, const void* actx,
                  void* dx, void* dqkv, void* o, void* xn, float* dgamma, float* part, float* G, void* adc, void* adcT,
                  float* dgp, void* wimg, int Nf, int HW, int C, float scale, float eps, int accumulate,
                  hipStream_t stream);
/* Fused SLA block backward with in-kernel weight gradients (C = 64): the forward runs cesm_slaf_fwd with
 * gamma_one (unit LN gamma) and wq_fold = bf16 W_qkv diag(gamma) (cesm_pack_scaled); this backward returns
 * dx and accumulates dwqkv (+)= dW_qkv [768][C], dgamma (+)= the LN gamma gradient (nullable) without the
 * 768-channel dqkv / xn intermediates of cesm_slaf_bwd.  nblk_dx from cesm_slaf_bwd_dw_nblk (0 = unsupported);
 * slab nblk_dx*768*C, tmp 768*C floats; wimg (2*768 + 256)*C bf16.  dwout [C][256] / dbout [C] (+)= the to_out
 * weight / bias gradients (both or neither; nullable) from the recomputed q~ and the forward's context, so the
 * forward need not write O: partm (cesm_slaf_nblk + 1) * Nf * 8 * 2048 floats, partb cesm_slaf_nblk * Nf * C.
 * Replaces video_net.py:313-347 (SLA) + :90-98 + :69-75 and the to_qkv / to_out weight gradients of its
 * backward. */
int cesm_slaf_bwd_dw_nblk(int Nf, int HW, int C);
int cesm_slaf_bwd_dw(const void* x, const void* dy, const float* gamma_one, const void* wq_fold, const float* wqkv_f32,
                     const float* gamma, const void* wout_t, const float* mz, const float* ctx32, const void* actT,
                     const void* actx, void* dx, float* dwqkv, float* dgamma, float* dwout, float* dbout, float* part,
                     float* G, void* adc, void* adcT, float* slab, float* tmp, float* partm, float* partb, void* wimg,
                     int nblk_dx, int Nf, int HW, int C, float scale, float eps, int accumulate, hipStream_t stream);
/* out = bf16(w diag(colscale)) for an fp32 row-major w [M][K] (trans = 1: written transposed, [K][M]) */
int cesm_pack_scaled(const float* w, const float* colscale, void* out, int M, int K, int trans, hipStream_t stream);
int cesm_slaf_bwd_nblk(int Nf, int HW, int C);

/* ---- small ops, loss, optimizer, data (csrc/misc.hip) ------------------------------------- */
/* SinusoidalPosEmb (video_net.py:101-113) */
int cesm_sinusoidal(const int64_t* t, float* emb, int B, int dim, hipStream_t stream);
/* y = bias + act(x) W^T, act = SiLU when silu_in (time_mlp video_net.py:651-656, ResnetBlock.mlp :238-242) */
int cesm_linear_small_fwd(const float* x, const float* w, const float* bias, float* y, int R, int I, int O,
                          int silu_in, hipStream_t stream);
int cesm_linear_small_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, float* db, int R,
                          int I, int O, int silu_in, int accumulate_dx, int accumulate_w, hipStream_t stream);
/* Diffusion.q_sample (model.py:196-201) and F.mse_loss (model.py:208) */
int cesm_q_sample(const float* x0, const float* noise, const int64_t* t, const float* sa, const float* s1a,
                  float* xt, int B, int64_t HW, hipStream_t stream);
/* Diffusion.p_sample DDPM update (model.py:168-183), fused: out = r_t (x - b_t/s1_t eps) + sqrt(pv_t) z,
 * coefficients gathered on device from the schedule buffers by t[B]; z may be null (no noise term);
 * out may alias x.  x, eps, z, out: [B][HW] fp32. */
int cesm_ddpm_step(const float* x, const float* eps, const float* z, const int64_t* t, const float* sqrt_recip_alphas,
                   const float* betas, const float* sqrt_one_minus_ac, const float* posterior_variance, float* out,
                   int B, int64_t HW, hipStream_t stream);
int cesm_mse(const float* pred, const float* tgt, float* loss, float* part, int64_t n, hipStream_t stream);
int cesm_mse_bwd(const float* pred, const float* tgt, const float* gscale, float* dpred, int64_t n,
                 hipStream_t stream);
/* clip_grad_norm_ (train.py:865; torch/nn/utils/clip_grad.py:165-180) over a flat grad buffer;
 * info = {norm, clamped clip coef, finite(loss & norm)} stays on device (no host sync). */
int cesm_grad_norm(const float* g, int64_t n, float max_norm, const float* loss, double* part, float* info,
                   hipStream_t stream);
/* AdamW step (train.py:1077-1083, torch/optim/adam.py:417-547) over flat buffers; skipped on device
 * when info[2] == 0 (non-finite), applies the clip coefficient info[1] when use_clip.  step: device int
 * step counter, advanced on device only for a finite step (info[3] <- the step number used for the bias
 * corrections), so a skipped step leaves the count consistent with exp_avg / exp_avg_sq. */
int cesm_adamw(float* p, float* g, float* m, float* v, float* info, int* step, int64_t n, float lr, float b1,
               float b2, float eps, float wd, int use_clip, hipStream_t stream);
/* out = a + b (gradient sums at residual / skip fan-outs) */
int cesm_add(int dtype, const void* a, const void* b, void* out, int64_t n, hipStream_t stream);
int cesm_cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, hipStream_t stream);
/* WindowedAllMembersDataset_random.__getitem__ gather (dataset_single_member.py:168-196);
 * items: nitems x {t0, m, anchor, reverse, crop_i, crop_j} int64 */
int cesm_window_gather(const float* cond, const float* tgt, const int64_t* items, float* cwin, float* x0,
                       int nitems, int K, int M, int H, int W, int h, int w, int center, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CESM_HIP_H */
