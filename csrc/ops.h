// Kernel launch interfaces (device side lives in *.hip, host glue in bindings.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "common.h"

namespace ddlpc {

// ---------------------------------------------------------------- conv 3x3 fwd / dgrad
struct ConvFwdArgs {
  int dims;                       // 2 or 3
  int N, D, H, W;                 // D = 1 for 2-D
  int C1, C2, Cin, CinW;          // X1 / X2 channels, Cin = C1 + C2, packed weight stride
  int Cout, Co1;                  // output channels; [0, Co1) -> Y1, rest -> Y2
  int taps;                       // 9 or 27
  const bf16_t* X1;
  const bf16_t* X2;
  const float* pscale;            // optional BN-apply + ReLU prologue on X1 (per channel)
  const float* pshift;
  const float* pscale2;           // optional prologue on X2 (a deferred skip tensor; C1 + C2 <= 512)
  const float* pshift2;
  const bf16_t* Wt;               // [Cout][taps][CinW]
  const float* bias;              // optional
  bf16_t* Y1;
  bf16_t* Y2;
  float* stats;                   // optional [grid][2][Cout] per-workgroup (sum, sum^2) of the fp32
                                  // outputs (before the bf16 store: the statistics an fp32
                                  // BatchNorm would see); rows of channels outside a
                                  // workgroup's n tile are not written.  (The resident
                                  // 96-channel variant — the concat data gradient: one input,
                                  // no prologue, no bias — writes sum^2 rows of zeros: its
                                  // sums are the up-conv's bias gradient)
  int TD, TH, TW;
  int tilesD, tilesH, tilesW;
  int nTilesM, nTilesN;
  int persist_blocks;             // grid cap (persistent workgroups); 0 = one per item
  int stat_rows;                  // out: rows written to `stats` (one per workgroup)
  int ksplit;                     // >1: split the channel chunks, fp32 partials to `part`
  float* part;                    // [ksplit][npix][Cout] fp32 (ksplit > 1)
  long long npix;                 // N * D * H * W
  // BN-backward epilogue (data gradient dA of a conv whose input went through BN + ReLU):
  // `stats` rows then hold (sum dyh, sum dyh * xhat) with dyh = [y*scale + shift > 0] * dA,
  // xhat = (y - mean) * invstd — the reduction pass of that BN's backward, fused.  2-D,
  // single output, no prologue.
  const bf16_t* bnb_y;            // y [N][H][W][Cout] (pre-BN activations of that layer)
  const float* bnb_s4;            // [4][Cout]: mean, invstd, scale, shift
  // per-micro-batch BatchNorm groups (a batched accumulation window, UNetEngine.bn_groups):
  // groups > 1 splits the batch into `groups` equal runs of images and walks the M tiles
  // GROUP-MAJOR — workgroup b serves group b / (R * nTilesN * ksplit) only (R = workgroups per
  // (group, n tile), launcher-chosen) — so every statistics row (forward (sum, sum^2) or the
  // BN-backward partials) belongs to one group: rows [groups][R * nTilesN][2][Cout], and the
  // prologue constants (pscale / pshift) and the BNB table (bnb_s4) of group g sit at
  // + g * gstride floats.  ksplit must be 1.
  int groups;
  long long gstride;
};
void conv3_splitk_finalize_launch(ConvFwdArgs& a, int grid, hipStream_t st);
void conv3_fwd_launch(ConvFwdArgs& a, int cfg, hipStream_t st);
int conv3_fwd_grid(const ConvFwdArgs& a);       // the streaming kernel's grid (= statistics rows)
int conv3_fwd_cfg_wm(int cfg);
// resident-weight kernel for high-resolution few-channel layers (conv3x3_res.hip)
int conv3_res_plan(ConvFwdArgs& a, int num_cus, int& grid, int& smem);
// 3-D 32-input-channel layers (32-channel output chunks): depth-streaming resident kernel
// (conv3x3x3_ds.hip); -1 = not eligible (grid = one workgroup per CU, statistics rows
// [grid][2][Cout])
int conv3d_ds_plan(const ConvFwdArgs& a, int num_cus, int& grid, int& smem);
void conv3d_ds_launch(ConvFwdArgs& a, int grid, int smem, hipStream_t st);
void conv3_res_launch(ConvFwdArgs& a, int variant, int grid, int smem, hipStream_t st);
int conv3_fwd_cfg_bn(int cfg);
int conv3_fwd_cfg_bm(int cfg);
int conv3_fwd_cfg_halo(int dims, int cfg);

// ---------------------------------------------------------------- fused 32-channel backward
// data + weight gradient of a 32 -> 32-channel 3x3 conv whose input is relu(bn1(Y)), from one
// read of dY and Y (conv3x3_bwd32.hip): dA [N][H][W][32] bf16, BN1-backward partial rows
// bnpart [grid][2][32] (sum dyh, sum dyh * xhat), weight-gradient slabs wpart [grid][32][9][32]
struct Bwd32Args {
  int N, H, W;
  const bf16_t* dY;
  const bf16_t* Y;
  const float* s4;                // [4][32] BN1 (mean, invstd, scale, shift)
  const bf16_t* Wd;               // data-gradient pack [32 ci][9][32 co] (flipped taps)
  bf16_t* dA;
  float* bnpart;
  float* wpart;
  int tilesH, tilesW, nTiles;     // 16 x 16 pixel tiles
  // BN groups (a batched window): `groups` equal runs of images with their own BN1 statistics
  // s4 [groups][4][32]; group-major workgroups, BN-partial rows [groups][R][2][32]
  int groups;
};
int conv3_bwd32_grid(int nTiles, int num_cus, int groups);
void conv3_bwd32_launch(const Bwd32Args& a, int grid, hipStream_t st);

// ---------------------------------------------------------------- conv 3x3 wgrad
struct ConvWgradArgs {
  int dims;
  int N, D, H, W;
  int C1, C2, Cin, Cout, taps;
  const bf16_t* dY;               // [pixels][Cout]
  const bf16_t* X1;
  const bf16_t* X2;
  const float* pscale;
  const float* pshift;
  const float* pscale2;           // prologue on X2 (deferred skip), C1 + C2 <= 512
  const float* pshift2;
  float* partial;                 // [splits][Cout][taps][Cin]
  int TD, TH, TW;
  int tilesD, tilesH, tilesW, nTiles;
  int coTiles, ciChunks, planes, splits;
  // BN-backward prologue on the output-gradient operand (v2 kernel, 2-D): dY holds dA (the
  // gradient w.r.t. the BN + ReLU output) and the kernel forms
  //   dY = k * (dA [y*scale + shift > 0] - m1 - xhat * m2)
  // on load (bn_bwd2_kernel's apply arithmetic): y = dyy, dys4 = [mean|invstd|scale|shift],
  // dycoef = [k|m1|m2] (each Cout floats)
  const bf16_t* dyy;
  const float* dys4;
  const float* dycoef;
  // (c32 kernel with the dY prologue: the formed dY is also stored here — the data gradient of
  // the same conv reads it instead of a separate BN-backward apply pass)
  bf16_t* dyout;
  int ciw;                        // v3: 32-channel input chunks per workgroup (1 or 2)
  // per-micro-batch BatchNorm groups (v3 only): images [g * gimg, (g+1) * gimg) use the
  // prologue constants pscale / pshift + g * gstride (the X1 prologue; no X2 prologue)
  int groups;
  int gimg;
  long long gstride;
};
void conv3_wgrad_launch(ConvWgradArgs& a, int bco, hipStream_t st);
// 3-D weight gradient (32-channel input / output chunks, >= 64x64 planes), depth-streaming
// (conv3x3x3_wgrad_ds.hip): -1 = not eligible, else the grid (sets ciChunks, splits, tiles;
// partial slab [splits][Cout][27][Cin])
int conv3d_wgrad_ds_plan(ConvWgradArgs& a, int num_cus);
void conv3d_wgrad_ds_launch(ConvWgradArgs& a, int grid, hipStream_t st);
// 2-D weight gradient of the 32-output-channel concat convs, every input chunk per workgroup
// (conv3x3_wgrad_c32.hip): -1 = not eligible, else the grid (partial slab [grid][32][9][Cin])
int conv3_wgrad_c32_plan(ConvWgradArgs& a, int num_cus);
void conv3_wgrad_c32_launch(ConvWgradArgs& a, int grid, hipStream_t st);
// LDS-DMA variant (1 x TH x 16 pixel tiles of conv3_wgrad2_pt(bco) pixels; 3-D: planes = 3,
// one depth tap plane per workgroup)
void conv3_wgrad2_launch(ConvWgradArgs& a, int bco, hipStream_t st);
int conv3_wgrad2_pt(int bco, int C2, int H, int W);
// 32x32x16-MFMA variant (conflict-free transposed reads; Cin % 32 == 0, pixel tiles of 128 / 256)
void conv3_wgrad3_launch(ConvWgradArgs& a, int bco, hipStream_t st);
// image layer (2-D, X1 = the 8-channel padded image with <= 4 real channels, no X2 / prologue;
// optional dY prologue): (tap, channel)-packed N, pixel tiles of conv3_wgrad_img_pt(bco);
// grid = coTiles x splits
void conv3_wgrad_img_launch(ConvWgradArgs& a, int bco, hipStream_t st);
int conv3_wgrad_img_pt(int bco);

int conv3_wgrad_halo_cap(int dims);

// ---------------------------------------------------------------- generic bf16 GEMM (convT)
// C[M][N] = sum_k A(m, k) * B(n, k)   with k-contiguous operands ("NT"), used by the
// transposed-conv forward / data-gradient, and a pixel-major ("TN") variant for its
// weight gradient.  Loader / epilogue modes are selected by `mode`.
struct GemmArgs {
  int mode;
  int M, N, K;
  const bf16_t* A;
  const bf16_t* B;
  const float* bias;
  void* C;
  float* partial;
  int splits;
  // geometry for the transposed-conv gathers / scatters
  int dims, Nimg, D, H, W;        // input (low-res) geometry
  int Cin, Cout;
  const float* pscale;            // unused (kept for layout)
  const float* pshift;
  // deferred BatchNorm of the convT INPUT tensor (bn4 = [mean|invstd|scale|shift] x Cin):
  //   FWD / WGRAD: x holds the pre-BN conv output; relu(x*scale+shift) is formed on load
  //   DGRAD: bny = that pre-BN tensor; the epilogue emits BN-backward partial rows
  //          bnpart[block][2][Cin] of the stored dx (zeros outside the block's channel tile)
  const float* bn4;
  const bf16_t* bny;
  float* bnpart;
  int wg2;                        // WGRAD: 1 = gemm_tn_wgrad2_kernel (tile from convt_wgrad2_tiles)
  const bf16_t* Wd2;              // fused backward: packed data-gradient weights [Cin][S*Cout]
};
enum GemmMode {
  GEMM_CONVT_FWD = 0,   // A = x[px][Cin], B = Wt[(sub, co)][Cin] -> scatter to 2x up, + bias
  GEMM_CONVT_DGRAD = 1, // A = dOut gathered [px][(sub, co)], B = Wd[ci][(sub, co)] -> dx[px][ci]
  GEMM_CONVT_WGRAD = 2, // TN: dW[ci][(sub, co)] = sum_px x[px][ci] * dOut[up(px, sub)][co]
};
void gemm_launch(GemmArgs& a, hipStream_t st);
int convt_bwd_fused_splits(long long K, int num_cus);   // workgroups of the fused 64-ch backward
int gemm_nt_bn(const GemmArgs& a);            // N tile of the forward / data-gradient GEMM
long long gemm_nt_grid(const GemmArgs& a);     // its workgroup count (= BN-partial rows)
int convt_wgrad2_tiles(const GemmArgs& a);
// fused data + weight gradient of a 2-D 64 -> 64-channel transposed conv (convt_gemm.hip):
// A = x [px][64], B = dOut, C = dx [px][64] (bf16), Wd2 = packed dgrad weights, partial =
// [splits][64][256] weight-gradient slab, bn4/bnpart = deferred BN of x and its partial rows
void convt_bwd_fused_launch(GemmArgs& a, hipStream_t st);
// resident-weight transposed-conv forward / data gradient (convt_res.hip): rows = BN-backward
// partial rows the DGRAD launch writes (0: shape not covered -> gemm_launch)
int convt_res_rows(const GemmArgs& a, int num_cus);
bool convt_res_launch(GemmArgs& a, int num_cus, hipStream_t st);


// ---------------------------------------------------------------- BatchNorm / ReLU / pool
// out may be null with pool (deferred skip: only the pooled tensor is materialised)
void bn_relu_apply_launch(const bf16_t* y, const float* scale, const float* shift, bf16_t* out,
                          bf16_t* pooled, int dims, int N, int D, int H, int W, int C,
                          hipStream_t st, int groups = 1, long long sstride = 0);
void bn_bwd_reduce_launch(const bf16_t* dA, const bf16_t* dP, const bf16_t* y,
                          const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* gscale, float* partial, int nblocks,
                          int dims, int N, int D, int H, int W, int C, hipStream_t st);
void bn_bwd_apply_launch(const bf16_t* dA, const bf16_t* dP, const bf16_t* y, const float* scale,
                         const float* shift, const float* mean, const float* invstd,
                         const float* coefs, const float* gscale, bf16_t* dY, int dims, int N,
                         int D, int H, int W, int C, hipStream_t st);
int bn_bwd_reduce_blocks(long long pixels_or_quads);
// per-micro-batch BatchNorm groups (bn.hip): `groups` statistics groups of gpix pixels each,
// the batch = the groups' tensors one after another; stats4 [groups][4][C]
bool bn_group_supported(int dims, bool pool, int D, int H, int W, int C);
int bn_group_stats_rows(long long gpix, int C, int groups);
// partial_scratch: [groups][nb][2][C]; arena (optional): row g at g * astride gets the
// group's (mean | unbiased var) for the in-order running-statistics update
void bn_group_stats_finalize_launch(const bf16_t* y, int groups, long long gpix, int C,
                                    const float* gamma, const float* beta, float eps, float* out4,
                                    float* arena, long long astride, float* partial_scratch,
                                    int nb, hipStream_t st);
int bn_group_bwd_rows(long long items_per_group, int groups);
// dY per group (N = images per group), coefs [groups][3][C], dgamma / dbeta summed over groups
void bn_group_backward_launch(const bf16_t* dA, const bf16_t* dP, const bf16_t* y,
                              const float* stats4, const float* gamma, float* dgamma, float* dbeta,
                              bool accumulate, float* coefs, float* partial_scratch, int nb,
                              bf16_t* dY, int dims, int groups, int N, int D, int H, int W, int C,
                              hipStream_t st, bool have_partial, double* gsum_scratch);
// per-group BatchNorm-backward coefficients [groups][3][C] and dgamma / dbeta (summed over the
// groups in order) from group-major partial rows [groups][nb][2][C]; dscale: optional device
// factor on the rows (rows reduced at a unit gradient scale)
void bn_group_grad_rows_launch(const float* partial, int nb, int groups, int C, double count,
                               const float* gamma, const float* stats4, float* dgamma, float* dbeta,
                               bool accumulate, float* coefs, double* gsum_scratch,
                               const float* dscale, hipStream_t st);
void bn_group_finalize_rows_launch(const float* partial, int nb, int groups, long long gpix, int C,
                                   const float* gamma, const float* beta, float eps, float* out4,
                                   float* arena, long long astride, hipStream_t st);

// ---------------------------------------------------------------- head + cross-entropy
bool head_supported(int C, int K);
// bn4 (optional, [mean | invstd | scale | shift] x C): the input holds a PRE-BatchNorm
// conv output whose BN + ReLU is applied on load (deferred activation)
void head_ce_fwd_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                        float* partial, float* out3, const float* bn4, int nblocks, long long P,
                        int C, int K, int ignore_index, hipStream_t st);
// bnpart (with bn4): [nblocks][2][C] BatchNorm-backward partial rows of the stored dA;
// nblocks from head_ce_bwd_blocks (one persistent wave of workgroups)
int head_ce_bwd_blocks(int C, int K, bool defer, long long P, int num_cus);
// groups > 1 (C = 32 head only): a batched window whose deferred BatchNorm has per-group
// statistics — group-major workgroups (grid = groups x Rb, BN partial rows [groups][Rb][2][C]),
// bn4 [groups][4][C], coefs [groups][3][C]; pixels per group a multiple of 16
int head_fwd_stats_blocks(int C, int K, long long P, int num_cus, int groups = 1);
void head_ce_bwd_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                        const float* gscale, const float* stats3, int unused, bf16_t* dA,
                        float* dW_partial, int nblocks, long long P, int C, int K,
                        int ignore_index, const float* bn4, float* bnpart, hipStream_t st);
// two-pass backward with the deferred BatchNorm of the last decoder block: dA == nullptr in
// head_ce_bwd_launch runs the stats pass (dWh, dbh, BN partials); this second pass
// recomputes dA and writes that BatchNorm's dY (coefs = [k | m1 | m2] x C)
// training forward with the deferred BN: loss rows -> out3 (ce_finalize) plus the backward
// statistics at a unit gradient scale (head_ce_bwd_kernel LOSS variant)
void head_ce_fwd_stats_launch(const bf16_t* a, const float* Wh, const float* bh,
                              const int64_t* labels, const float* bn4, float* dW_partial,
                              float* bnpart, float* loss_partial, float* out3, int nblocks,
                              long long P, int C, int K, int ignore_index, hipStream_t st,
                              int groups = 1);
void head_bn_apply_launch(const bf16_t* a, const float* Wh, const float* bh, const int64_t* labels,
                          const float* gscale, const float* stats3, const float* bn4,
                          const float* coefs, bf16_t* dY, long long P, int C, int K,
                          int ignore_index, hipStream_t st, int groups = 1);
void head_logits_launch(const bf16_t* a, const float* Wh, const float* bh, float* logits_nchw,
                        long long P, long long HW, int C, int K, const float* bn4, hipStream_t st);


// ---------------------------------------------------------------- optimizer / packing
void adam_launch(float* p, const float* g, float* m, float* v, long long n, float b1, float b2,
                 float eps, float wd, float step_size, float inv_sqrt_bc2, hipStream_t st,
                 const float* dscal = nullptr);
void adam_scalars_launch(float* s, double lr, double b1, double b2, hipStream_t st);
struct PackEntry {                 // one conv weight to pack into bf16 kernel layouts
  const float* src;                // OIHW fp32  (or IOHW for transposed conv)
  bf16_t* fwd;                     // conv: [co][tap][CinW]; convT: [(sub, co)][Cin]
  bf16_t* dgrad;                   // conv: [ci][8-tap][CoutW]; convT: [ci][(sub, co)]
  int kind;                        // 0 = conv3, 1 = convT2
  int Cout, Cin, taps, CinW, CoutW;
};
void weight_pack_launch(const PackEntry* entries_dev, int n_entries, long long max_elems,
                        hipStream_t st);

// ---------------------------------------------------------------- gradient codec
void codec_absmax_launch(const float* x, const int64_t* seg, int nseg, float* scales,
                         hipStream_t st);
void codec_encode_launch(const float* x, const int64_t* seg, int nseg, const float* scales,
                         void* out, int codec, long long n, hipStream_t st);
void codec_decode_sum_launch(float* out, const void* q, const float* scales, const float* w,
                             const int64_t* seg, int nseg, int world, int codec, long long n,
                             hipStream_t st);

// ---------------------------------------------------------------- deterministic reductions
int reduce_rows_chunks(int R);
void reduce_rows_launch(const float* in, int R, long long N, double* tmp, double* sums,
                        hipStream_t st);
void bn_stats_finalize_launch(const double* sums, int C, double count, const float* gamma,
                              const float* beta, float* running_mean, float* running_var,
                              float momentum, float eps, float* out4, bool update_running,
                              int64_t* nbt, hipStream_t st);
void bn_grad_finalize_launch(const double* sums, int C, double count, const float* gamma,
                             const float* invstd, float* dgamma, float* dbeta, float* coefs,
                             bool accumulate, hipStream_t st, const float* dscale = nullptr);
void meter_add_launch(double* buf, const float* loss, const float* correct, double pixels,
                      double n, hipStream_t st);
void head_grad_scale_launch(const float* out3, const float* gs, float* scale, hipStream_t st);
void scatter_sums_dscale_launch(const double* sums, long long N, float* dst, const float* dscale,
                                bool accumulate, hipStream_t st);
// single-kernel variants reading the partial rows directly (P small): one block per channel
void bn_stats_finalize_rows_launch(const float* partial, int P, int C, double count,
                                   const float* gamma, const float* beta, float* running_mean,
                                   float* running_var, float momentum, float eps, float* out4,
                                   bool update_running, int64_t* nbt, hipStream_t st);
void bn_grad_finalize_rows_launch(const float* partial, int P, int C, double count,
                                  const float* gamma, const float* invstd, float* dgamma,
                                  float* dbeta, float* coefs, bool accumulate, hipStream_t st,
                                  const float* dscale = nullptr);
void reduce_rows_scatter_launch(const float* in, int R, long long N, double* tmp, float* dst,
                                int mode, int A, int T, int B, bool accumulate, hipStream_t st,
                                long long ld = -1);
void scatter_sums_launch(const double* sums, long long N, float* dst, int mode, int A, int T,
                         int B, float scale, bool accumulate, hipStream_t st);

// ---------------------------------------------------------------- misc
void bilinear_up2_launch(const bf16_t* x, bf16_t* y, int dims, int N, int D, int H, int W, int C,
                         bool backward, hipStream_t st);
void bilinear_up2_bwd_launch(const bf16_t* dy, float* dx_f32, bf16_t* dx, int dims, int N, int D,
                             int H, int W, int C, hipStream_t st);
void channel_sum_launch(const bf16_t* x, long long P, int C, float* partial, int nblocks,
                        hipStream_t st);
void to_nhwc_pad_launch(const void* x, int in_dtype, bf16_t* y, int N, int C, int Cp, long long S,
                        long long sN, long long sC, long long sS, hipStream_t st);

// ---------------------------------------------------------------- input pipeline (data.hip)
void synth_tiles_launch(const int64_t* idx, int B, uint32_t seed, int classes, int in_ch, int tile,
                        int dims, int grid, float k, const float* palette, int cpad, bf16_t* x,
                        int64_t* y, hipStream_t st);
void tile_gather_launch(const uint8_t* src, const uint8_t* lab, const int64_t* idx, int B,
                        long long S, int in_ch, int cpad, long long N, bf16_t* x, int64_t* y,
                        hipStream_t st);

void bn_running_apply_launch(float* rm, float* rv, const float* slots, int K, int C, long long stride,
                             float momentum, int64_t* nbt, hipStream_t st);
void bn_running_apply_all_launch(const int64_t* entries, int L, int maxC, const float* arena, int K,
                                 long long stride, float momentum, hipStream_t st);

// ---------------------------------------------------------------- A/B switches (bindings.cpp)
// knob("NAME", def): an in-process override (torch.ops.ddlpc.set_knob, for interleaved
// same-process A/B runs) or else the environment variable DDLPC_NAME, or else def — for
// experiments in progress only: no shipped kernel reads one
int knob(const char* name, int def);

// ---------------------------------------------------------------- comm proxy (reduce.hip)
void comm_proxy_launch(float* g, long long n, int blocks, int passes, hipStream_t st);

}  // namespace ddlpc
