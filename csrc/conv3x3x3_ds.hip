// 3x3x3 convolution (stride 1, zero padding 1) of the 3-D U-Net's 32-channel level —
// 32 -> 32 channels at full resolution (enc1.b / dec1.b of the 3-D model at width/2 and their
// data gradients; BASELINE config #5, SURVEY K21: nn.Conv3d(32, 32, 3, padding=1)) — as a
// DEPTH-STREAMING RESIDENT kernel.
//
// The streaming kernel (conv3x3_fwd.hip) tiles 3-D boxes and re-stages each box's
// (TD+2)(TH+2)(TW+2) halo (2.5x the box) per 32-channel chunk, and streams the 27 x 32 x 32
// weights through LDS per (kd, kh) stage.  Here one persistent workgroup per CU owns whole
// tile COLUMNS: a 16 x 16 (h, w) tile of one volume, marched through every depth d.  Its LDS
// holds
//   * all 27 x 32 x 32 weights (55 KB, loaded once per workgroup), and
//   * a ring of four 18 x 18 x 32 input PLANES (20.7 KB each): planes d-1, d, d+1 serve
//     output plane d while plane d+2 arrives by LDS-DMA (buffer_load ... lds) —
// so every input plane is read from HBM once per column (1.27x for the (h, w) halo only) and
// the output plane costs one barrier.  8 waves (two per SIMD), each 32 pixels x 32 output
// channels of v_mfma_f32_16x16x32_bf16; fragment addresses are per-lane registers plus
// immediates (the plane halo is swizzled by its COLUMN, conflict-free 16-pixel reads); the
// previous layer's BatchNorm + ReLU (prologue) is applied in place by the lanes that DMA'd each
// piece, padding left zero; the epilogue stores bf16 and accumulates the BN (sum, sum^2) of the
// fp32 outputs, one statistics row per workgroup (conv3_fwd_kernel's contract).
//
// More than 32 output channels (enc2.a's 32 -> 64 forward at 64^3, dec1.a's 32 -> 96 data
// gradient at 128^3 — its outputs split at Co1 into the two concat inputs' gradients): work
// items are (32-channel output chunk, column) pairs dealt to the workgroups as even contiguous
// ranges of the chunk-major order; at a chunk change the workgroup re-loads that chunk's
// 27 x 32 x 32 weight slice and bias and flushes the finished chunk's statistics into its row
// ([grid][2][Cout]; chunks it never met stay zero).
#include "common.h"
#include "conv_lds.h"
#include "ops.h"

namespace ddlpc {

namespace {

using namespace convlds;

constexpr int DS_T = 16, DS_HW2 = 18;                 // 16 x 16 (h, w) tiles
constexpr int DS_HALO = DS_HW2 * DS_HW2;              // 324 pixels per plane halo
constexpr int DS_INSTR = (DS_HALO * 4 + 63) / 64;     // 21 DMA wave-instructions per plane
constexpr int DS_ITERS = (DS_INSTR + 7) / 8;          // per wave: 3 (waves 0-4) or 2
constexpr int DS_PBYTES = DS_INSTR * 1024;            // one plane slot
constexpr int DS_WBYTES = 27 * 32 * ROWB;             // resident weights: rows (tap, co)
constexpr int DS_SMEM = 2 * 32 * 4 + DS_WBYTES + 4 * DS_PBYTES;

__global__ __launch_bounds__(512, 1) void conv3d_ds_kernel(ConvFwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_pro = reinterpret_cast<float*>(smem);                 // prologue scale | shift [2][32]
  char* sW = smem + 2 * 32 * 4;
  char* sP = sW + DS_WBYTES;
  auto slot = [&](int plane) { return sP + (plane & 3) * DS_PBYTES; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesH = (p.H + DS_T - 1) / DS_T, tilesW = (p.W + DS_T - 1) / DS_T;
  const int ncol = p.N * tilesH * tilesW;
  const int nco = p.Cout / 32;                       // output chunks
  const int it_begin = (int)((long long)nco * ncol * blockIdx.x / gridDim.x);
  const int it_end = (int)((long long)nco * ncol * (blockIdx.x + 1) / gridDim.x);
  const long long plane_px = (long long)p.H * p.W;
  const long long vol_px = (long long)p.D * plane_px;
  const bool has_pro = p.pscale != nullptr;
  if (has_pro && tid < 32) { s_pro[tid] = p.pscale[tid]; s_pro[32 + tid] = p.pshift[tid]; }
  // ---- resident weights of output chunk cc: row (tap, co) of 32 ci, piece q at q ^ swz(co)
  auto load_weights = [&](int cc) {
    const auto rW = make_rsrc(p.Wt, (unsigned)(p.Cout * 27 * p.CinW * 2));
    for (int b = wave * 64; b < DS_WBYTES / 16; b += 512) {
      const int e = b + lane;
      const int row = e >> 2;
      const int t = row >> 5, co = row & 31;
      const int sub = (e & 3) ^ swz(co);
      dma16(rW, sW + b * 16, (unsigned)(((cc * 32 + co) * 27 + t) * p.CinW + sub * 8) * 2u);
    }
  };

  // ---- plane DMA: piece e = (i * 8 + wave) * 64 + lane -> halo pixel e >> 2, its channel
  // piece (e & 3) ^ swz(column) (the column swizzle: see the header)
  const int nins = (DS_INSTR - wave + 7) / 8;
  uint32_t vmasks = 0;                               // in-image pieces per ring slot, 8 bits each
  int col_n = 0, col_h0 = 0, col_w0 = 0;             // the current column
  auto issue = [&](int d) {
    const auto r = make_rsrc(p.X1 + (long long)col_n * vol_px * 32, (unsigned)(vol_px * 64));
    uint32_t valid = 0;
#pragma unroll
    for (int i = 0; i < DS_ITERS; ++i) {
      if (i * 8 + wave >= DS_INSTR) break;           // (wave-uniform)
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int hc = px % DS_HW2;
      const int gh = col_h0 + px / DS_HW2 - 1, gw = col_w0 + hc - 1;
      const bool ok = px < DS_HALO && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W;
      const unsigned pix = (unsigned)(d * plane_px + gh * p.W + gw);
      dma16(r, slot(d) + (i * 8 + wave) * 1024, ok ? (pix * 32 + (((lane & 3) ^ swz(hc)) << 3)) * 2u : kOOB);
      valid |= (ok ? 1u : 0u) << i;
    }
    vmasks = (vmasks & ~(0xffu << (8 * (d & 3)))) | (valid << (8 * (d & 3)));
  };
  // prologue BN + ReLU on this lane's own landed pieces of plane d (its 8 channels:
  // ((lane & 3) ^ swz(column)) * 8), padding re-zeroed
  auto transform_body = [&](char* __restrict__ P, int d) __attribute__((always_inline)) {
    const uint32_t valid = (vmasks >> (8 * (d & 3))) & 0xffu;
    uint4 v[DS_ITERS];
#pragma unroll
    for (int i = 0; i < DS_ITERS; ++i)
      if (i * 8 + wave < DS_INSTR) v[i] = *reinterpret_cast<const uint4*>(P + ((i * 8 + wave) * 64 + lane) * 16);
#pragma unroll
    for (int i = 0; i < DS_ITERS; ++i) {
      if (i * 8 + wave >= DS_INSTR) break;
      const int px = ((i * 8 + wave) * 64 + lane) >> 2;
      const int c8 = ((lane & 3) ^ swz(px % DS_HW2)) * 8;
      const float4* kp = reinterpret_cast<const float4*>(s_pro + opaque_zero() + c8);
      const float4 sa = kp[0], sb = kp[1], ha = kp[8], hb = kp[9];
      const float sc[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
      const float sh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
      const bool ok = (valid >> i) & 1u;
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x2_t x = {lo_bf(w[j]), hi_bf(w[j])};
        const f32x2_t y2 = __builtin_elementwise_fma(x, f32x2_t{sc[2 * j], sc[2 * j + 1]},
                                                     f32x2_t{sh[2 * j], sh[2 * j + 1]});
        const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(y2, bf16x2_t));
        const i16x2_t m = __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, pk), i16x2_t{0, 0});
        o[j] = ok ? __builtin_bit_cast(uint32_t, m) : 0u;
      }
      *reinterpret_cast<uint4*>(P + ((i * 8 + wave) * 64 + lane) * 16) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };

  // ---- fragments: wave w owns tile rows 2w, 2w + 1 (MT = 2) x 32 co (NT = 2); A = weights
  // (rows co), B = plane-halo pixels (K = 32 ci).  Per-lane offsets for the three tap columns
  // dw (the row, tap-row and tap terms are immediates)
  const int g = lane >> 4, c16 = lane & 15;
  int xo[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) xo[dw] = (2 * wave * DS_HW2 + c16 + dw) * ROWB + ((g ^ swz(c16 + dw)) << 4);
  const int wo = c16 * ROWB + ((g ^ swz(c16)) << 4);
  float st1[2][4], st2[2][4];                        // BN statistics of this workgroup's outputs
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) { st1[nt][i] = 0.f; st2[nt][i] = 0.f; }
  const bool want_stats = p.stats != nullptr;
  // bias of the lane's output channels of chunk cc, loaded before any DMA of the chunk (a
  // global load in the epilogue would make the compiler drain the in-flight plane DMA first)
  float bias_r[2][4];
  auto load_bias = [&](int cc) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) bias_r[nt][i] = p.bias != nullptr ? p.bias[cc * 32 + nt * 16 + 4 * g + i] : 0.f;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      asm volatile("" ::"v"(bias_r[nt][0]), "v"(bias_r[nt][1]), "v"(bias_r[nt][2]), "v"(bias_r[nt][3]));
  };
  // the current chunk's output tensor (Y1: channels < Co1, else Y2), its channel count and
  // the chunk's channel offset in it
  bf16_t* ybase = p.Y1;
  int ych = p.Co1, yoff = 0;

  auto compute = [&](int d, const char* __restrict__ Pm, const char* __restrict__ P0,
                     const char* __restrict__ Pp, const char* __restrict__ Wc) __attribute__((always_inline)) {
    f32x4_t acc[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // planes d - 1 / d + 1 exist? (wave-uniform: the kd taps past the volume are skipped)
    const bool lo_ok = d > 0, hi_ok = d + 1 < p.D;
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      if ((kd == 0 && !lo_ok) || (kd == 2 && !hi_ok)) continue;
      const char* __restrict__ P = kd == 0 ? Pm : kd == 1 ? P0 : Pp;
      uint4 xf[2][2], wf[2][2];
      auto load = [&](int j, uint4 (&x)[2], uint4 (&w)[2]) __attribute__((always_inline)) {
        const int dh = j / 3, dw = j % 3;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) x[mt] = lds128(P + xo[dw] + (mt + dh) * DS_HW2 * ROWB);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) w[nt] = lds128(Wc + wo + ((kd * 9 + j) * 32 + nt * 16) * ROWB);
      };
      load(0, xf[0], wf[0]);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        if (j + 1 < 9) load(j + 1, xf[(j + 1) & 1], wf[(j + 1) & 1]);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma16x16x32(wf[j & 1][nt], xf[j & 1][mt], acc[mt][nt]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // epilogue: + bias, bf16 16-byte channel-pair stores, BN statistics of the fp32 values
    // (lane: channels nt*16 + 4g .. + 3 of pixel c16 of tile row 2w + mt)
    const auto ry = make_rsrc(ybase + (long long)col_n * vol_px * ych, (unsigned)(vol_px * ych * 2));
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int gh = col_h0 + 2 * wave + mt, gw = col_w0 + c16;
      const bool ok = gh < p.H && gw < p.W;
      uint2 pk[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[mt][nt][i] + bias_r[nt][i];
          const float z = ok ? v[i] : 0.f;
          st1[nt][i] += z;
          st2[nt][i] = fmaf(z, z, st2[nt][i]);
        }
        pk[nt] = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
      const uint4 q = pair16(pk[0], pk[1]);
      unsigned off = ok ? (unsigned)((d * plane_px + gh * p.W + gw) * ych + yoff + pair16_ch(lane)) * 2u : kOOB;
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{q.x, q.y, q.z, q.w}, ry, off, 0, 0);
    }
  };

  // ---- one BN-statistics row per workgroup and output chunk: 16 pixel lanes, then the 8
  // waves (fixed order) — after every DMA landed and every wave is done with the planes (the
  // reduction reuses the plane ring)
  auto flush_stats = [&](int cc) {
    dma_wait<0>();
    lds_sync();
    float* red = reinterpret_cast<float*>(sP);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a1 = row16_sum(st1[nt][i]), a2 = row16_sum(st2[nt][i]);
        st1[nt][i] = 0.f;
        st2[nt][i] = 0.f;
        if (c16 == 0) {
          const int co = nt * 16 + 4 * g + i;
          red[(wave * 2) * 32 + co] = a1;
          red[(wave * 2 + 1) * 32 + co] = a2;
        }
      }
    lds_sync();
    if (tid < 64) {
      const int half = tid >> 5, co = tid & 31;
      float v = 0.f;
      for (int w = 0; w < 8; ++w) v += red[(w * 2 + half) * 32 + co];
      p.stats[((long long)blockIdx.x * 2 + half) * p.Cout + cc * 32 + co] = v;
    }
    lds_sync();
  };

  // ---- items (output chunk, column) it_begin .. it_end, each column marched through
  // d = 0 .. D-1.  Counted waits from a per-wave ledger of issued vector-memory ops (a plane:
  // nins DMAs; a step's epilogue: 2 stores)
  __syncthreads();                                   // prologue constants visible
  int issued = 0;
  int cc = -1;
  uint32_t met = 0;                                  // output chunks of this workgroup
  for (int it = it_begin; it < it_end; ++it) {
    const int ck = it / ncol, c = it - ck * ncol;
    if (ck != cc) {                                  // (the previous item ended with a barrier)
      if (cc >= 0 && want_stats) flush_stats(cc);
      cc = ck;
      met |= 1u << ck;
      load_bias(ck);
      load_weights(ck);
      const bool second = ck * 32 >= p.Co1;
      ybase = second ? p.Y2 : p.Y1;
      ych = second ? p.Cout - p.Co1 : p.Co1;
      yoff = second ? ck * 32 - p.Co1 : ck * 32;
      dma_wait<0>();
      lds_sync();                                    // weights visible
    }
    col_n = c / (tilesH * tilesW);
    const int rr = c - col_n * tilesH * tilesW;
    col_h0 = (rr / tilesW) * DS_T;
    col_w0 = (rr % tilesW) * DS_T;
    // planes 0 and 1; m0 / m1 = ledger counts right after the DMAs of planes d + 1, d + 2
    issue(0);
    issued += nins;
    const int m_p0 = issued;
    int m1 = m_p0;                                   // plane 1's mark (plane d + 1 at d = 0)
    if (p.D > 1) { issue(1); issued += nins; m1 = issued; }
    vm_wait_dyn(issued - m_p0);                      // plane 0 landed
    if (has_pro) transform_body(slot(0), 0);
    int m0 = m1;                                     // mark of plane d + 1 (d = 0: plane 1)
    for (int d = 0; d < p.D; ++d) {
      if (d + 1 < p.D) {
        vm_wait_dyn(issued - m0);                    // plane d + 1 landed
        if (has_pro) transform_body(slot(d + 1), d + 1);
      }
      lds_sync();                                    // planes visible; step d - 1 done by all
      int m2 = m0;
      if (d + 2 < p.D) {                             // into the slot of plane d - 2
        issue(d + 2);
        issued += nins;
        m2 = issued;
      }
      compute(d, slot(d + 3), slot(d), slot(d + 1), sW);   // (plane d - 1 = slot (d + 3) & 3)
      issued += 2;                                   // the two epilogue stores
      m0 = m2;
    }
    lds_sync();                                      // the column's last planes read by all
  }
  if (want_stats) {
    if (cc >= 0) flush_stats(cc);
    if (tid < 64)                                    // chunks this workgroup never met
      for (int k = 0; k < nco; ++k)
        if (!((met >> k) & 1u)) p.stats[((long long)blockIdx.x * 2 + (tid >> 5)) * p.Cout + k * 32 + (tid & 31)] = 0.f;
  }
}

}  // namespace

// planner: the 3-D layers with 32 input channels and 32-channel output chunks (outputs split
// at Co1 on a chunk boundary) with enough (chunk, column) items to fill the chip (one per CU
// at least); -1 = the streaming kernel
int conv3d_ds_plan(const ConvFwdArgs& a, int num_cus, int& grid, int& smem) {
  if (a.dims != 3 || a.C1 != 32 || a.C2 != 0 || a.Cin != 32 || a.Cout % 32 != 0 || a.Cout > 32 * 32 ||
      a.Co1 % 32 != 0 || a.CinW != 32 || a.pscale2 != nullptr || a.bnb_y != nullptr || a.groups > 1)
    return -1;
  if ((long long)a.D * a.H * a.W * a.Cout * 2 >= (1LL << 31)) return -1;
  const long long items = (long long)(a.Cout / 32) * a.N * ((a.H + DS_T - 1) / DS_T) * ((a.W + DS_T - 1) / DS_T);
  if (items < num_cus || items >= (1LL << 31)) return -1;
  grid = num_cus;
  smem = DS_SMEM;
  return 0;
}

void conv3d_ds_launch(ConvFwdArgs& a, int grid, int smem, hipStream_t st) {
  hipLaunchKernelGGL(conv3d_ds_kernel, dim3(grid), dim3(512), smem, st, a);
}

}  // namespace ddlpc
