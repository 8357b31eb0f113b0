// Host-side AddressSanitizer + UndefinedBehaviorSanitizer check of the launch planners
// (SURVEY.md §5.2 "host-side ASan for the C++ extension").  GPU ASan is not available on
// this pool, so the device code is covered by the guard-buffer bounds tests
// (tests/test_kernels_gpu.py::test_out_params_respect_bounds); this harness covers the host
// code that decides grids, tiles, LDS sizes and split counts for every kernel, sweeping the
// geometry range the U-Net uses (2-D 8^2..1024^2, 3-D 8^3..128^3, batch 1..256) and
// asserting the invariants the kernels rely on.  No GPU is touched (no HIP API calls).
//
// Build + run (scripts/host_sanitize.sh):
//   hipcc --offload-arch=gfx950 -O1 -g -Xarch_host -fsanitize=address \
//         -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all ...
#include <cstdio>
#include <cstdlib>

#include "../csrc/ops.h"

using namespace ddlpc;

// the planners read tuning knobs; bindings.cpp (torch-linked) is not part of this harness,
// so knobs resolve to their DDLPC_<NAME> environment value or the default here
int ddlpc::knob(const char* name, int def) {
  char env[128];
  std::snprintf(env, sizeof(env), "DDLPC_%s", name);
  const char* e = std::getenv(env);
  return e ? std::atoi(e) : def;
}

static long long g_checks = 0;
#define EXPECT(c, ...)                                                              \
  do {                                                                              \
    ++g_checks;                                                                     \
    if (!(c)) {                                                                     \
      std::fprintf(stderr, "FAIL %s:%d: %s  ", __FILE__, __LINE__, #c);             \
      std::fprintf(stderr, __VA_ARGS__);                                            \
      std::fprintf(stderr, "\n");                                                   \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

static const int kCUs = 256;
static const int kLds = 160 * 1024;

static void sweep_conv_fwd() {
  const int chans[][3] = {  // C1, C2, Cout (U-Net widths, both directions, concat layers)
      {8, 0, 32},    {32, 0, 32},   {32, 0, 64},   {64, 0, 64},   {64, 0, 128},
      {128, 0, 128}, {128, 0, 256}, {256, 0, 256}, {256, 256, 256}, {256, 128, 128},
      {128, 64, 64}, {64, 32, 32},  {32, 0, 8},    {64, 0, 32},   {128, 0, 64},
      {256, 0, 128}, {512, 0, 256}, {384, 0, 128}, {96, 0, 32},   {192, 0, 64}};
  const int sizes[] = {8, 16, 24, 32, 40, 64, 72, 128, 200, 256, 512, 1024};
  const int batches[] = {1, 2, 8, 32, 128, 256};
  for (auto& ch : chans)
    for (int hw : sizes)
      for (int n : batches) {
        for (int pro = 0; pro < 2; ++pro) {
          ConvFwdArgs a{};
          a.dims = 2; a.N = n; a.D = 1; a.H = hw; a.W = hw;
          a.C1 = ch[0]; a.C2 = ch[1]; a.Cin = a.C1 + a.C2;
          a.CinW = (a.Cin + 7) / 8 * 8;
          a.Cout = ch[2]; a.Co1 = ch[2]; a.taps = 9;
          static float dummy = 0.f;
          a.pscale = pro ? &dummy : nullptr;
          a.pshift = pro ? &dummy : nullptr;
          a.npix = (long long)n * hw * hw;
          int grid = 0, smem = 0;
          const int v = conv3_res_plan(a, kCUs, grid, smem);
          if (v < 0) continue;
          EXPECT(grid > 0 && grid <= 2 * kCUs, "grid=%d C=%d/%d/%d hw=%d n=%d", grid, ch[0], ch[1], ch[2], hw, n);
          EXPECT(smem > 0 && smem <= kLds, "smem=%d", smem);
          EXPECT(grid % a.nTilesN == 0, "grid %d not a multiple of nTilesN %d", grid, a.nTilesN);
          EXPECT((long long)a.tilesH * a.TH >= a.H && (long long)a.tilesW * a.TW >= a.W,
                 "tiles do not cover the image");
          EXPECT(a.nTilesM == a.N * a.tilesH * a.tilesW, "nTilesM");
        }
      }
  for (int cfg = 0; cfg <= 4; ++cfg) {
    EXPECT(conv3_fwd_cfg_bm(cfg) > 0 && conv3_fwd_cfg_bn(cfg) > 0, "cfg %d", cfg);
    EXPECT(conv3_fwd_cfg_halo(2, cfg) > 0, "halo cfg %d", cfg);
  }
}

static void sweep_wgrad() {
  const int c2s[] = {0, 32, 64, 128, 256};
  const int sizes[] = {16, 24, 32, 64, 128, 256, 512, 1024};
  for (int bco : {32, 64})
    for (int c2 : c2s)
      for (int hw : sizes) {
        const int pt = conv3_wgrad2_pt(bco, c2, hw, hw);
        EXPECT(pt == 64 || pt == 96 || pt == 128 || pt == 256, "pt=%d", pt);
        EXPECT(pt % 16 == 0, "pixel tile must be whole 16-wide rows");
      }
  EXPECT(conv3_wgrad_halo_cap(2) > 0 && conv3_wgrad_halo_cap(3) > 0, "halo caps");
}

static void sweep_reductions() {
  for (long long items = 1; items < (1LL << 34); items = items * 3 + 1) {
    const int nb = bn_bwd_reduce_blocks(items);
    EXPECT(nb >= 1 && nb <= 2048, "nb=%d items=%lld", nb, items);
  }
  for (int r = 1; r < (1 << 20); r = r * 2 + 1) {
    const int ch = reduce_rows_chunks(r);
    EXPECT(ch >= 1 && ch <= r, "chunks=%d rows=%d", ch, r);
  }
  EXPECT(head_supported(32, 6), "flagship head (32 -> 6 classes)");
  EXPECT(!head_supported(7, 6), "head rejects C %% 8 != 0");
}

int main() {
  sweep_conv_fwd();
  sweep_wgrad();
  sweep_reductions();
  std::printf("host_sanitize: %lld planner checks passed (ASan + UBSan)\n", g_checks);
  return 0;
}
